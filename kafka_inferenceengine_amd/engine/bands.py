"""Assembly of per-band kernel descriptors (``BandDesc``) from an operator
spec (``models.operators.OperatorSpec``) and device-resident observations.

An observation band on the active-pixel grid is either the compact Sentinel-2
encoding — uint16 digital numbers, reflectance = DN x scale, validity DN > 0,
sigma = max(rel_unc x reflectance, floor) (``Sentinel2_Observations.py:163-179``)
— decoded inside the analysis kernel, or explicit float32 ``(y, w, mask)``
with ``w`` the inverse variance (the reference's ``uncertainty``).
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace

import numpy as np
import torch

from ..models.gp import mfma_tables
from ..models.operators import OP_GP, OP_LINEAR, OP_PRECOMP, OP_SAR, OperatorSpec
from ..ops import kernels as K


@dataclass
class DeviceBand:
    """One observation band on the active-pixel grid (device or CPU tensors)."""
    kind: int                                   # K.OBS_DN16 | K.OBS_F32 | K.OBS_BF16 | K.OBS_BF16Y
    dn: torch.Tensor | None = None              # uint16 bit patterns, stored as int16 [N]
    y: torch.Tensor | None = None               # float32 [N]
    w: torch.Tensor | None = None               # float32 [N] inverse variance
    mask: torch.Tensor | None = None            # uint8 [N]
    scale: float = 1e-4
    rel_unc: float = 0.05
    unc_floor: float = 0.0
    metadata: dict = field(default_factory=dict)
    emulator: object = None
    aux: torch.Tensor | None = None             # float32 [N] (SAR incidence angle)

    @property
    def device(self):
        t = self.dn if self.dn is not None else self.y
        return t.device

    def decode(self):
        """(y, w) float32 on the same device (host-side reference of decode_obs)."""
        if self.kind == K.OBS_DN16:
            dn = self.dn.to(torch.int32) & 0xFFFF
            y = dn.to(torch.float32) * self.scale
            sig = torch.clamp(self.rel_unc * y, min=self.unc_floor)
            valid = (dn > 0) & (sig > 0)
            w = torch.where(valid, 1.0 / torch.where(valid, sig * sig, torch.ones_like(sig)), torch.zeros_like(y))
            return torch.where(dn > 0, y, torch.zeros_like(y)), w
        if self.kind == K.OBS_BF16Y:
            yy = (self.y.to(torch.int32) << 16).view(torch.float32)
            sig = torch.clamp(self.rel_unc * yy.abs(), min=self.unc_floor)
            ok = torch.isfinite(yy) & (sig > 0)
            if self.mask is not None:
                ok = ok & self.mask.bool()
            w = torch.where(ok, 1.0 / torch.where(ok, sig * sig, torch.ones_like(sig)), torch.zeros_like(yy))
            return torch.where(ok, yy, torch.zeros_like(yy)), w
        if self.kind == K.OBS_BF16:
            yy = (self.y.to(torch.int32) << 16).view(torch.float32)
            w = (self.w.to(torch.int32) << 16).view(torch.float32)
        else:
            yy, w = self.y, self.w.clone()
        if self.mask is not None:
            w = torch.where(self.mask.bool(), w, torch.zeros_like(w))
        bad = ~torch.isfinite(w) | ~(w > 0) | ~torch.isfinite(yy)
        return torch.where(bad, torch.zeros_like(yy), yy), torch.where(bad, torch.zeros_like(w), w)

    def _decode_f32(self):
        w = self.w.clone()
        if self.mask is not None:
            w = torch.where(self.mask.bool(), w, torch.zeros_like(w))
        bad = ~torch.isfinite(w) | ~(w > 0) | ~torch.isfinite(self.y)
        return torch.where(bad, torch.zeros_like(self.y), self.y), torch.where(bad, torch.zeros_like(w), w)


class RecordCache:
    """Uploads GP training records (and their split-f16 MFMA tables) once per
    (emulator, device)."""

    def __init__(self):
        self._c = {}
        self._m = {}

    def get_mfma(self, spec: OperatorSpec, device):
        """(table tensor, n_chunks, scale) of the matrix-core GP path, or None
        (D > 10, or values outside f16 range; the VALU loop is the analysis
        variant Variant.VALU_ORACLE)."""
        key = (id(spec.emulator) if spec.emulator is not None else id(spec.records), str(device))
        hit = self._m.get(key)
        if hit is None:
            built = mfma_tables(spec.records, spec.gp_pos_pairs, spec.coef)
            if built is None:
                hit = (None, spec.records)
            else:
                tab, nch, scale = built
                # + one zero fragment after the chunks (the global-table kernel's
                # rows past D read it: kf_gp_mfma.h:gp_mfma_sums_g)
                flat = np.concatenate([np.ascontiguousarray(tab).reshape(-1, 8), np.zeros((1, 8), np.float16)])
                t = torch.from_numpy(flat.view(np.int16)).to(device)
                hit = ((t, nch, scale), spec.records)
            self._m[key] = hit
        return hit[0]

    def get(self, spec: OperatorSpec, device) -> torch.Tensor:
        key = (id(spec.emulator) if spec.emulator is not None else id(spec.records), str(device))
        t = self._c.get(key)
        if t is None:
            t = torch.from_numpy(np.ascontiguousarray(spec.records, dtype=np.float32)).to(device)
            self._c[key] = (t, spec.records)  # keep the source alive so id() stays unique
        else:
            t = t[0]
        return t


def band_desc(spec: OperatorSpec, obs: DeviceBand | None, n_params: int, cache: RecordCache, h0_out=None,
              pre_h0=None, pre_h=None, device=None, aux=None):
    """Build one ``BandDesc``; returns (desc, tensors to keep alive)."""
    E = K.ext()
    d = E.BandDesc()
    keep = []
    device = obs.device if obs is not None else device
    d.op = int(spec.kind)
    if obs is not None:
        d.obs = int(obs.kind)
        d.scale, d.rel_unc, d.unc_floor = float(obs.scale), float(obs.rel_unc), float(obs.unc_floor)
    d.offset = float(spec.offset)
    if spec.kind == OP_GP:
        if spec.d > 12 or spec.d > n_params:
            raise ValueError(f"GP with {spec.d} inputs exceeds the compiled limit for n_params={n_params}")
        rec = cache.get(spec, device)
        if rec.dim() != 3 or rec.shape[1] != spec.d + 1 or rec.shape[2] != 2:
            raise ValueError(f"GP records must be [T/2, d+1, 2], got {tuple(rec.shape)}")
        if not 0 <= int(spec.gp_pos_pairs) <= int(rec.shape[0]):
            raise ValueError(f"gp_pos_pairs={spec.gp_pos_pairs} outside [0, {rec.shape[0]}]")
        d.d, d.T, d.Tp = spec.d, 2 * int(rec.shape[0]), int(spec.gp_pos_pairs)
        d.gp = rec.data_ptr()
        keep.append(rec)
        mt = cache.get_mfma(spec, device)
        if mt is not None:
            d.gpm, d.gpm_nchunk, d.gpm_scale = mt[0].data_ptr(), int(mt[1]), float(mt[2])
            keep.append(mt[0])
    elif spec.kind == OP_SAR:
        d.d, d.T = 2, 0
    elif spec.kind == OP_LINEAR:
        d.d, d.T = n_params, 0
    elif spec.kind == OP_PRECOMP:
        if pre_h0 is None or pre_h is None:
            raise ValueError("precomputed operator needs pre_h0/pre_h")
        d.pre_h0, d.pre_h, d.pre_ld = pre_h0.data_ptr(), pre_h.data_ptr(), int(pre_h.shape[1])
        keep += [pre_h0, pre_h]
    else:
        raise ValueError(f"unknown operator kind {spec.kind}")
    smap = [int(i) for i in spec.state_map]
    if any(i < 0 or i >= n_params for i in smap):
        raise ValueError(f"state map {smap} out of range for n_params={n_params}")
    d.map = smap
    d.map_identity = int(len(smap) >= int(d.d) > 0 and smap[:int(d.d)] == list(range(int(d.d))))
    # compile-time JRC-TIP maps (kf_core.h GPM_MAP_*): only for 7-parameter states
    d.map_kind = 0
    if spec.kind == OP_GP and n_params == 7 and int(d.d) == 4:
        d.map_kind = {(0, 1, 6, 2): 2, (3, 4, 6, 5): 3}.get(tuple(smap[:4]), 0)
    d.coef = [float(c) for c in spec.coef]
    d.center = [float(c) for c in spec.center]
    if spec.kind == OP_GP and getattr(spec, "domain_lo", None) is not None:
        d.dom_lo, d.dom_hi = [float(v) for v in spec.domain_lo], [float(v) for v in spec.domain_hi]
        d.dom_check = 1
    if obs is None:
        d.obs = K.OBS_NONE
    elif obs.kind == K.OBS_DN16:
        d.dn = obs.dn.data_ptr()
        keep.append(obs.dn)
    else:
        d.y, d.w = obs.y.data_ptr(), (obs.w.data_ptr() if obs.w is not None else 0)
        keep += [t for t in (obs.y, obs.w) if t is not None]
        if obs.mask is not None:
            d.mask = obs.mask.data_ptr()
            keep.append(obs.mask)
    aux = obs.aux if (obs is not None and obs.aux is not None) else aux
    if spec.kind == OP_SAR and aux is not None:
        d.aux = aux.data_ptr()
        keep.append(aux)
    if h0_out is not None:
        d.h0_out = h0_out.data_ptr()
        keep.append(h0_out)
    return d, keep


def _ptr(t):
    return 0 if t is None else t.data_ptr()


class TableCache:
    """Band descriptor tables by content: a table holds only pointers and
    scalars, so two dates whose bands sit in the same buffers (streamer slots,
    resident pools) with the same operators share one device table.  The key
    is every descriptor input (operator spec identity, observation encoding and
    scalars, tensor addresses); cached tables do not keep observation tensors
    alive (an address that is reused by a later band IS that band's buffer).
    Specs are held so their ids stay unique while cached."""

    def __init__(self, size: int = 16):
        from collections import OrderedDict
        self.size = size
        self._d = OrderedDict()
        self.hits = self.misses = 0

    @staticmethod
    def key(specs, obs_list, n_params, device):
        return (n_params, str(device)) + tuple(
            (id(sp), ob.kind, _ptr(ob.dn), _ptr(ob.y), _ptr(ob.w), _ptr(ob.mask), _ptr(ob.aux), float(ob.scale),
             float(ob.rel_unc), float(ob.unc_floor)) for sp, ob in zip(specs, obs_list))

    def get(self, specs, obs_list, n_params, cache, device) -> K.BandTable:
        k = self.key(specs, obs_list, n_params, device)
        hit = self._d.get(k)
        if hit is not None:
            self._d.move_to_end(k)
            self.hits += 1
            return hit[0]
        self.misses += 1
        tab = build_table(specs, obs_list, n_params, cache, device)
        # keep the GP record / MFMA tables (cache-owned) and the specs, not the observations
        obs_ids = {id(t) for ob in obs_list for t in (ob.dn, ob.y, ob.w, ob.mask, ob.aux) if t is not None}
        tab = replace(tab, keepalive=tuple(t for t in tab.keepalive if id(t) not in obs_ids))
        self._d[k] = (tab, tuple(specs))
        while len(self._d) > self.size:
            self._d.popitem(last=False)
        return tab


def build_table(specs, obs_list, n_params, cache, device, h0_outs=None, pre=None) -> K.BandTable:
    descs, keep = [], []
    want = torch.device(device)
    for i, (spec, ob) in enumerate(zip(specs, obs_list)):
        for t in (ob.dn, ob.y, ob.w, ob.mask, ob.aux):
            if t is not None and (t.device.type != want.type or
                                  (want.type == "cuda" and want.index is not None and t.device.index != want.index)):
                raise ValueError(f"band {i}: observation tensor on {t.device}, engine runs on {want}")
        h0 = None if h0_outs is None else h0_outs[i]
        ph0, ph = (None, None) if pre is None or pre[i] is None else pre[i]
        dsc, kp = band_desc(spec, ob, n_params, cache, h0, ph0, ph)
        descs.append(dsc)
        keep += kp
    return K.make_band_table(descs, device, keep, specs)


def operator_table(specs, n_params, cache, device, aux=None) -> K.BandTable:
    """Descriptors for operator evaluation only (no observations attached)."""
    descs, keep = [], []
    for spec in specs:
        dsc, kp = band_desc(spec, None, n_params, cache, device=device, aux=aux)
        descs.append(dsc)
        keep += kp
    return K.make_band_table(descs, device, keep)
