"""Synthetic observation sources with the reference observation protocol.

No satellite data ships with the reference (its drivers read private paths,
SURVEY.md §4), so every sensor here is synthetic but *shaped* like the real
reader:

* ``SyntheticObservations`` — generic source: a spatially smooth "truth" state
  field (deterministic in the global pixel index, so any strip partition sees
  the same data), pushed through each band's observation operator (the same
  gfx950 kernel the analysis uses), perturbed with relative Gaussian noise,
  quantised like Sentinel-2 L2A (uint16 DN, reflectance = DN x 1e-4, 0 = no
  data) and cut by spatially coherent clouds.
* ``SyntheticS2Observations`` / ``SyntheticBHRObservations`` /
  ``SyntheticS1Observations`` / ``SyntheticOLCIObservations`` — presets
  mirroring ``Sentinel2_Observations.py``, ``observations.py:214-310``
  (MCD43 BHR), ``Sentinel1_Observations.py`` and an OLCI-like 21-band sensor.

Protocol: ``dates``, ``bands_per_observation``, ``get_band_data(date, band)``
(reference namedtuple on the strip raster) and the device fast path
``get_device_band_data(date, band)`` / ``prefetch(date)``.
"""
from __future__ import annotations

import datetime as dt
import math

import numpy as np
import scipy.sparse as sp
import torch

from ..engine.bands import DeviceBand, RecordCache
from ..models.gp import GaussianProcessEmulator
from ..models.operators import OP_GP, OperatorSpec, gp_spec
from ..ops import kernels as K
from .streaming import DateStreamer

from .records import S2MSIdata

M32 = 0xFFFFFFFF


def _hash(x: torch.Tensor) -> torch.Tensor:
    x = x & M32
    x = ((x ^ (x >> 16)) * 0x45D9F3B) & M32
    x = ((x ^ (x >> 16)) * 0x45D9F3B) & M32
    return x ^ (x >> 16)


def hash_normal(gidx: torch.Tensor, salt: int) -> torch.Tensor:
    """Counter-based N(0,1) per global pixel index (partition independent)."""
    s = (salt * 0x9E3779B1) & M32
    h1 = _hash(gidx * 2 + s)
    h2 = _hash(gidx * 2 + 1 + s)
    u1 = (h1.to(torch.float64) + 0.5) / 4294967296.0
    u2 = (h2.to(torch.float64) + 0.5) / 4294967296.0
    return (torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(2 * math.pi * u2)).to(torch.float32)


class SmoothField:
    """Bilinear interpolation of a coarse N(0,1) grid: deterministic, smooth,
    evaluated only at the requested global pixels."""

    def __init__(self, shape, cell: int, seed: int):
        H, W = shape
        self.cell = max(1, int(cell))
        gh, gw = H // self.cell + 2, W // self.cell + 2
        rng = np.random.default_rng(seed)
        self.grid = torch.from_numpy(rng.standard_normal((gh, gw)).astype(np.float32))
        self.W = W

    def at(self, gidx: torch.Tensor) -> torch.Tensor:
        g = self.grid.to(gidx.device)
        r = (gidx // self.W).to(torch.float32) / self.cell
        c = (gidx % self.W).to(torch.float32) / self.cell
        r0, c0 = r.floor().long(), c.floor().long()
        fr, fc = r - r0, c - c0
        gw = g.shape[1]
        flat = g.reshape(-1)

        def G(rr, cc):
            return flat[rr * gw + cc]
        top = G(r0, c0) * (1 - fc) + G(r0, c0 + 1) * fc
        bot = G(r0 + 1, c0) * (1 - fc) + G(r0 + 1, c0 + 1) * fc
        return top * (1 - fr) + bot * fr


class SyntheticObservations:
    """Generic synthetic multi-band source (see module docstring)."""

    sensor = "synthetic"
    band_specs_static = True     # band_spec(date, b) does not depend on the date

    def __init__(self, state_mask, dates, band_specs, truth_center, truth_spread, truth_lo=None, truth_hi=None,
                 *, partition=None, encoding: str = "dn16", scale: float = 1e-4, rel_unc: float = 0.05,
                 unc_floor: float = 0.0, cloud_fraction: float = 0.2, seed: int = 0, device=None,
                 n_pool: int | None = None, stream: bool = True, field_cell: int = 64, metadata=None,
                 temporal_params=(), aux=None):
        from ..parallel.partition import StripPartition

        self.state_mask = np.asarray(state_mask).astype(bool)
        self.partition = partition or StripPartition(self.state_mask)
        self.dates = list(dates)
        self.band_specs = list(band_specs)
        self.n_bands = len(self.band_specs)
        self.bands_per_observation = {d: self.n_bands for d in self.dates}
        self.truth_center = np.asarray(truth_center, dtype=np.float64)
        self.truth_spread = np.asarray(truth_spread, dtype=np.float64)
        n = self.truth_center.size
        self.n_params = n
        self.truth_lo = np.full(n, -np.inf) if truth_lo is None else np.asarray(truth_lo, dtype=np.float64)
        self.truth_hi = np.full(n, np.inf) if truth_hi is None else np.asarray(truth_hi, dtype=np.float64)
        self.encoding = encoding
        self.scale, self.rel_unc, self.unc_floor = float(scale), float(rel_unc), float(unc_floor)
        self.cloud_fraction = float(cloud_fraction)
        self.seed = int(seed)
        self.device = torch.device(device if device is not None else ("cuda" if torch.cuda.is_available() else "cpu"))
        self.n_pool = len(self.dates) if n_pool is None else max(1, min(int(n_pool), len(self.dates)))
        self.stream_mode = bool(stream)
        self.field_cell = min(int(field_cell), max(2, min(self.state_mask.shape) // 2))
        self.metadata = metadata or {}
        self.temporal_params = tuple(temporal_params)
        self.aux = aux                              # e.g. SAR incidence angle raster
        self._cache = RecordCache()
        self._gidx = None
        self._pool = {}                              # k -> device tensor [n_bands, N] (resident mode)
        self._streamer = None
        self._truth_fields = [(SmoothField(self.state_mask.shape, self.field_cell, self.seed * 1000 + 2 * j),
                               SmoothField(self.state_mask.shape, self.field_cell, self.seed * 1000 + 2 * j + 1))
                              for j in range(n)]

    # ----------------------------------------------------------- helpers
    @property
    def N(self) -> int:
        return self.partition.N

    def _global_idx(self):
        if self._gidx is None:
            self._gidx = torch.from_numpy(self.partition.global_index()).to(self.device)
        return self._gidx

    def pool_index(self, date) -> int:
        pos = self.__dict__.get("_date_pos")
        if pos is None or len(pos) != len(self.dates):
            pos = self._date_pos = {d: i for i, d in enumerate(self.dates)}
        return pos[date] % self.n_pool

    def truth(self, k: int) -> torch.Tensor:
        """True state [n_params, N] for pool entry k (smooth in space and time)."""
        g = self._global_idx()
        phase = 2 * math.pi * k / max(self.n_pool, 4)
        out = torch.empty((self.n_params, self.N), dtype=torch.float32, device=self.device)
        for j, (fa, fb) in enumerate(self._truth_fields):
            f = fa.at(g)
            if j in self.temporal_params:
                f = math.cos(phase) * f + math.sin(phase) * fb.at(g)
            v = self.truth_center[j] + self.truth_spread[j] * f
            out[j] = torch.clamp(v, float(self.truth_lo[j]), float(self.truth_hi[j]))
        return out

    def _aux_local(self):
        if self.aux is None:
            return None
        if getattr(self, "_aux_t", None) is not None:
            return self._aux_t
        a = np.asarray(self.aux, dtype=np.float32)
        if a.ndim == 2:
            a = a.ravel()[self.partition.global_index()]
        else:
            a = np.broadcast_to(a, (self.N,))
        self._aux_t = torch.from_numpy(np.ascontiguousarray(a)).to(self.device)
        return self._aux_t

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """Noise-free observations [n_bands, N] of state x through the band operators."""
        from ..engine.bands import operator_table

        N = x.shape[1]
        aux = self._aux_local()
        tab = operator_table(self.band_specs, self.n_params, self._cache, x.device, aux=aux)
        out = torch.empty((self.n_bands, N), dtype=torch.float32, device=x.device)
        for b in range(self.n_bands):
            K.operator_eval(self.n_params, tab, b, x.contiguous(), out[b])
        return out

    def _synthesize(self, k: int) -> torch.Tensor:
        g = self._global_idx()
        x = self.truth(k)
        y = self.forward(x)
        cloud = SmoothField(self.state_mask.shape, max(2, self.field_cell // 2), self.seed * 7919 + k)
        thr = float(np.quantile(cloud.grid.numpy(), 1.0 - self.cloud_fraction)) if self.cloud_fraction > 0 else np.inf
        clear = cloud.at(g) <= thr
        if self.encoding in ("dn16", "bf16y"):
            out = torch.empty((self.n_bands, self.N), dtype=torch.int16, device=self.device)
        elif self.encoding == "bf16":
            out = torch.empty((2 * self.n_bands, self.N), dtype=torch.int16, device=self.device)
        else:
            out = torch.empty((2 * self.n_bands, self.N), dtype=torch.float32, device=self.device)
        for b in range(self.n_bands):
            z = hash_normal(g, self.seed * 100003 + k * 101 + b)
            yb = y[b] * (1.0 + self.rel_unc * z)
            ok = clear & torch.isfinite(yb)
            if self.encoding == "dn16":
                dn = torch.clamp(torch.round(yb / self.scale), 1, 65535)
                dn = torch.where(ok, dn, torch.zeros_like(dn)).to(torch.int32)
                out[b] = torch.where(dn > 32767, dn - 65536, dn).to(torch.int16)  # uint16 bit pattern
            elif self.encoding == "bf16y":
                # y only; the kernel derives w from rel_unc / unc_floor; NaN = cloud
                yv = torch.where(ok, yb, torch.full_like(yb, float("nan")))
                out[b] = yv.to(torch.bfloat16).view(torch.int16)
            else:
                sig = torch.clamp(self.rel_unc * yb.abs(), min=max(self.unc_floor, 1e-12))
                yv = torch.where(ok, yb, torch.zeros_like(yb))
                wv = torch.where(ok, 1.0 / (sig * sig), torch.zeros_like(yb))
                if self.encoding == "bf16":
                    out[b] = yv.to(torch.bfloat16).view(torch.int16)
                    out[self.n_bands + b] = wv.to(torch.bfloat16).view(torch.int16)
                else:
                    out[b] = yv
                    out[self.n_bands + b] = wv
        return out

    def _entry_shape(self):
        return (self.n_bands, self.N) if self.encoding in ("dn16", "bf16y") else (2 * self.n_bands, self.N)

    def _ensure_pool(self):
        if self._streamer is not None or self._pool:
            return
        if self.stream_mode:
            dtype = torch.int16 if self.encoding in ("dn16", "bf16", "bf16y") else torch.float32
            self._streamer = DateStreamer(self.n_pool, self._entry_shape(), dtype, self.device,
                                          n_bufs=3 if self.n_pool >= 3 else 2)
            for k in range(self.n_pool):
                data = self._synthesize(k)
                self._streamer.host_view(k).copy_(data.cpu())
                del data
            self._streamer.warm()
        else:
            for k in range(self.n_pool):
                self._pool[k] = self._synthesize(k)

    def _entry(self, k: int, key=None) -> torch.Tensor:
        """Pool entry k on the device; streamed per date (``key``): a recycled
        host entry is copied again for every date that uses it."""
        self._ensure_pool()
        if self._streamer is not None:
            return self._streamer.acquire(k, key)
        return self._pool[k]

    # ------------------------------------------------------ protocol
    def prefetch(self, date):
        if date not in self.bands_per_observation:
            return
        self._ensure_pool()
        if self._streamer is not None:
            self._streamer.prefetch(self.pool_index(date), date)

    @property
    def max_prefetch(self) -> int:
        """Dates the engine may prefetch ahead of the one being assimilated."""
        self._ensure_pool()
        return self._streamer.max_ahead if self._streamer is not None else 1

    def ingest_bytes(self) -> int:
        return 0 if self._streamer is None else self._streamer.bytes_h2d

    def band_spec(self, date, band):
        return self.band_specs[band]

    def get_device_band_data(self, date, band) -> DeviceBand:
        return self._band(self._entry(self.pool_index(date), date), band, self._aux_local())

    def _band(self, e, band, aux) -> DeviceBand:
        meta = dict(self.metadata)
        spec = self.band_specs[band]
        if self.encoding == "dn16":
            return DeviceBand(K.OBS_DN16, dn=e[band],
                              scale=self.scale, rel_unc=self.rel_unc, unc_floor=self.unc_floor, metadata=meta,
                              emulator=spec.emulator, aux=aux)
        if self.encoding == "bf16y":
            return DeviceBand(K.OBS_BF16Y, y=e[band], rel_unc=self.rel_unc, unc_floor=self.unc_floor, metadata=meta,
                              emulator=spec.emulator, aux=aux)
        kind = K.OBS_BF16 if self.encoding == "bf16" else K.OBS_F32
        return DeviceBand(kind, y=e[band], w=e[self.n_bands + band], metadata=meta, emulator=spec.emulator,
                          aux=aux)

    def get_device_bands(self, date):
        """Every band of ``date`` from one pool-entry acquire (one stream wait).
        A pool entry's band records are built once and handed out again for
        every date that uses the entry (the same buffers, scalars and
        operators), so the engine can reuse what it derived from them."""
        e = self._entry(self.pool_index(date), date)
        aux = self._aux_local()
        nb = self.bands_per_observation[date]
        key = (e.data_ptr(), tuple(e.shape), e.dtype, nb, None if aux is None else aux.data_ptr(), self.encoding,
               self.scale, self.rel_unc, self.unc_floor, id(self.metadata), tuple(map(id, self.band_specs)))
        lists = self.__dict__.setdefault("_band_lists", {})
        hit = lists.get(key)
        if hit is None:
            if len(lists) >= 64:
                lists.clear()
            hit = lists[key] = [self._band(e, b, aux) for b in range(nb)]
        return hit

    def get_band_data(self, date, band):
        """Reference record on this rank's strip raster (numpy, float64)."""
        db = self.get_device_band_data(date, band)
        y, w = db.decode()
        y, w = y.cpu().numpy().astype(np.float64), w.cpu().numpy().astype(np.float64)
        shape = self.partition.strip_shape
        idx = self.partition.local_idx
        obs = np.zeros(shape)
        obs.ravel()[idx] = y
        wr = np.zeros(shape[0] * shape[1])
        wr[idx] = w
        mask = np.zeros(shape, dtype=bool)
        mask.ravel()[idx] = w > 0
        unc = sp.dia_matrix((wr, 0), shape=(wr.size, wr.size)).tocsr()
        meta = dict(self.metadata)
        if self.aux is not None:
            a = np.asarray(self.aux, dtype=np.float64)
            meta["incidence_angle"] = a[self.partition.r0:self.partition.r1] if a.ndim == 2 else a
        return S2MSIdata(obs, unc, mask, meta, self.band_specs[band].emulator)

    def define_output(self):
        return "", [0.0, 1.0, 0.0, 0.0, 0.0, -1.0]


# ------------------------------------------------------------------ presets
def _date_list(start, n, step_days):
    return [start + dt.timedelta(days=int(step_days * i)) for i in range(n)]


def _truth_box(emulators, maps, n_params, center, spread, margin=0.1):
    lo = np.full(n_params, -np.inf)
    hi = np.full(n_params, np.inf)
    for em, mp in zip(emulators, maps):
        tlo, thi = em.inputs.min(0), em.inputs.max(0)
        pad = margin * (thi - tlo)
        for d, j in enumerate(mp):
            lo[j] = max(lo[j], tlo[d] + pad[d])
            hi[j] = min(hi[j], thi[d] - pad[d])
    c = np.clip(center, lo, hi)
    return lo, hi, c


class SyntheticBHRObservations(SyntheticObservations):
    """MCD43-like broadband BHR (VIS, NIR) for the 7-parameter JRC-TIP state
    (``observations.py:214-310``): 2 bands, 5 % relative uncertainty with a
    2.5e-3 floor, TIP band mapper, GP emulators with 4 inputs."""

    sensor = "BHR"

    def __init__(self, state_mask, dates=None, emulators=None, n_train=500, **kw):
        from ..models.gp import make_tip_emulators
        from ..models.operators import TIP_BAND_MAPPER
        from ..models.priors import tip_prior

        ems = emulators or make_tip_emulators(n_train=n_train, seed=kw.get("seed", 0))
        specs = [gp_spec(ems[b], TIP_BAND_MAPPER[b]) for b in range(2)]
        mean, cov, _ = tip_prior()
        spread = 0.5 * np.sqrt(np.diag(cov))
        lo, hi, c = _truth_box(ems, TIP_BAND_MAPPER, 7, mean, spread)
        dates = dates or _date_list(dt.datetime(2017, 1, 1), 23, 16)
        kw.setdefault("unc_floor", 2.5e-3)
        kw.setdefault("temporal_params", (6,))
        super().__init__(state_mask, dates, specs, c, spread, lo, hi, **kw)
        self.emulators = ems


class SyntheticS2Observations(SyntheticObservations):
    """Sentinel-2 L2A-shaped source (``Sentinel2_Observations.py:85-185``): uint16
    DN, reflectance = DN/1e4, mask = DN>0, 5 % relative uncertainty, one GP
    emulator per band over the 10 PROSAIL parameters (or a custom state map)."""

    sensor = "S2"
    BAND_NAMES = ["02", "03", "04", "05", "06", "07", "08", "8A", "09", "12", "01", "10", "11"]

    def __init__(self, state_mask, dates=None, n_bands=10, emulators=None, n_train=250, n_params=10,
                 state_maps=None, spread_scale: float = 0.5, hard: bool = False, **kw):
        from ..models.gp import make_prosail_emulators
        from ..models.priors import sail_prior

        ems = emulators or make_prosail_emulators(n_bands, n_train, kw.get("seed", 0), n_params, hard=hard)
        maps = state_maps or [list(range(ems[b].n_inputs)) for b in range(n_bands)]
        specs = [gp_spec(ems[b], maps[b]) for b in range(n_bands)]
        mean, cov, _ = sail_prior()
        mean, cov = mean[:n_params], cov[:n_params, :n_params]
        spread = float(spread_scale) * np.maximum(np.sqrt(np.diag(cov)), 0.02)
        lo, hi, c = _truth_box(ems, maps, n_params, mean, spread)
        dates = dates or _date_list(dt.datetime(2017, 7, 3), 10, 2)
        kw.setdefault("temporal_params", (6,))
        super().__init__(state_mask, dates, specs, c, spread, lo, hi, **kw)
        self.emulators = ems
        self.band_map = self.BAND_NAMES[:n_bands]


class SyntheticOLCIObservations(SyntheticS2Observations):
    """OLCI-like 21-band sensor sharing the PROSAIL state (multi-sensor config)."""

    sensor = "OLCI"

    def __init__(self, state_mask, dates=None, n_bands=21, **kw):
        kw.setdefault("seed", 21)
        super().__init__(state_mask, dates, n_bands=n_bands, **kw)


class SyntheticS1Observations(SyntheticObservations):
    """Sentinel-1-shaped SAR (``Sentinel1_Observations.py``): VV/VH sigma0 (linear),
    5 % uncertainty, per-pixel incidence angle, Water Cloud Model operator on
    the (LAI, SM) state."""

    sensor = "S1"

    def __init__(self, state_mask, dates=None, theta=None, n_params=2, **kw):
        from ..models.operators import _sar_device_spec

        specs = [_sar_device_spec(n_params, None, None, b) for b in range(2)]
        shape = np.asarray(state_mask).shape
        if theta is None:
            theta = np.broadcast_to(np.linspace(30.0, 45.0, shape[1], dtype=np.float32), shape).copy()
        center = np.array([2.0, 0.25] + [0.0] * (n_params - 2))
        spread = np.array([0.8, 0.08] + [0.0] * (n_params - 2))
        lo = np.array([0.2, 0.05] + [-np.inf] * (n_params - 2))
        hi = np.array([6.0, 0.5] + [np.inf] * (n_params - 2))
        dates = dates or _date_list(dt.datetime(2017, 4, 1), 20, 6)
        kw.setdefault("encoding", "f32")
        kw.setdefault("temporal_params", (0, 1))
        super().__init__(state_mask, dates, specs, center, spread, lo, hi, aux=theta, **kw)


class SyntheticIdentityObservations(SyntheticObservations):
    """Direct (identity) observations of every state element — band k observes
    parameter k (BASELINE config 2; the reference's identity operator,
    utils.py:119-126, fixed).  Default encoding: bf16 y with the weight derived
    in-kernel from the relative-uncertainty model (``bf16y``: 2 B per band and
    pixel; ``encoding="bf16"`` streams explicit (y, w) pairs)."""

    sensor = "identity"

    def __init__(self, state_mask, dates=None, n_params=7, mean=None, sigma=None, **kw):
        from ..models.operators import _linear_device_spec
        from ..models.priors import tip_prior

        if mean is None:
            mean, cov, _ = tip_prior()
            sigma = np.sqrt(np.diag(cov))
        mean = np.asarray(mean, dtype=np.float64)[:n_params]
        sigma = np.asarray(sigma, dtype=np.float64)[:n_params]
        specs = [_linear_device_spec(n_params, None, None, b) for b in range(n_params)]
        dates = dates or _date_list(dt.datetime(2017, 1, 1), 30, 5)
        kw.setdefault("encoding", "bf16y")
        kw.setdefault("rel_unc", 0.1)
        kw.setdefault("unc_floor", 0.01)
        super().__init__(state_mask, dates, specs, mean, 0.5 * sigma, mean - 2 * sigma, mean + 2 * sigma, **kw)


class MultiSensorObservations:
    """Joint observation operator over several sources sharing one state: each
    date carries the concatenated bands of every source observing it
    (S2 13-band + OLCI-like 21-band = 34 bands, BASELINE config 5)."""

    def __init__(self, sources):
        self.sources = list(sources)
        dates = sorted(set(d for s in self.sources for d in s.dates))
        self.dates = dates
        self.bands_per_observation = {d: sum(s.bands_per_observation.get(d, 0) for s in self.sources)
                                      for d in dates}
        self.state_mask = self.sources[0].state_mask
        self.partition = self.sources[0].partition

    def _locate(self, date, band):
        for s in self.sources:
            nb = s.bands_per_observation.get(date, 0)
            if band < nb:
                return s, band
            band -= nb
        raise IndexError(band)

    def get_band_data(self, date, band):
        s, b = self._locate(date, band)
        return s.get_band_data(date, b)

    def band_groups(self, date):
        """Source index of each band of ``date`` (the bands of one sensor
        share its clouds): the observation classes of the engine's pixel order."""
        out = []
        for i, s in enumerate(self.sources):
            out += [i] * s.bands_per_observation.get(date, 0)
        return out

    def get_device_band_data(self, date, band):
        s, b = self._locate(date, band)
        return s.get_device_band_data(date, b)

    def band_spec(self, date, band):
        s, b = self._locate(date, band)
        return s.band_specs[b]

    def prefetch(self, date):
        for s in self.sources:
            if date in s.bands_per_observation:
                s.prefetch(date)

    @property
    def max_prefetch(self) -> int:
        """Dates the engine may prefetch ahead of the one being assimilated
        (the tightest source: every source prefetches each date)."""
        return min(int(getattr(s, "max_prefetch", 1)) for s in self.sources)

    def ingest_bytes(self) -> int:
        return sum(s.ingest_bytes() for s in self.sources)


def synthesize_s2_archive(root, state_mask, n_dates: int = 4, n_train: int = 250, seed: int = 0, device=None,
                          cloud_fraction: float = 0.2, geotransform=None, projection=None):
    """Write a Sentinel-2 archive in the reader's on-disk layout
    (``sentinel.write_s2_archive``: tiled-DEFLATE uint16 DN GeoTIFFs per band,
    metadata.xml, angle-named emulator npz) whose reflectances are the
    SyntheticS2Observations fields pushed through its PROSAIL-like emulators on
    ``device`` — so a file-driven run converges like the synthetic one.
    Returns (data folder, emulator folder, dates)."""
    from .sentinel import S2_EMULATOR_BANDS, write_s2_archive

    mask = np.asarray(state_mask).astype(bool)
    dates = _date_list(dt.datetime(2017, 7, 3), n_dates, 2)
    src = SyntheticS2Observations(mask, dates=dates, n_bands=10, n_train=n_train, seed=seed, device=device,
                                  cloud_fraction=cloud_fraction, stream=False, n_pool=n_dates)
    idx = src.partition.global_index()
    H, W = mask.shape
    dn_by_date = {}
    for k, d in enumerate(dates):
        e = src._synthesize(k).cpu().numpy().view(np.uint16)        # [10, N] active pixels
        r = np.zeros((10, H * W), dtype=np.uint16)
        r[:, idx] = e
        dn_by_date[d] = r.reshape(10, H, W)
        del e
    ems = {f"S2A_MSI_{S2_EMULATOR_BANDS[b]:02d}": src.emulators[b] for b in range(10)}
    data, emus = write_s2_archive(root, dn_by_date, ems, geotransform, projection)
    return data, emus, dates
