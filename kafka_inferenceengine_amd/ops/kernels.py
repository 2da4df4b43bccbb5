"""Torch-facing wrappers of the gfx950 kernels (``csrc/kf_kernels.hip``).

Every op takes SoA tensors — state ``[n_p, ld]``, packed symmetric blocks
``[n_p(n_p+1)/2, ld]``, per-pixel vectors ``[N]`` — validates shape, dtype,
device and contiguity on the host (the kernels trust their arguments), and
launches on the current HIP stream of the tensors' device.  CPU tensors run
the identical per-pixel source through the OpenMP host runner.
"""
from __future__ import annotations

from dataclasses import dataclass
from enum import IntEnum

import numpy as np
import torch

from ..models.gp import gpm_frags_per_chunk
from ..utils.blocks import ntri
from . import _ext

OBS_NONE, OBS_F32, OBS_DN16, OBS_BF16, OBS_BF16Y = 0, 1, 2, 3, 4
ST_NONSPD, ST_NONFINITE, ST_BAD_OP, ST_NO_OBS, ST_FALLBACK, ST_OUT_OF_DOMAIN = 1, 2, 4, 8, 16, 32
SUPPORTED_NP = (1, 2, 3, 4, 7, 10)


def ext():
    return _ext.require_ext()


def _ptr(t):
    return 0 if t is None else int(t.data_ptr())


def _dev(t: torch.Tensor) -> bool:
    return t.device.type == "cuda"


# the current HIP stream of a device as a raw handle: torch's C accessor when it
# has one (torch.cuda.current_stream builds a Stream object through several
# Python layers: ~10 us of the per-date host path over a date's launches)
_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def current_raw_stream(device: torch.device) -> int:
    """Raw handle of ``device``'s current HIP stream."""
    if _RAW_STREAM is not None:
        return int(_RAW_STREAM(device.index if device.index is not None else torch.cuda.current_device()))
    return int(torch.cuda.current_stream(device).cuda_stream)


def _sig(t):
    """Identity of an operand for the launch memos: address, shape, strides, dtype, device."""
    return None if t is None else (t.data_ptr(), tuple(t.shape), t.stride(), t.dtype, t.device)


# validated analysis argument blocks by operand identity (analysis(): launch memo)
_ANALYSIS_MEMO: dict = {}


def _table_key(bands) -> tuple:
    """What an argument block takes from a band table (computed once per table)."""
    k = bands.__dict__.get("_memo_key")
    if k is None:
        dom = None if bands.dom is None else (tuple(bands.dom[0]), tuple(bands.dom[1]))
        k = bands.__dict__["_memo_key"] = (bands.ptr, bands.n, bands.fast_d, bands.fast_obs, bands.gpm_frags,
                                           bool(bands.gpm_global), bands.layout, dom)
    return k


def _stream(t: torch.Tensor) -> int:
    return current_raw_stream(t.device) if _dev(t) else 0


def _check_soa(t, rows, N, name, dtype=torch.float32, device=None):
    if t is None:
        return
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if t.dim() != 2 or t.shape[0] != rows or t.shape[1] < N:
        raise ValueError(f"{name}: expected [{rows}, >={N}], got {tuple(t.shape)}")
    if t.stride(1) != 1 or t.stride(0) != t.shape[1]:
        raise ValueError(f"{name}: must be a contiguous [rows, ld] tensor")
    if device is not None and t.device != device:
        raise ValueError(f"{name}: on {t.device}, expected {device}")


def _check_vec(t, N, name, dtype, device):
    if t is None:
        return
    if t.dtype != dtype or t.dim() != 1 or t.shape[0] < N or not t.is_contiguous():
        raise ValueError(f"{name}: expected contiguous {dtype}[>={N}], got {t.dtype}{tuple(t.shape)}")
    if t.device != device:
        raise ValueError(f"{name}: on {t.device}, expected {device}")


def check_np(n_params: int):
    if n_params not in SUPPORTED_NP:
        raise ValueError(f"n_params={n_params} has no compiled kernel (supported: {SUPPORTED_NP}); "
                         "pad the state (engine.padding) to a supported size")


def grid_for(N: int) -> int:
    return int(ext().grid(int(N)))


def partials_buffer(N: int, device) -> torch.Tensor:
    """Norm partials of one launch over N pixels: one f64 per workgroup of the
    grid-stride kernels."""
    return torch.zeros(grid_for(N), dtype=torch.float64, device=device)


def _set_valid(partials, n):
    """Entries of ``partials`` the last producer wrote (read by reduce_partials)."""
    if partials is not None:
        partials._kf_n = int(n)


@dataclass
class BandTable:
    """Packed ``BandDesc`` array resident on the target device plus the tensors
    it points into (kept alive as long as the table).  ``fast_d``/``fast_obs``
    select the specialised analysis kernel when every band is a GP with the
    same input count and observation encoding (0: generic kernel)."""
    buf: torch.Tensor
    n: int
    keepalive: tuple
    fast_d: int = 0
    fast_obs: int = 0
    gpm_frags: int = 0      # > 0: GP on the matrix cores, LDS fragments of all bands (kf_gp_mfma.h)
    gpm_global: bool = False  # GP on the matrix cores, tables read from global memory (too large for LDS)
    layout: int = 0         # BAND_LAYOUT_*: a band layout the kernels know at compile time (0: runtime)
    dom: tuple | None = None  # GP domain box in state space (lo, hi lists; ST_OUT_OF_DOMAIN)
    specs: tuple = ()       # the bands' OperatorSpecs (line tables of the first iteration at the forecast)

    @property
    def ptr(self) -> int:
        return int(self.buf.data_ptr())


OP_PRECOMP = 0
OP_LINEAR = 1
OP_GP = 2


# LDS budget of the matrix-core GP analysis (every band's table staged per workgroup)
GPM_MAX_LDS = 160 * 1024
GPM_MAX_BANDS = 4          # kf_gp_mfma.h: bands of the LDS-staged matrix-core path
GPM_GLOBAL_D = (7, 10)     # full-state GP input counts with a global-table instantiation

# kf_core.h BAND_LAYOUT_TIP: exactly two GP bands with the JRC-TIP VIS then NIR maps
# (BandDesc.map_kind 2, 3), 4 inputs each: the matrix-core kernel unrolls the band loop
BAND_LAYOUT_TIP = 1
# kf_core.h BAND_LAYOUT_SHARED_X: every band a full-state GP (identity map) around the
# same centre, matrix-core tables in global memory: one exponent operand per iteration
BAND_LAYOUT_SHARED_X = 2
FD_PRECOMP = -1   # kf_core.h: fast analysis kernel for all-precomputed operators
FD_LINEAR = -2    # kf_core.h: fast analysis kernel for all-linear (identity/selection) operators


class Variant(IntEnum):
    """``AnalysisArgs.variant`` (kf_core.h ``AnalysisVariant``): the production
    analysis kernel or an alternate device path kept as a test oracle (each is
    bit-identical to the default or pinned against it by a GPU test)."""
    DEFAULT = 0
    VALU_ORACLE = 4          # GP sums on the f32 VALU record loop instead of the matrix cores
    GT_PREFETCH = 7          # global tables: next chunk's fragments loaded under the current one
    RUNTIME_LAYOUT = 10      # JRC-TIP bands through the runtime-layout kernel
    PER_BAND_OPERAND = 14    # BAND_LAYOUT_SHARED_X: exponent operand rebuilt per band
    BLOCK_ORDER = 16         # exponent MFMAs block by block
    GENERIC_SPEC = 18        # fused forecast through the generic launch instead of SPEC_PROP


# analysis variant of launches that pass none (tests switch it to an oracle path;
# no environment variable reaches it)
DEFAULT_VARIANT = Variant.DEFAULT


class _PinnedRing:
    """Pinned staging ring for small host->device copies (descriptor tables,
    launch-argument blocks): allocated once per device, so no copy pays for a
    pinned allocation (which can stall the host for milliseconds).  A slot is
    reused only after the copy that last read it has run (its event)."""

    SLOT = 16 << 10
    SLOTS = 64

    def __init__(self, device):
        self.device = device
        self.buf = torch.empty(self.SLOT * self.SLOTS, dtype=torch.uint8, pin_memory=True)
        self.events = [None] * self.SLOTS
        self.i = 0

    def copy(self, cpu: torch.Tensor) -> torch.Tensor:
        n = cpu.numel() * cpu.element_size()
        j = self.i
        self.i = (self.i + 1) % self.SLOTS
        if self.events[j] is not None:
            self.events[j].synchronize()         # 64 copies ago: normally long done
        stage = self.buf[j * self.SLOT:j * self.SLOT + n]
        stage.copy_(cpu.reshape(-1).view(torch.uint8))
        out = torch.empty(n, dtype=torch.uint8, device=self.device)
        out.copy_(stage, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self.events[j] = ev
        return out.view(cpu.dtype).view(cpu.shape)


_RINGS = {}


def small_h2d(cpu: torch.Tensor, device) -> torch.Tensor:
    """Copy a small host buffer (descriptor table, launch arguments) to the
    device without blocking the host: staged in a pinned ring and queued on the
    current stream.  A pageable ``.to(device)`` would wait for every kernel
    already queued, which stalls the host's preparation of the next launch."""
    device = torch.device(device)
    if device.type != "cuda":
        return cpu.clone()
    cpu = cpu.contiguous()
    if cpu.numel() * cpu.element_size() <= _PinnedRing.SLOT:
        idx = device.index if device.index is not None else torch.cuda.current_device()
        ring = _RINGS.get(idx)
        if ring is None:
            ring = _RINGS[idx] = _PinnedRing(torch.device("cuda", idx))
        return ring.copy(cpu)
    return cpu.pin_memory().to(device, non_blocking=True)


def make_band_table(descs: list, device, keepalive=(), specs=()) -> BandTable:
    raw = ext().pack_band_descs(descs)
    cpu = torch.frombuffer(bytearray(raw), dtype=torch.uint8) if raw else torch.zeros(8, dtype=torch.uint8)
    buf = small_h2d(cpu, device)
    fast_d = fast_obs = 0
    obs = {d.obs for d in descs}
    one_obs = next(iter(obs)) if len(obs) == 1 else None
    if descs and all(d.op == OP_GP for d in descs):
        ds = {d.d for d in descs}
        if len(ds) == 1 and one_obs in (OBS_F32, OBS_DN16):
            fast_d, fast_obs = next(iter(ds)), one_obs
    elif descs and one_obs in (OBS_F32, OBS_DN16, OBS_BF16, OBS_BF16Y) and all(d.op == OP_PRECOMP for d in descs):
        fast_d, fast_obs = FD_PRECOMP, one_obs
    elif descs and one_obs in (OBS_F32, OBS_DN16, OBS_BF16, OBS_BF16Y) and all(d.op == OP_LINEAR for d in descs):
        fast_d, fast_obs = FD_LINEAR, one_obs
    gpm_frags, gpm_global = 0, False
    if fast_d > 0 and all(d.gpm_nchunk > 0 for d in descs):
        gpm_frags = sum(d.gpm_nchunk for d in descs) * gpm_frags_per_chunk(fast_d) + 1   # + zero fragment
        if gpm_frags * 16 > GPM_MAX_LDS or len(descs) > GPM_MAX_BANDS:
            # too large for LDS: the global-table kernel (compiled for full-state
            # GPs of 7 and 10 parameters, kf_device.h:analysis_mfma_g_kernel)
            gpm_frags, gpm_global = 0, fast_d in GPM_GLOBAL_D
    layout = 0
    if fast_d == 4 and gpm_frags > 0 and [d.map_kind for d in descs] == [2, 3]:
        layout = BAND_LAYOUT_TIP
    elif (gpm_global and fast_d % 2 == 0 and all(d.map_identity for d in descs)
          and len({tuple(d.center[:fast_d]) for d in descs}) == 1):
        layout = BAND_LAYOUT_SHARED_X
    return BandTable(buf, len(descs), tuple(keepalive), fast_d, fast_obs, gpm_frags, gpm_global, layout,
                     _state_domain(descs), tuple(specs))


def _state_domain(descs):
    """The GP bands' input training boxes (BandDesc.dom_*, centred) folded into
    one box in state space: input i of a band reads state map[i], so
    x[map[i]] in [dom_lo[i] + center[i], dom_hi[i] + center[i]]; the
    intersection over bands and inputs (+-inf where nothing constrains)."""
    lo, hi, any_ = [-np.inf] * 16, [np.inf] * 16, False
    for d in descs:
        if d.op != OP_GP or not d.dom_check:
            continue
        m, c, dl, dh = d.map, d.center, d.dom_lo, d.dom_hi
        for i in range(int(d.d)):
            j = int(m[i])
            lo[j] = max(lo[j], float(dl[i]) + float(c[i]))
            hi[j] = min(hi[j], float(dh[i]) + float(c[i]))
            any_ = True
    return (lo, hi) if any_ else None


# ------------------------------------------------------ line tables
# The matrix-core kernels' first Gauss-Newton iteration at a fused partial-reset
# forecast reads every band's value and gradient from cubic line tables
# (kf_gp_mfma.h line_pos / line_eval, models/gp.py:line_table) instead of
# running the GP sums: at the forecast every parameter but the propagated one
# is the reset mean.  On by default; tests and bench A/B switch it per call.
LINE_TABLES = True
_LINE_CACHE: dict = {}


def _prop_single(mask: int):
    """The one propagated parameter of a partial-reset forecast, -1 for none
    (prior reset), None for several (no line)."""
    mask = int(mask)
    if mask == 0:
        return -1
    return mask.bit_length() - 1 if mask & (mask - 1) == 0 else None


def line_fields(bands: BandTable, prop, n_params: int, dev):
    """(table, t0, inv_h, n, j) of the launch's first iteration at the fused
    forecast ``prop``, or None (no GP matrix-core bands, several propagated
    parameters, no table range, or the host runner).  Built once per (band
    specs, reset mean, j) in float64 and kept on the device."""
    if dev.type != "cuda" or prop is None or bands.fast_d <= 0 or not bands.specs or \
            not (bands.gpm_frags > 0 or bands.gpm_global):
        return None
    if any(getattr(sp, "kind", None) != OP_GP or len(sp.state_map) != bands.fast_d for sp in bands.specs):
        return None
    j = _prop_single(prop.args.prop_mask)
    if j is None:
        return None
    fixed = tuple(float(v) for v in list(prop.args.reset_mean)[:n_params])
    key = (tuple(id(sp) for sp in bands.specs), fixed, j, dev)
    hit = _LINE_CACHE.get(key)
    if hit is None:
        from ..models.gp import line_table

        r = line_table(list(bands.specs), np.asarray(fixed, dtype=np.float64), j)
        tab = None if r is None else torch.from_numpy(np.ascontiguousarray(r[0])).to(dev)
        if len(_LINE_CACHE) >= 32:
            _LINE_CACHE.clear()
        hit = _LINE_CACHE[key] = (bands.specs, None if r is None else (tab, r[1], r[2], r[3], j))
    return hit[1]


def _set_line(a, bands, prop, n_params, dev, x_prev, line):
    if x_prev is not None or not (LINE_TABLES if line is None else line):
        return
    lf = line_fields(bands, prop, n_params, dev)
    if lf is not None:
        a.line_tab, a.line_t0, a.line_inv_h, a.line_n, a.line_j = _ptr(lf[0]), lf[1], lf[2], lf[3], lf[4]


# ------------------------------------------------------------------ ops
def gp_operator(n_params, bands: BandTable, x, h0, h, N=None, d=None):
    """K2 split path: GP value/Jacobian of every band of ``bands`` at x into
    h0 [nb, ldh] and h [nb*n_params, ldh] (masked pixels: zeros)."""
    check_np(n_params)
    N = int(x.shape[1] if N is None else N)
    _check_soa(x, n_params, N, "x")
    nb = bands.n
    d = bands.fast_d if d is None else d
    if h0.shape[0] != nb or h.shape[0] != nb * n_params or h0.shape[1] != h.shape[1] or h0.shape[1] < N:
        raise ValueError("h0 must be [nb, ldh] and h [nb*n_params, ldh]")
    if _dev(x) and not ext().gp_operator_supported(n_params, int(d)):
        raise ValueError(f"no gp_operator kernel for n_params={n_params}, d={d}")
    ext().gp_operator(n_params, int(d), bands.ptr, nb, _ptr(x), N, x.shape[1], _ptr(h0), _ptr(h), h0.shape[1],
                      _dev(x), _stream(x))


def gp_operator_supported(n_params, d) -> bool:
    return bool(ext().gp_operator_supported(int(n_params), int(d)))


def analysis(n_params, bands: BandTable, x_prev, x_f, pf_inv, x_out=None, a_out=None, b_out=None, status=None,
             partials=None, N=None, solve=True, fast=True, variant=None, a_in=None, b_in=None, prop=None,
             out=None, reg=None, x0_out=None, gn_fused=1, partials_first=None, order=None, n_visit=None,
             dn_out=None, a_rows=None, n_visit_dev=None, line=None):
    """K1 fused Gauss-Newton analysis (information form).

    ``gn_fused=2`` runs two Gauss-Newton iterations in this launch: the first
    (which cannot end the loop, min_iterations = 2) stays in registers, its
    norm partials go to ``partials_first``; ``x_out``/``a_out``/``out`` and
    ``partials`` are those of the second.  Bit-identical to two launches.

    ``prop`` (from :func:`prop_args`) fuses the propagation: the forecast is
    computed per pixel from the previous analysis inside the kernel and
    ``x_f``/``pf_inv`` must be None; ``x_prev=None`` then linearises at the
    forecast (first Gauss-Newton iteration).

    ``out = (mean, unc, idx)`` additionally writes x and 1/sqrt(diag A) into
    output rasters ``[n_params, plane]`` at raster positions ``idx`` (int64 [N],
    None = identity) — the unpack pass fused into the final iteration.

    ``reg = dict(gamma, mask, v_out, nbr=None, geo=None)`` replaces the solve by
    the K9 regulariser prepare (kf_core.h): a_out <- A + g deg E_R, x_out <- u =
    A_reg^-1 b, v_out [k*n, ld] <- A_reg^-1 E_R; no partials.  ``x0_out``
    receives the linearisation point (the fused forecast when x_prev is None).
    With ``gn_fused=2`` the first iteration is the plain solve (its norm to
    ``partials_first``) and the regulariser prepares the second, linearised
    at x_1 (written to ``x0_out``).

    ``order`` (int32 [N], from :func:`obs_order`): the pixel visiting order --
    the observed pixels first, so cloudy pixels fill whole waves that skip the
    GP; each pixel's result is the same in any order (the per-workgroup norm
    partials sum different pixel sets).  ``n_visit``: visit only
    ``order[:n_visit]`` (the per-chunk Gauss-Newton loop's active pixels;
    needs ``order``).  ``n_visit_dev`` (int32 [>= 1], device): the count to
    visit read by the kernel itself (at most ``n_visit``, which then only
    sizes the grid) -- a launch queued before the host has read the count.

    ``dn_out`` (float32 [N]): each visited pixel's |x - x0|^2 of the launch's
    last iteration, at its pixel index (per-chunk convergence norms).
    ``a_rows``: bit mask of the packed precision rows stored to ``a_out``
    (None / 0: every row; EngineConfig.store_precision).  ``line``: the first
    iteration at the fused forecast from line tables (:func:`line_fields`;
    None: ``LINE_TABLES``).

    Launch memo: the engine's steady state repeats the same operands date
    after date (buffers alternate, arguments are memoised upstream), so a call
    whose tensors (address, shape, stride, dtype) and options equal an earlier
    validated one reuses its argument block: no re-validation and none of the
    ~50 per-field writes into the native struct on the per-date host path."""
    ref = next(t for t in (x_prev, x_f, x_out, a_out) if t is not None)
    key = None
    if reg is None:
        key = (n_params, _table_key(bands), N, bool(solve), bool(fast),
               DEFAULT_VARIANT if variant is None else variant, gn_fused, n_visit, _sig(n_visit_dev), a_rows,
               None if prop is None else (prop.device_copy().data_ptr(), prop.args.ld, prop.args.N, prop.fused,
                                          prop.device),
               _sig(x_prev), _sig(x_f), _sig(pf_inv), _sig(x_out), _sig(a_out), _sig(b_out), _sig(status),
               _sig(partials), _sig(a_in), _sig(b_in), _sig(x0_out), _sig(partials_first), _sig(order), _sig(dn_out),
               None if out is None else (_sig(out[0]), _sig(out[1]), _sig(out[2])),
               LINE_TABLES if line is None else bool(line))
        hit = _ANALYSIS_MEMO.get(key)
        if hit is not None:
            a, grid = hit
            n_part = ext().analysis(n_params, a, grid, _dev(ref), _stream(ref))
            _set_valid(partials, n_part)
            _set_valid(partials_first if gn_fused == 2 else None, n_part)
            return partials
    check_np(n_params)
    N = int(ref.shape[1] if N is None else N)
    dev = ref.device
    nt = ntri(n_params)
    if prop is None and (x_prev is None or x_f is None or pf_inv is None):
        raise ValueError("x_prev, x_f and pf_inv are required unless the propagation is fused")
    if prop is not None and (x_f is not None or pf_inv is not None or a_in is not None):
        raise ValueError("fused propagation replaces x_f/pf_inv and excludes a_in")
    for t, r, nm in ((x_prev, n_params, "x_prev"), (x_f, n_params, "x_f"), (pf_inv, nt, "pf_inv"),
                     (x_out, n_params, "x_out"), (a_out, nt, "a_out"), (b_out, n_params, "b_out")):
        _check_soa(t, r, N, nm, device=dev)
    ld = ref.shape[1]
    for t in (x_prev, x_f, pf_inv, x_out, a_out, b_out):
        if t is not None and t.shape[1] != ld:
            raise ValueError("all SoA operands must share the leading dimension")
    if prop is not None and (prop.args.ld != ld or prop.args.N < N or prop.device != dev):
        raise ValueError("fused propagation arguments do not match the analysis layout/device")
    if prop is not None and not prop.fused:
        raise ValueError("analysis(prop=...) needs prop_args(..., fused=True)")
    if solve and x_out is None:
        raise ValueError("solve=True needs x_out")
    _check_vec(status, N, "status", torch.uint8, dev)
    if partials is not None and (partials.dtype != torch.float64 or partials.numel() < grid_for(N)):
        raise ValueError("partials must be float64 with >= grid_for(N) entries")
    if gn_fused not in (1, 2):
        raise ValueError("gn_fused must be 1 or 2")
    if gn_fused == 2 and (a_in is not None or not solve):
        raise ValueError("gn_fused=2 runs the solve path only (no band chunks or solve=False)")
    if gn_fused == 2 and reg is not None and x0_out is None:
        raise ValueError("gn_fused=2 with reg needs x0_out (x_1, the second iteration's linearisation point)")
    if partials_first is not None and (partials_first.dtype != torch.float64 or partials_first.numel() < grid_for(N)):
        raise ValueError("partials_first must be float64 with >= grid_for(N) entries")
    a = ext().AnalysisArgs()
    a.N, a.ld, a.n_bands, a.solve = N, ld, bands.n, int(bool(solve))
    a.gn_fused = int(gn_fused)
    a.partials_first = _ptr(partials_first) if gn_fused == 2 else 0
    a.fast_d, a.fast_obs = (bands.fast_d, bands.fast_obs) if fast else (0, 0)
    a.band_layout = int(bands.layout) if (fast and (bands.layout != BAND_LAYOUT_TIP or n_params == 7)) else 0
    v = DEFAULT_VARIANT if variant is None else variant
    a.variant = int(Variant(int(v)))     # unknown numbers raise
    a.gpm_frags = bands.gpm_frags if fast else 0
    a.gpm_global = int(bool(bands.gpm_global) and fast and bands.fast_d == n_params)
    a.bands = bands.ptr
    a.x_prev, a.x_f, a.pf_inv = _ptr(x_prev), _ptr(x_f), _ptr(pf_inv)
    a.x_out, a.a_out, a.b_out = _ptr(x_out), _ptr(a_out), _ptr(b_out)
    if (a_in is None) != (b_in is None):
        raise ValueError("a_in and b_in go together")
    _check_soa(a_in, nt, N, "a_in", device=dev)
    _check_soa(b_in, n_params, N, "b_in", device=dev)
    a.a_in, a.b_in = _ptr(a_in), _ptr(b_in)
    a.status, a.partials = _ptr(status), _ptr(partials)
    if prop is not None:
        a.prop = _ptr(prop.device_copy())
    if out is not None:
        # (mean, unc, idx); with ``reg`` the mean is None: the regulariser's
        # prepare writes the uncertainty raster (1/sqrt of the regularised
        # precision's diagonal) and reg_finish the mean
        mean, unc, idx = out
        if not solve:
            raise ValueError("fused output needs solve=True")
        if unc is None or (reg is not None and mean is not None):
            raise ValueError("out = (mean, unc, idx); with reg the mean is None (reg_finish writes it)")
        plane = unc.shape[1]
        if mean is None and reg is None and (idx is not None or x_out is None or x_out.shape[1] != plane):
            # the state's x is the mean raster (DeviceOutput alias): identity map, x's layout
            raise ValueError("out mean None needs the identity map and x_out of the raster's plane")
        for t, nm in ((mean, "out mean"), (unc, "out unc")):
            if t is None:
                continue
            _check_soa(t, n_params, 0, nm, device=dev)
            if t.shape[1] != plane:
                raise ValueError("out mean / unc planes differ")
        if idx is not None:
            _check_vec(idx, N, "out idx", torch.int64, dev)
        elif plane < N:
            raise ValueError("identity output needs plane >= N")
        a.out_mean, a.out_unc, a.out_idx, a.out_plane = _ptr(mean), _ptr(unc), _ptr(idx), plane
    if x0_out is not None:
        _check_soa(x0_out, n_params, N, "x0_out", device=dev)
        if x0_out.shape[1] != ld:
            raise ValueError("x0_out must share the leading dimension")
        a.x0_out = _ptr(x0_out)
    if reg is not None:
        k = bin(int(reg["mask"])).count("1")
        v_out = reg["v_out"]
        _check_soa(v_out, k * n_params, N, "reg v_out", device=dev)
        if x_out is None or v_out.shape[1] != ld or k == 0:
            raise ValueError("regulariser prepare needs x_out (u), v_out [k*n, ld] and a non-empty mask")
        _check_nbr(reg.get("nbr"), N, reg.get("geo"))
        if partials is not None:
            raise ValueError("regulariser prepare produces no partials (reg_finish does)")
        a.reg_gamma, a.reg_mask = float(reg["gamma"]), int(reg["mask"])
        a.reg_nbr, a.reg_v = _ptr(reg.get("nbr")), _ptr(v_out)
        geo = reg.get("geo")
        if geo is not None:
            if geo["w"] <= 0 or geo["h"] * geo["w"] != N:
                raise ValueError(f"dense geometry {geo} does not cover N={N} pixels")
            a.geo_w, a.geo_h, a.geo_halo, a.geo_n_up = int(geo["w"]), int(geo["h"]), int(geo["halo"]), \
                int(geo["n_up"])
    if order is not None:
        _check_vec(order, N, "order", torch.int32, dev)
        a.order = _ptr(order)
    nv = N
    if n_visit is not None:
        nv = int(n_visit)
        if order is None or not 0 < nv <= N:
            raise ValueError(f"n_visit={n_visit} needs an order and 0 < n_visit <= N={N}")
        if gn_fused != 1 or reg is not None:
            raise ValueError("n_visit: single-iteration launches without the regulariser")
        a.n_visit = nv
    if n_visit_dev is not None:
        if n_visit is None:
            raise ValueError("n_visit_dev needs n_visit (the bound that sizes the grid)")
        _check_vec(n_visit_dev, 1, "n_visit_dev", torch.int32, dev)
        a.n_visit_dev = _ptr(n_visit_dev)
    if dn_out is not None:
        _check_vec(dn_out, N, "dn_out", torch.float32, dev)
        a.dn_out = _ptr(dn_out)
    if bands.dom is not None:
        a.dom_check, a.dom_lo, a.dom_hi = 1, list(bands.dom[0]), list(bands.dom[1])
    if a_rows:
        if int(a_rows) >> nt:
            raise ValueError(f"a_rows has bits past the {nt} packed rows")
        a.a_rows = int(a_rows)
    if fast:
        _set_line(a, bands, prop, n_params, dev, x_prev, line)
    grid = grid_for(nv)
    if partials is not None and partials.numel() < grid:
        raise ValueError("partials must hold one entry per workgroup (partials_buffer)")
    n_part = ext().analysis(n_params, a, grid, _dev(ref), _stream(ref))
    if key is not None:
        if len(_ANALYSIS_MEMO) >= 64:
            _ANALYSIS_MEMO.clear()
        _ANALYSIS_MEMO[key] = (a, grid)
    _set_valid(partials, n_part)
    _set_valid(partials_first if gn_fused == 2 else None, n_part)
    return partials


# ------------------------------------------------ per-chunk convergence
CHUNK_GROUP_RUNS = 16   # kf_core.h: runs summed per stage-1 workgroup


def chunk_groups(lc_ptr) -> int:
    """Stage-1 groups per local chunk (the most runs of any chunk / CHUNK_GROUP_RUNS)."""
    runs = np.diff(np.asarray(lc_ptr, dtype=np.int64))
    return max(1, int(-(-runs.max() // CHUNK_GROUP_RUNS))) if runs.size else 1


def chunk_partials(dn, seg_start, seg_len, lc_ptr, lc_gid, active, part, gpart, groups, qinv, clamp):
    """part[g] = this rank's pixels' dn of each active chunk g in integer quanta
    (kf_core.h:chunk_quant with ``qinv[g]`` quanta per unit and ``clamp``
    quanta at most per pixel; exact sums, kf_kernels.hip:chunk_group_kernel /
    chunk_total_kernel); other entries kept.  ``part`` int64 [nc], ``gpart``
    [n_local * groups] int64 scratch, ``groups`` from :func:`chunk_groups`."""
    n_local = int(lc_gid.numel())
    if gpart.numel() < n_local * groups or gpart.dtype != torch.int64 or part.dtype != torch.int64:
        raise ValueError("chunk_partials: int64 part / group scratch of the right size")
    if qinv.dtype != torch.float64 or qinv.numel() != part.numel():
        raise ValueError("chunk_partials: qinv must be float64 [nc]")
    ext().chunk_partials(_ptr(dn), _ptr(seg_start), _ptr(seg_len), _ptr(lc_ptr), _ptr(lc_gid), n_local,
                         _ptr(active), _ptr(part), _ptr(gpart), int(groups), _ptr(qinv), int(clamp), _dev(part),
                         _stream(part))


def chunk_decide(part_all, world, len_x, local_count, tol, n_iter, min_iter, max_iter, active, newly, iters, info,
                 px_out=None, unit=1.0):
    """The reference's exit test per chunk (linear_kf.py:297-304) on the
    all-gathered integer partials [world, nc] (norm = sqrt(total * unit));
    info <- (active chunks, largest norm tested, this rank's active pixels,
    chunks stopped now); ``px_out`` (int32 [>= 1]) <- this rank's active
    pixels (the next launch's device count)."""
    nc = int(active.numel())
    if part_all.numel() != world * nc or len_x.numel() != nc or local_count.numel() != nc:
        raise ValueError("chunk_decide: inconsistent chunk vectors")
    if part_all.dtype != torch.int64:
        raise ValueError("chunk_decide: int64 partials")
    ext().chunk_decide(_ptr(part_all), int(world), nc, _ptr(len_x), _ptr(local_count), float(tol), int(n_iter),
                       int(min_iter), int(max_iter), _ptr(active), _ptr(newly), _ptr(iters), _ptr(info),
                       _ptr(px_out), float(unit), _dev(active), _stream(active))


def chunk_compact_scratch(n: int, device) -> torch.Tensor:
    return torch.empty(int(ext().chunk_compact_blocks(max(int(n), 1))) + 1, dtype=torch.int32, device=device)


def chunk_compact(order_in, n_in, chunk_of, active, newly, counts, order_out, x_src=None, x_dst=None, n_in_dev=None):
    """order_out <- the slots of order_in[:n_in] (None: 0..n_in-1) whose chunk
    is active, stable; x of the pixels whose chunk stopped now copied x_src ->
    x_dst ([n_p, ld]).  ``n_in_dev`` (int32 [>= 1]): the slot count read on the
    device (at most ``n_in``, which then only sizes the grid).  Returns the
    kept count on the host runner, None on the device (chunk_decide's info
    holds it)."""
    n_in = int(n_in)
    if n_in_dev is not None and (n_in_dev.dtype != torch.int32 or n_in_dev.device != chunk_of.device):
        raise ValueError("chunk_compact: n_in_dev must be an int32 tensor on the chunk map's device")
    if order_in is not None and order_in.data_ptr() == order_out.data_ptr():
        raise ValueError("chunk_compact: order_out must not alias order_in")
    np_, ld = (0, 0) if x_src is None else (int(x_src.shape[0]), int(x_src.shape[1]))
    if x_src is not None and (x_dst is None or x_dst.shape != x_src.shape):
        raise ValueError("chunk_compact: x_src / x_dst of one shape")
    r = ext().chunk_compact(_ptr(order_in), n_in, _ptr(chunk_of), _ptr(active), _ptr(newly), _ptr(counts),
                            _ptr(order_out), _ptr(x_src), _ptr(x_dst), np_, ld, _ptr(n_in_dev), _dev(chunk_of),
                            _stream(chunk_of))
    return None if r < 0 else int(r)


_GROUP_IDS = {}   # (device, band groups) -> int32 device tensor of obs_order


def obs_order(bands: BandTable, N: int, device, out=None, scratch=None, groups=None, local=False):
    """Stable partition of the pixels 0..N-1 by observation class
    (``AnalysisArgs.order``): ``groups`` gives each band's group (bands of one
    sensor share its cloud mask; None: one group, at most 3 groups); pixels
    observed in every group come first, then the partial classes, the
    unobserved last -- each class fills whole waves, which skip the GP of the
    groups they have no data for.  ``local=False`` (default): one global
    partition (count, scan, scatter); True: each 4096-pixel chunk (64 waves)
    partitioned in place, one pass (A/B, EngineConfig.observed_first_local).  ``out`` int32 [>= N] and
    ``scratch`` (device int32) may be reused; returns (order [N], scratch)."""
    dev = torch.device(device)
    N = int(N)
    if out is None or out.numel() < N:
        out = torch.empty(max(N, 1), dtype=torch.int32, device=dev)
    grp = None
    G = 1
    if groups is not None:
        groups = [int(g) for g in groups]
        if len(groups) != bands.n or min(groups) < 0 or max(groups) > 2:
            raise ValueError("obs_order: one group id in 0..2 per band")
        G = max(groups) + 1
        key = (str(dev), tuple(groups))
        grp = _GROUP_IDS.get(key)
        if grp is None:   # once per layout: a pageable H2D copy waits for the stream
            grp = _GROUP_IDS[key] = torch.tensor(groups, dtype=torch.int32, device=dev)
    # [chunks][classes] prefixes, then the class totals
    nc = (int(ext().obs_order_chunks(N)) + 1) * (1 << G)
    if dev.type == "cuda" and not local and (scratch is None or scratch.numel() < nc):
        scratch = torch.empty(max(nc, 9), dtype=torch.int32, device=dev)
    ext().obs_order(bands.ptr, _ptr(grp), bands.n, G, N, _ptr(scratch), _ptr(out), bool(local), dev.type == "cuda",
                    _stream(out))
    return out[:N], scratch


def gain(n_params, bands: BandTable, x_prev, x_f, p_f, x_out, p_out=None, status=None, partials=None, N=None,
         joseph=False, prop=None, out=None, fast=True, gn_fused=1, partials_first=None, order=None, n_visit=None,
         dn_out=None, pdiag_rows=0, n_visit_dev=None, line=None):
    """K1g covariance/gain-form analysis (sequential scalar band updates).

    ``prop`` (:func:`prop_args` with ``fused=True`` over the analysis
    COVARIANCE) fuses the forecast as for :func:`analysis` (x_f / p_f None;
    ``x_prev=None`` linearises at it); ``out = (mean, unc, idx)`` writes the
    output rasters (x, 1/sqrt(diag P^-1)) from the kernel (mean None: the
    state's x is the mean raster -- identity map, x_out's plane); ``p_out`` may
    be None in iterations that cannot end the Gauss-Newton loop.

    K1's launch features (:func:`analysis`): ``gn_fused=2`` runs iterations 1
    and 2 in this launch (the first iteration's norm partials to
    ``partials_first``); ``order`` / ``n_visit`` / ``n_visit_dev`` the visiting
    order and the per-chunk subset; ``dn_out`` every visited pixel's |x - x0|^2.
    ``pdiag_rows`` (bit j): store only the analysis precision diagonal entries
    (P^-1)_jj of these parameters, into ``p_out`` rows tri(j, j) -- the rows a
    fused forecast with ``PropArgs.pa_pdiag`` reads (the stored-rows policy);
    0 stores the full covariance.  ``line``: line tables for the first
    iteration at the fused forecast, as :func:`analysis`."""
    check_np(n_params)
    ref = next(t for t in (x_prev, x_f, x_out) if t is not None)
    N = int(ref.shape[1] if N is None else N)
    dev = ref.device
    nt = ntri(n_params)
    if prop is None and (x_prev is None or x_f is None or p_f is None):
        raise ValueError("x_prev, x_f and p_f are required unless the propagation is fused")
    if prop is not None and (x_f is not None or p_f is not None):
        raise ValueError("fused propagation replaces x_f/p_f")
    for t, r, nm in ((x_prev, n_params, "x_prev"), (x_f, n_params, "x_f"), (p_f, nt, "p_f"),
                     (x_out, n_params, "x_out"), (p_out, nt, "p_out")):
        _check_soa(t, r, N, nm, device=dev)
    ld = ref.shape[1]
    for t in (x_prev, x_f, p_f, x_out, p_out):
        if t is not None and t.shape[1] != ld:
            raise ValueError("all SoA operands must share the leading dimension")
    if prop is not None and (prop.args.ld != ld or prop.args.N < N or prop.device != dev or not prop.fused):
        raise ValueError("fused propagation arguments do not match the gain layout/device")
    _check_vec(status, N, "status", torch.uint8, dev)
    if gn_fused not in (1, 2):
        raise ValueError("gn_fused must be 1 or 2")
    if partials_first is not None and (partials_first.dtype != torch.float64 or partials_first.numel() < grid_for(N)):
        raise ValueError("partials_first must be float64 with >= grid_for(N) entries")
    a = ext().GainArgs()
    a.N, a.ld, a.n_bands, a.joseph = N, ld, bands.n, int(bool(joseph))
    a.fast_d, a.fast_obs = (bands.fast_d, bands.fast_obs) if fast else (0, 0)
    if a.fast_d < 0:     # precomputed / linear fast paths exist for K1 only
        a.fast_d, a.fast_obs = 0, 0
    # GP on the matrix cores with LDS tables (kf_device.h:gain_mfma_kernel, JRC-TIP)
    a.gpm_frags = bands.gpm_frags if (fast and DEFAULT_VARIANT != Variant.VALU_ORACLE) else 0
    a.bands = bands.ptr
    a.x_prev, a.x_f, a.p_f, a.x_out, a.p_out = map(_ptr, (x_prev, x_f, p_f, x_out, p_out))
    a.status, a.partials = _ptr(status), _ptr(partials)
    a.gn_fused = int(gn_fused)
    a.partials_first = _ptr(partials_first) if gn_fused == 2 else 0
    if prop is not None:
        a.prop = _ptr(prop.device_copy())
    if out is not None:
        mean, unc, idx = out
        if unc is None:
            raise ValueError("out = (mean, unc, idx) needs the uncertainty planes")
        plane = unc.shape[1]
        if mean is None and (idx is not None or x_out is None or x_out.shape[1] != plane):
            raise ValueError("out mean None needs the identity map and x_out of the raster's plane")
        for t, nm in ((mean, "out mean"), (unc, "out unc")):
            if t is None:
                continue
            _check_soa(t, n_params, 0, nm, device=dev)
            if t.shape[1] != plane:
                raise ValueError("out mean / unc planes differ")
        if idx is not None:
            _check_vec(idx, N, "out idx", torch.int64, dev)
        elif plane < N:
            raise ValueError("identity output needs plane >= N")
        a.out_mean, a.out_unc, a.out_idx, a.out_plane = _ptr(mean), _ptr(unc), _ptr(idx), plane
    if order is not None:
        _check_vec(order, N, "order", torch.int32, dev)
        a.order = _ptr(order)
    nv = N
    if n_visit is not None:
        nv = int(n_visit)
        if order is None or not 0 < nv <= N:
            raise ValueError(f"n_visit={n_visit} needs an order and 0 < n_visit <= N={N}")
        if gn_fused != 1:
            raise ValueError("n_visit: single-iteration launches")
        a.n_visit = nv
    if n_visit_dev is not None:
        if n_visit is None:
            raise ValueError("n_visit_dev needs n_visit (the bound that sizes the grid)")
        _check_vec(n_visit_dev, 1, "n_visit_dev", torch.int32, dev)
        a.n_visit_dev = _ptr(n_visit_dev)
    if dn_out is not None:
        _check_vec(dn_out, N, "dn_out", torch.float32, dev)
        a.dn_out = _ptr(dn_out)
    if pdiag_rows:
        if int(pdiag_rows) >> n_params:
            raise ValueError(f"pdiag_rows has bits past the {n_params} parameters")
        a.pdiag_rows = int(pdiag_rows)
    if a.gpm_frags > 0:
        _set_line(a, bands, prop, n_params, dev, x_prev, line)
    grid = grid_for(nv)
    ext().gain(n_params, a, grid, _dev(ref), _stream(ref))
    _set_valid(partials, grid)
    _set_valid(partials_first if gn_fused == 2 else None, grid)
    return partials


def jacobi(n_params, a_in, b_in, x_ext, nbr, x_ref, x_out, gamma, reg_mask, N, a_out=None, partials=None,
           geo=None):
    """K9 block-Jacobi sweep of the GMRF spatial regulariser."""
    check_np(n_params)
    dev = a_in.device
    _check_soa(a_in, ntri(n_params), N, "a_in", device=dev)
    _check_soa(b_in, n_params, N, "b_in", device=dev)
    _check_soa(x_ref, n_params, N, "x_ref", device=dev)
    _check_soa(x_out, n_params, N, "x_out", device=dev)
    _check_soa(x_ext, n_params, N, "x_ext", device=dev)
    _check_nbr(nbr, N, geo)
    a = ext().JacobiArgs()
    _set_geo(a, geo, N)
    a.N, a.ld, a.ld_ext = N, a_in.shape[1], x_ext.shape[1]
    a.gamma, a.reg_mask = float(gamma), int(reg_mask)
    a.a_in, a.b_in, a.x_ext, a.nbr, a.x_ref, a.x_out = map(_ptr, (a_in, b_in, x_ext, nbr, x_ref, x_out))
    a.a_out, a.partials = _ptr(a_out), _ptr(partials)
    ext().jacobi(n_params, a, grid_for(N), _dev(a_in), _stream(a_in))
    _set_valid(partials, grid_for(N))
    return partials


JACOBI_PREPARE, JACOBI_SWEEP, JACOBI_FINISH = 1, 2, 3


def _set_geo(a, geo, N, prefix="geo"):
    """Dense strip geometry (StripPartition.dense_geometry) into an args struct."""
    if geo is None:
        return
    if geo["w"] <= 0 or geo["h"] * geo["w"] != N:
        raise ValueError(f"dense geometry {geo} does not cover N={N} pixels")
    a.geo_w, a.geo_h, a.geo_halo, a.geo_n_up = int(geo["w"]), int(geo["h"]), int(geo["halo"]), int(geo["n_up"])


def _check_nbr(nbr, N, geo):
    if geo is not None and nbr is None:
        return
    if nbr is None or nbr.dtype != torch.int32 or nbr.shape != (4, N) or not nbr.is_contiguous():
        raise ValueError("nbr must be contiguous int32 [4, N] (or pass the dense geometry)")


def _reg_args(n_params, mode, N, ld, gamma, reg_mask, nbr, geo=None):
    _check_nbr(nbr, N, geo)
    a = ext().JacobiArgs()
    a.N, a.ld = N, ld
    a.gamma, a.reg_mask = float(gamma), int(reg_mask)
    a.mode, a.k = mode, bin(int(reg_mask)).count("1")
    a.nbr = _ptr(nbr)
    _set_geo(a, geo, N)
    return a


def reg_prepare(n_params, a_in, b_in, nbr, u_out, v_out, gamma, reg_mask, N, a_out=None, geo=None, x_ref=None):
    """K9 affine form, once per GN iteration: A_reg = A + g deg E_R (written to
    ``a_out``, may alias ``a_in``), u = A_reg^-1 b, V = A_reg^-1 E_R ([k*n, ld]).
    A non-SPD / non-finite pixel gets V = 0 and u = ``x_ref`` (0 without it)."""
    check_np(n_params)
    dev = a_in.device
    k = bin(int(reg_mask)).count("1")
    _check_soa(a_in, ntri(n_params), N, "a_in", device=dev)
    _check_soa(b_in, n_params, N, "b_in", device=dev)
    _check_soa(u_out, n_params, N, "u_out", device=dev)
    _check_soa(v_out, k * n_params, N, "v_out", device=dev)
    _check_soa(a_out, ntri(n_params), N, "a_out", device=dev)
    ld = a_in.shape[1]
    for t in (b_in, u_out, v_out, a_out):
        if t is not None and t.shape[1] != ld:
            raise ValueError("all SoA operands must share the leading dimension")
    if x_ref is not None:
        _check_soa(x_ref, n_params, N, "x_ref", device=dev)
        if x_ref.shape[1] != ld:
            raise ValueError("all SoA operands must share the leading dimension")
    a = _reg_args(n_params, JACOBI_PREPARE, N, ld, gamma, reg_mask, nbr, geo)
    a.a_in, a.b_in, a.x_out, a.v, a.a_out = map(_ptr, (a_in, b_in, u_out, v_out, a_out))
    a.x_ref = _ptr(x_ref)
    ext().jacobi(n_params, a, grid_for(N), _dev(a_in), _stream(a_in))


def reg_sweep(n_params, u, v, z_ext, nbr, z_out, gamma, reg_mask, N, geo=None, rows=None, z_prev=None,
              omega=1.0):
    """K9 affine sweep of the k regularised fields: z_out[:, :N] = u_R + g V_RR s(z_ext).
    ``rows = (p0, n)`` restricts it to local pixels [p0, p0 + n) (C2 overlap: the
    boundary rows first, then the interior while the halo is in flight).
    ``z_prev``/``omega``: Chebyshev step z_out = z_prev + omega (jacobi - z_prev)."""
    check_np(n_params)
    dev = u.device
    k = bin(int(reg_mask)).count("1")
    _check_soa(u, n_params, N, "u", device=dev)
    _check_soa(v, k * n_params, N, "v", device=dev)
    _check_soa(z_ext, k, N, "z_ext", device=dev)
    _check_soa(z_out, k, N, "z_out", device=dev)
    if z_out.shape[1] != z_ext.shape[1] or v.shape[1] != u.shape[1]:
        raise ValueError("z_out must share z_ext's leading dimension and v u's")
    a = _reg_args(n_params, JACOBI_SWEEP, N, u.shape[1], gamma, reg_mask, nbr, geo)
    a.ld_ext = z_ext.shape[1]
    a.u, a.v, a.x_ext, a.z_out = map(_ptr, (u, v, z_ext, z_out))
    if z_prev is not None:
        _check_soa(z_prev, k, N, "z_prev", device=dev)
        if z_prev.shape[1] != z_ext.shape[1] or z_prev.data_ptr() in (z_out.data_ptr(),):
            raise ValueError("z_prev must share z_ext's leading dimension and differ from z_out")
        a.z_prev, a.omega = _ptr(z_prev), float(omega)
    n = N
    if rows is not None:
        p0, n = int(rows[0]), int(rows[1])
        if p0 < 0 or n < 0 or p0 + n > N:
            raise ValueError(f"sweep rows {rows} outside [0, {N})")
        if n == 0:
            return
        a.p0, a.pn = p0, n
    ext().jacobi(n_params, a, grid_for(n), _dev(u), _stream(u))


REG_TILE_MAX_SWEEPS = 8


REG_TILE_ROWS = 64    # kf_reg_tiled.hip RT_TH: strip rows per tile row


def reg_tile_rows(h: int) -> int:
    """Tile rows of the tiled sweep kernel over a strip of ``h`` rows."""
    return -(-int(h) // REG_TILE_ROWS)


def reg_boundary_tile_rows(h: int, depth: int, up: bool, down: bool):
    """``(a, b)``: the tile rows [0, a) and [b, tiles) hold the strip rows the
    neighbours need ([0, depth) with a neighbour above, [h - depth, h) with one
    below); [a, b) is the interior a pass can run while they are on the wire."""
    ty = reg_tile_rows(h)
    a = reg_tile_rows(min(depth, h)) if up else 0
    b = (max(h - depth, 0) // REG_TILE_ROWS) if down else ty
    a = min(a, ty)
    return a, max(a, b)


def reg_sweeps_tiled(n_params, u, v, z, z_prev, z_out, zp_out, gamma, reg_mask, N, geo, omegas=None,
                     chebyshev=None, *, sched=None, s_base=0, nsweep=None, halo=None, tile_rows=None):
    """K9 temporal blocking (csrc/kf_reg_tiled.hip): up to 8 sweeps of the one
    regularised field of a dense strip in one launch.  Sweep s is
    ``reg_sweep(..., z_prev=previous iterate, omega=omegas[s])`` when
    ``chebyshev[s]``, the plain Jacobi sweep otherwise; bit-identical to those
    launches.  Writes the last iterate to ``z_out`` and the one before to
    ``zp_out`` (local parts, [1, >= N]).

    ``sched = (sched_i32, omega_tab)``: the device schedule of :func:`reg_schedule`
    instead of host weights -- the pass runs sweeps ``s_base ..`` of it, at most
    ``nsweep`` (none left: the outputs are copies of the inputs).
    ``halo = (hu, hd, up, dn)``: deep halo of a tile-DP strip, ``up`` / ``dn``
    [4, >= depth * w] planes (u, v, z, zp rows) of the rows above / below, row-
    major from the outermost row (``HaloExchanger.deep_*``).  ``tile_rows = (ty0,
    ty1)``: only those tile rows (boundary-first C2 overlap)."""
    check_np(n_params)
    dev = u.device
    if bin(int(reg_mask)).count("1") != 1:
        raise ValueError("reg_sweeps_tiled: one regularised field")
    if geo is None:
        raise ValueError("reg_sweeps_tiled: dense strip geometry needed")
    hu, hd, up, dn = halo if halo is not None else (0, 0, None, None)
    gh = int(geo["halo"])
    if bool(hu) != bool(gh & 1) or bool(hd) != bool(gh & 2):
        raise ValueError("reg_sweeps_tiled: the deep halo must match the strip's halo rows")
    if sched is None:
        if omegas is None or chebyshev is None:
            raise ValueError("reg_sweeps_tiled: host weights or a device schedule")
        ns = len(omegas)
        if not 1 <= ns <= REG_TILE_MAX_SWEEPS or len(chebyshev) != ns:
            raise ValueError(f"reg_sweeps_tiled: 1..{REG_TILE_MAX_SWEEPS} sweeps, one flag per sweep")
        mask = sum(1 << s for s, c in enumerate(chebyshev) if c)
        if mask & 1 and z_prev is None:
            raise ValueError("reg_sweeps_tiled: the first sweep is a Chebyshev step but z_prev is None")
    else:
        if omegas is not None:
            raise ValueError("reg_sweeps_tiled: host weights and a device schedule")
        ns = int(nsweep or 0)
        if not 1 <= ns <= REG_TILE_MAX_SWEEPS:
            raise ValueError(f"reg_sweeps_tiled: 1..{REG_TILE_MAX_SWEEPS} sweeps per pass")
        mask = 0
        sch, om = sched
        if sch.dtype != torch.int32 or om.dtype != torch.float32 or sch.device != dev or om.device != dev:
            raise ValueError("reg_sweeps_tiled: schedule tensors (int32, float32) on the operands' device")
        # the kernel reads omega_tab[s] only for s < sched[0] <= omega_tab.numel() - 1
        if s_base < 0:
            raise ValueError("reg_sweeps_tiled: negative first sweep")
        if z_prev is None and s_base > 0:
            raise ValueError("reg_sweeps_tiled: a later pass needs the previous iterate")
    w, h = int(geo["w"]), int(geo["h"])
    for d in (hu, hd):
        if d and not ns <= d <= REG_TILE_MAX_SWEEPS:
            raise ValueError(f"reg_sweeps_tiled: halo depth {d} must cover the pass's {ns} sweeps")
    plane = 0
    for t, d, nm in ((up, hu, "halo up"), (dn, hd, "halo down")):
        if d:
            if t is None or t.dim() != 2 or t.shape[0] != 4 or t.shape[1] < d * w or not t.is_contiguous():
                raise ValueError(f"reg_sweeps_tiled: {nm} must be contiguous [4, >= {d * w}]")
            if t.device != dev or t.dtype != torch.float32:
                raise ValueError(f"reg_sweeps_tiled: {nm} float32 on {dev}")
            if plane and plane != t.shape[1]:
                raise ValueError("reg_sweeps_tiled: halo planes differ in size")
            plane = t.shape[1]
    _check_soa(u, n_params, N, "u", device=dev)
    _check_soa(v, n_params, N, "v", device=dev)
    if v.shape[1] != u.shape[1]:
        raise ValueError("v must share u's leading dimension")
    for t, nm in ((z, "z"), (z_out, "z_out"), (zp_out, "zp_out")):
        _check_soa(t, 1, N, nm, device=dev)
    if z_prev is not None:
        _check_soa(z_prev, 1, N, "z_prev", device=dev)
    ptrs = {t.data_ptr() for t in (z, z_out, zp_out)}
    if len(ptrs) != 3 or (z_prev is not None and z_prev.data_ptr() in (z_out.data_ptr(), zp_out.data_ptr())):
        raise ValueError("reg_sweeps_tiled: outputs must not alias the inputs")
    _set_geo(ext().JacobiArgs(), geo, N)   # validates w * h == N
    ty0, ty1 = tile_rows if tile_rows is not None else (0, 0)
    if tile_rows is not None:
        if not 0 <= ty0 <= ty1 <= reg_tile_rows(h):
            raise ValueError(f"reg_sweeps_tiled: tile rows {tile_rows} outside [0, {reg_tile_rows(h)}]")
        if ty0 == ty1:
            return
    j0 = (int(reg_mask) & -int(reg_mask)).bit_length() - 1
    ext().reg_tiled(u.shape[1], w, h, j0, mask, float(gamma), [] if sched is not None else [float(o) for o in omegas],
                    _ptr(u), _ptr(v), _ptr(z), _ptr(z_prev), _ptr(z_out), _ptr(zp_out), _dev(u), _stream(u),
                    nsweep=ns, hu=int(hu), hd=int(hd), halo_up=_ptr(up), halo_dn=_ptr(dn), halo_plane=plane,
                    ty0=int(ty0), ty1=int(ty1), sched=_ptr(sched[0]) if sched is not None else 0,
                    omega_tab=_ptr(sched[1]) if sched is not None else 0, s_base=int(s_base))


class RegSchedule:
    """Device-resident schedule of one GN iteration's coupled solve (K9): rho
    (Gershgorin bound of the Jacobi matrix, all-rank max), the sweep count and
    the Chebyshev weights, computed on the device so the host can queue the
    first tiled pass without reading rho back (kf_reg_tiled.hip)."""

    def __init__(self, N: int, max_sweeps: int, device):
        self.device = torch.device(device)
        self.max_sweeps = int(max_sweeps)
        self.npart = int(ext().reg_rho_blocks(max(int(N), 1))) if self.device.type == "cuda" else 1
        self.pmax = torch.zeros(self.npart, dtype=torch.float32, device=self.device)
        self.rho = torch.zeros(1, dtype=torch.float64, device=self.device)
        self.sched = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.omega = torch.zeros(max(self.max_sweeps, 1), dtype=torch.float32, device=self.device)
        self.info = torch.zeros(2, dtype=torch.float64, device=self.device)

    def rho_pass(self, v_row: torch.Tensor, geo, N: int, gamma: float):
        """rho[0] = gamma * max_p v_row[p] * deg(p) over a dense strip."""
        if v_row.dtype != torch.float32 or v_row.device != self.device or v_row.numel() < N:
            raise ValueError("reg rho: float32 v row of >= N entries on the schedule's device")
        if not v_row.is_contiguous():
            raise ValueError("reg rho: contiguous v row")
        ext().reg_rho(_ptr(v_row), int(geo["w"]), int(geo["h"]), int(geo["halo"]), int(N), _ptr(self.pmax),
                      self.npart, float(gamma), _ptr(self.rho), _dev(v_row), _stream(v_row))

    def schedule(self, tol: float):
        """sched[0] = sweeps before the finish, omega[:] their weights, info = (rho, S)."""
        ext().reg_schedule(_ptr(self.rho), float(tol), self.max_sweeps, _ptr(self.sched), _ptr(self.omega),
                           _ptr(self.info), _dev(self.rho), _stream(self.rho))


def reg_finish(n_params, u, v, z_ext, nbr, x_ref, x_out, gamma, reg_mask, N, partials=None, geo=None, out=None,
               a_prec=None):
    """K9 affine form, last sweep: x = u + g V s(z_ext) for every parameter, with
    the convergence partials of (x - x_ref).  ``out = (mean, unc, idx)`` also
    writes x and 1/sqrt(diag a_prec) into the output rasters (the unpack pass
    fused, as :func:`analysis` does for the unregularised path)."""
    check_np(n_params)
    dev = u.device
    k = bin(int(reg_mask)).count("1")
    _check_soa(u, n_params, N, "u", device=dev)
    _check_soa(v, k * n_params, N, "v", device=dev)
    _check_soa(z_ext, k, N, "z_ext", device=dev)
    _check_soa(x_ref, n_params, N, "x_ref", device=dev)
    _check_soa(x_out, n_params, N, "x_out", device=dev)
    ld = u.shape[1]
    for t in (v, x_ref, x_out):
        if t.shape[1] != ld:
            raise ValueError("all SoA operands must share the leading dimension")
    a = _reg_args(n_params, JACOBI_FINISH, N, ld, gamma, reg_mask, nbr, geo)
    a.ld_ext = z_ext.shape[1]
    a.u, a.v, a.x_ext, a.x_ref, a.x_out, a.partials = map(_ptr, (u, v, z_ext, x_ref, x_out, partials))
    if out is not None:
        # unc None: the analysis (regulariser prepare) already wrote it
        mean, unc, idx = out
        if (unc is None) != (a_prec is None):
            raise ValueError("the uncertainty raster needs a_prec (and only then)")
        if a_prec is not None:
            _check_soa(a_prec, ntri(n_params), N, "a_prec", device=dev)
            if a_prec.shape[1] != ld:
                raise ValueError("a_prec must share the leading dimension")
        plane = mean.shape[1]
        for t, nm in ((mean, "out mean"), (unc, "out unc")):
            if t is None:
                continue
            _check_soa(t, n_params, 0, nm, device=dev)
            if t.shape[1] != plane:
                raise ValueError("out mean / unc planes differ")
        if idx is not None:
            _check_vec(idx, N, "out idx", torch.int64, dev)
        elif plane < N:
            raise ValueError("identity output needs plane >= N")
        a.a_in = _ptr(a_prec)
        a.out_mean, a.out_unc, a.out_idx, a.out_plane = _ptr(mean), _ptr(unc), _ptr(idx), plane
    ext().jacobi(n_params, a, grid_for(N), _dev(u), _stream(u))
    _set_valid(partials, grid_for(N))
    return partials


def _reset_cov(n_params, reset_cinv):
    """Packed inverse of the (packed) reset precision C0 when it is SPD, else
    None (PROP_INFO_APPROX: C0 = 0) -- the constant the K1g fast forecast
    updates (kf_core.h:gain_forecast)."""
    if reset_cinv is None:
        return None
    from ..utils.blocks import pack_matrix, unpack_blocks
    C0 = unpack_blocks(np.asarray(reset_cinv, dtype=np.float64).reshape(-1, 1), n_params)[0]
    try:
        L = np.linalg.cholesky(C0)
    except np.linalg.LinAlgError:
        return None
    if not np.all(np.isfinite(L)) or np.min(np.diag(L)) <= 1e-12 * max(1.0, np.max(np.abs(C0))):
        return None
    return pack_matrix(np.linalg.inv(C0))


def prop_args(n_params, spec: dict, x_a, p_a, x_f=None, p_f=None, N=None, status=None, q_pix=None,
              blend_mean_pix=None, blend_cinv_pix=None, fused=False, pa_pdiag=False):
    """Validated ``PropArgs`` for :func:`propagate` or, with ``fused=True``, for
    a fused :func:`analysis`.  ``spec`` keys: mode, m, q, prop_mask,
    reset_mean, reset_cinv (packed), blend, quirk_blend, blend_mean,
    blend_cinv (packed).  The fused kernel evaluates one formula (partial
    prior reset, kf_core.h:forecast_partial); PROP_PRIOR and PROP_INFO_APPROX
    are mapped onto it here.  Fused arguments also carry C0^-1 for the K1g
    fast forecast (``cov_fast``) and ``pa_pdiag``: ``p_a``'s propagated
    diagonal rows hold the analysis precision diagonal (a gain-form analysis
    under the stored-rows policy)."""
    check_np(n_params)
    if fused:
        if not prop_is_light(spec["mode"], spec.get("blend", False)):
            raise ValueError("only PRIOR / PRIOR_PARTIAL / INFO_APPROX without blend can be fused")
        spec = dict(spec)
        mode = int(spec["mode"])
        if mode == 0:        # PROP_PRIOR: nothing propagated
            spec["prop_mask"] = 0
        elif mode == 2:      # PROP_INFO_APPROX: everything propagated, diagonal precision only
            spec["prop_mask"] = (1 << n_params) - 1
            spec["reset_mean"] = np.zeros(n_params)
            spec["reset_cinv"] = np.zeros(ntri(n_params))
        spec["mode"] = 1
        spec["blend"] = False
    N = int(x_a.shape[1] if N is None else N)
    dev = x_a.device
    nt = ntri(n_params)
    _check_soa(x_a, n_params, N, "x_a")
    _check_soa(p_a, nt, N, "p_a", device=dev)
    _check_soa(x_f, n_params, N, "x_f", device=dev)
    _check_soa(p_f, nt, N, "p_f", device=dev)
    _check_soa(q_pix, n_params, N, "q_pix", device=dev)
    _check_soa(blend_mean_pix, n_params, N, "blend_mean_pix", device=dev)
    _check_soa(blend_cinv_pix, nt, N, "blend_cinv_pix", device=dev)
    ld = x_a.shape[1]
    for t in (p_a, x_f, p_f, q_pix, blend_mean_pix, blend_cinv_pix):
        if t is not None and t.shape[1] != ld:
            raise ValueError("all SoA operands must share the leading dimension")
    a = ext().PropArgs()
    a.N, a.ld = N, ld
    a.mode = int(spec["mode"])
    a.blend = int(bool(spec.get("blend", False)))
    a.quirk_blend = int(bool(spec.get("quirk_blend", False)))
    a.prop_mask = int(spec.get("prop_mask", 0))
    a.m = [float(v) for v in spec.get("m", np.ones(n_params))]
    a.q = [float(v) for v in spec.get("q", np.zeros(n_params))]
    for key in ("reset_mean", "reset_cinv", "blend_mean", "blend_cinv"):
        if spec.get(key) is not None:
            setattr(a, key, [float(v) for v in np.asarray(spec[key]).ravel()])
    a.x_a, a.p_a, a.x_f, a.p_f = map(_ptr, (x_a, p_a, x_f, p_f))
    a.q_pix, a.blend_mean_pix, a.blend_cinv_pix = map(_ptr, (q_pix, blend_mean_pix, blend_cinv_pix))
    a.status = _ptr(status)
    if fused:
        a.pa_pdiag = int(bool(pa_pdiag))
        cov = _reset_cov(n_params, spec.get("reset_cinv"))
        if cov is not None:      # K1g: the forecast covariance by rank-1 updates of C0^-1
            a.cov_fast, a.reset_cov = 1, [float(v) for v in cov]
    return PropHandle(a, dev, (x_a, p_a, x_f, p_f, q_pix, blend_mean_pix, blend_cinv_pix, status), fused)


LIGHT_PROP_MODES = (0, 1, 2)   # PROP_PRIOR, PROP_PRIOR_PARTIAL, PROP_INFO_APPROX


def prop_is_light(mode, blend=False) -> bool:
    """Propagations the analysis kernel can evaluate in-kernel (kf_core.h:forecast_partial)."""
    return (not blend) and int(mode) in LIGHT_PROP_MODES


class PropHandle:
    """PropArgs plus the device and the tensors its pointers refer to (kept alive)."""

    def __init__(self, args, device, tensors, fused=False):
        self.args, self.device, self._tensors, self.fused = args, device, tensors, fused
        self._buf = None

    def device_copy(self) -> torch.Tensor:
        """The PropArgs bytes on the device (read by the kernel through s_load)."""
        if self._buf is None:
            raw = torch.frombuffer(bytearray(ext().pack_prop_args(self.args)), dtype=torch.uint8)
            self._buf = small_h2d(raw, self.device)
        return self._buf


def propagate(n_params, spec: dict, x_a, p_a, x_f, p_f, N=None, status=None, q_pix=None,
              blend_mean_pix=None, blend_cinv_pix=None):
    """K4/K5 propagation (+ optional prior blend); see :func:`prop_args`."""
    if x_f is None or p_f is None:
        raise ValueError("propagate needs x_f and p_f outputs")
    h = prop_args(n_params, spec, x_a, p_a, x_f, p_f, N, status, q_pix, blend_mean_pix, blend_cinv_pix)
    ext().propagate(n_params, h.args, _dev(x_a), _stream(x_a))


def invert(n_params, src, dst, N=None, status=None):
    """Packed SPD inverse (covariance <-> precision)."""
    check_np(n_params)
    N = int(src.shape[1] if N is None else N)
    _check_soa(src, ntri(n_params), N, "src")
    _check_soa(dst, ntri(n_params), N, "dst", device=src.device)
    if src.shape[1] != dst.shape[1]:
        raise ValueError("src/dst leading dims differ")
    ext().invert(n_params, _ptr(src), _ptr(dst), N, src.shape[1], _ptr(status), _dev(src), _stream(src))


def operator_eval(n_params, bands: BandTable, band: int, x, h0, h=None, ok=None, N=None):
    """Evaluate one band's operator and Jacobian at x (standalone K2/K3)."""
    check_np(n_params)
    N = int(x.shape[1] if N is None else N)
    _check_soa(x, n_params, N, "x")
    _check_vec(h0, N, "h0", torch.float32, x.device)
    _check_soa(h, n_params, N, "h", device=x.device)
    _check_vec(ok, N, "ok", torch.uint8, x.device)
    if not 0 <= band < bands.n:
        raise IndexError("band out of range")
    ext().operator_eval(n_params, bands.ptr, band, _ptr(x), N, x.shape[1], _ptr(h0), _ptr(h),
                        0 if h is None else h.shape[1], _ptr(ok), _dev(x), _stream(x))


def hessian(n_params, bands: BandTable, x, a, N=None):
    """K6: A -= sum_b w (y - f) d2f/dx2 over GP bands (in place)."""
    check_np(n_params)
    N = int(x.shape[1] if N is None else N)
    _check_soa(x, n_params, N, "x")
    _check_soa(a, ntri(n_params), N, "a", device=x.device)
    ext().hessian(n_params, bands.ptr, bands.n, _ptr(x), _ptr(a), N, x.shape[1], _dev(x), _stream(x))


class TileEncoder:
    """GeoTIFF tiles encoded on the device (csrc/kf_deflate.h): each 256 x 256
    tile of each float32 plane becomes one zlib stream (TIFF predictor 3,
    fixed-Huffman DEFLATE with run-length matches), packed back to back.
    ``encode(planes, H, W)`` -> (packed uint8, sizes int64, offsets int64), all
    on the planes' device and queued on the current stream; the scratch and
    packed buffers are kept for the next call of the same shape.  On the CPU
    the host runner of the same row encoder produces the same bytes."""

    def __init__(self):
        self._bufs = {}

    @staticmethod
    def tiles(H: int, W: int) -> tuple[int, int]:
        t = int(ext().DFL_TILE)
        return -(-int(W) // t), -(-int(H) // t)

    def _buf(self, key, n, dtype, device):
        b = self._bufs.get(key)
        if b is None or b.numel() < n or b.device != device:
            b = self._bufs[key] = torch.empty(n, dtype=dtype, device=device)
        return b[:n]

    def encode(self, planes: torch.Tensor, H: int, W: int, packed: torch.Tensor | None = None, base=None):
        """``packed``: the output buffer (default: the encoder's own); ``base``:
        an int64 scalar tensor added to the offsets (several rasters packed
        into one buffer back to back, device-side: no host read-back)."""
        if planes.dtype != torch.float32 or planes.dim() != 2 or planes.stride(1) != 1:
            raise ValueError("planes: [n, ld] float32 with unit column stride")
        n, ld = planes.shape
        if H * W > ld:
            raise ValueError(f"plane of {ld} values holds no {H} x {W} raster")
        tx, ty = self.tiles(H, W)
        nt = n * tx * ty
        bound = int(ext().DFL_BOUND)
        dev = planes.device
        scratch = self._buf("scratch", nt * bound, torch.uint8, dev)
        sizes = self._buf("sizes", nt, torch.int32, dev)        # uint32 byte counts (< 2^31)
        rows = self._buf("rows", nt * int(ext().DFL_ROW_SCRATCH), torch.uint8, dev) if _dev(planes) else None
        ext().deflate_tiles(_ptr(planes), planes.stride(0), int(H), int(W), int(n), _ptr(scratch), _ptr(sizes),
                            _dev(planes), _stream(planes), _ptr(rows))
        s64 = sizes.to(torch.int64)
        offs = torch.cumsum(s64, 0) - s64
        if base is not None:
            offs += base
        if packed is None:
            packed = self._buf("packed", nt * bound, torch.uint8, dev)
        if not _dev(planes):
            sz, of = s64.numpy(), offs.numpy()
            src = scratch.numpy().reshape(nt, bound)
            dst = packed.numpy()
            for i in range(nt):
                dst[of[i]:of[i] + sz[i]] = src[i, :sz[i]]
            return packed, s64, offs
        ext().deflate_pack(_ptr(scratch), _ptr(sizes), _ptr(offs), _ptr(packed), nt, _stream(planes))
        return packed, s64, offs


def unpack(n_params, x, a, mean=None, unc=None, idx=None, N=None):
    """Scatter mean and 1/sqrt(diag(P^-1)) onto raster planes [n_p, H*W]."""
    check_np(n_params)
    N = int(x.shape[1] if N is None else N)
    _check_soa(x, n_params, N, "x")
    if unc is not None:
        _check_soa(a, ntri(n_params), N, "a", device=x.device)
    plane = (mean if mean is not None else unc).shape[1]
    for t in (mean, unc):
        if t is not None:
            _check_soa(t, n_params, 0, "out", device=x.device)
    if idx is not None:
        _check_vec(idx, N, "idx", torch.int64, x.device)
    elif plane < N:
        raise ValueError("output plane smaller than N without an index map")
    ext().unpack(n_params, _ptr(x), _ptr(a), N, x.shape[1], _ptr(idx), _ptr(mean), _ptr(unc), plane, _dev(x),
                 _stream(x))


def reduce_partials(partials: torch.Tensor, out: torch.Tensor | None = None):
    """Fixed-order f64 sum of the partials the last producer wrote (device:
    one workgroup)."""
    n = min(int(getattr(partials, "_kf_n", partials.numel())), int(partials.numel()))
    if _dev(partials):
        if out is None:
            out = torch.empty(1, dtype=torch.float64, device=partials.device)
        ext().reduce_partials(_ptr(partials), n, _ptr(out), _stream(partials))
        return out
    val = float(np.sum(partials.numpy()[:n]))
    if out is None:
        return torch.tensor([val], dtype=torch.float64)
    out.fill_(val)
    return out


def gather(src, idx, out=None, rows=None):
    """out[r, p] = src[r, idx[p]] (compaction of raster rows onto active pixels);
    idx[p] < 0 gives 0 (a warped grid's pixels no source pixel covers)."""
    if src.dim() == 1:
        src2, squeeze = src.view(1, -1), True
    else:
        src2, squeeze = src, False
    n = idx.numel()
    if out is None:
        out = torch.empty((src2.shape[0], n), dtype=src.dtype, device=src.device)
    if not _dev(src):
        o = out.view(src2.shape[0], -1)
        o[:, :n] = src2[:, idx.clamp(min=0)]
        miss = idx < 0
        if bool(miss.any()):
            o[:, :n][:, miss] = 0
        return out.view(-1) if squeeze else out
    eb = src.element_size()
    ext().gather(eb, _ptr(src2), _ptr(idx), _ptr(out), n, src2.shape[0], src2.stride(0),
                 out.view(src2.shape[0], -1).stride(0), _stream(src))
    return out.view(-1) if squeeze else out


def lut_nearest(lut, x, out=None, N=None):
    """K7 nearest LUT row for every pixel (x as [D, ld])."""
    N = int(x.shape[1] if N is None else N)
    lut = lut.contiguous()
    M, D = lut.shape
    if out is None:
        out = torch.empty(N, dtype=torch.int32, device=x.device)
    ext().lut_nearest(_ptr(lut), M, D, _ptr(x), N, x.shape[1], _ptr(out), _dev(x), _stream(x))
    return out
