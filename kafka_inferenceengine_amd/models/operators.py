"""Observation-operator factories (reference plug-in point L2).

Each factory keeps the reference signature
``f(n_params, emulator, metadata, mask, state_mask, x_forecast, band)`` and,
called directly, returns the reference objects — ``(H0, H_csr)`` for
non-linear operators or ``H`` for linear ones — built with vectorised NumPy
instead of per-pixel ``lil_matrix`` writes (the 90-96 % hot spot of the
reference, ``kafka/inference/utils.py:197-215``).

The engine never calls them on its device path: it reads the factory's
``device_spec`` hook and evaluates the operator + Jacobian inside the fused
gfx950 analysis kernel.  A user factory without ``device_spec`` still works
(the engine calls it on the host each Gauss-Newton iteration and uploads the
per-pixel Jacobian rows — ``OP_PRECOMP``).
"""
from __future__ import annotations

import logging
from dataclasses import dataclass, field

import numpy as np
import scipy.sparse as sp
import torch

from .gp import GaussianProcessEmulator
from .sar import POLARISATIONS, WaterCloudModel, sar_observation_operator

LOG = logging.getLogger(__name__)

# keep in sync with csrc/kf_core.h
OP_PRECOMP, OP_LINEAR, OP_GP, OP_SAR = 0, 1, 2, 3

TIP_BAND_MAPPER = (np.array([0, 1, 6, 2]), np.array([3, 4, 6, 5]))


def band_selecta(band):
    """JRC-TIP state subset per band (kf_tools.py:19-23)."""
    return TIP_BAND_MAPPER[0] if band == 0 else TIP_BAND_MAPPER[1]


@dataclass
class OperatorSpec:
    """Device description of one band's observation operator."""
    kind: int
    state_map: list = field(default_factory=list)
    coef: list = field(default_factory=list)
    center: list = field(default_factory=list)
    offset: float = 0.0
    records: np.ndarray | None = None     # GP training records [T/2, D+1, 2] (models/gp.py)
    aux: np.ndarray | None = None         # per active pixel auxiliary (SAR theta)
    emulator: object = None
    gp_pos_pairs: int = 0                 # leading record pairs with alpha > 0
    # GP: the training box of the centred inputs widened by GP_DOMAIN_MARGIN of its
    # range per side (the kernels flag inputs outside it: ST_OUT_OF_DOMAIN)
    domain_lo: list | None = None
    domain_hi: list | None = None

    @property
    def d(self) -> int:
        return len(self.state_map)


@dataclass
class LinearOperator:
    """H0 = offset + coef . x ; identity/selection is coef = e_k."""
    coef: np.ndarray
    offset: float = 0.0

    @classmethod
    def select(cls, n_params: int, k: int):
        c = np.zeros(n_params)
        c[k] = 1.0
        return cls(c, 0.0)


# margin of a GP band's domain box beyond its training inputs, per side, as a
# fraction of the input's training range (ST_OUT_OF_DOMAIN)
GP_DOMAIN_MARGIN = 0.0


def gp_spec(emulator: GaussianProcessEmulator, state_map) -> OperatorSpec:
    """Device operator description of a GP band (memoised per emulator and state
    map: the engine asks for it on every observation date)."""
    state_map = [int(i) for i in state_map]
    cache = emulator.__dict__.setdefault("_spec_cache", {})
    key = tuple(state_map)
    if key not in cache:
        cache[key] = _gp_spec(emulator, state_map)
    return cache[key]


def _gp_spec(emulator: GaussianProcessEmulator, state_map) -> OperatorSpec:
    if emulator.n_inputs != len(state_map):
        raise ValueError(f"emulator has {emulator.n_inputs} inputs but state map has {len(state_map)}")
    lo = hi = None
    X = getattr(emulator, "inputs", None)
    if X is not None and np.asarray(X).ndim == 2 and np.asarray(X).shape[0] > 0:
        X = np.asarray(X, dtype=np.float64)
        c = np.asarray(emulator.center(), dtype=np.float64)
        tlo, thi = X.min(0), X.max(0)
        pad = GP_DOMAIN_MARGIN * (thi - tlo)
        lo, hi = list(map(float, tlo - pad - c)), list(map(float, thi + pad - c))
    return OperatorSpec(OP_GP, state_map, list(map(float, emulator.lam)), list(map(float, emulator.center())),
                        float(emulator.mean), emulator.records(), None, emulator, emulator.n_pos_pairs, lo, hi)


# ---------------------------------------------------------------- helpers
def _active(mask, state_mask):
    return np.asarray(mask)[np.asarray(state_mask)].ravel().astype(bool)


def _rows_to_csr(h_rows, valid, n_params, cols=None):
    """Per-pixel Jacobian rows -> CSR (N x n_params*N); empty rows where invalid."""
    N = h_rows.shape[0]
    if cols is None:
        cols = np.arange(n_params)
    cols = np.asarray(cols)
    k = cols.size
    idx = np.nonzero(valid)[0]
    data = h_rows[idx][:, :k].astype(np.float32).ravel()
    colidx = (idx[:, None] * n_params + cols[None, :]).ravel()
    counts = np.zeros(N + 1, dtype=np.int64)
    counts[idx + 1] = k
    indptr = np.cumsum(counts)
    return sp.csr_matrix((data, colidx, indptr), shape=(N, n_params * N))


def run_emulator(gp, x, tol=None, lut_threshold: float = 1e6, lut_size: int = 5000, seed=None):
    """Unique-row emulator evaluation (utils.py:68-106), vectorised.

    Above ``lut_threshold`` unique rows, the reference draws a 5000-sample
    MVN look-up table and assigns nearest neighbours (utils.py:75-84)."""
    if torch.is_tensor(x):
        return _run_emulator_device(gp, x, lut_threshold, lut_size, seed)
    x = np.asarray(x, dtype=np.float64)
    if x.shape[0] == 0:
        return np.zeros(0), np.zeros_like(x)
    uniq, inv = np.unique(x, axis=0, return_inverse=True)
    inv = np.asarray(inv).ravel()
    if len(uniq) > lut_threshold:
        LOG.info("Clustering parameter space")
        rng = np.random.default_rng(seed)
        uniq = rng.multivariate_normal(x.mean(0), np.cov(x, rowvar=False), lut_size)
        inv = locate_in_lut(uniq, x)
    out = gp.predict(uniq, do_unc=False)
    H_, dH_ = (out[0], out[-1])
    return np.asarray(H_)[inv], np.asarray(dH_)[inv]


def _run_emulator_device(gp, x, lut_threshold, lut_size, seed):
    """run_emulator for a resident (N, D) tensor: the unique-row pass and the
    LUT assignment stay on x's device (torch.unique, K7 ``lut_nearest``); only
    the emulator itself runs on the host, over at most ``lut_size`` rows or the
    unique rows.  Rows are deduplicated in x's own precision (float64 input:
    rows that differ only below float32 precision stay distinct, as on the
    host path, utils.py:72-84); the LUT nearest search runs in float32 (K7).
    Returns (H (N,), dH (N, D)) in x's float dtype (float64 or float32) on x's
    device."""
    from ..ops import kernels as K
    dev = x.device
    dt = torch.float64 if x.dtype == torch.float64 else torch.float32
    if x.shape[0] == 0:
        return (torch.zeros(0, dtype=dt, device=dev), torch.zeros_like(x, dtype=dt))
    xin = x.to(dt)
    uniq, inv = torch.unique(xin, dim=0, return_inverse=True)
    if uniq.shape[0] > lut_threshold:
        LOG.info("Clustering parameter space")
        xd = xin.double()
        mean = xd.mean(0)
        xc = xd - mean
        cov = (xc.T @ xc) / max(x.shape[0] - 1, 1)
        rng = np.random.default_rng(seed)
        lut = rng.multivariate_normal(mean.cpu().numpy(), cov.cpu().numpy(), lut_size)
        uniq = torch.as_tensor(lut, dtype=dt, device=dev)
        inv = K.lut_nearest(uniq.to(torch.float32), xin.to(torch.float32).T.contiguous()).long()
    out = gp.predict(uniq.double().cpu().numpy(), do_unc=False)
    H_ = torch.as_tensor(np.asarray(out[0]), dtype=dt, device=dev)
    dH_ = torch.as_tensor(np.asarray(out[-1]), dtype=dt, device=dev)
    return H_[inv], dH_[inv]


def locate_in_lut(lut, im, chunk: int = 8192):
    """Nearest LUT row for every row of im (utils.py:225-234), chunked."""
    lut = np.asarray(lut, dtype=np.float64)
    im = np.asarray(im, dtype=np.float64)
    assert lut.shape[1] == im.shape[1]
    out = np.empty(im.shape[0], dtype=np.int64)
    l2 = (lut * lut).sum(1)
    for s in range(0, im.shape[0], chunk):
        blk = im[s:s + chunk]
        d = l2[None, :] - 2 * blk @ lut.T
        out[s:s + chunk] = d.argmin(1)
    return out


# ------------------------------------------------------------- factories
def create_prosail_observation_operator(n_params, emulator, metadata, mask, state_mask, x_forecast, band):
    """GP emulator of the full state vector (utils.py:181-219)."""
    LOG.info("Creating the ObsOp for band %d" % band)
    valid = _active(mask, state_mask)
    N = int(np.asarray(x_forecast).shape[0] // n_params)
    x0 = np.asarray(x_forecast, dtype=np.float64).reshape(N, n_params)
    LOG.info("Running emulators")
    H0_, dH = run_emulator(emulator, x0[valid])
    H0 = np.zeros(N, dtype=np.float32)
    H0[valid] = H0_
    rows = np.zeros((N, n_params))
    rows[valid] = dH
    LOG.info("\tDone!")
    return H0, _rows_to_csr(rows, valid, n_params)


def _prosail_device_spec(n_params, emulator, metadata, band, band_mapper=None):
    if not isinstance(emulator, GaussianProcessEmulator):
        return None
    smap = getattr(emulator, "state_map", None)
    if smap is None:
        smap = band_mapper[band] if band_mapper is not None else range(emulator.n_inputs)
    return gp_spec(emulator, smap)


create_prosail_observation_operator.device_spec = _prosail_device_spec


def create_nonlinear_observation_operator(n_params, emulator, metadata, mask, state_mask, x_forecast, band):
    """JRC-TIP emulator on the band's 4-parameter subset (utils.py:130-177)."""
    LOG.info("Creating the ObsOp for band %d" % band)
    smap = band_selecta(band)
    valid = _active(mask, state_mask)
    N = int(np.asarray(x_forecast).shape[0] // n_params)
    x0 = np.asarray(x_forecast, dtype=np.float64).reshape(N, n_params)[:, smap]
    LOG.info("Running emulators")
    H0_, dH = run_emulator(emulator, x0[valid])
    H0 = np.zeros(N, dtype=np.float32)
    H0[valid] = H0_
    rows = np.zeros((N, len(smap)))
    rows[valid] = dH
    # duplicate columns cannot occur for the TIP mapper; keep generic sum anyway
    return H0, _rows_to_csr(rows, valid, n_params, cols=smap)


def _tip_device_spec(n_params, emulator, metadata, band, band_mapper=None):
    if not isinstance(emulator, GaussianProcessEmulator):
        return None
    smap = band_mapper[band] if band_mapper is not None else band_selecta(band)
    return gp_spec(emulator, smap)


create_nonlinear_observation_operator.device_spec = _tip_device_spec


def create_sar_observation_operator(n_params, forward_model, metadata, mask, state_mask, x_forecast, band):
    """Water Cloud Model operator (sar_forward_model.py:109-173).

    Fixes vs the reference: integer pixel count under Python 3 (:137) and the
    per-pixel incidence angle from ``metadata['incidence_angle']`` when present
    (the reference hard-codes 23 degrees, :156)."""
    LOG.info("Creating the ObsOp for band %d" % band)
    pol = POLARISATIONS[band]
    valid = _active(mask, state_mask)
    N = int(np.asarray(x_forecast).shape[0] // n_params)
    x0 = np.asarray(x_forecast, dtype=np.float64).reshape(N, n_params)
    theta = _theta(metadata, state_mask, N)
    fm = forward_model if callable(forward_model) else sar_observation_operator
    LOG.info("Running SAR forward model")
    H0_, dH = fm(x0[valid][:, :2], theta[valid], pol)
    H0 = np.zeros(N, dtype=np.float32)
    H0[valid] = H0_
    rows = np.zeros((N, 2))
    rows[valid] = dH
    return H0, _rows_to_csr(rows, valid, n_params, cols=[0, 1])


def _theta(metadata, state_mask, N):
    if isinstance(metadata, dict) and metadata.get("incidence_angle") is not None:
        th = np.asarray(metadata["incidence_angle"], dtype=np.float64)
        if th.ndim == 2:
            th = th[np.asarray(state_mask)]
        return np.broadcast_to(th.ravel(), (N,)).astype(np.float64)
    return np.full(N, 23.0)


def _sar_device_spec(n_params, forward_model, metadata, band, band_mapper=None):
    if callable(forward_model) and forward_model is not sar_observation_operator \
            and not isinstance(forward_model, WaterCloudModel):
        return None
    wcm = forward_model if isinstance(forward_model, WaterCloudModel) else WaterCloudModel(POLARISATIONS[band])
    smap = list(wcm.state_map) if band_mapper is None else list(band_mapper[band])
    coef = list(wcm.coefficients) + [wcm.default_theta]
    aux = None
    if isinstance(metadata, dict) and metadata.get("incidence_angle") is not None:
        aux = np.asarray(metadata["incidence_angle"], dtype=np.float32)
    return OperatorSpec(OP_SAR, smap, coef, [], 0.0, None, aux, wcm)


create_sar_observation_operator.device_spec = _sar_device_spec


def create_linear_observation_operator(n_params, emulator, metadata, mask, state_mask, x_forecast, band=None):
    """Linear/identity operator.  The reference version (utils.py:119-126) built a
    dense identity of the wrong shape; here band ``b`` observes state element
    ``b`` (identity when n_bands == n_params) unless ``emulator`` is a
    :class:`LinearOperator`.  Returns H (linear: no H0)."""
    valid = _active(mask, state_mask)
    N = int(np.asarray(x_forecast).shape[0] // n_params)
    op = emulator if isinstance(emulator, LinearOperator) else LinearOperator.select(n_params, band or 0)
    rows = np.broadcast_to(np.asarray(op.coef, dtype=np.float64), (N, n_params))
    return _rows_to_csr(np.ascontiguousarray(rows), valid, n_params)


_LINEAR_SPECS = {}


def _linear_device_spec(n_params, emulator, metadata, band, band_mapper=None):
    """Memoised (one OperatorSpec object per operator: band tables are cached by
    spec identity, engine/bands.py:TableCache)."""
    op = emulator if isinstance(emulator, LinearOperator) else LinearOperator.select(n_params, band or 0)
    coef = np.zeros(n_params)
    coef[:len(op.coef)] = op.coef
    key = (n_params, tuple(map(float, coef)), float(op.offset))
    spec = _LINEAR_SPECS.get(key)
    if spec is None:
        spec = _LINEAR_SPECS[key] = OperatorSpec(OP_LINEAR, list(range(n_params)), list(map(float, coef)), [],
                                                 float(op.offset))
    return spec


create_linear_observation_operator.device_spec = _linear_device_spec
create_linear_observation_operator.linear = True


def create_uncertainty(uncertainty, mask):
    """Diagonal sigma^2 for good observations (utils.py:109-116)."""
    good_obs = int(np.asarray(mask).sum())
    R = np.ones(good_obs) * uncertainty * uncertainty
    return sp.dia_matrix((R, 0), shape=(good_obs, good_obs))
