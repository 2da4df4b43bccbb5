"""State propagation, prior blending and Hessian corrections — reference API.

Signatures follow ``kafka/inference/kf_tools.py`` so a reference user can swap
imports; the bodies operate on per-pixel blocks (vectorised NumPy, float64)
instead of global SuperLU solves.  Every propagator carries a ``device_spec``
(mode + parameters of the gfx950 propagate kernel, ``csrc/kf_core.h``
``pixel_propagate``) that the engine uses on its device path.
"""
from __future__ import annotations

import logging
from dataclasses import dataclass, field

import numpy as np
import scipy.sparse as sp

from ..models.operators import band_selecta
from ..models.priors import tip_prior
from ..utils.blocks import blocks_to_sparse, sparse_to_blocks

LOG = logging.getLogger(__name__)

# keep in sync with csrc/kf_core.h PropMode
PROP_PRIOR, PROP_PRIOR_PARTIAL, PROP_INFO_APPROX, PROP_INFO_EXACT, PROP_STANDARD, PROP_IDENTITY = range(6)


class NoHessianMethod(Exception):
    """Forward model cannot provide a Hessian (kf_tools.py:13-17)."""

    def __init__(self, message):
        super().__init__(message)
        self.message = message


@dataclass
class PropagatorSpec:
    """Device description of a propagator."""
    mode: int
    output: str = "precision"                    # 'precision' | 'covariance'
    propagated: tuple = ()                       # PROP_PRIOR_PARTIAL
    reset_mean: np.ndarray | None = None         # PROP_PRIOR / PROP_PRIOR_PARTIAL
    reset_cinv: np.ndarray | None = None
    extra: dict = field(default_factory=dict)


def _diag(m, n_total=None):
    if m is None:
        return None
    if sp.issparse(m):
        return np.asarray(m.diagonal())
    m = np.asarray(m)
    return np.diag(m) if m.ndim == 2 else m


def _apply_M(M_matrix, x):
    if M_matrix is None:
        return np.asarray(x) * 1.0
    return np.asarray(M_matrix.dot(x)).ravel() if hasattr(M_matrix, "dot") else np.asarray(M_matrix) @ x


# ------------------------------------------------------------------ priors
def tip_prior_noLAI(prior):
    """Tiled TIP prior without LAI information (the reference called
    ``tip_prior`` with the wrong arity, kf_tools.py:118-120)."""
    return tip_prior_full(prior)


def tip_prior_full(prior):
    """TIP prior tiled over ``prior['n_pixels']`` (kf_tools.py:123-133)."""
    x_prior, _, c_inv_prior = tip_prior()
    n_pixels = int(prior["n_pixels"])
    mean = np.tile(x_prior, n_pixels)
    blocks = np.broadcast_to(c_inv_prior.astype(np.float32), (n_pixels, 7, 7))
    return mean, blocks_to_sparse(np.ascontiguousarray(blocks), "csr", np.float32)


def blend_prior(prior_mean, prior_cov_inverse, x_forecast, P_forecast_inverse, quirk: bool = True,
                n_params: int | None = None):
    """Gaussian product of prior and forecast (kf_tools.py:75-96).

    The reference swaps the operands of the right-hand side
    (``b = P_f^-1 mu + C^-1 x_f``); ``quirk=True`` (the reference-API default)
    reproduces that, ``quirk=False`` is the textbook product."""
    combined = P_forecast_inverse + prior_cov_inverse
    if quirk:
        b = P_forecast_inverse.dot(prior_mean) + prior_cov_inverse.dot(x_forecast)
    else:
        b = P_forecast_inverse.dot(x_forecast) + prior_cov_inverse.dot(prior_mean)
    b = np.asarray(b, dtype=np.float32).astype(np.float64)
    n = n_params or _guess_block(combined, len(b))
    blocks = sparse_to_blocks(combined, n, check=False).astype(np.float32).astype(np.float64)
    x = np.linalg.solve(blocks, b.reshape(-1, n, 1))[..., 0].ravel()
    return x, combined


def _guess_block(m, size):
    """Smallest n whose n x n diagonal blocks hold every non-zero of m."""
    coo = sp.coo_matrix(m) if sp.issparse(m) else sp.coo_matrix(np.asarray(m))
    for n in range(1, 65):
        if size % n == 0 and np.all((coo.row // n) == (coo.col // n)):
            return n
    raise ValueError("matrix is not block diagonal")


def propagate_and_blend_prior(x_analysis, P_analysis, P_analysis_inverse, M_matrix, Q_matrix,
                              prior=None, state_propagator=None, date=None, reference_quirks: bool = True):
    """Propagator then prior blend (kf_tools.py:136-171).  ``reference_quirks``
    selects the reference's swapped blend (default, the reference API) or the
    Gaussian product; ``LinearKalman`` passes its ``EngineConfig.reference_quirks``
    so host and device blends agree."""
    if state_propagator is not None:
        x_forecast, P_forecast, P_forecast_inverse = state_propagator(
            x_analysis, P_analysis, P_analysis_inverse, M_matrix, Q_matrix)
    if prior is not None:
        prior_mean, prior_cov_inverse = prior.process_prior(date, inv_cov=True)
    if prior is not None and state_propagator is not None:
        x_combined, combined_cov_inv = blend_prior(prior_mean, prior_cov_inverse, x_forecast, P_forecast_inverse,
                                                   quirk=reference_quirks)
        return x_combined, None, combined_cov_inv
    elif prior is not None:
        return prior_mean, None, prior_cov_inverse
    elif state_propagator is not None:
        return x_forecast, P_forecast, P_forecast_inverse
    return None, None, None


# ------------------------------------------------------------- propagators
def propagate_standard_kalman(x_analysis, P_analysis, P_analysis_inverse, M_matrix, Q_matrix,
                              prior=None, state_propagator=None, date=None):
    """x_f = M x_a, P_f = P_a + Q (kf_tools.py:174-205)."""
    x_forecast = M_matrix.dot(x_analysis)
    P_forecast = P_analysis + Q_matrix
    return x_forecast, P_forecast, None


propagate_standard_kalman.device_spec = PropagatorSpec(PROP_STANDARD, output="covariance")


def propagate_information_filter_SLOW(x_analysis, P_analysis, P_analysis_inverse, M_matrix, Q_matrix,
                                      prior=None, state_propagator=None, date=None, n_params=None):
    """Exact information propagation P_f^-1 = (I + P_a^-1 Q)^-1 P_a^-1 (kf_tools.py:208-245),
    solved block by block."""
    x_forecast = _apply_M(M_matrix, x_analysis)
    n = n_params or _guess_block(P_analysis_inverse, len(x_forecast))
    Ai = sparse_to_blocks(P_analysis_inverse, n, check=False).astype(np.float64)
    q = _diag(Q_matrix).reshape(-1, n)
    lhs = np.eye(n)[None] + Ai * q[:, None, :]
    Pf = np.linalg.solve(lhs, Ai)
    return x_forecast, None, blocks_to_sparse(Pf, "csr")


propagate_information_filter_SLOW.device_spec = PropagatorSpec(PROP_INFO_EXACT)


def propagate_information_filter_approx_SLOW(x_analysis, P_analysis, P_analysis_inverse, M_matrix, Q_matrix,
                                             prior=None, state_propagator=None, date=None):
    """Diagonal approximation D = 1/(1 + diag(P^-1) diag(Q)) (kf_tools.py:247-289)."""
    x_forecast = _apply_M(M_matrix, x_analysis)
    d = _diag(P_analysis_inverse)
    D = 1. / (1. + d * _diag(Q_matrix))
    n = len(d)
    return x_forecast, None, sp.dia_matrix((d * D, 0), shape=(n, n)).tocsr()


propagate_information_filter_approx_SLOW.device_spec = PropagatorSpec(PROP_INFO_APPROX)

# the reference test-suite imports this name (tests/test_kf.py:16); its golden
# diagonal is the diagonal approximation's.
propagate_information_filter = propagate_information_filter_approx_SLOW


def make_partial_prior_propagator(prior_mean, prior_cov_inverse, propagated, name="partial_prior"):
    """Generalised ``propagate_information_filter_LAI``: every parameter is reset to
    the prior except the ``propagated`` indices, whose mean is carried by M and
    whose variance is inflated by Q: P_f^-1[k,k] = 1/(1/P_a^-1[k,k] + Q[k])."""
    prior_mean = np.asarray(prior_mean, dtype=np.float64)
    prior_cov_inverse = np.asarray(prior_cov_inverse, dtype=np.float64)
    n = prior_mean.size
    propagated = tuple(int(k) for k in np.atleast_1d(propagated))

    def propagator(x_analysis, P_analysis, P_analysis_inverse, M_matrix, Q_matrix,
                   prior=None, state_propagator=None, date=None):
        x_forecast = _apply_M(M_matrix, x_analysis)
        n_pixels = len(x_analysis) // n
        x0 = np.tile(prior_mean, n_pixels)
        blocks = np.broadcast_to(prior_cov_inverse, (n_pixels, n, n)).copy()
        dA = _diag(P_analysis_inverse)
        dQ = _diag(Q_matrix)
        for k in propagated:
            x0[k::n] = x_forecast[k::n]
            blocks[:, k, k] = 1.0 / ((1.0 / dA[k::n]) + dQ[k::n])
        return x0, None, blocks_to_sparse(blocks.astype(np.float32), "csr")

    propagator.__name__ = name
    propagator.device_spec = PropagatorSpec(PROP_PRIOR_PARTIAL, propagated=propagated, reset_mean=prior_mean,
                                            reset_cinv=prior_cov_inverse)
    return propagator


_tip_mean, _, _tip_cinv = tip_prior()
propagate_information_filter_LAI = make_partial_prior_propagator(_tip_mean, _tip_cinv, (6,),
                                                                 "propagate_information_filter_LAI")
propagate_information_filter_LAI.__doc__ = (
    "JRC-TIP LAI-only propagation (kf_tools.py:292-314): all parameters reset to the TIP prior "
    "except TLAI (index 6), whose precision is inflated by Q.")


def make_no_propagation(prior_mean, prior_cov_inverse, name="no_propagation"):
    prior_mean = np.asarray(prior_mean, dtype=np.float64)
    prior_cov_inverse = np.asarray(prior_cov_inverse, dtype=np.float64)
    n = prior_mean.size

    def propagator(x_analysis, P_analysis, P_analysis_inverse, M_matrix, Q_matrix,
                   prior=None, state_propagator=None, date=None):
        n_pixels = len(x_analysis) // n
        blocks = np.broadcast_to(prior_cov_inverse.astype(np.float32), (n_pixels, n, n))
        return np.tile(prior_mean, n_pixels), None, blocks_to_sparse(np.ascontiguousarray(blocks), "csr")

    propagator.__name__ = name
    propagator.device_spec = PropagatorSpec(PROP_PRIOR, reset_mean=prior_mean, reset_cinv=prior_cov_inverse)
    return propagator


no_propagation = make_no_propagation(_tip_mean, _tip_cinv)
no_propagation.__doc__ = "Reset to the tiled TIP prior, ignoring inputs (kf_tools.py:316-353)."


def identity_propagation(x_analysis, P_analysis, P_analysis_inverse, M_matrix, Q_matrix,
                         prior=None, state_propagator=None, date=None):
    """x_f = M x_a with the analysis precision carried unchanged."""
    return _apply_M(M_matrix, x_analysis), P_analysis, P_analysis_inverse


identity_propagation.device_spec = PropagatorSpec(PROP_IDENTITY)


# ------------------------------------------------------- Hessian correction
def hessian_correction_pixel(gp, x0, C_obs_inv, innovation, band, nparams):
    selecta = band_selecta(band)
    ddH = np.asarray(gp.hessian(np.atleast_2d(x0[selecta]))).squeeze()
    big = np.zeros((nparams, nparams))
    big[np.ix_(selecta, selecta)] = ddH
    return big * C_obs_inv * innovation


def hessian_correction(gp, x0, R_mat, innovation, mask, state_mask, band, nparams, state_map=None):
    """Second-order GN correction of the likelihood Hessian (kf_tools.py:37-60),
    vectorised over pixels.  Returns 0. if the emulator has no ``hessian``."""
    if not hasattr(gp, "hessian"):
        return 0.
    C_obs_inv = _diag(R_mat)[np.asarray(state_mask).ravel()]
    m = np.asarray(mask)[np.asarray(state_mask)].ravel().astype(bool)
    smap = band_selecta(band) if state_map is None else np.asarray(state_map)
    N = m.size
    x = np.asarray(x0).reshape(N, nparams)
    blocks = np.zeros((N, nparams, nparams))
    idx = np.nonzero(m)[0]
    if idx.size:
        ddH = np.asarray(gp.hessian(x[idx][:, smap]))
        scale = (C_obs_inv[idx] * np.asarray(innovation)[idx])[:, None, None]
        blocks[np.ix_(idx, smap, smap)] = ddH * scale
    return blocks_to_sparse(blocks, "csr")


def hessian_correction_multiband(gp, x0, R_mats, innovations, masks, state_mask, n_bands, nparams):
    """Sum of per-band corrections (kf_tools.py:63-72)."""
    gps = gp if isinstance(gp, (list, tuple)) else [gp] * n_bands
    return sum(hessian_correction(g, x0, R, inn, mk, state_mask, b, nparams)
               for g, R, inn, mk, b in zip(gps, R_mats, innovations, masks, range(n_bands)))
