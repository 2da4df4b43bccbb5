"""Variational (information-form) Kalman analysis — reference API + float64 oracle.

``variational_kalman`` / ``variational_kalman_multiband`` / ``sort_band_data``
keep the signatures of ``kafka/inference/solvers.py:41-145``.  When the stacked
operator is per-pixel block structured (every operator in this package) the
normal equations are solved as N independent n_p x n_p systems; an arbitrary
user-supplied sparse H that couples pixels falls back to a global sparse LU,
exactly like the reference.

``analysis_blocks`` is the float64 oracle of the fused gfx950 kernel
(``csrc/kf_core.h`` ``pixel_analysis``): packed/SoA inputs, per-band
``(H0, h, y, w)``, returns x_a and the analysis precision.
"""
from __future__ import annotations

import logging

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spl

from ..utils.blocks import blocks_to_sparse, sparse_to_blocks

LOG = logging.getLogger(__name__ + ".solvers")


def _is_nonlinear(H):
    return isinstance(H, (tuple, list)) and len(H) == 2


def _weights(uncertainty, state_mask):
    sm = np.asarray(state_mask).ravel().astype(bool)
    if sp.issparse(uncertainty):
        R = np.asarray(uncertainty.diagonal())[sm]
    else:
        u = np.asarray(uncertainty)
        R = u.ravel()[sm] if u.ndim == 2 and u.shape == np.asarray(state_mask).shape else np.diag(u)[sm]
    return R


def sort_band_data(H_matrix, observations, uncertainty, mask, x0, x_forecast, state_mask):
    """Per-band (H, H0, R, y', y) with y' = y + H x0 - H0 (solvers.py:81-96)."""
    if _is_nonlinear(H_matrix):
        H0, H_ = H_matrix
        non_linear = True
    else:
        H0, H_ = 0., H_matrix
        non_linear = False
    R = _weights(uncertainty, state_mask)
    sm = np.asarray(state_mask).astype(bool)
    m = np.asarray(mask)[sm]
    y = np.where(m, np.asarray(observations)[sm], 0.)
    # masked pixels: zero weight (the reference relies on empty H rows with inf weights)
    R = np.where(m & np.isfinite(R), R, 0.)
    y_orig = y * 1.
    if non_linear:
        y = y + H_.dot(x0) - H0
    return H_, H0, R, y, y_orig


def _solve(A, b, n_params):
    """Solve the (float32-cast, as solvers.py:127-134) system; block path when possible."""
    A = A.astype(np.float32)
    b = np.asarray(b, dtype=np.float32)
    try:
        blocks = sparse_to_blocks(A, n_params, check=True)
    except ValueError:
        return spl.splu(sp.csc_matrix(A)).solve(b)
    x = np.linalg.solve(blocks.astype(np.float64), b.astype(np.float64).reshape(-1, n_params, 1))
    return x.ravel()


def variational_kalman(observations, mask, state_mask, uncertainty, H_matrix, n_params,
                       x_forecast, P_forecast, P_forecast_inv, the_metadata, approx_diagonal=True):
    """Single-band analysis linearised about x_forecast (solvers.py:41-78)."""
    H_, H0, R, y, y_orig = sort_band_data(H_matrix, observations, uncertainty, mask, x_forecast, x_forecast,
                                          state_mask)
    Rm = sp.diags(R)
    LOG.info("Creating linear problem")
    A = H_.T.dot(Rm).dot(H_) + P_forecast_inv
    b = H_.T.dot(Rm).dot(y) + P_forecast_inv.dot(x_forecast)
    LOG.info("Solving")
    x_analysis = _solve(sp.csr_matrix(A), b, n_params)
    fwd_modelled = H_.dot(x_analysis - x_forecast) + H0
    innovations = y_orig - fwd_modelled
    return x_analysis, None, A, innovations, fwd_modelled


def variational_kalman_multiband(observations_b, mask_b, state_mask, uncertainty_b, H_matrix_b, n_params,
                                 x0, x_forecast, P_forecast, P_forecast_inv, the_metadata_b,
                                 approx_diagonal=True):
    """Joint multi-band analysis (solvers.py:100-145).  Returns
    ``(x_a, None, A, innovations = y - H0, fwd_modelled)``."""
    n_bands = len(observations_b)
    Hs, H0s, Rs, ys, yos = [], [], [], [], []
    for i in range(n_bands):
        a, b, c, d, e = sort_band_data(H_matrix_b[i], observations_b[i], uncertainty_b[i], mask_b[i], x0,
                                       x_forecast, state_mask)
        Hs.append(a)
        H0s.append(np.broadcast_to(b, d.shape))
        Rs.append(c)
        ys.append(d)
        yos.append(e)
    H_ = sp.vstack(Hs).tocsr()
    H0 = np.hstack(H0s)
    R = sp.diags(np.hstack(Rs))
    y = np.hstack(ys)
    y_orig = np.hstack(yos)
    A = H_.T.dot(R).dot(H_) + P_forecast_inv
    b = H_.T.dot(R).dot(y) + P_forecast_inv.dot(x_forecast)
    LOG.info("Solving")
    x_analysis = _solve(sp.csr_matrix(A), b, n_params)
    fwd_modelled = H_.dot(x_analysis - x_forecast) + H0
    innovations = y_orig - H0  # intentional override (solvers.py:139-142)
    return x_analysis, None, A, innovations, fwd_modelled


# --------------------------------------------------------------- oracle
def analysis_blocks(x_prev, x_f, Pf_inv_blocks, bands):
    """float64 per-pixel analysis.

    x_prev, x_f: [N, n]; Pf_inv_blocks: [N, n, n];
    bands: iterable of (H0 [N], h [N, n], y [N], w [N]) evaluated at x_prev.
    Returns (x_a [N, n], A [N, n, n]).
    """
    A = np.array(Pf_inv_blocks, dtype=np.float64, copy=True)
    b = np.einsum("nij,nj->ni", A, x_f)
    for H0, h, y, w in bands:
        w = np.where(np.isfinite(w) & (w > 0), w, 0.0)
        yp = y + np.einsum("ni,ni->n", h, x_prev) - H0
        A += w[:, None, None] * h[:, :, None] * h[:, None, :]
        b += (w * yp)[:, None] * h
    x_a = np.linalg.solve(A, b[..., None])[..., 0]
    return x_a, A


def gain_blocks(x_prev, x_f, Pf_blocks, bands):
    """float64 covariance-form (Kalman gain) analysis; same linearisation."""
    P = np.array(Pf_blocks, dtype=np.float64, copy=True)
    x = np.array(x_f, dtype=np.float64, copy=True)
    for H0, h, y, w in bands:
        ok = np.isfinite(w) & (w > 0)
        ph = np.einsum("nij,nj->ni", P, h)
        s = np.einsum("ni,ni->n", h, ph) + np.where(ok, 1.0 / np.where(ok, w, 1.0), 1.0)
        innov = y - H0 + np.einsum("ni,ni->n", h, x_prev - x)
        k = np.where(ok[:, None], ph / s[:, None], 0.0)
        x = x + k * innov[:, None]
        P = P - k[:, :, None] * ph[:, None, :]
    return x, P
