"""K9 spatial prior against the exact coupled GMRF solve (SURVEY.md §2.7 K9,
BASELINE config 4).  The final Gauss-Newton iteration's linear system

    A_reg,p x_p - g E_R sum_{q ~ p} x_q,R = b_p,   A_reg,p = A_p + g deg_p E_R

(A_reg and u = A_reg^-1 b are what the engine keeps for that iteration) is
assembled over the whole tile and solved with SciPy's sparse direct solver;
the engine's state after the configured smoother is compared with it.  The
reference has no spatial coupling; it plugs into the GN loop of
/root/reference/kafka/linear_kf.py:253-307."""
import datetime as dt

import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spl

import kafka_inferenceengine_amd as k
from kafka_inferenceengine_amd.utils.blocks import unpack_blocks

GAMMA = 5.0


def _run(**cfg):
    mask = np.ones((48, 40), bool)
    mask[10:18, 5:22] = False          # irregular neighbourhoods around a hole
    obs = k.SyntheticBHRObservations(mask, n_train=80, device="cpu", stream=False, n_pool=2, seed=5, field_cell=8,
                                     cloud_fraction=0.3)
    kf = k.LinearKalman(obs, None, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS, device="cpu",
                        state_propagation=k.propagate_information_filter_LAI,
                        config=k.EngineConfig(spatial_gamma=GAMMA, spatial_params=[6], **cfg))
    kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
    prior = k.JRCPrior(k.TIP_PARAMETERS, mask)
    x0, Pi = prior.process_prior(None)
    grid = [obs.dates[0] - dt.timedelta(days=1), obs.dates[0] + dt.timedelta(days=1)]
    st = kf.run(grid, x0, None, Pi)
    return kf, st


def _exact(kf, st):
    n, N, R = kf.n_params, kf.N, 6
    A = unpack_blocks(st.P[:, :N].numpy().astype(np.float64), n)          # A_reg per pixel
    u = kf._reg_uv[0][:, :N].numpy().astype(np.float64).T                # A_reg^-1 b
    b = np.einsum("pij,pj->pi", A, u)
    rows, cols = np.nonzero(np.ones((n, n), bool))
    ii = (np.arange(N)[:, None] * n + rows[None, :]).ravel()
    jj = (np.arange(N)[:, None] * n + cols[None, :]).ravel()
    vals = A[:, rows, cols].ravel()
    nbr = kf.partition.neighbour_table()                                  # [4, N], one rank: no halo
    p_idx = np.repeat(np.arange(N)[None, :], 4, 0)
    ok = nbr >= 0
    ci = p_idx[ok] * n + R
    cj = nbr[ok].astype(np.int64) * n + R
    M = sp.csr_matrix((np.r_[vals, -GAMMA * np.ones(ci.size)], (np.r_[ii, ci], np.r_[jj, cj])), shape=(n * N, n * N))
    x = spl.spsolve(M.tocsc(), b.ravel()).reshape(N, n)
    return x.T, M, b


def _rel_err(st, x_exact):
    x = st.x[:, :x_exact.shape[1]].numpy().astype(np.float64)
    return np.abs(x - x_exact).max(1) / (np.abs(x_exact).max(1) + 1e-12)


def test_tight_chebyshev_solves_the_coupled_system():
    kf, st = _run(spatial_solver="chebyshev", spatial_tol=1e-7, spatial_max_sweeps=400)
    x_exact, M, b = _exact(kf, st)
    err = _rel_err(st, x_exact)
    assert err[6] < 2e-5 and err.max() < 2e-5, err


def test_default_solver_error_is_pinned_and_beats_four_jacobi_sweeps():
    """The default (Chebyshev, spatial_tol = 1e-3) reaches the coupled
    solution to ~1e-3 of the regularised field; the round-2 smoother (4 plain
    Jacobi sweeps per GN iteration) is reported next to it."""
    kf, st = _run()
    x_exact, _, _ = _exact(kf, st)
    err_c = _rel_err(st, x_exact)
    kj, sj = _run(spatial_solver="jacobi", jacobi_sweeps=4)
    xj_exact, _, _ = _exact(kj, sj)
    err_j = _rel_err(sj, xj_exact)
    print(f"TLAI rel. error vs exact coupled solve: chebyshev(tol 1e-3) {err_c[6]:.2e}, "
          f"jacobi x4 {err_j[6]:.2e}; chebyshev (rho, sweeps) per GN iteration "
          f"{[(r['rho'], r['sweeps']) for d in kf.metrics.records for r in d.get('spatial', [])]}")
    assert err_c[6] < 2e-3, err_c
    assert err_c[6] < err_j[6], (err_c[6], err_j[6])


def test_spatial_residual_logged_per_gn_iteration(tmp_path):
    kf, st = _run(metrics_path=str(tmp_path / "m.jsonl"))
    dates = [r for r in kf.metrics.records if r.get("event") == "date"]
    sp_rec = dates[-1]["spatial"]
    assert len(sp_rec) == dates[-1]["n_iter"]
    # the first GN iteration is the plain per-pixel solve (spatial_first_plain)
    assert sp_rec[0]["solver"] == "plain" and sp_rec[0]["sweeps"] == 0
    for r in sp_rec[1:]:
        assert r["solver"] == "chebyshev" and 0 < r["rho"] < 1 and r["sweeps"] >= 1
        assert np.isfinite(r["residual_rms"]) and r["residual_rms"] < 1e-2
