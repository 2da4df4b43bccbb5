"""Line tables of the first Gauss-Newton iteration at the fused forecast
(kf_gp_mfma.h line_pos / line_eval, models/gp.py:line_table, ops/kernels.py
line_fields): every band's value and gradient at a partial-reset forecast from
float64 cubic pieces instead of the matrix-core GP sums."""
from __future__ import annotations

import datetime as dt

import numpy as np
import pytest
import torch

import kafka_inferenceengine_amd as k
from kafka_inferenceengine_amd.ops import kernels as K
from kafka_inferenceengine_amd.utils.blocks import pack_matrix

import kernel_cases as C

pytestmark = pytest.mark.gpu


def _first_iteration_h0(device, prob, spec, xa, pa, line):
    n, N = prob["n"], prob["N"]
    h0 = [torch.zeros(N, dtype=torch.float32, device=device) for _ in range(2)]
    tab = C.table(prob, device, h0_outs=h0)
    xo = torch.zeros((n, N), device=device)
    ao = torch.zeros((n * (n + 1) // 2, N), device=device)
    st = torch.zeros(N, dtype=torch.uint8, device=device)
    h = K.prop_args(n, spec, xa, pa, fused=True)
    K.analysis(n, tab, None, None, None, xo, ao, None, st, None, prop=h, line=line)
    torch.cuda.synchronize()
    return [t.cpu().numpy().astype(np.float64) for t in h0], xo.cpu().numpy()


@pytest.mark.parametrize("pmask", [1 << 6, 0])
def test_line_first_iteration_h0_against_float64(cuda, pmask):
    """H0 at the forecast from the line tables equals the float64 emulator to
    float32 rounding, and is at least as close as the GP sums on the matrix
    cores (LAI propagator: TLAI varies, the rest at the prior mean; prior
    reset: one point for every pixel)."""
    prob = C.tip_problem(N=20000, seed=4, n_train=500, dn16=True)   # DN16: the SPEC_PROP kernels
    n, N = prob["n"], prob["N"]
    mu, _, Pi = k.tip_prior()
    rng = np.random.default_rng(4)
    A = C.spd_blocks(rng, N, n, 5.0) * 0.2 + prob["Pf"]
    spec = {"mode": 1, "m": np.ones(n), "q": np.full(n, 0.04), "prop_mask": pmask, "reset_mean": mu,
            "reset_cinv": pack_matrix(Pi)}
    xa, pa = C.soa(prob["x"], cuda), C.packed(A, cuda)
    xf = np.broadcast_to(np.asarray(mu, dtype=np.float32).astype(np.float64), (N, n)).copy()
    if pmask:
        xf[:, 6] = prob["x"][:, 6].astype(np.float32)
    errs = {}
    for line in (True, False):
        h0, _ = _first_iteration_h0(cuda, prob, spec, xa, pa, line)
        e = 0.0
        for b in range(2):
            obs = prob["bands"][b][1] > 0
            H, _ = prob["ems"][b].predict(xf[:, k.TIP_BAND_MAPPER[b]])
            e = max(e, float(np.abs(h0[b][obs] - H[obs]).max()))
        errs[line] = e
    assert errs[True] < 2e-6, errs
    assert errs[True] <= errs[False] + 1e-7, errs


def test_line_tables_are_used_and_cached(cuda):
    """A fused-forecast launch of the TIP bands gets a line table (built once per
    band specs and reset mean); an explicit forecast or several propagated
    parameters get none."""
    prob = C.tip_problem(N=512, seed=1, n_train=64)
    n = prob["n"]
    mu, _, Pi = k.tip_prior()
    tab = C.table(prob, cuda)
    xa = C.soa(prob["x"], cuda)
    pa = C.packed(prob["Pf"], cuda)
    spec = {"mode": 1, "m": np.ones(n), "q": np.full(n, 0.04), "prop_mask": 1 << 6, "reset_mean": mu,
            "reset_cinv": pack_matrix(Pi)}
    h = K.prop_args(n, spec, xa, pa, fused=True)
    lf = K.line_fields(tab, h, n, cuda)
    assert lf is not None and lf[4] == 6 and lf[0].is_cuda and lf[3] >= 256
    assert K.line_fields(tab, h, n, cuda)[0] is lf[0]
    h2 = K.prop_args(n, dict(spec, prop_mask=0b1000001), xa, pa, fused=True)
    assert K.line_fields(tab, h2, n, cuda) is None
    assert K.line_fields(tab, None, n, cuda) is None


@pytest.mark.parametrize("cfg", ["tip", "tip_gain", "prosail"])
def test_line_tables_engine_runs_close_to_gp_sums(cuda, cfg):
    """Whole runs with and without line tables: the same Gauss-Newton counts and
    states within the matrix-core GP's own float32 error."""
    mask = np.ones((96, 128), bool)
    mask[10:30, 40:90] = False
    outs = []
    for line in (True, False):
        cfg_e = k.EngineConfig(line_tables=line, analysis_form="gain" if cfg == "tip_gain" else "information")
        if cfg.startswith("tip"):
            grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(5)]
            obs = k.SyntheticBHRObservations(mask, n_train=500, device=cuda, stream=False, n_pool=3, field_cell=8)
            kf = k.LinearKalman(obs, None, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS,
                                device=cuda, state_propagation=k.propagate_information_filter_LAI, config=cfg_e)
            kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
            st = kf.run(grid, kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask)), None, None)
        else:
            grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=5 * i) for i in range(4)]
            obs = k.SyntheticS2Observations(mask, dates=grid, n_bands=10, n_train=250, device=cuda, stream=False,
                                            n_pool=2)
            prior = k.SAILPrior(k.SAIL_PARAMETERS, mask)
            kf = k.LinearKalman(obs, None, mask, k.create_prosail_observation_operator, k.SAIL_PARAMETERS,
                                state_propagation=None, prior=prior, device=cuda, config=cfg_e)
            st = kf.run([grid[0] - dt.timedelta(days=1)] + [d + dt.timedelta(days=1) for d in grid],
                        kf.state_from_prior(prior), None, None)
        torch.cuda.synchronize()
        outs.append((st.x[:, :st.N].cpu().numpy(), [h.get("gn_iterations") for h in kf.history],
                     kf.last_status[:st.N].cpu().numpy()))
    (xa, ia, sa), (xb, ib, sb) = outs
    assert ia == ib
    assert np.isfinite(xa).all()
    assert not np.array_equal(xa, xb)      # the line path ran (first iteration differs in the last bits)
    ok = (sa & K.ST_FALLBACK) == 0
    assert np.abs(xa - xb)[:, ok].max() < 2e-3, np.abs(xa - xb)[:, ok].max()
