#!/usr/bin/env python
"""Where a float32 pipeline loses precision on the SURVEY §7.3 slice: the
float64 torch oracle (tests/oracle.py) re-run with one part in float32 at a
time -- the GP's squared distances, its kernel-weighted sums, the solver's
float32 cast (the reference's own loss, solvers.py:127-134) -- each against
the plain float64 oracle on the same observations (max-norm x / P^-1, the
per-pixel tail), next to the engine's own errors.

    python scripts/mvp_precision_sources.py --size 1024
"""
import argparse
import json
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0] + "/tests")
sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])

import kafka_inferenceengine_amd as k  # noqa: E402
from kafka_inferenceengine_amd.utils.blocks import pack_blocks  # noqa: E402
from oracle import oracle_run_blocks_torch  # noqa: E402
from test_mvp import Q6, _grid  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--dates", type=int, default=10)
    a = ap.parse_args()
    import torch
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    mask = np.ones((a.size, a.size), bool)
    dates, grid = _grid(a.dates)
    jp = k.JRCPrior(k.TIP_PARAMETERS, mask)
    obs = k.SyntheticBHRObservations(mask, dates=dates, n_train=500, device=dev, stream=True, n_pool=a.dates)
    kf = k.LinearKalman(obs, k.DeviceOutput(k.TIP_PARAMETERS), mask, k.create_nonlinear_observation_operator,
                        k.TIP_PARAMETERS, state_propagation=k.propagate_information_filter_LAI, device=dev)
    kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, Q6]))
    st = kf.run(grid, kf.state_from_prior(jp), None, None)
    N = st.N
    mu, _, ci = k.tip_prior()

    def oracle(**kw):
        x, A, it = oracle_run_blocks_torch(obs, mask, k.TIP_BAND_MAPPER, grid, mu, ci, q=[0, 0, 0, 0, 0, 0, Q6],
                                           x0=jp.mean, A0=jp.inv_covar, device=dev, **kw)
        P = pack_blocks(A).astype(np.float64)
        return x.T, P, it

    xo, Po, it0 = oracle()
    if Po.shape[0] != xo.shape[0] * (xo.shape[0] + 1) // 2:
        Po = Po.T
    xs_scale = np.abs(xo).max(1) + 1e-12
    ps_scale = np.abs(Po).max(1) + 1e-12

    def errs(x, P, it):
        if P.shape != Po.shape:
            P = P.T
        px = (np.abs(x - xo) / xs_scale[:, None]).max(0)
        pp = (np.abs(P - Po) / ps_scale[:, None]).max(0)
        return {"gn_equal": it == it0, "x_rel": float(px.max()), "P_rel": float(pp.max()),
                "x_p99.99": float(np.percentile(px, 99.99)), "P_p99.99": float(np.percentile(pp, 99.99)),
                "n_over_pins": int(((px > 5e-4) | (pp > 1e-3)).sum())}

    out = {"size": a.size, "engine": errs(st.x[:, :N].cpu().numpy().astype(np.float64),
                                          st.P[:, :N].cpu().numpy().astype(np.float64),
                                          [h["gn_iterations"][0] for h in kf.history])}
    for name, kw in (("solver_f32_cast", dict(cast_f32=True)), ("gp_exponent_f32", dict(gp_f32=("exponent",))),
                     ("gp_sums_f32", dict(gp_f32=("sums",))), ("gp_all_f32", dict(gp_f32=("exponent", "sums")))):
        out[name] = errs(*oracle(**kw))
        print(name, json.dumps(out[name]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
