#!/usr/bin/env python
"""Headline benchmark: pixel-state updates/s on a full 10980² Sentinel-2 tile,
7-parameter JRC-TIP state (BASELINE.json).

One *step* = one 16-day time-grid step of ``LinearKalman``: propagation
(LAI propagator, Q[TLAI]=0.04, ``kafka_test.py:207-208``), ingest of one
observation date (2 bands as uint16 DN streamed from pinned host memory over a
side stream), Gauss-Newton iterations to the reference's global convergence
criterion (each iteration = GP emulator (T=500 training points, 4 inputs per
band) + Jacobian + normal equations + Cholesky for every pixel), and the
device output unpack (mean and 1/sqrt(diag P^-1) rasters).
A *pixel-state update* is one active pixel's full analysis for one date
(BASELINE.md), so updates/step = active pixels.

Multi-GPU: tile-DP over row strips, one process per GPU (torchrun), RCCL
collectives for the global convergence norm; the tile is fixed, so scaling is
strong.  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import datetime as dt
import json
import os
import sys
import time

import numpy as np
import torch

BASELINE_UPDATES_PER_S = 50250.0  # 8 Xeon cores, 7p-2b, chunk-parallel (kafka_test_Py36.py:254)


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=int, default=10980, help="tile edge (pixels)")
    ap.add_argument("--n-train", type=int, default=500, help="GP training points per band emulator")
    ap.add_argument("--cloud", type=float, default=0.2, help="cloud (masked) fraction per date")
    ap.add_argument("--pool", type=int, default=3, help="distinct synthetic dates kept in pinned host memory")
    ap.add_argument("--metrics", default=None)
    ap.add_argument("--device", default=None)
    ap.add_argument("--watchdog", type=float, default=0, help="dump Python stacks every N s (hang triage)")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()
    if a.watchdog > 0:
        import faulthandler
        faulthandler.dump_traceback_later(a.watchdog, repeat=True, file=sys.stderr)
    if a.verbose:
        import logging
        logging.basicConfig(level=logging.INFO, stream=sys.stderr)

    from kafka_inferenceengine_amd import (DeviceOutput, EngineConfig, JRCPrior, LinearKalman,
                                           SyntheticBHRObservations, TIP_PARAMETERS,
                                           create_nonlinear_observation_operator, propagate_information_filter_LAI)
    from kafka_inferenceengine_amd.inference import iterate_time_grid
    from kafka_inferenceengine_amd.parallel import Comm, StripPartition

    comm = Comm.from_env(device=a.device)
    if comm.distributed:
        dev = comm.device
    else:
        dev = torch.device(a.device or ("cuda" if torch.cuda.is_available() else "cpu"))
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        comm = Comm.single(dev)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    world, rank = comm.world, comm.rank
    if a.gpus != world:
        log(f"--gpus {a.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")

    H = W = a.size
    mask = np.ones((H, W), dtype=bool)
    part = StripPartition(mask, rank, world)
    t_setup = time.time()
    n_dates = a.warmup + a.steps + 1
    dates = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(n_dates)]
    obs = SyntheticBHRObservations(mask, dates=dates, n_train=a.n_train, partition=part, device=dev,
                                   n_pool=a.pool, stream=True, cloud_fraction=a.cloud, seed=0)
    prior = JRCPrior(TIP_PARAMETERS, mask)
    cfg = EngineConfig(metrics_path=a.metrics)
    kf = LinearKalman(obs, DeviceOutput(TIP_PARAMETERS), mask, create_nonlinear_observation_operator,
                      TIP_PARAMETERS, state_propagation=propagate_information_filter_LAI, prior=None, config=cfg,
                      comm=comm, partition=part)
    kf.set_trajectory_model()
    Q = np.zeros(7)
    Q[6] = 0.04
    kf.set_trajectory_uncertainty(Q)
    state = kf.state_from_prior(prior)
    obs._ensure_pool()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    log(f"rank {rank}/{world}: strip rows {part.r0}-{part.r1}, {part.N} px, setup {time.time() - t_setup:.1f}s, "
        f"pinned={obs._streamer.pinned}")

    grid = [dates[0] - dt.timedelta(days=1)] + [d + dt.timedelta(days=1) for d in dates]
    steps = list(iterate_time_grid(grid, dates))
    first = True
    times = []
    t_start = None
    for i, (t, loc, is_first) in enumerate(steps[:a.warmup + a.steps]):
        if i == a.warmup:
            comm.barrier()
            if dev.type == "cuda":
                torch.cuda.synchronize()
            t_start = time.perf_counter()
        t0 = time.perf_counter()
        state = kf.step(t, loc, state, advance=not first, all_dates=dates)
        first = False
        if dev.type == "cuda" and (i < a.warmup):
            torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        log(f"step {i} {'(warmup)' if i < a.warmup else ''} {times[-1] * 1e3:.1f} ms "
            f"gn_iters={kf.history[-1].get('gn_iterations')}")
    comm.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    elapsed = comm.max_float(elapsed)
    ok = bool(torch.isfinite(state.x[:, :state.N]).all().item())
    updates = float(part.N_total) * a.steps
    value = updates / elapsed
    if rank == 0:
        gn = [h.get("gn_iterations") for h in kf.history[a.warmup:]]
        rec = {"metric": "pixel-state updates/sec (whole node), 10980^2 S2 tile, 7-param state",
               "value": round(value, 1), "unit": "pixel-state updates/s", "n_gpus": world, "steps": a.steps,
               "warmup": a.warmup, "ms_per_step": round(1e3 * elapsed / a.steps, 3), "higher_is_better": True,
               "scaling": "strong", "vs_baseline": round(value / BASELINE_UPDATES_PER_S, 2), "dtype": "fp32",
               "data": f"synthetic (smooth random truth -> GP emulators -> 5% noise, {a.cloud:.0%} clouds, "
                       f"uint16 DN), random-init GP emulators (T={a.n_train})",
               "config": {"model": "JRC-TIP 7-param, 2-band GP-emulator operator, LAI propagator",
                          "tile": f"{H}x{W}", "active_pixels": part.N_total, "global_batch": part.N_total,
                          "seq_len": 1, "bands": 2, "gp_train_points": a.n_train,
                          "parallelism": f"tile-dp{world}", "gn_iterations": gn, "finite": ok,
                          "ingest_bytes_per_step": obs.ingest_bytes() // max(1, len(steps))}}
        print(json.dumps(rec), flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
