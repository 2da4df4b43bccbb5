#!/usr/bin/env python
"""Host time between a date's decision read-back and the next date's analysis
launch (the GPU idles through it): wraps PendingSum.result and the native
analysis launch with perf_counter stamps, runs bench-like steps, and prints the
per-date gap distribution plus a cProfile of the host work inside the gaps.

    python scripts/host_gap_probe.py --size 3882 --steps 30 [--set convergence_chunk=tile]
"""
import argparse
import cProfile
import datetime as dt
import io
import json
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])

import kafka_inferenceengine_amd as k  # noqa: E402
from kafka_inferenceengine_amd.ops import _ext  # noqa: E402
from kafka_inferenceengine_amd.parallel import comm as C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=3882)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--set", action="append", default=[])
    a = ap.parse_args()
    over = {}
    for kv in a.set:
        key, val = kv.split("=", 1)
        over[key] = val
    dev = torch.device("cuda", 0)
    mask = np.ones((a.size, a.size), bool)
    n = a.warmup + a.steps + 11       # + 10 profiled dates after the stamped ones
    dates = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(n)]
    obs = k.SyntheticBHRObservations(mask, dates=dates, n_train=500, device=dev, n_pool=3, stream=True)
    cfg = dict(convergence_chunk=[256, 256])
    cfg.update(over)
    kf = k.LinearKalman(obs, k.DeviceOutput(k.TIP_PARAMETERS), mask, k.create_nonlinear_observation_operator,
                        k.TIP_PARAMETERS, state_propagation=k.propagate_information_filter_LAI, device=dev,
                        config=k.EngineConfig(**cfg))
    kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
    state = kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask))
    obs._ensure_pool()
    stamps = []
    real_result = C.PendingSum.result
    ext = _ext.require_ext()
    real_analysis = ext.analysis

    def result(self, j=0):
        v = real_result(self, j)
        stamps.append(("result", time.perf_counter()))
        return v

    def analysis(*args):
        stamps.append(("launch", time.perf_counter()))
        return real_analysis(*args)

    real_step = kf.step

    def step(*args, **kw):
        stamps.append(("step_start", time.perf_counter()))
        v = real_step(*args, **kw)
        stamps.append(("step_end", time.perf_counter()))
        return v

    C.PendingSum.result = result
    ext.analysis = analysis
    kf.step = step
    grid = [dates[0] - dt.timedelta(days=1)] + [d + dt.timedelta(days=1) for d in dates]
    from kafka_inferenceengine_amd.inference import iterate_time_grid
    steps = list(iterate_time_grid(grid, dates))
    prof = cProfile.Profile()
    first = True
    for i, (t, loc, _) in enumerate(steps[:a.warmup + a.steps + 10]):
        if i == a.warmup:
            torch.cuda.synchronize()
            stamps.clear()
        if i == a.warmup + a.steps:      # the stamped dates ran without the profiler
            torch.cuda.synchronize()
            stamps.append(("stop", time.perf_counter()))
            prof.enable()
        state = kf.step(t, loc, state, advance=not first, all_dates=dates)
        first = False
    prof.disable()
    torch.cuda.synchronize()
    stamps = stamps[:[k for k, _ in stamps].index("stop")]
    # per date: last read-back -> end of step (tail), end of step -> next step
    # (the caller), next step start -> its first analysis launch (head)
    tail, caller, head, gaps = [], [], [], []
    last_result = last_end = start = None
    for kind, ts in stamps:
        if kind == "result":
            last_result = ts
        elif kind == "step_end":
            if last_result is not None:
                tail.append(ts - last_result)
            last_end = ts
        elif kind == "step_start":
            if last_end is not None:
                caller.append(ts - last_end)
            start = ts
        elif kind == "launch" and start is not None:
            head.append(ts - start)
            if last_result is not None:
                gaps.append(ts - last_result)
            start = last_result = None

    def stat(v):
        g = 1e6 * np.array(v)
        return {"n": int(g.size), "median": round(float(np.median(g)), 1), "p90": round(float(np.percentile(g, 90)), 1)} \
            if g.size else None
    print(json.dumps({"size": a.size, "set": over, "dates": a.steps, "gap_us": stat(gaps), "tail_us": stat(tail),
                      "caller_us": stat(caller), "head_us": stat(head)}))
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("cumulative").print_stats(40)
    print(s.getvalue())


if __name__ == "__main__":
    main()
