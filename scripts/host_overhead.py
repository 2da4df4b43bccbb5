#!/usr/bin/env python
"""Host (Python) overhead per time-grid step: the headline engine on a tiny
tile (device time negligible); times steps, then profiles them with cProfile."""
import argparse
import cProfile
import datetime as dt
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from kafka_inferenceengine_amd.inference import iterate_time_grid  # noqa: E402
from kafka_inferenceengine_amd.parallel import Comm, StripPartition  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=256)
ap.add_argument("--steps", type=int, default=100)
ap.add_argument("--config", default="tip7")
a0 = ap.parse_args()
a = argparse.Namespace(warmup=3, steps=2 * a0.steps, n_train=None, pool=3, cloud=0.2, metrics=None, band_parallel=1)
dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
comm = Comm.single(dev)
mask = np.ones((a0.size, a0.size), bool)
part = StripPartition(mask, 0, 1)
obs, kf, state, dates = bench.build(a0.config, a, mask, part, dev, comm)
grid = [dates[0] - dt.timedelta(days=1)] + [d + dt.timedelta(days=1) for d in dates]
steps = list(iterate_time_grid(grid, dates))
first = True


def run(sl):
    global state, first
    for t, loc, _ in sl:
        state = kf.step(t, loc, state, advance=not first, all_dates=dates)
        first = False


run(steps[:3])
torch.cuda.synchronize() if dev.type == "cuda" else None
t0 = time.perf_counter()
run(steps[3:3 + a0.steps])
torch.cuda.synchronize() if dev.type == "cuda" else None
print(f"host+device ms/step at {a0.size}^2: {(time.perf_counter() - t0) * 1e3 / a0.steps:.3f}")
prof = cProfile.Profile()
prof.enable()
run(steps[3 + a0.steps:3 + 2 * a0.steps])
torch.cuda.synchronize() if dev.type == "cuda" else None
prof.disable()
st = pstats.Stats(prof)
st.sort_stats("cumulative").print_stats(45)
st.sort_stats("tottime").print_stats(30)
