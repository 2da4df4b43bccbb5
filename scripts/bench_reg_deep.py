#!/usr/bin/env python
"""K9 deep-halo timing on one MI355X: the LDS-tiled sweep pass over one rank's
strip at the N = 8 share of a 10980^2 granule (1373 x 10980), halo-free vs
with an 8-row deep halo on both sides (an interior rank), as one launch and as
the boundary-first split (boundary tile rows, then the interior), host weights
vs the device schedule.  Interleaved rounds in one process; prints one JSON
line per variant (median / min ms per pass of 8 sweeps)."""
import argparse
import json
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])

from kafka_inferenceengine_amd.ops import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--h", type=int, default=1373)
    ap.add_argument("--w", type=int, default=10980)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    h, w, d = a.h, a.w, a.depth
    N = h * w
    n, j0 = 7, 6
    g = torch.Generator(device=dev).manual_seed(0)
    u = torch.randn(n, N, device=dev, generator=g)
    v = torch.rand(n, N, device=dev, generator=g) * 0.2
    z = torch.randn(1, N + 2 * w, device=dev, generator=g)
    zp = torch.randn(1, N + 2 * w, device=dev, generator=g)
    zo = torch.empty_like(z)
    zpo = torch.empty_like(z)
    up = torch.randn(4, d * w, device=dev, generator=g)
    dn = torch.randn(4, d * w, device=dev, generator=g)
    om = [1.0, 1.3, 1.2, 1.25, 1.22, 1.21, 1.2, 1.2][:d]
    ch = [s > 0 for s in range(d)]
    rs = K.RegSchedule(N, 64, dev)
    rs.rho.fill_(0.833)
    rs.schedule(1e-3)
    geo0 = {"w": w, "h": h, "halo": 0, "n_up": 0}
    geo3 = {"w": w, "h": h, "halo": 3, "n_up": w}
    halo = (d, d, up, dn)
    T = K.reg_tile_rows(h)
    ta, tb = K.reg_boundary_tile_rows(h, d, True, True)
    mask = 1 << j0

    def plain():
        K.reg_sweeps_tiled(n, u, v, z, zp, zo, zpo, 0.9, mask, N, geo0, om, ch)

    def deep():
        K.reg_sweeps_tiled(n, u, v, z, zp, zo, zpo, 0.9, mask, N, geo3, om, ch, halo=halo)

    def deep_split():
        for tr in ((0, ta), (tb, T), (ta, tb)):
            K.reg_sweeps_tiled(n, u, v, z, zp, zo, zpo, 0.9, mask, N, geo3, om, ch, halo=halo, tile_rows=tr)

    def deep_sched():
        for tr in ((0, ta), (tb, T), (ta, tb)):
            K.reg_sweeps_tiled(n, u, v, z, zp, zo, zpo, 0.9, mask, N, geo3, halo=halo, tile_rows=tr,
                               sched=(rs.sched, rs.omega), s_base=1, nsweep=d)

    variants = {"halo_free": plain, "deep_halo": deep, "deep_halo_split": deep_split,
                "deep_halo_split_device_sched": deep_sched}
    times = {k: [] for k in variants}
    for r in range(a.rounds + 2):
        for name, fn in variants.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            e.synchronize()
            if r >= 2:
                times[name].append(s.elapsed_time(e))
    base = float(np.median(times["halo_free"]))
    for name, t in times.items():
        t = np.array(t)
        print(json.dumps({"variant": name, "strip": [h, w], "depth": d, "median_ms": round(float(np.median(t)), 4),
                          "min_ms": round(float(t.min()), 4),
                          "ratio_vs_halo_free": round(float(np.median(t)) / base, 4)}), flush=True)


if __name__ == "__main__":
    main()
