#!/usr/bin/env python
"""Interleaved A/B timing of analysis-kernel variants in ONE process
(cdna_hip_programming.md §5.4 rule 24) on the bench problem (TIP, 2 GP bands,
DN16 observations)."""
import argparse
import json
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])

import kafka_inferenceengine_amd as k  # noqa: E402
from kafka_inferenceengine_amd.engine.bands import RecordCache, build_table  # noqa: E402
from kafka_inferenceengine_amd.ops import kernels as K  # noqa: E402
from kafka_inferenceengine_amd.utils.blocks import pack_matrix  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--n-train", type=int, default=500)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="4,0")
    ap.add_argument("--uniform", action="store_true", help="every pixel at the prior mean (old behaviour)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    mask = np.ones((a.size, a.size), bool)
    obs = k.SyntheticBHRObservations(mask, n_train=a.n_train, device=dev, stream=False, n_pool=1)
    date = obs.dates[0]
    bands = [(obs.band_specs[b], obs.get_device_band_data(date, b)) for b in range(2)]
    tab = build_table([s for s, _ in bands], [d for _, d in bands], 7, RecordCache(), dev)
    N = obs.N
    mu, P, Pi = k.tip_prior()
    if a.uniform:
        xf = torch.tensor(mu, dtype=torch.float32, device=dev)[:, None].expand(7, N).contiguous()
    else:
        # per-pixel states spread like a real tile's (a uniform state makes every
        # column of the MFMA operands identical, which lets the chip clock higher)
        g = torch.Generator(device=dev).manual_seed(0)
        sd = torch.tensor(np.sqrt(np.diag(P)) * 0.3, dtype=torch.float32, device=dev)[:, None]
        xf = torch.tensor(mu, dtype=torch.float32, device=dev)[:, None] + sd * torch.randn(7, N, device=dev,
                                                                                            generator=g)
        xf[6].clamp_(0.05, 0.95)
    Pf = torch.tensor(pack_matrix(Pi), dtype=torch.float32, device=dev)[:, None].expand(28, N).contiguous()
    xo = torch.empty_like(xf)
    ao = torch.empty_like(Pf)
    variants = a.variants.split(",")   # "V" or "V@MAXBLOCKS" (grid cap; 0 = default)
    ext = K.ext()
    default_cap = ext.get_max_blocks()
    parts = {}
    for v in variants:
        cap = int(v.split("@")[1]) if "@" in v else 0
        ext.set_max_blocks(cap or default_cap)
        parts[v] = K.partials_buffer(N, dev)
    times = {v: [] for v in variants}
    outs = {}
    for r in range(a.rounds + 1):
        for v in variants:
            vv, cap = (v.split("@") + ["0"])[:2]
            ext.set_max_blocks(int(cap) or default_cap)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            K.analysis(7, tab, xf, xf, Pf, xo, ao, None, None, parts[v], fast=(vv != "g"),
                       variant=0 if vv == "g" else int(vv))
            e.record()
            e.synchronize()
            if r:
                times[v].append(s.elapsed_time(e))
            outs[v] = xo.clone()
    ref = outs[variants[0]]
    # GP point evaluations per launch: valid (unmasked) pixel-bands x training points
    pts = sum(int((d.decode()[1] > 0).sum().item()) for _, d in bands) * a.n_train
    res = {}
    for v in variants:
        t = np.array(times[v])
        res[v] = {"median_ms": float(np.median(t)), "min_ms": float(t.min()),
                  "gpoints_per_s": round(pts / (np.median(t) * 1e-3) / 1e9, 1),
                  "max_abs_diff_vs_first": float((outs[v] - ref).abs().max())}
    print(json.dumps({"size": a.size, "N": N, "n_train": a.n_train, "points": pts, "variants": res}))


if __name__ == "__main__":
    main()
