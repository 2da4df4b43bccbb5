"""Per-chunk Gauss-Newton iteration histograms of a hard-PROSAIL tile for a few
tolerances (picks the GPU test's problem; prints one JSON line per setting).

    python scripts/chunk_probe.py [--size 1024] [--block 256] [--tols 1e-5,2e-5,5e-5]"""
import argparse
import datetime as dt
import json
import time

import numpy as np
import torch

import kafka_inferenceengine_amd as k


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--block", type=int, default=256)
    ap.add_argument("--tols", default="1e-5,2e-5,5e-5,1e-4")
    ap.add_argument("--n-train", type=int, default=100)
    a = ap.parse_args()
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    dates = [dt.datetime(2017, 7, 3) + dt.timedelta(days=2 * i) for i in range(3)]
    grid = [dates[0] - dt.timedelta(days=1)] + [d + dt.timedelta(days=1) for d in dates]
    mask = np.ones((a.size, a.size), bool)
    for tol in [float(t) for t in a.tols.split(",")]:
        obs = k.SyntheticS2Observations(mask, dates=dates, n_bands=10, n_train=a.n_train, device=dev, stream=False,
                                        n_pool=3, hard=True, spread_scale=1.0, rel_unc=0.02, seed=1)
        prior = k.SAILPrior(k.SAIL_PARAMETERS, mask)
        kf = k.LinearKalman(obs, None, mask, k.create_prosail_observation_operator, k.SAIL_PARAMETERS,
                            state_propagation=None, prior=prior, device=dev,
                            config=k.EngineConfig(convergence_tolerance=tol, convergence_chunk=[a.block, a.block]))
        t0 = time.perf_counter()
        kf.run(grid, kf.state_from_prior(prior), None, None)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        print(json.dumps({"tol": tol, "block": a.block, "size": a.size, "s": round(time.perf_counter() - t0, 3),
                          "chunk_iters": [h["chunk_iters"][0] for h in kf.history]}), flush=True)


if __name__ == "__main__":
    main()
