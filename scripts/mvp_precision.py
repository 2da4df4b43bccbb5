#!/usr/bin/env python
"""SURVEY §7.3 MVP slice on one device against the float64 block oracle,
for several analysis variants (0: matrix-core GP, 4: f32 VALU record loop) and
the host runner: one JSON line each (final x / packed P errors, per-date
drift).  Where the device loses precision relative to the host runner.

    python scripts/mvp_precision.py [--size 256] [--variants 0,4] [--host] [--torch-oracle]"""
import argparse
import json
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]
sys.path.insert(0, ROOT)
sys.path.insert(0, ROOT + "/tests")

import torch  # noqa: E402

from kafka_inferenceengine_amd.ops import kernels as K  # noqa: E402
from test_mvp import mvp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--variants", default="0,4")
    ap.add_argument("--host", action="store_true")
    ap.add_argument("--n-dates", type=int, default=10)
    ap.add_argument("--torch-oracle", action="store_true", help="the float64 oracle's torch twin on the device (1024^2)")
    a = ap.parse_args()
    runs = []
    if torch.cuda.is_available():
        runs += [("cuda", int(v)) for v in a.variants.split(",") if v != ""]
    if a.host:
        runs.append(("cpu", 0))
    for dev, v in runs:
        K.DEFAULT_VARIANT = K.Variant(v)
        r = mvp(torch.device("cuda", 0) if dev == "cuda" else "cpu", a.size, n_dates=a.n_dates, progress=True,
                torch_oracle=a.torch_oracle and dev == "cuda")
        r.update(device=dev, variant=v)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
