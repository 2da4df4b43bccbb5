"""Compare two bench.py --dump-state runs of one tile (any rank counts): the
strips of each are concatenated in rank order and compared, and the chunk
Gauss-Newton histograms of their bench records (the last JSON line of each
log) must match.

    python scripts/compare_strips.py PREFIX_A LOG_A PREFIX_B LOG_B
"""
import glob
import json
import sys

import numpy as np


def load(prefix):
    files = sorted(glob.glob(f"{prefix}.strip*.npy"), key=lambda f: int(f.rsplit("strip", 1)[1].split(".")[0]))
    if not files:
        raise SystemExit(f"no strips for {prefix}")
    return np.concatenate([np.load(f) for f in files], axis=1), len(files)


def record(log):
    lines = [ln for ln in open(log) if ln.startswith("{")]
    return json.loads(lines[-1])


def main():
    pa, la, pb, lb = sys.argv[1:5]
    xa, na = load(pa)
    xb, nb = load(pb)
    ra, rb = record(la), record(lb)
    ha, hb = ra["config"].get("chunk_gn_histogram"), rb["config"].get("chunk_gn_histogram")
    d = float(np.abs(xa - xb).max()) if xa.shape == xb.shape else None
    out = {"strips": [na, nb], "shape": [list(xa.shape), list(xb.shape)], "max_abs_diff": d,
           "bit_identical": bool(xa.shape == xb.shape and np.array_equal(xa, xb)),
           "histograms": [ha, hb], "histograms_equal": ha == hb,
           "gn_iterations": [ra["config"]["gn_iterations"], rb["config"]["gn_iterations"]]}
    print(json.dumps(out))
    if xa.shape != xb.shape or ha != hb or d > 1e-4:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
