"""Throughput of the native GeoTIFF writer on one 10980^2 Float32 plane
(one output raster of a Sentinel-2 granule): DEFLATE levels / strategies x
thread counts, plus a raw sequential write of the same bytes (disk bound).

    python scripts/bench_tiff_write.py [--size 10980] [--dir /tmp] [--threads 8 16 32]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=10980)
    ap.add_argument("--dir", default="/tmp")
    ap.add_argument("--threads", type=int, nargs="+", default=[8, 16, 32])
    ap.add_argument("--levels", type=int, nargs="+", default=[0, 1, 6])
    ap.add_argument("--deflate-backend", default="auto", choices=["auto", "zlib"],
                    help="DEFLATE encoder: libdeflate when present (auto) or zlib")
    a = ap.parse_args()
    from kafka_inferenceengine_amd.ops import kernels as K
    fast = K.ext().tiff_deflate_backend(a.deflate_backend)
    print(json.dumps({"deflate_backend": "libdeflate" if fast else "zlib"}), flush=True)
    from kafka_inferenceengine_amd.input_output.tiff import write_tiff

    rng = np.random.default_rng(0)
    n = a.size
    fields = {
        "noisy": (2.0 + 0.3 * rng.standard_normal((n, n), dtype=np.float32)),
        "smooth": (2.0 + np.cumsum(0.01 * rng.standard_normal((n, n), dtype=np.float32), 1)).astype(np.float32),
    }
    path = os.path.join(a.dir, "kafka_write_bench.tif")
    for name, f in fields.items():
        t = time.perf_counter()
        with open(path, "wb") as fh:
            fh.write(f.tobytes())
        dt = time.perf_counter() - t
        print(json.dumps({"field": name, "mode": "raw_write", "MBps": round(f.nbytes / dt / 1e6, 1)}), flush=True)
        for lvl in a.levels:
            for th in a.threads:
                t = time.perf_counter()
                write_tiff(path, f, [0, 10, 0, 0, 0, -10], "EPSG:32630", level=lvl, threads=th)
                dt = time.perf_counter() - t
                print(json.dumps({"field": name, "level": lvl, "threads": th, "s": round(dt, 3),
                                  "MBps": round(f.nbytes / dt / 1e6, 1),
                                  "ratio": round(os.path.getsize(path) / f.nbytes, 3)}), flush=True)
    os.remove(path)


if __name__ == "__main__":
    main()
