"""Compare the matrix-core analysis against the VALU record loop per pixel on a
realistic TIP problem, with a small grid cap so every wave walks many tiles.
    python scripts/debug_mfma_tiles.py [--size 512] [--max-blocks 16] [--variants 0]"""
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
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--max-blocks", type=int, default=16)
    ap.add_argument("--variants", default="0")
    ap.add_argument("--partials", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    mask = np.ones((a.size, a.size), bool)
    obs = k.SyntheticBHRObservations(mask, n_train=500, device=dev, stream=False, n_pool=1)
    date = obs.dates[0]
    bands = [(obs.band_specs[b], obs.get_device_band_data(date, b)) for b in range(2)]
    tab = build_table([s for s, _ in bands], [d for _, d in bands], 7, RecordCache(), dev)
    N = obs.N
    mu, P, Pi = k.tip_prior()
    g = torch.Generator(device=dev).manual_seed(0)
    sd = torch.tensor(np.sqrt(np.diag(P)) * 0.3, dtype=torch.float32, device=dev)[:, None]
    xf = torch.tensor(mu, dtype=torch.float32, device=dev)[:, None] + sd * torch.randn(7, N, device=dev, generator=g)
    xf[6].clamp_(0.05, 0.95)
    Pf = torch.tensor(pack_matrix(Pi), dtype=torch.float32, device=dev)[:, None].expand(28, N).contiguous()
    ext = K.ext()
    res = {}
    outs = {}
    for cap in (0, a.max_blocks):
        ext.set_max_blocks(cap or K.ext().MAX_BLOCKS)
        for v in [4] + [int(x) for x in a.variants.split(",")]:
            xo = torch.zeros_like(xf)
            part = K.partials_buffer(N, dev) if a.partials else None
            K.analysis(7, tab, xf, xf, Pf, xo, torch.zeros_like(Pf), None, None, part, variant=v)
            torch.cuda.synchronize()
            outs[(cap, v)] = xo.cpu().numpy()
    ref = outs[(0, 4)]
    for key, x in outs.items():
        d = np.abs(x - ref).max(0)
        bad = np.nonzero(d > 1e-2)[0]
        res[str(key)] = {"max": float(d.max()), "n_bad": int(bad.size),
                         "first_bad": bad[:8].tolist(), "bad_tiles": np.unique(bad // 64)[:12].tolist(),
                         "bad_lane_hist": np.bincount(bad % 64, minlength=64).tolist()
                         if bad.size else []}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
