"""Command-line drivers (the reference's de-facto CLI are its three driver
scripts):

  run    — assimilation run: TIP/BHR (kafka_test.py), S2 PROSAIL (kafka_test_S2.py),
           S1 SAR, identity, multi-sensor; synthetic sensors or file readers;
           GeoTIFF or in-memory output; checkpoint/resume; metrics JSONL.
           Launch with torchrun for tile-DP over GPUs.
  farm   — chunk farming over ranks (kafka_test_Py36.py: get_chunks + client.map).
  chunks — print get_chunks(nx, ny, block).
  info   — device, native extension and compiled kernel sizes.

Examples:
  python -m kafka_inferenceengine_amd run --sensor bhr --size 2400 2400 --steps 23 --out /tmp/kafka
  torchrun --nproc-per-node 8 -m kafka_inferenceengine_amd run --sensor s2 --size 10980 10980
  python -m kafka_inferenceengine_amd run --sensor s2 --s2-folder DATA --emulator-folder EMUS --mask mask.tif
"""
from __future__ import annotations

import argparse
import datetime as dt
import json
import logging
import sys

import numpy as np


def _mask(args):
    from .input_output.tiff import read_tiff, tiff_info

    if args.mask:
        m, info = read_tiff(args.mask)
        return m.astype(bool), info
    ref = _file_reference_raster(args)
    if ref is not None:                 # file-driven run: the grid of the data (ROI-cropped)
        info = tiff_info(ref)
        h, w = info["shape"]
        roi = getattr(args, "roi", None)
        if roi:
            h, w = roi[3] - roi[1], roi[2] - roi[0]
            gt = list(info.get("geotransform", [0, 1, 0, 0, 0, -1]))
            gt[0] += roi[0] * gt[1]
            gt[3] += roi[1] * gt[5]
            info["geotransform"] = gt
        return np.ones((h, w), dtype=bool), info
    h, w = args.size
    return np.ones((h, w), dtype=bool), {}


def _file_reference_raster(args):
    """First raster of a file-driven BHR / S2 / S1 run (defines the grid when no --mask)."""
    import glob
    import os

    if getattr(args, "bhr_folder", None):
        f = sorted(glob.glob(os.path.join(args.bhr_folder, "*_kernels_b0_k0.tif")))
    elif getattr(args, "s2_folder", None):
        f = sorted(glob.glob(os.path.join(args.s2_folder, "**", "B02_sur.tif"), recursive=True))
    elif getattr(args, "s1_folder", None):
        f = sorted(glob.glob(os.path.join(args.s1_folder, "S1_*", "theta.tif")))
    else:
        return None
    if not f:
        raise SystemExit("no input rasters found in the data folder")
    return f[0]


# The reference drivers' chunking: one LinearKalman per get_chunks tile, so the
# Gauss-Newton exit test is taken per chunk -- 256^2 for the MCD43 / TIP driver
# (kafka_test_Py36.py:241), 128^2 for the Sentinel-2 driver (kafka_test_S2.py:202)
DRIVER_CHUNK = {"bhr": 256, "identity": 256, "s2": 128, "multisensor": 128}


def _engine_config(args):
    """EngineConfig of a run: the command line / YAML, with the reference
    driver's per-chunk convergence as the default (``--convergence-chunk tile``
    tests over the whole state instead)."""
    from .engine.config import EngineConfig

    cfg = EngineConfig.from_args(args)
    explicit = getattr(args, "convergence_chunk", None) is not None
    if not explicit and getattr(args, "config_file", None):
        import yaml
        with open(args.config_file) as f:
            explicit = "convergence_chunk" in (yaml.safe_load(f) or {})
    if not explicit and cfg.convergence_chunk is None and args.sensor in DRIVER_CHUNK and cfg.spatial_gamma <= 0:
        b = DRIVER_CHUNK[args.sensor]
        cfg.convergence_chunk = [b, b]
        cfg.validate()
    return cfg


def _build(args, comm):
    import kafka_inferenceengine_amd as k
    from .parallel import StripPartition

    mask, info = _mask(args)
    part = StripPartition(mask, comm.rank, comm.world)
    dev = comm.device
    cfg = _engine_config(args)
    syn = dict(partition=part, device=dev, stream=True, cloud_fraction=args.cloud, seed=args.seed)
    if args.sensor == "bhr":
        if args.bhr_folder:      # MCD43 kernel-weight rasters (kafka_test.py:156-217)
            from .input_output.sentinel import BHRObservations
            emu = args.emulator or k.make_tip_emulators(n_train=args.n_train or 500)
            roi = args.roi or [0, 0, None, None]
            obs = BHRObservations(emu, args.bhr_folder, period=args.period, ulx=roi[0], uly=roi[1], lrx=roi[2],
                                  lry=roi[3])
        else:
            obs = k.SyntheticBHRObservations(mask, n_train=args.n_train or 500, **syn)
        params, factory = k.TIP_PARAMETERS, k.create_nonlinear_observation_operator
        prior = k.JRCPrior(params, mask)
        prop = k.propagate_information_filter_LAI
        q = np.array([0, 0, 0, 0, 0, 0, 0.04])
        step = 16
    elif args.sensor in ("s2", "multisensor"):
        if args.s2_folder:
            from .input_output.sentinel import Sentinel2Observations
            if not args.emulator_folder:
                raise SystemExit("--s2-folder needs --emulator-folder")
            # a --mask GeoTIFF is the state grid every band is warped onto
            # (kafka_test_S2.py:155-162); without one the granule grid (ROI-cropped)
            obs = Sentinel2Observations(args.s2_folder, args.emulator_folder, args.mask or mask,
                                        roi=None if args.mask else args.roi)
        elif args.sensor == "s2":
            obs = k.SyntheticS2Observations(mask, n_bands=10, n_train=args.n_train or 250, **syn)
        else:
            obs = k.MultiSensorObservations([
                k.SyntheticS2Observations(mask, n_bands=13, n_train=args.n_train or 250, **syn),
                k.SyntheticOLCIObservations(mask, n_bands=21, n_train=args.n_train or 250,
                                            **{**syn, "seed": args.seed + 21})])
        params, factory = k.SAIL_PARAMETERS, k.create_prosail_observation_operator
        prior = k.SAILPrior(params, mask)
        prop, q, step = None, None, 2
    elif args.sensor == "s1":
        if args.s1_folder:       # sigma0_VV / sigma0_VH / theta GeoTIFFs per acquisition
            from .input_output.sentinel import S1Observations
            obs = S1Observations(args.s1_folder, args.mask or mask, roi=None if args.mask else args.roi)
        else:
            obs = k.SyntheticS1Observations(mask, **syn)
        params, factory = ["lai", "sm"], k.create_sar_observation_operator
        prior = k.GaussianPrior(params, mask, [2.0, 0.25], np.diag([1.0, 0.01]))
        prop, q, step = None, None, 6
    elif args.sensor == "identity":
        obs = k.SyntheticIdentityObservations(mask, **syn)
        params, factory = k.TIP_PARAMETERS, k.create_linear_observation_operator
        prior = k.JRCPrior(params, mask)
        prop = k.propagate_information_filter_LAI
        q = np.array([0, 0, 0, 0, 0, 0, 0.04])
        step = 5
    else:
        raise SystemExit(f"unknown sensor {args.sensor}")
    if args.s2_folder or args.s1_folder or args.bhr_folder:   # file readers define the output grid (as the reference drivers)
        projection, geotransform = obs.define_output()
    else:
        projection, geotransform = info.get("projection", ""), info.get("geotransform", [0, 1, 0, 0, 0, -1])
    if args.out:
        out = k.KafkaOutput(params, geotransform, projection,
                            args.out, prefix=args.prefix, level=args.out_level, gather=args.out_gather,
                            predictor=3 if args.out_fast else 1, strategy="rle" if args.out_fast else None,
                            keep_timesteps=args.out_keep, encoder=args.out_encoder)
    else:
        out = k.DeviceOutput(params)
    kf = k.LinearKalman(obs, out, mask, factory, params, state_propagation=prop,
                        prior=None if prop is not None else prior, config=cfg, comm=comm, partition=part)
    kf.set_trajectory_model()
    if q is not None:
        kf.set_trajectory_uncertainty(q)
    dates = sorted(obs.dates)
    n = min(args.steps, len(dates)) if args.steps else len(dates)
    grid = [dates[0] - dt.timedelta(days=1)] + [dates[0] + dt.timedelta(days=step * (i + 1) - 1) for i in range(n)]
    return kf, prior, grid, out


def cmd_run(args):
    from .parallel import Comm

    import kafka_inferenceengine_amd as k

    cfg = _engine_config(args)
    comm = Comm.from_env(device=args.device, band_parallel=getattr(args, "band_parallel", None) or 1,
                         timeout_s=cfg.comm_timeout_s)
    if not comm.distributed and comm.band is None:
        import torch
        dev = args.device or ("cuda" if torch.cuda.is_available() else "cpu")
        comm = Comm.single(dev if dev != "cuda" else torch.device("cuda", torch.cuda.current_device()))
    kf, prior, grid, out = _build(args, comm)
    import time
    t_run = time.perf_counter()
    start = None
    if args.resume:
        from .input_output.checkpoint import CheckpointManager
        path = CheckpointManager.resolve(args.resume)
        state = kf.run(grid, None, None, None, resume_from=path)
    else:
        start = kf.state_from_prior(prior)
        state = kf.run(grid, start, None, None)
    t_flush = time.perf_counter()
    if hasattr(out, "flush"):
        out.flush()
    t_end = time.perf_counter()
    if comm.rank == 0:
        rec = {"timesteps": len(kf.history), "pixels": kf.n_total,
               "gn_iterations": [h.get("gn_iterations") for h in kf.history],
               "finite": bool(np.isfinite(state.x[:, :state.N].cpu().numpy()).all()),
               # end to end (ingest, assimilation, output drained) and per timestep
               "wall_s": round(t_end - t_run, 3), "output_drain_s": round(t_end - t_flush, 3),
               "timestep_wall_ms": [round(1e3 * h["wall_s"], 1) for h in kf.history if "wall_s" in h]}
        if kf.timer.enabled:
            rec["phases_ms"] = kf.timer.cumulative()
            ing = getattr(kf.observations, "_ingest", None)
            if ing is not None:
                rec["ingest"] = {"bytes_read": ing.bytes_read, "bytes_h2d": ing.bytes_h2d, "pinned": ing.pinned}
        ck = getattr(kf, "checkpointer", None)
        if ck is not None and ck.stats["bytes"]:
            rec["checkpoint"] = {k_: [round(v, 3) for v in vals] for k_, vals in ck.stats.items() if k_ != "bytes"}
            rec["checkpoint"]["GB"] = [round(b / 1e9, 2) for b in ck.stats["bytes"]]
        if getattr(out, "write_s", None):
            # writer telemetry: queue depth, engine waits on the writer, encode time, bytes
            rec["output"] = {"files": len(out.written), "write_ms": [round(1e3 * t, 1) for t in out.write_s],
                             **out.writer_stats()}
        print(json.dumps(rec))
    comm.destroy()


def cmd_farm(args):
    """Independent engine per chunk, chunks round-robin over ranks."""
    import torch

    import kafka_inferenceengine_amd as k
    from .parallel import Comm
    from .parallel.farm import run_chunks

    comm = Comm.from_env(device=args.device)
    mask, _ = _mask(args)
    H, W = mask.shape

    def fn(chunk):
        x0, y0, w, h, no = chunk
        sub = mask[y0:y0 + h, x0:x0 + w]
        dev = comm.device if comm.distributed else torch.device("cuda" if torch.cuda.is_available() else "cpu")
        obs = k.SyntheticBHRObservations(sub, n_train=args.n_train or 200, device=dev, stream=False,
                                         seed=args.seed + no)
        out = k.KafkaOutput(k.TIP_PARAMETERS, None, "", args.out, prefix=hex(no)) if args.out else None
        kf = k.LinearKalman(obs, out, sub, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS, device=dev)
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.025]))
        grid = [obs.dates[0] - dt.timedelta(days=1)] + [d + dt.timedelta(days=1) for d in obs.dates[:args.steps]]
        st = kf.run(grid, kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, sub)), None, None)
        if out is not None:
            out.flush()
        return int(st.N)

    res = run_chunks(W, H, args.block, fn, comm if comm.distributed else None, skip_empty_mask=mask)
    if res is not None:
        print(json.dumps({"chunks": len(res), "pixels": sum(v or 0 for v in res.values())}))
    comm.destroy()


def cmd_synth_s2(args):
    """Write a synthetic Sentinel-2 archive (tiled-DEFLATE GeoTIFF granules +
    emulators) for file-driven runs: ``run --sensor s2 --s2-folder OUT/data
    --emulator-folder OUT/emus``."""
    import torch

    from .input_output.synthetic import synthesize_s2_archive

    h, w = args.size
    dev = args.device or ("cuda" if torch.cuda.is_available() else "cpu")
    data, emus, dates = synthesize_s2_archive(args.out, np.ones((h, w), bool), args.dates, args.n_train, args.seed,
                                              dev, args.cloud)
    print(json.dumps({"data": data, "emulators": emus, "dates": [d.isoformat() for d in dates]}))


def cmd_chunks(args):
    from .input_output.utils import get_chunks

    for c in get_chunks(args.nx, args.ny, args.block):
        print(*c)


def cmd_info(args):
    import torch

    from .ops import SUPPORTED_NP, ext_path

    print(json.dumps({"torch": torch.__version__, "hip": torch.version.hip, "gpu": torch.cuda.is_available(),
                      "device_name": torch.cuda.get_device_name(0) if torch.cuda.is_available() else None,
                      "extension": ext_path(), "compiled_n_params": list(SUPPORTED_NP)}))


def main(argv=None):
    from .engine.config import EngineConfig

    ap = argparse.ArgumentParser(prog="kafka_inferenceengine_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run", help="assimilation run")
    r.add_argument("--sensor", default="bhr", choices=["bhr", "s2", "s1", "identity", "multisensor"])
    r.add_argument("--size", type=int, nargs=2, default=[512, 512], metavar=("H", "W"))
    r.add_argument("--mask", default=None, help="state mask GeoTIFF (non-zero = active)")
    r.add_argument("--s2-folder", default=None)
    r.add_argument("--emulator-folder", default=None)
    r.add_argument("--bhr-folder", default=None, help="MCD43 kernel rasters A%%Y%%j_kernels_b{0,1}_k{0,1,2}.tif + _qa")
    r.add_argument("--s1-folder", default=None, help="S1_* acquisition folders with sigma0_VV/VH and theta")
    r.add_argument("--emulator", default=None, help="emulator-set .npz for --bhr-folder (default: synthetic TIP)")
    r.add_argument("--period", type=int, default=16, help="take every period-th BHR date")
    r.add_argument("--roi", type=int, nargs=4, default=None, metavar=("ULX", "ULY", "LRX", "LRY"))
    r.add_argument("--steps", type=int, default=0, help="time steps (0: all dates)")
    r.add_argument("--n-train", type=int, default=None)
    r.add_argument("--cloud", type=float, default=0.2)
    r.add_argument("--seed", type=int, default=0)
    r.add_argument("--out", default=None, help="GeoTIFF output folder (default: device-resident output)")
    r.add_argument("--prefix", default=None)
    r.add_argument("--out-level", type=int, default=6, help="DEFLATE level of the output GeoTIFFs (1: fastest)")
    r.add_argument("--out-fast", action="store_true",
                   help="floating-point predictor + run-length DEFLATE (zlib's Z_RLE: about 3x faster encoding "
                        "than zlib level 6; always zlib, also where libdeflate is present -- writer_stats reports "
                        "the encoder)")
    r.add_argument("--out-encoder", default="auto", choices=["auto", "device", "host"],
                   help="DEFLATE tiles encoded on the GPU (device: predictor 3 + fixed-Huffman run-length streams, "
                        "only compressed tiles cross PCIe) or by the host thread pool; auto: device on a GPU")
    r.add_argument("--out-keep", type=int, default=None,
                   help="keep only the newest N timesteps' output files on local disk")
    r.add_argument("--out-gather", action="store_true", help="gather strips to rank 0 and write one raster")
    r.add_argument("--resume", default=None, help="checkpoint directory (latest) or checkpoint path")
    r.add_argument("--log-level", default="WARNING")
    EngineConfig.add_arguments(r)
    r.set_defaults(fn=cmd_run)
    f = sub.add_parser("farm", help="chunk farming over ranks (kafka_test_Py36.py)")
    f.add_argument("--size", type=int, nargs=2, default=[512, 512], metavar=("H", "W"))
    f.add_argument("--mask", default=None)
    f.add_argument("--block", type=int, nargs=2, default=[256, 256])
    f.add_argument("--steps", type=int, default=4)
    f.add_argument("--n-train", type=int, default=None)
    f.add_argument("--seed", type=int, default=0)
    f.add_argument("--out", default=None)
    f.add_argument("--device", default=None)
    f.set_defaults(fn=cmd_farm)
    y = sub.add_parser("synth-s2", help="write a synthetic Sentinel-2 GeoTIFF archive")
    y.add_argument("--out", required=True)
    y.add_argument("--size", type=int, nargs=2, default=[512, 512], metavar=("H", "W"))
    y.add_argument("--dates", type=int, default=4)
    y.add_argument("--n-train", type=int, default=250)
    y.add_argument("--seed", type=int, default=0)
    y.add_argument("--cloud", type=float, default=0.2)
    y.add_argument("--device", default=None)
    y.set_defaults(fn=cmd_synth_s2)
    c = sub.add_parser("chunks", help="print get_chunks")
    c.add_argument("nx", type=int)
    c.add_argument("ny", type=int)
    c.add_argument("--block", type=int, nargs=2, default=[256, 256])
    c.set_defaults(fn=cmd_chunks)
    i = sub.add_parser("info")
    i.set_defaults(fn=cmd_info)
    args = ap.parse_args(argv)
    if getattr(args, "log_level", None):
        logging.basicConfig(level=getattr(logging, args.log_level.upper()), stream=sys.stderr)
    args.fn(args)


if __name__ == "__main__":
    main()
