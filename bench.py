#!/usr/bin/env python
"""Benchmarks: pixel-state updates/s (BASELINE.json).

Headline (default ``--config tip7``): full 10980² Sentinel-2 tile, 7-parameter
JRC-TIP state.  One *step* = one 16-day time-grid step of ``LinearKalman``:
propagation (LAI propagator, Q[TLAI]=0.04, ``kafka_test.py:207-208``), ingest
of one observation date (2 bands of uint16 DN streamed from pinned host memory
on a side stream), Gauss-Newton iterations to the reference's global
convergence criterion (each iteration = GP emulator (T=500 training points, 4
inputs per band) + Jacobian + normal equations + Cholesky for every pixel), and
the device output unpack (mean and 1/sqrt(diag P^-1) rasters).  A pixel-state
update is one active pixel's full analysis for one date, so
updates/step = active pixels.

Other BASELINE.json configs: ``identity7`` (1024² tile, identity operator,
bf16 observations), ``prosail10`` (S2 granule, 10-param PROSAIL, 10 band GP
emulators, SAIL prior reset — kafka_test_S2.py), ``spatial`` (TIP with the GMRF
spatial prior and RCCL halo exchange), ``multisensor`` (S2 13-band + OLCI-like
21-band joint operator on the PROSAIL state).

Multi-GPU: tile-DP over row strips, one process per GPU (torchrun), RCCL for
the global convergence norm (and halos); the tile is fixed, so scaling is
strong.  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import datetime as dt
import json
import os
import sys
import time

import numpy as np
import torch

# 8 Xeon cores, chunk-parallel (kafka_test_Py36.py:254): 7p-2b 50,250/s;
# 10p-10b ~4,600/s (581/s x 8, linear scaling assumed).
BASELINE_7P = 50250.0
BASELINE_10P = 4600.0
HEADLINE_METRIC = "pixel-state updates/sec (whole node), 10980^2 S2 tile, 7-param state"

CONFIGS = {
    # chunk: the reference drivers' Gauss-Newton exit test per get_chunks tile
    # (one LinearKalman per chunk: 256^2 in the MCD43/TIP driver, kafka_test_Py36.py:241;
    # 128^2 in the S2 driver, kafka_test_S2.py:202); --set convergence_chunk=tile
    # tests over the whole state instead
    "tip7": dict(size=10980, n_train=500, chunk=256,
                 model="JRC-TIP 7-param, 2-band GP-emulator operator, LAI propagator, GN to convergence per 256^2 "
                       "chunk", baseline=BASELINE_7P),
    "identity7": dict(size=1024, chunk=256, model="7-param state, identity observation operator (7 bands), "
                                                  "bf16 observations, LAI propagator", baseline=BASELINE_7P),
    "prosail10": dict(size=10980, n_train=250, chunk=128,
                      model="PROSAIL 10-param, 10-band S2 GP emulators, SAIL prior reset, GN to convergence per "
                            "128^2 chunk", baseline=BASELINE_10P),
    # harder 10p-10b problem: T=500, strongly non-linear
    # emulators (Beer-law gap fraction, saturating leaf optics), wider truth.
    # Convergence-driven with the reference driver's semantics: the exit test
    # ||dx|| / len(x) < 1e-3 per 128^2 chunk (kafka_test_S2.py:202 chunks the S2
    # tile into 128^2 LinearKalman runs; engine/chunks.py), each chunk frozen
    # when it converges -- over the whole tile the test is met after 2
    # iterations by any problem
    "prosail10_hard": dict(size=10980, n_train=500, hard=True, spread=1.0, rel_unc=0.04, chunk=128,
                           model="PROSAIL 10-param, 10-band S2 GP emulators (T=500, non-linear), SAIL prior reset, "
                                 "GN to convergence per 128^2 chunk", baseline=BASELINE_10P),
    "spatial": dict(size=10980, n_train=500, gamma=5.0, tol=1e-3,
                    model="JRC-TIP 7-param + GMRF spatial prior on TLAI (coupled solve per GN iteration: "
                          "Chebyshev-accelerated block Jacobi to 1e-3, halo exchange)",
                    baseline=BASELINE_7P),
    "multisensor": dict(size=10980, n_train=250, chunk=128,
                        model="PROSAIL 10-param, S2 13-band + OLCI-like 21-band joint GP operator, GN to convergence "
                              "per 128^2 chunk", baseline=BASELINE_10P),
}


def socket_name():
    import socket
    return socket.gethostname()


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def build(cfg_name, a, mask, part, dev, comm):
    import kafka_inferenceengine_amd as k

    c = CONFIGS[cfg_name]
    n_dates = a.warmup + a.steps + 1
    stream = not a.resident
    seed = 0
    over = {}
    for kv in getattr(a, "set", None) or []:        # --set field=value (EngineConfig A/B knobs)
        key, val = kv.split("=", 1)
        dflt = getattr(k.EngineConfig(), key)
        if isinstance(dflt, bool):
            over[key] = val.lower() in ("1", "true", "yes")
        elif dflt is None:
            over[key] = val            # parsed by EngineConfig.validate (e.g. convergence_chunk=128)
        else:
            over[key] = type(dflt)(val)

    def mkout(params):
        # --output DIR: the reference's GeoTIFF granule writer (KafkaOutput: fused
        # device rasters -> pinned host -> writer thread -> tiled DEFLATE GeoTIFF);
        # default: device-resident rasters only (DeviceOutput)
        if not a.output:
            return k.DeviceOutput(params)
        return k.KafkaOutput(params, [0.0, 10.0, 0.0, 0.0, 0.0, -10.0], "EPSG:32630", a.output,
                             prefix=f"r{comm.rank}" if comm.world > 1 else None, level=a.output_level,
                             predictor=3, strategy="rle" if a.output_level else None,
                             keep_timesteps=a.output_keep, encoder=a.output_encoder)

    def mkcfg(**kw):
        # phase_timing: hipEvent pairs around each phase on the compute stream
        # (device time, resolved after the timed region) for the per-rank record
        if "chunk" in c:
            kw.setdefault("convergence_chunk", [c["chunk"], c["chunk"]])
        return k.EngineConfig(metrics_path=a.metrics, band_parallel=a.band_parallel,
                              phase_timing=not a.no_telemetry, **{**kw, **over})
    if cfg_name in ("tip7", "spatial"):
        dates = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(n_dates)]
        obs = k.SyntheticBHRObservations(mask, dates=dates, n_train=a.n_train or c["n_train"], partition=part,
                                         device=dev, n_pool=a.pool, stream=stream, cloud_fraction=a.cloud, seed=seed)
        cfg = mkcfg()
        if cfg_name == "spatial":
            cfg = mkcfg(spatial_gamma=c["gamma"], spatial_params=[6], spatial_tol=c["tol"])
        kf = k.LinearKalman(obs, mkout(k.TIP_PARAMETERS), mask, k.create_nonlinear_observation_operator,
                            k.TIP_PARAMETERS, state_propagation=k.propagate_information_filter_LAI, config=cfg,
                            comm=comm, partition=part)
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
        state = kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask))
    elif cfg_name == "identity7":
        dates = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(n_dates)]
        obs = k.SyntheticIdentityObservations(mask, dates=dates, partition=part, device=dev, n_pool=a.pool,
                                              stream=stream, cloud_fraction=a.cloud, seed=seed)
        kf = k.LinearKalman(obs, mkout(k.TIP_PARAMETERS), mask, k.create_linear_observation_operator,
                            k.TIP_PARAMETERS, state_propagation=k.propagate_information_filter_LAI,
                            config=mkcfg(), comm=comm, partition=part)
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
        state = kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask))
    else:
        dates = [dt.datetime(2017, 7, 3) + dt.timedelta(days=2 * i) for i in range(n_dates)]
        T = a.n_train or c["n_train"]
        if cfg_name == "prosail10":
            obs = k.SyntheticS2Observations(mask, dates=dates, n_bands=10, n_train=T, partition=part, device=dev,
                                            n_pool=a.pool, stream=stream, cloud_fraction=a.cloud, seed=seed)
        elif cfg_name == "prosail10_hard":
            obs = k.SyntheticS2Observations(mask, dates=dates, n_bands=10, n_train=T, partition=part, device=dev,
                                            n_pool=a.pool, stream=stream, cloud_fraction=a.cloud, seed=seed,
                                            hard=True, spread_scale=c["spread"], rel_unc=c["rel_unc"])
        else:
            s2 = k.SyntheticS2Observations(mask, dates=dates, n_bands=13, n_train=T, partition=part, device=dev,
                                           n_pool=a.pool, stream=stream, cloud_fraction=a.cloud, seed=seed)
            olci = k.SyntheticOLCIObservations(mask, dates=dates, n_bands=21, n_train=T, partition=part,
                                               device=dev, n_pool=a.pool, stream=stream, cloud_fraction=a.cloud,
                                               seed=seed + 21)
            obs = k.MultiSensorObservations([s2, olci])
        prior = k.SAILPrior(k.SAIL_PARAMETERS, mask)
        kf = k.LinearKalman(obs, mkout(k.SAIL_PARAMETERS), mask, k.create_prosail_observation_operator,
                            k.SAIL_PARAMETERS, state_propagation=None, prior=prior,
                            config=mkcfg(), comm=comm, partition=part)
        state = kf.state_from_prior(prior)
    return obs, kf, state, dates


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="tip7", choices=sorted(CONFIGS))
    ap.add_argument("--size", type=int, default=None, help="tile edge (pixels); default per config")
    ap.add_argument("--n-train", type=int, default=None, help="GP training points per band emulator")
    ap.add_argument("--cloud", type=float, default=0.2, help="cloud (masked) fraction per date")
    ap.add_argument("--pool", type=int, default=3, help="distinct synthetic dates kept in pinned host memory")
    ap.add_argument("--metrics", default=None)
    ap.add_argument("--device", default=None)
    ap.add_argument("--profile", default=None, help="write a torch.profiler chrome trace here (rank 0)")
    ap.add_argument("--watchdog", type=float, default=0, help="dump Python stacks every N s (hang triage)")
    ap.add_argument("--host-profile", default=None, metavar="PATH",
                    help="cProfile of the timed steps' host work (rank 0) written to PATH (pstats)")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--set", action="append", default=[], metavar="FIELD=VALUE",
                    help="override an EngineConfig field (A/B runs), e.g. --set gp_split=never")
    ap.add_argument("--kernel-variant", type=int, default=0,
                    help="analysis kernel variant (ops/kernels.py Variant; A/B of a test-oracle path, e.g. 4 = "
                         "the f32 VALU record loop)")
    ap.add_argument("--band-parallel", type=int, default=1,
                    help="ranks per band group (strips x band groups; multi-band configs)")
    ap.add_argument("--band-parallel-force", action="store_true",
                    help="keep --band-parallel even where the cost model says strips are faster")
    ap.add_argument("--resident", action="store_true",
                    help="keep the synthetic observation pool in HBM (compute-only: no per-step H2D; "
                         "the default re-uploads every date from pinned host memory)")
    ap.add_argument("--rehearse-gloo", action="store_true",
                    help="multi-rank rehearsal on one GPU: gloo for device tensors (RehearsalComm), not RCCL")
    ap.add_argument("--no-telemetry", action="store_true",
                    help="no per-phase hipEvent timers (the per_rank record then has no phase times)")
    ap.add_argument("--telemetry", default="auto", choices=["auto", "on", "off"],
                    help="per-phase hipEvent timers in the timed steps: auto = on unless a warm-up step takes "
                         "under 2 ms (their event records would then be a visible share of the step)")
    ap.add_argument("--dump-state", default=None, metavar="PREFIX",
                    help="after the timed region, write each strip's final state x [n_p, N] to "
                         "PREFIX.strip<r>.npy (band slot 0 only; rehearsal checks against one rank)")
    ap.add_argument("--output", default=None, metavar="DIR",
                    help="write every timestep's mean/unc GeoTIFFs here (KafkaOutput; the timed region ends "
                         "after the writer has drained); default: device rasters only")
    ap.add_argument("--output-level", type=int, default=1, help="DEFLATE level of --output (0: uncompressed)")
    ap.add_argument("--output-encoder", default="auto", choices=["auto", "device", "host"],
                    help="DEFLATE tiles of --output encoded on the GPU (auto / device) or on the host thread pool")
    ap.add_argument("--output-keep", type=int, default=2,
                    help="keep only the newest N timesteps' files of --output on disk")
    a = ap.parse_args()
    if a.watchdog > 0:
        import faulthandler
        faulthandler.dump_traceback_later(a.watchdog, repeat=True, file=sys.stderr)
    if a.verbose:
        import logging
        logging.basicConfig(level=logging.INFO, stream=sys.stderr)

    from kafka_inferenceengine_amd.inference import iterate_time_grid
    from kafka_inferenceengine_amd.parallel import Comm, StripPartition

    from kafka_inferenceengine_amd.engine.config import EngineConfig
    from kafka_inferenceengine_amd.ops import kernels as K0
    K0.DEFAULT_VARIANT = K0.Variant(a.kernel_variant)

    # band-parallel only where its C5 all-reduce pays (parallel/policy.py); else pure strips
    from kafka_inferenceengine_amd.parallel.policy import band_parallel_decision
    c0 = CONFIGS[a.config]
    dev_type = (a.device or ("cuda" if torch.cuda.is_available() else "cpu")).split(":")[0]
    nb, npar = {"tip7": (2, 7), "spatial": (2, 7), "identity7": (7, 7), "prosail10": (10, 10),
                "prosail10_hard": (10, 10), "multisensor": (34, 10)}[a.config]
    T = 0 if a.config == "identity7" else (a.n_train or c0["n_train"])
    bp_req = a.band_parallel
    a.band_parallel, bp_why = band_parallel_decision(npar, nb, T, a.band_parallel, dev_type,
                                                     force=a.band_parallel_force)
    if bp_why:
        log(bp_why)
    if a.band_parallel_force:
        a.set.append("band_parallel_force=true")
    if a.rehearse_gloo:       # several ranks on one GPU: the gloo harness (parallel/rehearsal.py)
        from kafka_inferenceengine_amd.parallel.rehearsal import RehearsalComm as Comm
    comm = Comm.from_env(device=a.device, band_parallel=a.band_parallel, timeout_s=EngineConfig().comm_timeout_s)
    if comm.distributed or comm.band is not None:
        dev = comm.device
    else:
        dev = torch.device(a.device or ("cuda" if torch.cuda.is_available() else "cpu"))
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        comm = Comm.single(dev)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    world, rank = comm.world, comm.rank                 # strips (tile-DP)
    B = comm.band.world if comm.band is not None else 1  # band groups
    n_ranks = world * B
    g_rank = comm.ranks[rank] if comm.band is None else comm.band.ranks[comm.band.rank]
    if a.gpus != n_ranks:
        log(f"--gpus {a.gpus} but WORLD_SIZE {n_ranks}; using WORLD_SIZE")
    c = CONFIGS[a.config]
    H = W = a.size or c["size"]
    mask = np.ones((H, W), dtype=bool)
    part = StripPartition(mask, rank, world)
    t_setup = time.time()
    obs, kf, state, dates = build(a.config, a, mask, part, dev, comm)
    srcs = getattr(obs, "sources", [obs])
    for s in srcs:
        s._ensure_pool()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    log(f"rank {g_rank}/{n_ranks}: {a.config} strip rows {part.r0}-{part.r1}, {part.N} px, "
        f"setup {time.time() - t_setup:.1f}s")

    grid = [dates[0] - dt.timedelta(days=1)] + [d + dt.timedelta(days=1) for d in dates]
    steps = list(iterate_time_grid(grid, dates))
    # setup objects (torch, the engine, the pools) to the permanent generation:
    # the collector's full passes otherwise stall sub-millisecond steps by ~6 ms
    import gc
    gc.collect()
    gc.freeze()
    prof = None
    first = True
    warm_ms = None          # fastest warm-up step after the first (telemetry auto)
    telemetry = "off" if a.no_telemetry else "on"
    msgs = []   # per-step lines of the timed steps are printed after the timed region
    for i, (t, loc, is_first) in enumerate(steps[:a.warmup + a.steps]):
        if i == a.warmup:
            if a.telemetry == "off" or (a.telemetry == "auto" and warm_ms is not None
                                        and comm.max_float(warm_ms) < 2.0):
                kf.timer.enabled = False      # sub-2 ms steps: no per-phase event records
                telemetry = "off"
            comm.barrier()
            if dev.type == "cuda":
                torch.cuda.synchronize()
            if a.output:
                kf.output.flush()         # the warm-up dates' files are out of the timed region
                w0 = kf.output.writer_stats()
            ph0 = kf.timer.cumulative()   # phase totals of the warm-up steps (subtracted below)
            h2d0 = sum(s.ingest_bytes() for s in srcs)
            t_start = time.perf_counter()
            if a.profile and g_rank == 0:
                prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                                          torch.profiler.ProfilerActivity.CUDA])
                prof.__enter__()
            if a.host_profile and g_rank == 0:
                import cProfile
                hprof = cProfile.Profile()
                hprof.enable()
        t0 = time.perf_counter()
        state = kf.step(t, loc, state, advance=not first, all_dates=dates)
        first = False
        if dev.type == "cuda" and i == a.warmup - 1:
            torch.cuda.synchronize()
        step_ms = (time.perf_counter() - t0) * 1e3
        if i < a.warmup and i > 0:
            warm_ms = step_ms if warm_ms is None else min(warm_ms, step_ms)
        msgs.append(f"step {i}{' (warmup)' if i < a.warmup else ''} {step_ms:.1f} ms "
                    f"gn_iters={kf.history[-1].get('gn_iterations')}")
        if i < a.warmup:
            for m in msgs:
                log(m)
            msgs = []
    if a.host_profile and g_rank == 0 and a.steps:
        hprof.disable()
        hprof.dump_stats(a.host_profile)
    t_drain = time.perf_counter()
    if a.output:
        kf.output.flush()                 # every timed date's files are on disk
    t_drain = time.perf_counter() - t_drain
    comm.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t_local = time.perf_counter() - t_start
    elapsed = comm.max_float(t_local)
    kf.resolve_pending()      # deferred read-backs (lazy norms, per-chunk histograms) of the timed dates
    for m in msgs:
        log(m)
    # per-rank telemetry of the timed steps (device time per phase from the
    # engine's hipEvent pairs): where a multi-GPU run loses efficiency --
    # analysis kernels (load), C1 norm all-gather (waits for the slowest rank),
    # C2 halos, ingest -- gathered to rank 0 after the timed region
    ph1 = kf.timer.cumulative()
    phases = {kk: round(v - ph0.get(kk, 0.0), 3) for kk, v in ph1.items()}
    mine = {"rank": g_rank, "strip_rank": rank, "N": int(part.N), "wall_ms": round(1e3 * t_local, 3),
            "device": str(dev), "host": socket_name(),
            "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
            "analysis_ms": phases.get("analysis", 0.0), "c1_ms": phases.get("converge", 0.0),
            "halo_ms": round(phases.get("halo", 0.0) + phases.get("band_allreduce", 0.0), 3),
            "ingest_ms": phases.get("ingest", 0.0), "phases_ms": phases,
            "h2d_bytes": int(sum(s.ingest_bytes() for s in srcs) - h2d0),
            "gn_iterations": [h.get("gn_iterations") for h in kf.history[a.warmup:]]}
    if a.output:
        # granule writer over the timed dates: encode+write time per date, how long
        # the engine blocked on the writer (full queue / pinned slot), the drain
        w1 = kf.output.writer_stats()
        n_w = w1["timesteps_written"] - w0["timesteps_written"]
        ws = kf.output.write_s[w0["timesteps_written"]:]
        mine["output"] = {"dir": a.output, "deflate_level": a.output_level, "timesteps": n_w,
                          "encoder": w1.get("deflate_backend"),
                          "write_ms_mean": round(1e3 * sum(ws) / max(1, len(ws)), 3),
                          "write_ms_max": round(1e3 * max(ws), 3) if ws else None,
                          "raster_MB_per_date": round((w1["raster_bytes"] - w0["raster_bytes"]) / max(1, n_w) / 1e6, 1),
                          "file_MB_per_date": round((w1["file_bytes"] - w0["file_bytes"]) / max(1, n_w) / 1e6, 1),
                          "queue_depth_max": w1.get("queue_depth_max"),
                          "queue_wait_ms": round(1e3 * (w1.get("queue_wait_s", 0) - w0.get("queue_wait_s", 0)), 3),
                          "slot_wait_ms": round(1e3 * (w1["slot_wait_s"] - w0["slot_wait_s"]), 3),
                          "d2h_wait_ms": round(1e3 * (w1["d2h_s"] - w0["d2h_s"]), 3),
                          "prune_ms": round(1e3 * (w1["prune_s"] - w0["prune_s"]), 3),
                          "drain_ms": round(1e3 * t_drain, 3)}
    # per-chunk convergence (config.convergence_chunk): {GN iterations: chunks},
    # summed over the timed dates (the chunk decisions are the same on every rank)
    chunk_hist = {}
    for h in kf.history[a.warmup:]:
        for d in h.get("chunk_iters") or []:
            for it, n in d.items():
                chunk_hist[it] = chunk_hist.get(it, 0) + n
    per_rank = [mine]
    if n_ranks > 1:
        import torch.distributed as dist
        per_rank = [None] * dist.get_world_size()
        dist.all_gather_object(per_rank, mine)   # every rank of the job (strips x band groups)
    if hasattr(kf, "cache_stats"):
        log(f"host caches: {kf.cache_stats()}")
    from kafka_inferenceengine_amd.ops import kernels as K
    if dev.type == "cuda" and hasattr(K.ext(), "phase_clocks"):
        # measuring build (KAFKA_PROF=1): shader cycles per phase of the fused
        # analysis kernel, summed over waves, warm-up steps included
        names = ("prologue", "forecast", "band_in", "gp", "band_out", "solve", "groups")
        log("phase_clocks " + json.dumps(dict(zip(names, K.ext().phase_clocks(kf.n_params, False)))))
    if prof is not None:
        prof.__exit__(None, None, None)
        prof.export_chrome_trace(a.profile)
    # numerical health over the WHOLE job: finite everywhere (min over ranks) and
    # the fraction of pixels whose solve fell back to the forecast (should be ~0)
    ok_local = bool(torch.isfinite(state.x[:, :state.N]).all().item())
    if a.dump_state and (comm.band is None or comm.band.rank == 0):
        np.save(f"{a.dump_state}.strip{rank}.npy", state.x[:, :state.N].cpu().numpy())
    st_last = getattr(kf, "last_status", None)
    n_fb = 0 if st_last is None or not state.N else int(((st_last[:state.N] & K.ST_FALLBACK) > 0).sum().item())
    # GP inputs outside the emulators' training box (models/operators.py GP_DOMAIN_MARGIN) at the last date
    n_ood = 0 if st_last is None or not state.N else \
        int(((st_last[:state.N] & K.ST_OUT_OF_DOMAIN) > 0).sum().item())
    ok = comm.max_float(0.0 if ok_local else 1.0) == 0.0
    fallback = comm.sum_int(n_fb) / max(1, part.N_total)
    out_of_domain = comm.sum_int(n_ood) / max(1, part.N_total)
    # distinct GPUs behind the ranks (a one-GPU multi-rank rehearsal is not scaling)
    n_dev = n_ranks
    if n_ranks > 1:
        import torch.distributed as dist
        ids = [None] * dist.get_world_size()
        # GPU ranks sharing a device count once; CPU ranks (gloo harness) each count
        dist.all_gather_object(ids, (socket_name(), str(dev)) if dev.type == "cuda" else (socket_name(), g_rank))
        n_dev = len(set(ids))
    value = float(part.N_total) * a.steps / elapsed
    if g_rank == 0:
        gn = [h.get("gn_iterations") for h in kf.history[a.warmup:]]
        metric = HEADLINE_METRIC if a.config == "tip7" and H == 10980 else \
            f"pixel-state updates/sec (whole node), {H}x{W} tile, {a.config}"
        ingest = sum(s.ingest_bytes() for s in srcs) // max(1, a.warmup + a.steps)
        n_gn = sum(sum(g) if isinstance(g, (list, tuple)) else (g or 0) for g in gn)
        rec = {"metric": metric, "value": round(value, 1), "unit": "pixel-state updates/s", "n_gpus": n_dev,
               "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(1e3 * elapsed / a.steps, 3),
               "higher_is_better": True, "scaling": "strong",
               "vs_baseline": round(value / c["baseline"], 2), "dtype": "fp32" if a.config != "identity7"
               else "fp32 state / bf16 observations",
               "data": f"synthetic (smooth random truth -> observation operators -> noise, {a.cloud:.0%} clouds), "
                       "random-init GP emulators" + ("; observations device-resident (compute-only, no per-step H2D)"
                                                     if a.resident else "; observations re-uploaded from pinned host "
                                                     "memory every step"),
               "config": {"name": a.config, "model": c["model"], "tile": f"{H}x{W}", "active_pixels": part.N_total,
                          "global_batch": part.N_total, "seq_len": 1,
                          "gp_train_points": a.n_train or c.get("n_train"), "parallelism": f"tile-dp{world}" + (f" x band-tp{B}" if B > 1 else ""),
                          "gn_iterations": gn, "ms_per_gn_iteration": round(1e3 * elapsed / max(1, n_gn), 3),
                          "finite": ok, "fallback_frac": round(fallback, 6),
                          "out_of_domain_frac": round(out_of_domain, 6), "ingest_bytes_per_step": ingest,
                          "baseline_updates_per_s": c["baseline"]}}
        # the engine settings that decide what a step computes (reference semantics)
        ec = kf.config
        rec["config"]["engine"] = {"convergence_tolerance": ec.convergence_tolerance,
                                   "min_iterations": ec.min_iterations, "max_iterations": ec.max_iterations,
                                   "convergence": "per chunk" if ec.convergence_chunk else "tile",
                                   "store_precision": ec.store_precision, "observed_first": ec.observed_first,
                                   "fuse_gn": ec.fuse_gn, "analysis_form": ec.analysis_form,
                                   "line_tables": ec.line_tables, "phase_telemetry": telemetry}
        if chunk_hist:
            rec["config"]["convergence_chunk"] = kf.config.convergence_chunk
            rec["config"]["chunk_gn_histogram"] = {str(i): chunk_hist[i] for i in sorted(chunk_hist)}
            n_ch = sum(chunk_hist.values())
            rec["config"]["chunk_gn_mean"] = round(sum(i * n for i, n in chunk_hist.items()) / max(1, n_ch), 3)
        rec["per_rank"] = sorted(per_rank, key=lambda r: r["rank"])
        if a.output:
            rec["output"] = [r.get("output") for r in rec["per_rank"]]
        # what torch.distributed saw: the driver can confirm from the record alone
        # that the N-GPU line came from N RCCL ranks on N distinct devices
        import torch.distributed as dist
        rec["dist"] = {"initialized": dist.is_initialized(),
                       "backend": dist.get_backend() if dist.is_initialized() else None,
                       "world_size": dist.get_world_size() if dist.is_initialized() else 1,
                       "devices": [r["device"] for r in rec["per_rank"]],
                       "hosts": sorted({r["host"] for r in rec["per_rank"]}),
                       "distinct_devices": n_dev}
        if bp_why:
            rec["band_parallel_fallback"] = {"requested": bp_req, "reason": bp_why}
        if n_dev != n_ranks:
            rec["rehearsal"] = f"{n_ranks} ranks on {n_dev} device(s): logic rehearsal, not a scaling point"
        print(json.dumps(rec), flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
