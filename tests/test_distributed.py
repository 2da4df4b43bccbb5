"""Tile-DP over row strips with world_size 2 on the CPU (gloo) — the logic
harness of the RCCL path (tier 3b)."""
import datetime as dt
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem(world, rank, dense=False, rows=30):
    import kafka_inferenceengine_amd as k
    from kafka_inferenceengine_amd.parallel import Comm, StripPartition

    mask = np.ones((rows, 22), bool)
    if not dense:   # dense strips take the index geometry and the overlapped C2 path
        mask[4:9, 3:12] = False
    comm = Comm(rank, world, "cpu") if world > 1 else Comm.single("cpu")
    part = StripPartition(mask, rank, world)
    obs = k.SyntheticBHRObservations(mask, n_train=60, device="cpu", stream=True, n_pool=4, partition=part,
                                     field_cell=6, seed=3)
    return k, mask, comm, part, obs


def _run(world, rank, cfg, out_q):
    cfg = dict(cfg)
    dense = cfg.pop("_dense", False)
    rows = cfg.pop("_rows", 30)
    if world > 1:
        torch.set_num_threads(1)   # 8 ranks on the 8 CPUs
    k, mask, comm, part, obs = _problem(world, rank, dense, rows)
    kf = k.LinearKalman(obs, None, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS, device="cpu",
                        comm=comm, partition=part, config=k.EngineConfig(**cfg))
    kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
    prior = k.JRCPrior(k.TIP_PARAMETERS, mask)
    x0, Pinv = prior.process_prior(None)
    grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(5)]
    st = kf.run(grid, x0, None, Pinv)
    norms = [r["norms"] for r in kf.metrics.records if r.get("event") == "date"]
    sweeps = [[e["sweeps"] for e in r.get("spatial", [])] for r in kf.metrics.records if r.get("event") == "date"]
    reg = kf._reg
    out_q.put((rank, part.offset, st.x.numpy().copy(), st.P.numpy().copy(), norms, kf.reg_overlapped_sweeps,
               {"tiled": kf.reg_tiled_launches, "exchanges": reg.exchanges if reg is not None else 0,
                "sweeps": sweeps, "depth": kf._reg_tiled_depth(1)}))


def _worker(rank, world, port, cfg, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _run(world, rank, cfg, q)
    finally:
        dist.destroy_process_group()


def _gather(world, cfg):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    if world == 1:
        _run(1, 0, cfg, q)
        res = [q.get()]
    else:
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, world, port, cfg, q)) for r in range(world)]
        for p in procs:
            p.start()
        res = [q.get(timeout=300) for _ in range(world)]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    res.sort(key=lambda t: t[0])
    x = np.concatenate([r[2] for r in res], 1)
    P = np.concatenate([r[3] for r in res], 1)
    _gather.overlapped = [r[5] for r in res]
    _gather.reg = [r[6] for r in res]
    return x, P, [r[4] for r in res]


@pytest.mark.parametrize("cfg", [{}, {"spatial_gamma": 30.0, "spatial_params": [6], "jacobi_sweeps": 5},
                                 {"convergence_tolerance": 1e-7, "max_iterations": 4}],
                         ids=["independent", "regularised-halo", "extra-iterations"])
def test_two_ranks_equal_one_rank(cfg):
    x1, P1, n1 = _gather(1, cfg)
    x2, P2, n2 = _gather(2, cfg)
    assert x1.shape == x2.shape
    # per-pixel math is identical; only the f64 norm summation order differs
    assert np.allclose(x1, x2, rtol=1e-5, atol=1e-6)
    assert np.allclose(P1, P2, rtol=1e-5, atol=1e-3)
    # the global convergence decision is identical on every rank
    assert n2[0] == n2[1]
    assert [len(a) for a in n1[0]] == [len(a) for a in n2[0]]


@pytest.mark.parametrize("dense", [False, True], ids=["masked", "dense-overlap"])
def test_four_ranks_regularised_halo_equal_one_rank(dense):
    """Interior strips (ranks 1 and 2) exchange halos with BOTH neighbours, which
    world_size 2 never exercises (C2 up and down in the same Jacobi sweep).  On a
    dense tile the sweeps run boundary rows -> posted exchange -> interior rows ->
    wait (C2 overlap); the result must not change."""
    cfg = {"spatial_gamma": 30.0, "spatial_params": [6], "jacobi_sweeps": 5, "_dense": dense}
    x1, P1, n1 = _gather(1, cfg)
    x4, P4, n4 = _gather(4, cfg)
    # C2 overlap on dense and masked strips alike (boundary rows split by index range)
    assert all(c > 0 for c in _gather.overlapped), _gather.overlapped
    assert x1.shape == x4.shape
    assert np.allclose(x1, x4, rtol=1e-5, atol=1e-6)
    assert np.allclose(P1, P4, rtol=1e-5, atol=1e-3)
    assert all(n == n4[0] for n in n4[1:])
    assert [len(a) for a in n1[0]] == [len(a) for a in n4[0]]


@pytest.mark.parametrize("cfg", [{"_rows": 48}, {"_rows": 48, "_dense": True, "spatial_gamma": 30.0,
                                                 "spatial_params": [6], "jacobi_sweeps": 5}],
                         ids=["tip7-independent", "spatial-dense-halo"])
def test_eight_ranks_equal_one_rank(cfg):
    """SURVEY.md §4 tier 3 at the node's full width: 8 strips (6 rows each; the
    6 interior strips exchange halos with two neighbours) give the 1-rank
    result and the same global convergence decisions on every rank."""
    x1, P1, n1 = _gather(1, cfg)
    reg1 = _gather.reg[0]
    x8, P8, n8 = _gather(8, cfg)
    assert x1.shape == x8.shape
    assert np.allclose(x1, x8, rtol=1e-5, atol=1e-6)
    assert np.allclose(P1, P8, rtol=1e-5, atol=1e-3)
    assert all(n == n8[0] for n in n8[1:])
    assert [len(a) for a in n1[0]] == [len(a) for a in n8[0]]
    if cfg.get("spatial_gamma"):
        assert all(c > 0 for c in _gather.overlapped), _gather.overlapped
        _check_deep_halo(x1, P1, reg1, x8, P8, _gather.reg)


def _check_deep_halo(x1, P1, reg1, xw, Pw, regw):
    """Communication-avoiding coupled solve (K9 + C2 deep halo): every rank
    runs the LDS-tiled passes, the state equals one rank's bit for bit, and the
    halo exchanges per GN iteration are one per pass plus the initial u, v, z
    one (the finish takes its row from the last pass's exchange)."""
    assert reg1["tiled"] > 0
    assert all(r["tiled"] > 0 for r in regw), regw
    assert np.array_equal(x1, xw) and np.array_equal(P1, Pw)
    for r in regw:
        depth = r["depth"]
        per_it = [s for date in r["sweeps"] for s in date]
        assert per_it and per_it == [s for date in reg1["sweeps"] for s in date]
        # sweeps before the finish, `depth` per pass; + 1: the u, v, z0 exchange
        bound = sum(max(1, -(-(s - 1) // depth)) + 1 for s in per_it)
        assert 0 < r["exchanges"] <= bound, (r["exchanges"], bound, per_it, depth)
        assert r["exchanges"] <= sum(-(-s // 8) + 1 for s in per_it) or depth < 8


def test_four_ranks_deep_halo_passes_of_eight():
    """Strips of 16 rows: passes of the full 8 sweeps, interior strips read a
    deep halo from both neighbours; equal to one rank bit for bit."""
    cfg = {"_rows": 64, "_dense": True, "spatial_gamma": 30.0, "spatial_params": [6]}
    x1, P1, n1 = _gather(1, cfg)
    reg1 = _gather.reg[0]
    x4, P4, n4 = _gather(4, cfg)
    assert all(r["depth"] == 8 for r in _gather.reg)
    assert all(n == n4[0] for n in n4[1:])
    _check_deep_halo(x1, P1, reg1, x4, P4, _gather.reg)


def test_strip_partition_balances_active_pixels():
    from kafka_inferenceengine_amd.parallel import StripPartition
    rng = np.random.default_rng(0)
    mask = rng.random((400, 50)) < np.linspace(0.1, 0.9, 400)[:, None]
    parts = [StripPartition(mask, r, 4) for r in range(4)]
    counts = [p.N for p in parts]
    assert sum(counts) == mask.sum()
    assert max(counts) - min(counts) <= mask.sum(1).max()
    assert parts[0].offset == 0 and parts[3].offset == sum(counts[:3])
    g = np.concatenate([p.global_index() for p in parts])
    assert np.array_equal(g, np.flatnonzero(mask.ravel()))


@pytest.mark.parametrize("extra", [[], ["--config", "prosail10", "--size", "40", "--band-parallel", "2"]],
                         ids=["tile-dp", "band-parallel"])
def test_bench_torchrun_gloo_two_ranks(extra):
    """bench.py under torch.distributed.run with 2 CPU ranks (gloo)."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--size", "96", "--n-train", "40", "--device", "cpu"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["value"] > 0 and rec["config"]["finite"]
    assert rec["config"]["fallback_frac"] < 0.01
    # per-rank telemetry of the timed steps, gathered from every rank of the job
    pr = rec["per_rank"]
    assert [r["rank"] for r in pr] == [0, 1]
    for r in pr:
        assert r["N"] > 0 and r["analysis_ms"] > 0 and r["c1_ms"] >= 0 and r["h2d_bytes"] > 0
        assert set(r) >= {"analysis_ms", "c1_ms", "halo_ms", "h2d_bytes", "N", "gn_iterations"}
        assert len(r["gn_iterations"]) == 2


@pytest.mark.parametrize("config", ["tip7", "spatial"])
def test_forced_one_rank_process_group_equals_single_process(tmp_path, config):
    """KAFKA_FORCE_DIST=1 under torch.distributed.run with one rank: the
    collectives run through the process group (gloo here, RCCL on a GPU box,
    tests/test_gpu.py) and the state equals the plain single-process run."""
    args = ["--config", config, "--size", "64", "--n-train", "24", "--steps", "2", "--warmup", "1", "--device", "cpu"]
    recs = []
    for forced in (False, True):
        env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + args
        if forced:
            env["KAFKA_FORCE_DIST"] = "1"
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                   "--master-addr=127.0.0.1", f"--master-port={_free_port()}"] + cmd[1:]
        cmd += ["--dump-state", str(tmp_path / f"f{int(forced)}")]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-3000:]
        import json
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1
        recs.append(json.loads(lines[0]))
    assert recs[1]["dist"]["initialized"] and recs[1]["dist"]["world_size"] == 1
    assert not recs[0]["dist"]["initialized"]
    assert np.array_equal(np.load(tmp_path / "f0.strip0.npy"), np.load(tmp_path / "f1.strip0.npy"))


def _comm_one_rank(env):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "tests", "comm_one_rank.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=dict(env, KAFKA_FORCE_DIST="1"), cwd=ROOT)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    import json
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["sum_f64"] == 1.25 and out["sum_f64_async"] == [0.5, 2.0] and out["sum_int"] == 7
    assert out["max_float"] == 3.5 and out["all_reduce"] == [0.0, 1.0, 2.0, 3.0, 4.0, 5.0]
    assert out["broadcast_packed"] == [[["k", 3]], [0.0, 1.0, 2.0]] and out["broadcast_object"] == {"a": 1}
    assert out["gather_object"] == [{"r": 0}] and out["gather_to_root"] == [2, 3]
    return out


def test_comm_collectives_one_rank_process_group():
    """Every Comm collective through a one-rank process group (gloo here;
    tests/test_gpu.py runs the same script over RCCL on the device)."""
    out = _comm_one_rank(dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES=""))
    assert out["backend"] == "gloo"


# (config, args of both runs, args of the 8-rank run only).  The defaults run the
# reference drivers' per-chunk exit test (tip7 / identity7 256^2, prosail10 /
# multisensor / prosail10_hard 128^2); "chunk64" cuts tip7's 256^2 rehearsal tile
# into 16 chunks and "tile" runs the tile-global test
SCALE_CASES = [("tip7", [], []), ("tip7", ["--set", "convergence_chunk=64"], []),
               ("tip7", ["--set", "convergence_chunk=tile"], []), ("spatial", [], []), ("prosail10", [], []),
               ("prosail10_hard", [], []), ("identity7", [], []), ("multisensor", [], []),
               ("multisensor", ["--set", "convergence_chunk=tile"], ["--band-parallel", "2"])]


def _case_id(c, both, eight):
    tag = c
    if both:
        tag += "-" + both[-1].split("=")[-1]
    if eight:
        tag += "-bp2"
    return tag


def _bench(nproc, config, extra, prefix, size=256):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    args = [os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--steps", "2", "--warmup", "1", "--size",
            str(size), "--n-train", "24", "--device", "cpu", "--config", config, "--dump-state", prefix] + extra
    if nproc > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}"] + args
    else:
        cmd = [sys.executable] + args
        env["OMP_NUM_THREADS"] = "8"
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("config,both,extra", SCALE_CASES, ids=[_case_id(*c) for c in SCALE_CASES])
def test_bench_eight_rank_rehearsal(tmp_path, config, both, extra):
    """The driver's SCALE run, rehearsed on the CPU: bench.py under
    torch.distributed.run with 8 ranks (gloo) at 256^2 -- one JSON line with 8
    per-rank records, what torch.distributed saw (backend, world size, the
    devices), the same GN iterations on every rank, and a final state equal to
    a one-rank run (reference analogue: the dask farm of
    kafka_test_Py36.py:241-255)."""
    one = _bench(1, config, both, str(tmp_path / "one"))
    rec = _bench(8, config, both + extra, str(tmp_path / "eight"))
    assert rec["n_gpus"] == 8 and rec["value"] > 0 and rec["config"]["finite"]
    assert rec["config"]["fallback_frac"] < 0.01
    d = rec["dist"]
    assert d["initialized"] and d["backend"] == "gloo" and d["world_size"] == 8
    assert len(d["devices"]) == 8 and d["distinct_devices"] == 8
    pr = rec["per_rank"]
    assert [r["rank"] for r in pr] == list(range(8))
    assert all(r["gn_iterations"] == pr[0]["gn_iterations"] for r in pr)
    assert pr[0]["gn_iterations"] == one["per_rank"][0]["gn_iterations"]
    # per-chunk convergence: the same chunk decisions at 1 and 8 ranks
    assert rec["config"]["engine"]["convergence"] == one["config"]["engine"]["convergence"]
    assert rec["config"].get("chunk_gn_histogram") == one["config"].get("chunk_gn_histogram")
    if not any("=tile" in b for b in both) and not extra and config != "spatial":
        assert rec["config"]["engine"]["convergence"] == "per chunk" and rec["config"]["chunk_gn_histogram"]
    assert sorted(r["local_rank"] for r in pr) == list(range(8))
    S = 4 if extra else 8
    x8 = np.concatenate([np.load(tmp_path / f"eight.strip{s}.npy") for s in range(S)], axis=1)
    x1 = np.load(tmp_path / "one.strip0.npy")
    assert x8.shape == x1.shape
    assert np.allclose(x8, x1, rtol=1e-5, atol=1e-5), float(np.abs(x8 - x1).max())
    if config == "spatial":
        assert np.array_equal(x8, x1)   # deep-halo tiled passes: bit-identical at any rank count


def _bp_worker(rank, world, port, B, q, chunk=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import kafka_inferenceengine_amd as k
    from kafka_inferenceengine_amd.parallel import Comm, StripPartition

    torch.set_num_threads(1)
    comm = Comm.from_env(device="cpu", band_parallel=B)
    try:
        q.put(_bp_run(k, comm, StripPartition, chunk))
    finally:
        comm.destroy()


def _bp_run(k, comm, StripPartition, chunk=None):
    mask = np.ones((20, 18), bool)
    mask[3:6, 2:9] = False
    part = StripPartition(mask, comm.rank, comm.world)
    obs = k.SyntheticS2Observations(mask, n_bands=5, n_train=24, device="cpu", stream=False, n_pool=2,
                                    partition=part, field_cell=6, seed=4)
    prior = k.SAILPrior(k.SAIL_PARAMETERS, mask)
    kf = k.LinearKalman(obs, None, mask, k.create_prosail_observation_operator, k.SAIL_PARAMETERS,
                        state_propagation=None, prior=prior, device="cpu", comm=comm, partition=part,
                        config=k.EngineConfig(gp_split="never", convergence_chunk=chunk,
                                              convergence_tolerance=2e-4 if chunk else 1e-3))
    grid = [obs.dates[0] - dt.timedelta(days=1)] + [d + dt.timedelta(days=1) for d in obs.dates[:2]]
    st = kf.run(grid, kf.state_from_prior(prior), None, None)
    g = comm.ranks[comm.rank] if comm.band is None else comm.band.ranks[comm.band.rank]
    its = [h["gn_iterations"] for h in kf.history] if chunk is None else [h["chunk_iters"] for h in kf.history]
    return (g, part.offset, st.x.numpy().copy(), its, kf.last_status.numpy().copy())


@pytest.mark.parametrize("world,B", [(2, 2), (4, 2), (8, 2)],
                         ids=["1strip-x-2bands", "2strips-x-2bands", "4strips-x-2bands"])
def test_band_parallel_equals_single_rank(world, B, chunk=None):
    """Band-parallel (TP-like) decomposition: bands split over the ranks of a
    strip, normal equations all-reduced (C5) — same result as one rank."""
    import kafka_inferenceengine_amd as k
    from kafka_inferenceengine_amd.parallel import Comm, StripPartition

    ref = _bp_run(k, Comm.single("cpu"), StripPartition, chunk)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bp_worker, args=(r, world, port, B, q, chunk)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    S = world // B
    for s in range(S):
        members = res[s * B:(s + 1) * B]
        for m in members[1:]:      # every member of a band group holds the identical state
            assert np.array_equal(m[2], members[0][2]) and np.array_equal(m[4], members[0][4])
    x = np.concatenate([res[s * B][2] for s in range(S)], 1)
    st = np.concatenate([res[s * B][4][:res[s * B][2].shape[1]] for s in range(S)])
    assert np.allclose(x, ref[2], rtol=1e-4, atol=1e-5)
    assert all(r[3] == ref[3] for r in res)
    assert np.array_equal(st, ref[4][:ref[2].shape[1]])


def test_band_parallel_per_chunk_convergence():
    """Band-parallel with the per-chunk exit test (6 x 6 chunks): the chunk
    decisions are taken on the all-reduced solve's per-pixel norms, so every
    band group stops the same chunks on the same iteration as one rank."""
    test_band_parallel_equals_single_rank(4, 2, chunk=[6, 6])


def test_metrics_summary_aggregates_ranks(tmp_path):
    import json
    path = str(tmp_path / "m.jsonl")
    _gather(2, {"metrics_path": path})
    summary = json.load(open(tmp_path / "m.summary.json"))
    assert [r["rank"] for r in summary["ranks"]] == [0, 1]
    assert summary["n_pixels"] == sum(r["n_pixels"] for r in summary["ranks"])
    assert os.path.exists(str(tmp_path / "m.rank1.jsonl"))


def _bp_ck_worker(rank, world, port, B, ckdir, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import kafka_inferenceengine_amd as k
    from kafka_inferenceengine_amd.parallel import Comm, StripPartition

    torch.set_num_threads(1)
    comm = Comm.from_env(device="cpu", band_parallel=B)
    try:
        mask = np.ones((12, 10), bool)
        part = StripPartition(mask, comm.rank, comm.world)
        obs = k.SyntheticS2Observations(mask, n_bands=4, n_train=20, device="cpu", stream=False, n_pool=2,
                                        partition=part, field_cell=5, seed=2)
        prior = k.SAILPrior(k.SAIL_PARAMETERS, mask)
        kf = k.LinearKalman(obs, None, mask, k.create_prosail_observation_operator, k.SAIL_PARAMETERS,
                            state_propagation=None, prior=prior, device="cpu", comm=comm, partition=part,
                            config=k.EngineConfig(gp_split="never", checkpoint_dir=ckdir, checkpoint_every=1))
        grid = [obs.dates[0] - dt.timedelta(days=1)] + [d + dt.timedelta(days=1) for d in obs.dates[:3]]
        st = kf.run(grid, kf.state_from_prior(prior), None, None)
        q.put((comm.band.rank if comm.band is not None else 0, st.x.numpy().copy()))
    finally:
        comm.destroy()


def test_band_parallel_checkpoint_single_writer(tmp_path):
    """with band groups every member holds the same strip state, so
    only band slot 0 writes; a checkpoint per timestep is committed and loads
    back to the final state."""
    import kafka_inferenceengine_amd as k

    ck = str(tmp_path / "ck")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bp_ck_worker, args=(r, 2, port, 2, ck, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    dirs = sorted(p for p in os.listdir(ck))
    assert len(dirs) == 3
    for d in dirs:
        files = sorted(os.listdir(os.path.join(ck, d)))
        assert files == ["manifest.json", "state.rank0.P.f32", "state.rank0.x.f32", "state_mask.u8"], files
    last = k.CheckpointManager.resolve(ck)
    x = np.fromfile(last / "state.rank0.x.f32", dtype="<f4").reshape(10, -1)
    assert np.array_equal(x, res[0][1][:, :x.shape[1]])


def _gather_worker(rank, world, port, folder, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        k, mask, comm, part, obs = _problem(world, rank)
        out = k.KafkaOutput(k.TIP_PARAMETERS, [500000., 10., 0., 4000000., 0., -10.], "EPSG:32630", folder,
                            gather=True)
        kf = k.LinearKalman(obs, out, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS,
                            device="cpu", comm=comm, partition=part)
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
        x0, Pinv = k.JRCPrior(k.TIP_PARAMETERS, mask).process_prior(None)
        grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(3)]
        kf.run(grid, x0, None, Pinv)
        out.flush()
        q.put((rank, sorted(os.path.basename(f) for f in out.written)))
    finally:
        if world > 1:
            dist.destroy_process_group()


def test_output_gather_to_root_writes_one_raster(tmp_path):
    """C3: with gather=True the strips are gathered to rank 0 (Comm.gather_to_root)
    and written as one full-tile GeoTIFF equal to the single-rank output."""
    import kafka_inferenceengine_amd as k
    ctx = mp.get_context("spawn")
    res = {}
    for world in (1, 2):
        q = ctx.Queue()
        folder = str(tmp_path / f"w{world}")
        port = _free_port()
        procs = [ctx.Process(target=_gather_worker, args=(r, world, port, folder, q)) for r in range(world)]
        for p in procs:
            p.start()
        got = dict(q.get(timeout=300) for _ in range(world))
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        assert got[0] and all(not v for r, v in got.items() if r)   # only rank 0 writes
        res[world] = (folder, got[0])
    assert res[1][1] == res[2][1]
    for name in res[1][1]:
        a, ia = k.read_tiff(os.path.join(res[1][0], name))
        b, ib = k.read_tiff(os.path.join(res[2][0], name))
        assert a.shape == b.shape == (30, 22)
        assert np.allclose(a, b, rtol=1e-5, atol=1e-6), name
        assert ia["geotransform"] == ib["geotransform"]


def _s2_worker(rank, world, port, data, emus, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import kafka_inferenceengine_amd as k
        from kafka_inferenceengine_amd.input_output import sentinel as S
        from kafka_inferenceengine_amd.parallel import Comm, StripPartition
        if rank > 0:   # C4: only rank 0 may read emulator files
            def _no_read(path):
                raise AssertionError(f"rank {rank} read {path}")
            S.load_emulator_set = _no_read
        mask = np.ones((16, 12), bool)
        comm = Comm(rank, world, "cpu") if world > 1 else Comm.single("cpu")
        part = StripPartition(mask, rank, world)
        obs = S.Sentinel2Observations(data, emus, mask)
        prior = k.SAILPrior(k.SAIL_PARAMETERS, mask)
        kf = k.LinearKalman(obs, None, mask, k.create_prosail_observation_operator, k.SAIL_PARAMETERS,
                            state_propagation=None, prior=prior, device="cpu", comm=comm, partition=part)
        x0, Pinv = prior.process_prior(None)
        grid = [obs.dates[0] - dt.timedelta(days=1)] + [d + dt.timedelta(days=1) for d in obs.dates]
        st = kf.run(grid, x0, None, Pinv)
        q.put((rank, st.x.numpy().copy(), getattr(obs, "c4_broadcasts", 0)))
    finally:
        if world > 1:
            dist.destroy_process_group()


def test_s2_emulators_broadcast_from_rank0(tmp_path):
    """C4: with two ranks only rank 0 reads the emulator files; rank 1 receives
    the packed set by tensor broadcast, and the run equals one rank."""
    import kafka_inferenceengine_amd as k
    from kafka_inferenceengine_amd.input_output.synthetic import synthesize_s2_archive
    data, emus, _ = synthesize_s2_archive(str(tmp_path), np.ones((16, 12), bool), n_dates=2, n_train=30,
                                          device="cpu")
    ctx = mp.get_context("spawn")
    xs = {}
    for world in (1, 2):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_s2_worker, args=(r, world, port, data, emus, q)) for r in range(world)]
        for p in procs:
            p.start()
        got = sorted((q.get(timeout=300) for _ in range(world)), key=lambda t: t[0])
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        if world == 2:
            assert all(c >= 1 for _, _, c in got)
        xs[world] = np.concatenate([g[1] for g in got], 1)
    assert np.allclose(xs[1], xs[2], rtol=1e-5, atol=1e-6)
