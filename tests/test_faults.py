"""Fault injection: corrupted observations and degenerate
blocks must be contained to their pixels and flagged."""
import datetime as dt

import numpy as np
import torch

import kafka_inferenceengine_amd as k
from kafka_inferenceengine_amd.engine.bands import DeviceBand
from kafka_inferenceengine_amd.ops import kernels as K


class NaNInjected:
    """Wraps a source and corrupts a tile of every band with NaN/inf."""

    def __init__(self, src, rows, cols):
        self.src = src
        self.dates = src.dates
        self.bands_per_observation = src.bands_per_observation
        self.partition = src.partition
        self.rows, self.cols = rows, cols

    def get_band_data(self, date, band):
        r = self.src.get_band_data(date, band)
        obs = r.observations.copy()
        obs[self.rows, self.cols] = np.nan
        unc = r.uncertainty.tolil()
        W = obs.shape[1]
        for rr in range(*self.rows.indices(obs.shape[0])):
            for cc in range(*self.cols.indices(W)):
                unc[rr * W + cc, rr * W + cc] = np.inf
        return r._replace(observations=obs, uncertainty=unc.tocsr())


import pytest


@pytest.mark.parametrize("gamma", [0.0, 2.0], ids=["plain", "spatial"])
def test_nan_tile_is_contained_and_flagged(gamma):
    mask = np.ones((16, 12), bool)
    src = k.SyntheticBHRObservations(mask, n_train=40, device="cpu", stream=False, n_pool=2, field_cell=4)
    bad = NaNInjected(src, slice(2, 5), slice(3, 7))
    grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(3)]
    res = []
    for obs in (src, bad):
        cfg = k.EngineConfig(spatial_gamma=gamma, spatial_params=[6], jacobi_sweeps=3)
        kf = k.LinearKalman(obs, None, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS,
                            device="cpu", config=cfg)
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
        st = kf.run(grid, kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask)), None, None)
        res.append((st.x.clone(), kf.last_status.clone()))
    (xa, sa), (xb, sb) = res
    assert torch.isfinite(xb).all()
    img = np.zeros(mask.shape, bool)
    img[2:5, 3:7] = True
    inside = torch.from_numpy(img.ravel())
    assert torch.all((sb[inside] & K.ST_NO_OBS) > 0)       # corrupted pixels saw no valid observation
    if gamma == 0.0:
        # pixels outside the tile: identical physics, only the global norm could differ
        assert torch.allclose(xa[:, ~inside], xb[:, ~inside], rtol=1e-5, atol=1e-6)
    else:
        # coupled: far from the tile (> 3 sweeps of 4-neighbour influence) nothing changes
        far = np.ones(mask.shape, bool)
        far[0:9, 0:11] = False
        far = torch.from_numpy(far.ravel())
        assert torch.allclose(xa[:, far], xb[:, far], rtol=1e-3, atol=1e-4)


def test_nonspd_forecast_falls_back_per_pixel():
    n, N = 7, 64
    mu, _, Pi = k.tip_prior()
    x = torch.tensor(np.tile(mu[:, None], (1, N)), dtype=torch.float32)
    from kafka_inferenceengine_amd.utils.blocks import pack_matrix
    P = torch.tensor(np.tile(pack_matrix(Pi)[:, None], (1, N)), dtype=torch.float32)
    P[:, :5] = torch.tensor(pack_matrix(-np.eye(7)), dtype=torch.float32)[:, None]
    P[:, 5] = float("nan")
    y = torch.full((N,), 0.1)
    w = torch.zeros(N)   # no observations: A = P_f^-1 only
    spec = k.models.operators._linear_device_spec(n, None, None, 0)
    from kafka_inferenceengine_amd.engine.bands import RecordCache, build_table
    tab = build_table([spec], [DeviceBand(K.OBS_F32, y=y, w=w)], n, RecordCache(), "cpu")
    xo, ao = torch.zeros_like(x), torch.zeros_like(P)
    st = torch.zeros(N, dtype=torch.uint8)
    K.analysis(n, tab, x, x, P, xo, ao, None, st, K.partials_buffer(N, "cpu"))
    assert torch.all(st[:6] & K.ST_FALLBACK)
    assert torch.equal(xo[:, :6], x[:, :6])
    assert not torch.any(st[6:] & K.ST_FALLBACK)
    assert torch.isfinite(xo).all()


def test_nonspd_forecast_falls_back_in_spatial_epilogue():
    """The regularised (reg_v) epilogue: non-SPD / NaN pixels keep the forecast,
    are decoupled (V = 0) and nothing non-finite reaches the sweeps."""
    n, H, W = 7, 4, 16
    N = H * W
    mu, _, Pi = k.tip_prior()
    from kafka_inferenceengine_amd.utils.blocks import pack_matrix, ntri
    x = torch.tensor(np.tile(mu[:, None], (1, N)), dtype=torch.float32)
    P = torch.tensor(np.tile(pack_matrix(Pi)[:, None], (1, N)), dtype=torch.float32)
    P[:, :5] = torch.tensor(pack_matrix(-np.eye(7)), dtype=torch.float32)[:, None]
    P[:, 5] = float("nan")
    y = torch.full((N,), 0.1)
    w = torch.zeros(N)
    spec = k.models.operators._linear_device_spec(n, None, None, 0)
    from kafka_inferenceengine_amd.engine.bands import RecordCache, build_table
    tab = build_table([spec], [DeviceBand(K.OBS_F32, y=y, w=w)], n, RecordCache(), "cpu")
    u, ao = torch.zeros_like(x), torch.zeros_like(P)
    v = torch.full((n, N), 7.0)
    st = torch.zeros(N, dtype=torch.uint8)
    geo = {"w": W, "h": H, "halo": 0, "n_up": 0}
    K.analysis(n, tab, x, x, P, u, ao, None, st, None, N=N,
               reg=dict(gamma=2.0, mask=1 << 6, v_out=v, nbr=None, geo=geo))
    assert torch.all(st[:6] & K.ST_FALLBACK) and not torch.any(st[6:] & K.ST_FALLBACK)
    assert torch.equal(u[:, :6], x[:, :6])
    assert torch.all(v[:, :6] == 0) and torch.isfinite(v).all() and torch.isfinite(u).all()
    keep = torch.ones(N, dtype=torch.bool)
    keep[5] = False            # its forecast precision is NaN, and the fallback keeps the forecast
    assert torch.isfinite(ao[:, keep]).all()


# ----------------------------------------------------------- rank failure
def _rank_worker(rank, world, port, ckdir, die_at, q):
    import os
    import torch.distributed as dist

    from kafka_inferenceengine_amd.parallel import Comm, StripPartition

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=dt.timedelta(seconds=60))
    try:
        mask = np.ones((24, 16), bool)
        part = StripPartition(mask, rank, world)
        obs = k.SyntheticBHRObservations(mask, n_train=30, device="cpu", stream=False, n_pool=2, partition=part,
                                         field_cell=6, seed=9)
        kf = k.LinearKalman(obs, None, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS,
                            device="cpu", comm=Comm(rank, world, "cpu"), partition=part,
                            config=k.EngineConfig(checkpoint_dir=ckdir, checkpoint_every=1 if ckdir else 0))
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
        grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(6)]
        if die_at is not None and rank == 1:
            step = kf.step
            count = [0]

            def dying_step(*a, **kw):
                count[0] += 1
                if count[0] == die_at:
                    os._exit(17)          # the rank disappears mid-run (no cleanup)
                return step(*a, **kw)
            kf.step = dying_step
        resume = k.CheckpointManager.latest(ckdir) if (ckdir and die_at is None) else None
        try:
            start = None if resume else kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask))
            st = kf.run(grid, start, None, None, resume_from=resume)
            q.put((rank, "ok", st.x.numpy().copy()))
        except Exception as e:  # the survivor sees the failed peer as a collective error
            q.put((rank, "error", type(e).__name__))
    finally:
        try:
            dist.destroy_process_group()
        except Exception:
            pass


def _launch(world, ckdir, die_at):
    import socket
    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_worker, args=(r, world, port, ckdir, die_at, q)) for r in range(world)]
    for p in procs:
        p.start()
    expected = world - (1 if die_at is not None else 0)
    res = [q.get(timeout=240) for _ in range(expected)]
    for p in procs:
        p.join(timeout=120)
    return sorted(res, key=lambda t: t[0]), [p.exitcode for p in procs]


def test_rank_failure_detected_and_resumed_from_checkpoint(tmp_path):
    """a rank dies mid-run -> the survivor's collective fails
    (no hang), the job restarts from the last per-timestep checkpoint and ends
    on the same state as an uninterrupted run."""
    ref, codes = _launch(2, None, None)
    assert codes == [0, 0] and all(r[1] == "ok" for r in ref)
    ck = str(tmp_path / "ck")
    res, codes = _launch(2, ck, die_at=4)
    assert codes[1] == 17
    assert res[0][1] == "error"
    assert k.CheckpointManager.latest(ck) is not None
    res, codes = _launch(2, ck, None)
    assert codes == [0, 0]
    for (r0, s0, x0), (r1, s1, x1) in zip(ref, res):
        assert s1 == "ok" and np.allclose(x0, x1, rtol=1e-6, atol=1e-7)
