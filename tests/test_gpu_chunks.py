"""Per-chunk Gauss-Newton convergence on the MI355X (engine/chunks.py): the
device kernels against the host runner, and a 1024^2 hard-PROSAIL tile
against a farm of one engine per 256^2 chunk (the reference's driver model,
kafka_test_Py36.py:147-187, 241)."""
import datetime as dt

import numpy as np
import pytest
import torch

import kafka_inferenceengine_amd as k
from kafka_inferenceengine_amd.engine.chunks import ChunkConvergence
from kafka_inferenceengine_amd.input_output.utils import get_chunks
from kafka_inferenceengine_amd.ops import kernels as K
from kafka_inferenceengine_amd.parallel import Comm, StripPartition

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("block", [[64, 48], [300, 40]])
def test_chunk_kernels_match_host(cuda, block):
    """chunk_partials is bit-identical on the device and the host runner (same
    summation order; 300-wide chunks take the runs-longer-than-a-workgroup
    loop); chunk_decide and chunk_compact agree exactly."""
    rng = np.random.default_rng(0)
    H, W = 700, 530
    mask = rng.random((H, W)) > 0.1
    part = StripPartition(mask, 0, 1)
    N = part.N
    cc0 = ChunkConvergence(part, block, 7, "cpu", Comm.single("cpu"))
    flags = ((rng.random(cc0.nc) > 0.3) & (cc0.counts > 0)).astype(np.uint8)
    # odd chunks far below the tolerance, even ones above: some chunks stop, some go on
    dn = (rng.random(N) * np.where(cc0.chunk_of.numpy() % 2 == 1, 1e-9, 1e-3)).astype(np.float32)
    perm = rng.permutation(N).astype(np.int32)
    xs = rng.random((7, N)).astype(np.float32)
    outs = {}
    for dev in ("cpu", cuda):
        cc = ChunkConvergence(part, block, 7, dev, Comm.single(dev))
        cc.dn.copy_(torch.from_numpy(dn))
        cc.active.copy_(torch.from_numpy(flags))
        pend = cc.decide(n_iter=3, tol=2e-6, min_iter=2, max_iter=25)
        info = [pend.result(j) for j in range(4)]
        order = torch.from_numpy(perm).to(dev)
        x_src = torch.from_numpy(xs).to(dev)
        x_dst = torch.zeros_like(x_src)
        out = cc.compact(order, N, int(info[2]), x_src, x_dst)
        if dev != "cpu":
            torch.cuda.synchronize()
        outs[str(dev)] = (cc.part.cpu().numpy(), cc.active.cpu().numpy(), cc.iters.cpu().numpy(), info,
                          out[:int(info[2])].cpu().numpy(), x_dst.cpu().numpy())
    a, b = outs["cpu"], outs[str(cuda)]
    assert np.array_equal(a[0], b[0])          # partials: bit-identical
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2]) and a[3] == b[3]
    assert 0 < a[3][2] < N and a[3][3] > 0
    assert np.array_equal(a[4], b[4])           # stable compaction
    assert np.array_equal(a[5], b[5])           # frozen copy


DATES = [dt.datetime(2017, 7, 3) + dt.timedelta(days=2 * i) for i in range(3)]
GRID = [DATES[0] - dt.timedelta(days=1)] + [d + dt.timedelta(days=1) for d in DATES]


def _engine(mask, cfg, dev, emulators=None):
    obs = k.SyntheticS2Observations(mask, dates=DATES, n_bands=10, n_train=100, device=dev, stream=False, n_pool=3,
                                    hard=True, spread_scale=1.0, rel_unc=0.02, seed=1, emulators=emulators)
    prior = k.SAILPrior(k.SAIL_PARAMETERS, mask)
    kf = k.LinearKalman(obs, None, mask, k.create_prosail_observation_operator, k.SAIL_PARAMETERS,
                        state_propagation=None, prior=prior, device=dev,
                        config=k.EngineConfig(convergence_tolerance=2e-5, **cfg))
    return kf, obs, prior


def test_chunked_1024_hard_prosail_equals_farm(cuda):
    """on a 1024^2 tile with the hard PROSAIL emulators
    every 256^2 chunk runs the Gauss-Newton iterations of its own engine
    (one LinearKalman per chunk, parallel/farm.py), date by date, and the state
    matches the farm's."""
    S, B = 1024, 256
    mask = np.ones((S, S), bool)
    mask[100:300, 600:700] = False
    kf, obs, prior = _engine(mask, {"convergence_chunk": [B, B]}, cuda)
    st = kf.run(GRID, kf.state_from_prior(prior), None, None)
    torch.cuda.synchronize()
    hist = [h["chunk_iters"][0] for h in kf.history]
    iters = kf._chunks.iters.cpu().numpy()
    x = st.x[:, :st.N].cpu().numpy()
    pos = np.full(S * S, -1, np.int64)
    pos[kf.partition.global_index()] = np.arange(st.N)
    want = [{} for _ in DATES]
    worst = 0.0
    for x0, y0, nx, ny, no in get_chunks(S, S, [B, B]):
        m = np.zeros_like(mask)
        m[y0:y0 + ny, x0:x0 + nx] = mask[y0:y0 + ny, x0:x0 + nx]
        kc, _, pc = _engine(m, {}, cuda, obs.emulators)
        sc = kc.run(GRID, kc.state_from_prior(pc), None, None)
        its = [h["gn_iterations"][0] for h in kc.history]
        for d, it in enumerate(its):
            want[d][it] = want[d].get(it, 0) + 1
        assert iters[no - 1] == its[-1], (no, iters[no - 1], its)
        cols = pos[kc.partition.global_index()]
        worst = max(worst, float(np.abs(x[:, cols] - sc.x[:, :sc.N].cpu().numpy()).max()))
    assert hist == want, (hist, want)
    assert any(len(h) > 1 for h in hist), f"chunks should need different iteration counts: {hist}"
    assert worst <= 1e-5, worst
    print(f"per-chunk GN histograms {hist}; max |x - farm| {worst:g}")


def test_chunk_tail_lookahead_on_device(cuda):
    """The tail's queued iterations on the device (counts read by the
    kernels, decisions read late) equal reading every decision first, and the
    host runner."""
    from test_chunks import _chunked_run, _mask

    mask = _mask()
    ref = _chunked_run(mask, 0, device=cuda)
    got = _chunked_run(mask, 3, device=cuda, emulators=ref[-1])
    assert max(ref[3]) > 4
    assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1])
    assert got[2] == ref[2] and got[3] == ref[3] and got[4] == ref[4]
    assert np.array_equal(got[5], ref[5])
