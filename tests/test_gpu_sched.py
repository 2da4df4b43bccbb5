"""Tile-queue scheduling of the matrix-core analysis kernels (kf_device.h
analysis_tiles / launch_tiles, Variant.TILE_QUEUE): a persistent grid whose
waves pull 64-slot tiles from per-XCD device counters.  Each pixel's analysis
is the same whichever wave runs it, so the state is bit-identical to the
default static grid-stride schedule, and the per-tile norm partials sum to the
same norm."""
import datetime as dt

import numpy as np
import pytest
import torch

import kafka_inferenceengine_amd as k
from kafka_inferenceengine_amd.ops import kernels as K

pytestmark = pytest.mark.gpu


def _run(cuda, config, variant, size=768):
    old = K.DEFAULT_VARIANT
    K.DEFAULT_VARIANT = K.Variant(variant)
    try:
        mask = np.ones((size, size), bool)
        mask[50:90, 10:500] = False
        if config == "tip7":
            obs = k.SyntheticBHRObservations(mask, n_train=200, device=cuda, stream=True, n_pool=3, seed=2,
                                             cloud_fraction=0.3)
            kf = k.LinearKalman(obs, k.DeviceOutput(k.TIP_PARAMETERS), mask, k.create_nonlinear_observation_operator,
                                k.TIP_PARAMETERS, device=cuda, config=k.EngineConfig(store_precision="always"))
            kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
            x0, Pinv = k.JRCPrior(k.TIP_PARAMETERS, mask).process_prior(None)
            grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(4)]
            st = kf.run(grid, x0, None, Pinv)
        else:
            obs = k.SyntheticS2Observations(mask, n_bands=10, n_train=120, device=cuda, stream=True, n_pool=3, seed=2,
                                            cloud_fraction=0.3)
            prior = k.SAILPrior(k.SAIL_PARAMETERS, mask)
            kf = k.LinearKalman(obs, k.DeviceOutput(k.SAIL_PARAMETERS), mask, k.create_prosail_observation_operator,
                                k.SAIL_PARAMETERS, state_propagation=None, prior=prior, device=cuda,
                                config=k.EngineConfig(store_precision="always"))
            grid = [obs.dates[0] - dt.timedelta(days=1)] + [d + dt.timedelta(days=1) for d in obs.dates[:3]]
            st = kf.run(grid, kf.state_from_prior(prior), None, None)
        torch.cuda.synchronize()
        norms = [r["norms"] for r in kf.history]
        return (st.x[:, :st.N].cpu().numpy(), st.P[:, :st.N].cpu().numpy(), kf.last_status[:st.N].cpu().numpy(),
                norms, [r["gn_iterations"] for r in kf.history])
    finally:
        K.DEFAULT_VARIANT = old


@pytest.mark.parametrize("config", ["tip7", "prosail10"])
def test_tile_queue_bit_identical_to_static_grid(cuda, config):
    xq, Pq, sq, nq, gq = _run(cuda, config, K.Variant.TILE_QUEUE)
    xs, Ps, ss, ns, gs = _run(cuda, config, K.Variant.DEFAULT)
    assert np.array_equal(xq, xs) and np.array_equal(Pq, Ps) and np.array_equal(sq, ss)
    assert gq == gs
    # the norm: the same f64 sum in another association (per tile vs per workgroup)
    for a, b in zip(nq, ns):
        np.testing.assert_allclose(np.array(a, dtype=float), np.array(b, dtype=float), rtol=1e-12)


def test_tile_queue_is_bit_reproducible(cuda):
    """Which wave ran which tile changes from run to run; the partials do not
    (one per tile, reduced in tile order): the norms repeat bit for bit."""
    a = _run(cuda, "tip7", K.Variant.TILE_QUEUE, size=512)
    b = _run(cuda, "tip7", K.Variant.TILE_QUEUE, size=512)
    assert np.array_equal(a[0], b[0]) and a[3] == b[3]


def test_two_level_reduction_matches_host(cuda):
    g = torch.Generator().manual_seed(0)
    v = torch.rand(2_500_000, generator=g, dtype=torch.float64)
    d = v.to(cuda)
    out = K.reduce_partials(d)
    ref = float(np.sum(v.numpy()))
    assert abs(float(out.cpu()) - ref) <= 1e-12 * ref
    d._kf_n = 1_000_001          # only the entries the producer wrote
    out2 = K.reduce_partials(d)
    ref2 = float(np.sum(v.numpy()[:1_000_001]))
    assert abs(float(out2.cpu()) - ref2) <= 1e-12 * ref2
