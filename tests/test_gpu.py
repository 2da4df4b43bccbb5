"""HIP kernels on an MI355X: each compared with the host runner of the same
source, the float64 oracle, or a plain PyTorch fp32 reference."""
import datetime as dt

import numpy as np
import pytest
import torch

import kafka_inferenceengine_amd as k
from kafka_inferenceengine_amd.inference import analysis_blocks
from kafka_inferenceengine_amd.ops import kernels as K
from kafka_inferenceengine_amd.utils.blocks import unpack_blocks

import kernel_cases as C

pytestmark = pytest.mark.gpu


def close(a, b, tol=1e-3, floor=0.05):
    """Row-scaled comparison: f32 kernels on device vs host differ in exp2/sqrt/
    division rounding and FMA contraction; ill-conditioned per-pixel solves
    amplify that to ~1e-4 relative."""
    a, b = torch.as_tensor(a).double(), torch.as_tensor(b).double()
    scale = b.abs().amax(dim=-1, keepdim=True).clamp(min=floor) if b.dim() > 1 else b.abs().max().clamp(min=floor)
    return float(((a - b).abs() / scale).max()) < tol


def _analysis(prob, device, variant=None):
    N, n = prob["N"], prob["n"]
    tab = C.table(prob, device)
    xo = torch.zeros((n, N), device=device)
    ao = torch.zeros((28, N), device=device)
    st = torch.zeros(N, dtype=torch.uint8, device=device)
    part = K.partials_buffer(N, device)
    K.analysis(n, tab, C.soa(prob["x"], device), C.soa(prob["xf"], device), C.packed(prob["Pf"], device), xo, ao,
               None, st, part, variant=variant)
    red = K.reduce_partials(part)
    return xo.cpu(), ao.cpu(), st.cpu(), float(red.cpu().item())


def test_native_extension_is_loaded(cuda):
    from kafka_inferenceengine_amd.ops import ext_path
    assert ext_path() is not None and ext_path().endswith(".so")


@pytest.mark.parametrize("dn16", [False, True])
def test_analysis_device_vs_host_and_oracle(cuda, dn16):
    """VALU record loop (variant 4) vs the host runner of the same source, and
    the default matrix-core GP (kf_gp_mfma.h) vs the float64 oracle."""
    prob = C.tip_problem(N=20000, dn16=dn16, seed=11)
    xd, ad, sd, rd = _analysis(prob, cuda, variant=4)
    xh, ah, sh, rh = _analysis(prob, "cpu")
    assert torch.equal(sd, sh)
    assert close(xd, xh)
    assert close(ad, ah, 1e-5)
    assert abs(rd - rh) / rh < 1e-4
    xr, Ar = analysis_blocks(prob["x"], prob["xf"], prob["Pf"], C.oracle_bands(prob, prob["x"]))
    assert np.max(np.abs(xd.numpy().T - xr) / (np.abs(xr) + 0.05)) < 2e-3
    xm, am, sm, rm = _analysis(prob, cuda)
    assert torch.equal(sm, sh)
    assert np.max(np.abs(xm.numpy().T - xr) / (np.abs(xr) + 0.05)) < 2e-3
    # A against the oracle, entries scaled by sqrt(A_ii A_jj); the f32 VALU path
    # on the host is the yardstick (both f32 Jacobians of cancelling GP sums)
    d = np.sqrt(np.einsum("nii->ni", Ar))
    norm = d[:, :, None] * d[:, None, :]
    err_m = np.max(np.abs(unpack_blocks(am.numpy(), 7) - Ar) / norm)
    err_h = np.max(np.abs(unpack_blocks(ah.numpy(), 7) - Ar) / norm)
    assert err_m < max(2e-4, 1.5 * err_h), (err_m, err_h)
    assert abs(rm - rh) / rh < 1e-2


def test_propagate_and_invert_device(cuda):
    """Device propagate vs the host runner (the reference-API oracle of every
    mode is tests/test_oracles.py::test_propagate_modes_vs_reference_api);
    invert vs torch.linalg.inv."""
    rng = np.random.default_rng(1)
    N, n = 5000, 7
    A = C.spd_blocks(rng, N, n)
    xa = rng.normal(size=(N, n))
    mu, _, Pi = k.tip_prior()
    from kafka_inferenceengine_amd.utils.blocks import pack_matrix
    for mode in range(6):
        spec = {"mode": mode, "m": np.ones(n), "q": np.full(n, 0.05), "prop_mask": 1 << 6, "reset_mean": mu,
                "reset_cinv": pack_matrix(Pi), "blend": mode != 4, "blend_mean": mu, "blend_cinv": pack_matrix(Pi)}
        outs = []
        for dev in (cuda, "cpu"):
            xf = torch.zeros((n, N), device=dev)
            pf = torch.zeros((28, N), device=dev)
            K.propagate(n, spec, C.soa(xa, dev), C.packed(A, dev), xf, pf)
            outs.append((xf.cpu(), pf.cpu()))
        assert close(outs[0][0], outs[1][0]), mode
        assert close(outs[0][1], outs[1][1]), mode
    out = torch.zeros((28, N), device=cuda)
    K.invert(n, C.packed(A, cuda), out)
    ref = torch.linalg.inv(torch.tensor(A, dtype=torch.float32))
    assert torch.allclose(torch.tensor(unpack_blocks(out.cpu().numpy(), n)), ref, rtol=1e-4, atol=1e-6)


def test_gain_jacobi_hessian_unpack_device(cuda):
    """Independent references: the GP Hessian against the NumPy emulator
    Hessian, the Jacobi sweep against per-pixel NumPy solves, unpack / gather /
    LUT against closed forms and torch (gain: tests/test_oracles.py)."""
    from test_kernels import hessian_vs_numpy, jacobi_sweep_vs_numpy, unpack_gather_lut_vs_torch
    hessian_vs_numpy(cuda)
    jacobi_sweep_vs_numpy(cuda)
    unpack_gather_lut_vs_torch(cuda)


def test_operator_device_vs_numpy(cuda):
    prob = C.tip_problem(N=10000, seed=13)
    tab = C.table(prob, cuda)
    xs = C.soa(prob["x"], cuda)
    for b in range(2):
        h0 = torch.zeros(10000, device=cuda)
        h = torch.zeros((7, 10000), device=cuda)
        K.operator_eval(7, tab, b, xs, h0, h)
        H, dH = prob["ems"][b].predict(prob["x"][:, k.TIP_BAND_MAPPER[b]])
        assert np.allclose(h0.cpu().numpy(), H, atol=5e-6)
        full = np.zeros((10000, 7))
        full[:, k.TIP_BAND_MAPPER[b]] = dH
        assert np.allclose(h.cpu().numpy().T, full, atol=5e-5)


def test_engine_gpu_matches_cpu_and_oracle(cuda):
    """The device engine against the float64 NumPy oracle of the reference run
    loop (tests/oracle.py) and against the host runner."""
    from oracle import oracle_run
    from kafka_inferenceengine_amd.utils.blocks import interleaved_to_soa, pack_blocks, sparse_to_blocks
    mask = np.ones((48, 40), bool)
    mask[:5, :6] = False
    grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(5)]
    outs = []
    for dev in (cuda, "cpu"):
        obs = k.SyntheticBHRObservations(mask, n_train=100, device=dev, stream=True, n_pool=3, field_cell=8)
        prior = k.JRCPrior(k.TIP_PARAMETERS, mask)
        kf = k.LinearKalman(obs, k.DeviceOutput(k.TIP_PARAMETERS), mask, k.create_nonlinear_observation_operator,
                            k.TIP_PARAMETERS, device=dev)
        kf.set_trajectory_model()
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
        st = kf.run(grid, kf.state_from_prior(prior), None, None)
        outs.append((st.x.cpu(), st.P.cpu(), [h.get("gn_iterations") for h in kf.history]))
    assert outs[0][2] == outs[1][2]
    assert close(outs[0][0], outs[1][0], 2e-3)
    assert close(outs[0][1], outs[1][1], 2e-3, floor=1.0)
    obs = k.SyntheticBHRObservations(mask, n_train=100, device="cpu", stream=True, n_pool=3, field_cell=8)
    x0, Pinv = k.JRCPrior(k.TIP_PARAMETERS, mask).process_prior(None)
    Q = np.zeros_like(x0)
    Q[6::7] = 0.04
    xr, Pr, iters = oracle_run(obs, mask, k.create_nonlinear_observation_operator, 7, grid, x0, Pinv,
                               propagator=k.propagate_information_filter_LAI, Q=Q)
    N = int(mask.sum())
    xs = outs[0][0][:, :N].numpy()
    assert [g[0] for g in outs[0][2]] == iters
    xo = interleaved_to_soa(xr, 7)
    assert np.max(np.abs(xs - xo) / (np.abs(xo).max(axis=1, keepdims=True) + 1e-3)) < 2e-3
    Po = pack_blocks(sparse_to_blocks(Pr, 7, check=False))
    Ps = outs[0][1][:, :N].numpy()
    assert np.max(np.abs(Ps - Po) / (np.abs(Po).max(axis=1, keepdims=True) + 1e-6)) < 2e-3


@pytest.mark.parametrize("config", ["tip7", "spatial", "prosail"])
def test_observed_first_order_equals_natural_order_gpu(cuda, config):
    """EngineConfig.observed_first on the device (matrix-core kernels, obs_order
    kernels): every pixel's state, precision and output raster equal the
    natural visiting order's bit for bit, GN counts equal."""
    mask = np.ones((96, 160), bool)
    mask[5:20, 30:70] = False
    outs = []
    for on in (False, True):
        out = k.DeviceOutput(k.TIP_PARAMETERS if config != "prosail" else k.SAIL_PARAMETERS, keep_history=True)
        if config == "prosail":
            grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=5 * i) for i in range(4)]
            obs = k.SyntheticS2Observations(mask, dates=grid, n_bands=10, n_train=250, device=cuda, stream=False,
                                            n_pool=2)
            prior = k.SAILPrior(k.SAIL_PARAMETERS, mask)
            kf = k.LinearKalman(obs, out, mask, k.create_prosail_observation_operator, k.SAIL_PARAMETERS,
                                state_propagation=None, prior=prior, device=cuda,
                                config=k.EngineConfig(observed_first=on))
            st = kf.run([grid[0] - dt.timedelta(days=1)] + [d + dt.timedelta(days=1) for d in grid],
                        kf.state_from_prior(prior), None, None)
        else:
            grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(5)]
            obs = k.SyntheticBHRObservations(mask, n_train=500, device=cuda, stream=False, n_pool=3, field_cell=8)
            reg = dict(spatial_gamma=5.0, spatial_params=[6]) if config == "spatial" else {}
            kf = k.LinearKalman(obs, out, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS,
                                device=cuda, state_propagation=k.propagate_information_filter_LAI,
                                config=k.EngineConfig(observed_first=on, **reg))
            kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
            st = kf.run(grid, kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask)), None, None)
        assert (kf._visit is not None) == on
        outs.append((st.x.cpu(), st.P.cpu(), [h.get("gn_iterations") for h in kf.history],
                     {t: (m.cpu(), u.cpu()) for t, (m, u) in out.history.items()}))
    (xa, Pa, ia, ha), (xb, Pb, ib, hb) = outs
    assert ia == ib
    assert torch.equal(xa, xb) and torch.equal(Pa, Pb)
    for t in ha:
        assert torch.equal(ha[t][0], hb[t][0]) and torch.equal(ha[t][1], hb[t][1])


@pytest.mark.parametrize("stream", [False, True])
def test_obs_order_device_equals_host(cuda, stream):
    """The obs_order kernels (chunk-local: the scatter alone; global: count,
    scan, scatter) give the host runner's stable partitions, on a tile spanning many 4096-pixel chunks
    (N = 620 x 331: a partial last chunk and 16-pixel tile).
    stream: DN16 observations, the kernels' two-vector-load path."""
    from kafka_inferenceengine_amd.engine.bands import build_table
    from kafka_inferenceengine_amd.ops import kernels as K
    mask = np.ones((700, 331), bool)
    mask[100:180, :] = False
    res = []
    for dev in (cuda, torch.device("cpu")):
        obs = k.SyntheticBHRObservations(mask, n_train=40, device=dev, stream=stream, n_pool=1, field_cell=8)
        kf = k.LinearKalman(obs, None, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS, device=dev)
        bands = kf._device_bands(obs.dates[0])
        table = build_table([s for s, _ in bands], [d for _, d in bands], kf.n_params, kf._cache, kf.device)
        for local in (True, False):
            res.append(K.obs_order(table, kf.N, kf.device, local=local)[0].cpu())
            # band groups (one band per group): the 4-class partition
            res.append(K.obs_order(table, kf.N, kf.device, groups=[0, 1], local=local)[0].cpu())
    assert all(torch.equal(res[i], res[i + 4]) for i in range(4))


def _orders(mask, devs, make_obs, groups_list, locals_=(True, False)):
    from kafka_inferenceengine_amd.engine.bands import build_table
    from kafka_inferenceengine_amd.ops import kernels as K
    res = []
    for dev in devs:
        obs = make_obs(dev)
        kf = k.LinearKalman(obs, None, mask, k.create_nonlinear_observation_operator if obs.__class__.__name__.
                            startswith("SyntheticBHR") else k.create_prosail_observation_operator,
                            k.TIP_PARAMETERS if obs.__class__.__name__.startswith("SyntheticBHR") else
                            k.SAIL_PARAMETERS, device=dev)
        bands = kf._device_bands(obs.dates[0])
        table = build_table([s for s, _ in bands], [d for _, d in bands], kf.n_params, kf._cache, kf.device)
        out = []
        for groups in groups_list:
            for local in locals_:
                out.append(K.obs_order(table, kf.N, kf.device, groups=groups, local=local)[0].cpu())
        res.append(out)
        del kf, table, bands, obs
    return res


def test_obs_order_cross_tile_scan_carry(cuda):
    """The global partition past one scan tile (obs_scan_kernel: 1024 x 8
    chunks of 4096 pixels per tile, the carry between tiles): 6000^2 pixels =
    8790 chunks, two tiles (a 10980^2 production tile has 29.4k chunks, four),
    device equal to the host runner."""
    mask = np.ones((6000, 6000), bool)
    mask[:37, :] = False
    mk = lambda dev: k.SyntheticBHRObservations(mask, n_train=20, device=dev, stream=True, n_pool=1,  # noqa: E731
                                                field_cell=8)
    dev_res, host_res = _orders(mask, (cuda, torch.device("cpu")), mk, [None], locals_=(False,))
    assert int(mask.sum()) > 8192 * 4096
    assert torch.equal(dev_res[0], host_res[0])


def test_obs_order_eight_classes_partial_chunk(cuda):
    """Three band groups (G = 3: eight observation classes) on a tile whose
    last 4096-pixel chunk is partial: device equal to the host runner, chunk-
    local and global."""
    mask = np.ones((700, 331), bool)
    mask[100:180, :] = False
    mk = lambda dev: k.SyntheticS2Observations(mask, n_bands=3, n_train=20, device=dev, stream=True,  # noqa: E731
                                               n_pool=1, cloud_fraction=0.4)
    dev_res, host_res = _orders(mask, (cuda, torch.device("cpu")), mk, [[0, 1, 2], None])
    assert int(mask.sum()) % 4096 != 0
    for a, b in zip(dev_res, host_res):
        assert torch.equal(a, b)


def test_streamer_async_copies_keep_stream_order(cuda):
    """DateStreamer copies issued by the HostRing submitter thread (h2d_async)
    under running kernels: every acquired buffer holds its own date's entry,
    and no copy overwrites a buffer a queued kernel still reads (each step's
    kernel reduces the acquired buffer after a slow kernel in front of it)."""
    from kafka_inferenceengine_amd.input_output.streaming import DateStreamer
    s = DateStreamer(3, (4, 1 << 18), torch.int16, cuda, n_bufs=3)
    for kk in range(3):
        s.host_view(kk).fill_(kk + 1)
    s.warm()
    x = torch.ones(1 << 22, device=cuda)
    sums = []
    for i in range(30):
        buf = s.acquire(i % 3, key=i)
        s.prefetch((i + 1) % 3, key=i + 1)
        s.prefetch((i + 2) % 3, key=i + 2)
        for _ in range(20):
            x.mul_(1.0000001)       # keep the compute stream busy ahead of the read
        sums.append(buf.float().sum())
    got = [int(v.item()) for v in sums]
    assert got == [((i % 3) + 1) * 4 * (1 << 18) for i in range(30)]


def test_streamer_pinned_and_overlaps(cuda):
    from kafka_inferenceengine_amd.input_output.streaming import DateStreamer
    s = DateStreamer(3, (2, 1 << 20), torch.int16, cuda)
    assert s.pinned
    for kk in range(3):
        s.host_view(kk).fill_(kk + 1)
    a = s.acquire(0)
    s.prefetch(1)
    assert int(a[0, 0]) == 1
    b = s.acquire(1)
    assert int(b[1, -1]) == 2
    c = s.acquire(2)
    assert int(c.sum()) == 3 * 2 * (1 << 20)


def test_spatial_regulariser_gpu_matches_cpu(cuda):
    mask = np.ones((32, 32), bool)
    grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(3)]
    outs = []
    for dev in (cuda, "cpu"):
        obs = k.SyntheticBHRObservations(mask, n_train=60, device=dev, stream=False, n_pool=2, field_cell=8)
        kf = k.LinearKalman(obs, None, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS, device=dev,
                            config=k.EngineConfig(spatial_gamma=20.0, spatial_params=[6]))
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
        st = kf.run(grid, kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask)), None, None)
        outs.append(st.x.cpu())
    assert close(outs[0], outs[1], 2e-3)


def test_split_gp_path_gpu_matches_fused(cuda):
    mask = np.ones((40, 32), bool)
    outs = []
    for mode in ("never", "always"):
        obs = k.SyntheticS2Observations(mask, n_bands=10, n_train=40, device=cuda, stream=False, n_pool=2,
                                        field_cell=8)
        prior = k.SAILPrior(k.SAIL_PARAMETERS, mask)
        kf = k.LinearKalman(obs, None, mask, k.create_prosail_observation_operator, k.SAIL_PARAMETERS,
                            state_propagation=None, prior=prior, device=cuda,
                            config=k.EngineConfig(gp_split=mode, band_chunk=4))
        grid = [obs.dates[0] - dt.timedelta(days=1), obs.dates[1] + dt.timedelta(days=1)]
        outs.append(kf.run(grid, kf.state_from_prior(prior), None, None).x.cpu())
    assert close(outs[0], outs[1], 1e-3)


@pytest.mark.parametrize("mode,blend,quirk,pmask", C.FUSED_CASES[:3])
def test_fused_propagation_device(cuda, mode, blend, quirk, pmask):
    """Fused forecast in the gfx950 analysis kernel vs the propagate kernel +
    analysis on the device, and vs the host runner."""
    ref, fused = C.fused_vs_materialized(cuda, mode, blend, quirk, pmask, N=20000)
    host, _ = C.fused_vs_materialized("cpu", mode, blend, quirk, pmask, N=20000)
    for (x1, a1, s1), (x2, a2, s2), (x3, a3, s3) in zip(ref, fused, host):
        assert np.array_equal(s1, s2)
        assert close(x2, x1, 1e-4) and close(a2, a1, 1e-5)
        assert close(x2, x3) and close(a2, a3, 1e-4)


def test_gpu_runs_are_bit_reproducible(cuda):
    """SURVEY.md §5.2 deterministic-reduction mode: fixed-order f64 partials,
    no atomics -> two runs give bit-identical states and norms."""
    mask = np.ones((64, 48), bool)
    grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(4)]
    outs = []
    for _ in range(2):
        obs = k.SyntheticBHRObservations(mask, n_train=100, device=cuda, stream=True, n_pool=3, field_cell=8)
        kf = k.LinearKalman(obs, None, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS, device=cuda)
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
        st = kf.run(grid, kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask)), None, None)
        outs.append((st.x.cpu(), st.P.cpu(), [r["norms"] for r in kf.metrics.records if r.get("event") == "date"]))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert outs[0][2] == outs[1][2]




@pytest.mark.parametrize("op", ["tip", "identity"])
def test_fused_gn_launch_equals_separate_launches_gpu(cuda, op):
    """EngineConfig.fuse_gn on the device (matrix-core GP kernel for TIP, the
    FD_LINEAR kernel for the identity operator): GN iterations 1 + 2 in one
    launch are bit-identical to one launch per iteration (states, output
    rasters, iteration counts, final norms)."""
    mask = np.ones((96, 160), bool)
    mask[5:20, 30:70] = False
    grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(5)]
    outs = []
    for fuse in (False, True):
        out = k.DeviceOutput(k.TIP_PARAMETERS, keep_history=True)
        if op == "tip":
            obs = k.SyntheticBHRObservations(mask, n_train=500, device=cuda, stream=False, n_pool=3, field_cell=8)
            fac = k.create_nonlinear_observation_operator
        else:
            obs = k.SyntheticIdentityObservations(mask, device=cuda, stream=False, n_pool=3, field_cell=8)
            fac = k.create_linear_observation_operator
        kf = k.LinearKalman(obs, out, mask, fac, k.TIP_PARAMETERS, device=cuda,
                            state_propagation=k.propagate_information_filter_LAI,
                            config=k.EngineConfig(fuse_gn=fuse))
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
        st = kf.run(grid, kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask)), None, None)
        outs.append((st.x.cpu(), st.P.cpu(), [h.get("gn_iterations") for h in kf.history],
                     [h.get("norms") for h in kf.history], {t: (m.cpu(), u.cpu()) for t, (m, u) in out.history.items()}))
    (xa, Pa, ia, na, ha), (xb, Pb, ib, nb, hb) = outs
    assert ia == ib and na == nb
    assert torch.equal(xa, xb) and torch.equal(Pa, Pb)
    for t in ha:
        assert torch.equal(ha[t][0], hb[t][0]) and torch.equal(ha[t][1], hb[t][1])


def test_fused_spatial_first_iteration_equals_separate_launches_gpu(cuda):
    """spatial_first_plain on the device (matrix-core TIP kernel): the plain
    first Gauss-Newton iteration fused with the regularised prepare of the
    second is bit-identical to the two launches (states, output rasters,
    iteration counts, norms)."""
    mask = np.ones((96, 160), bool)
    mask[5:20, 30:70] = False
    grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(5)]
    outs = []
    for fuse in (False, True):
        out = k.DeviceOutput(k.TIP_PARAMETERS, keep_history=True)
        obs = k.SyntheticBHRObservations(mask, n_train=500, device=cuda, stream=False, n_pool=3, field_cell=8)
        kf = k.LinearKalman(obs, out, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS, device=cuda,
                            state_propagation=k.propagate_information_filter_LAI,
                            config=k.EngineConfig(fuse_gn=fuse, spatial_gamma=5.0, spatial_params=[6]))
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
        st = kf.run(grid, kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask)), None, None)
        outs.append((st.x.cpu(), st.P.cpu(), [h.get("gn_iterations") for h in kf.history],
                     [h.get("norms") for h in kf.history], {t: (m.cpu(), u.cpu()) for t, (m, u) in out.history.items()}))
    (xa, Pa, ia, na, ha), (xb, Pb, ib, nb, hb) = outs
    assert ia == ib and na == nb
    assert torch.equal(xa, xb) and torch.equal(Pa, Pb)
    for t in ha:
        assert torch.equal(ha[t][0], hb[t][0]) and torch.equal(ha[t][1], hb[t][1])


def test_specialised_prosail_kernel_equals_generic_gpu(cuda):
    """PROSAIL (global-table matrix-core kernel) with the fused forecast: the
    SPEC_PROP kernel gives the same bits as the generic one (variant 18)."""
    from kafka_inferenceengine_amd.ops import kernels as K
    mask = np.ones((64, 80), bool)
    grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=5 * i) for i in range(4)]
    outs = []
    old, old_line = K.DEFAULT_VARIANT, K.LINE_TABLES
    K.LINE_TABLES = False   # variant 18 has no line tables (kf_gp_mfma.h)
    try:
        for variant in (0, 18):
            K.DEFAULT_VARIANT = variant
            obs = k.SyntheticS2Observations(mask, dates=grid, n_bands=10, n_train=250, device=cuda, stream=False,
                                            n_pool=2)
            prior = k.SAILPrior(k.SAIL_PARAMETERS, mask)
            kf = k.LinearKalman(obs, None, mask, k.create_prosail_observation_operator, k.SAIL_PARAMETERS,
                                state_propagation=None, prior=prior, device=cuda)
            st = kf.run([grid[0] - dt.timedelta(days=1)] + [d + dt.timedelta(days=1) for d in grid],
                        kf.state_from_prior(prior), None, None)
            outs.append((st.x.cpu(), st.P.cpu(), [h.get("norms") for h in kf.history]))
    finally:
        K.DEFAULT_VARIANT, K.LINE_TABLES = old, old_line
    assert outs[0][2] == outs[1][2]
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("spatial,n_train", [(False, 500), (True, 500), (False, 32)])
def test_specialised_tip_kernel_equals_generic_gpu(cuda, spatial, n_train):
    """The JRC-TIP kernels specialised for the fused forecast (SPEC_PROP, and
    SPEC_PROP_REG with the spatial prior: explicit-forecast / regulariser code
    compiled out; SPEC_PROP_PF for small emulators, T = 32: the next pixel
    group's forecast inputs loaded ahead) give the same bits as the generic
    kernel (variant 18)."""
    from kafka_inferenceengine_amd.ops import kernels as K
    mask = np.ones((96, 160), bool)
    mask[5:20, 30:70] = False
    grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(5)]
    reg = dict(spatial_gamma=5.0, spatial_params=[6]) if spatial else {}
    outs = []
    old, old_line = K.DEFAULT_VARIANT, K.LINE_TABLES
    K.LINE_TABLES = False   # variant 18 has no line tables (kf_gp_mfma.h)
    try:
        for variant in (0, 18):
            K.DEFAULT_VARIANT = variant
            out = k.DeviceOutput(k.TIP_PARAMETERS, keep_history=True)
            obs = k.SyntheticBHRObservations(mask, n_train=n_train, device=cuda, stream=False, n_pool=3,
                                             field_cell=8)
            kf = k.LinearKalman(obs, out, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS,
                                device=cuda, state_propagation=k.propagate_information_filter_LAI,
                                config=k.EngineConfig(**reg))
            kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
            st = kf.run(grid, kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask)), None, None)
            outs.append((st.x.cpu(), st.P.cpu(), [h.get("norms") for h in kf.history],
                         {t: (m.cpu(), u.cpu()) for t, (m, u) in out.history.items()}))
    finally:
        K.DEFAULT_VARIANT, K.LINE_TABLES = old, old_line
    (xa, Pa, na, ha), (xb, Pb, nb, hb) = outs
    assert na == nb and torch.equal(xa, xb) and torch.equal(Pa, Pb)
    for t in ha:
        assert torch.equal(ha[t][0], hb[t][0]) and torch.equal(ha[t][1], hb[t][1])


@pytest.mark.parametrize("spatial", [False, True])
def test_fused_output_gpu(cuda, spatial):
    """Fused output (analysis kernel, or the regulariser finish pass with a
    spatial prior) equals the separate unpack kernel on the device."""
    reg = dict(spatial_gamma=50.0, spatial_params=[6], jacobi_sweeps=4) if spatial else {}
    mask = np.ones((40, 36), bool)
    mask[3:9, 2:20] = False
    grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(4)]
    outs = []
    for fuse in (False, True):
        obs = k.SyntheticBHRObservations(mask, n_train=80, device=cuda, stream=False, n_pool=2, field_cell=8)
        out = k.DeviceOutput(k.TIP_PARAMETERS)
        kf = k.LinearKalman(obs, out, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS, device=cuda,
                            config=k.EngineConfig(fuse_output=fuse, **reg))
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
        kf.run(grid, kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask)), None, None)
        outs.append((out.mean.cpu(), out.unc.cpu()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.allclose(outs[0][1], outs[1][1], rtol=1e-6)


def test_gain_form_equals_information_form_gpu(cuda):
    """K1g on the matrix cores with K1's launch features (GN 1 + 2 in one
    launch, observed-first order, the stored precision diagonal read by the
    Sherman-Morrison fast forecast, fused output) against the information form
    on the device, and against the host runner of the same gain code."""
    mask = np.ones((64, 60), bool)
    mask[5:12, 3:30] = False
    grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(5)]

    def run(dev, **cfg):
        obs = k.SyntheticBHRObservations(mask, n_train=100, device=dev, stream=False, n_pool=3, field_cell=8, seed=2)
        out = k.DeviceOutput(k.TIP_PARAMETERS)
        kf = k.LinearKalman(obs, out, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS, device=dev,
                            state_propagation=k.propagate_information_filter_LAI, config=k.EngineConfig(**cfg))
        kf.set_trajectory_model()
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
        st = kf.run(grid, kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask)), None, None)
        return st, out, [h.get("gn_iterations") for h in kf.history]

    si, oi, gi = run(cuda)
    sg, og, gg = run(cuda, analysis_form="gain")
    sh, oh, gh = run("cpu", analysis_form="gain")
    assert gi == gg == gh
    N = si.N
    assert close(sg.x[:, :N].cpu(), si.x[:, :N].cpu(), 2e-3)
    assert close(og.unc.cpu(), oi.unc.cpu(), 5e-3)
    assert close(sg.x[:, :N].cpu(), sh.x[:, :N].cpu(), 1e-3)
    assert close(og.unc.cpu(), oh.unc.cpu(), 1e-3)


def test_masked_strip_geotiff_mean_not_overwritten_by_next_date(cuda, tmp_path):
    """A masked strip's mean planes are owned by the output (not the state's
    x): the next date's fused analysis must not overwrite them while this
    date's side-stream device-to-host copy still reads them.  A 2048^2 x 7
    plane pair takes milliseconds to copy against a sub-millisecond identity
    analysis, so without the double-buffered mean the GeoTIFF of date t would
    hold date t+1's mean."""
    from kafka_inferenceengine_amd.input_output.tiff import read_tiff
    mask = np.ones((2048, 2048), bool)
    mask[::7] = False
    grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=5 * i) for i in range(6)]

    def run(out):
        obs = k.SyntheticIdentityObservations(mask, device=cuda, stream=False, n_pool=2, seed=3)
        kf = k.LinearKalman(obs, out, mask, k.create_linear_observation_operator, k.TIP_PARAMETERS, device=cuda,
                            state_propagation=k.propagate_information_filter_LAI)
        kf.set_trajectory_model()
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
        kf.run(grid, kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask)), None, None)
        if torch.device(cuda).type == "cuda":
            torch.cuda.synchronize()
        return kf

    ref = k.DeviceOutput(k.TIP_PARAMETERS, keep_history=True)
    run(ref)
    out = k.KafkaOutput(k.TIP_PARAMETERS, None, "", str(tmp_path), compress=None)
    run(out)
    out.flush()
    assert len(ref.history) >= 4
    for ts, (m, u) in ref.history.items():
        for p in (0, 6):
            got = read_tiff(tmp_path / f"{k.TIP_PARAMETERS[p]}_{ts.strftime('A%Y%j')}.tif")[0]
            assert np.array_equal(got.reshape(-1), m[p].cpu().numpy()), (ts, p)
            gu = read_tiff(tmp_path / f"{k.TIP_PARAMETERS[p]}_{ts.strftime('A%Y%j')}_unc.tif")[0]
            assert np.array_equal(gu.reshape(-1), u[p].cpu().numpy()), (ts, p)


@pytest.mark.parametrize("regmask", [0b1000000, 0b1000101])
def test_affine_jacobi_equals_classic_gpu(cuda, regmask):
    from test_kernels import affine_vs_classic_jacobi
    affine_vs_classic_jacobi(cuda, regmask=regmask)


def test_identity_linear_fast_path_gpu_matches_cpu(cuda):
    """The all-linear bf16 analysis kernel (FD_LINEAR, OBS_BF16) on the device
    vs the generic host runner."""
    mask = np.ones((40, 36), bool)
    grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(4)]
    outs = []
    for dev in (cuda, "cpu"):
        obs = k.SyntheticIdentityObservations(mask, device=dev, stream=False, n_pool=3, field_cell=8)
        kf = k.LinearKalman(obs, None, mask, k.create_linear_observation_operator, k.TIP_PARAMETERS, device=dev,
                            state_propagation=k.propagate_information_filter_LAI)
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
        st = kf.run(grid, kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask)), None, None)
        outs.append((st.x.cpu(), st.P.cpu(), [h.get("gn_iterations") for h in kf.history]))
    assert outs[0][2] == outs[1][2]
    assert close(outs[0][0], outs[1][0], 1e-4) and close(outs[0][1], outs[1][1], 1e-4, floor=1.0)


@pytest.mark.parametrize("config", ["tip7", "spatial"])
def test_bench_rccl_one_rank_equals_single_process(cuda, tmp_path, config):
    """bench.py under torch.distributed.run with KAFKA_FORCE_DIST=1: a one-rank
    job whose collectives (C1 all-gather of the norms, the per-rank record
    gather, C4 broadcasts, device barriers) go through RCCL ("nccl") on the
    GPU -- the code the driver's multi-GPU runs take and the gloo rehearsals
    do not.  The final state equals the plain single-process run bit for bit."""
    import json
    import os
    import socket
    import subprocess
    import sys
    from pathlib import Path

    root = str(Path(__file__).resolve().parents[1])
    args = [os.path.join(root, "bench.py"), "--config", config, "--size", "512", "--steps", "2", "--warmup", "1"]
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    recs = []
    for forced in (False, True):
        env = dict(os.environ, PYTHONPATH=root)
        cmd = [sys.executable] + args
        if forced:
            env["KAFKA_FORCE_DIST"] = "1"
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                   "--master-addr=127.0.0.1", f"--master-port={port}"] + args
        cmd += ["--dump-state", str(tmp_path / f"f{int(forced)}")]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=100, env=env, cwd=root)
        assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, r.stdout[-2000:]
        recs.append(json.loads(lines[0]))
    assert recs[1]["dist"]["backend"] == "nccl" and recs[1]["dist"]["world_size"] == 1, recs[1]["dist"]
    assert recs[0]["dist"]["initialized"] is False
    a = np.load(tmp_path / "f0.strip0.npy")
    b = np.load(tmp_path / "f1.strip0.npy")
    assert np.array_equal(a, b)


def test_comm_collectives_one_rank_rccl(cuda):
    """Every Comm collective (C1 sums, band all-reduce, C3 gather, C4
    broadcasts, object gathers, device barrier, empty C2 batch) through a
    one-rank RCCL process group with device tensors."""
    import os
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parent))
    from test_distributed import _comm_one_rank

    root = str(Path(__file__).resolve().parents[1])
    out = _comm_one_rank(dict(os.environ, PYTHONPATH=root))
    assert out["backend"] == "nccl" and out["device"].startswith("cuda"), out


def test_checked_build_smoke_on_device(cuda):
    """The debug variant (KF_CHECKED index assertions in the gfx950 kernels) runs the
    smoke step on the GPU without a failed check."""
    import os
    import subprocess
    import sys
    from pathlib import Path

    from kafka_inferenceengine_amd import _build

    if not _build.CHECKED_EXT_PATH.exists():
        pytest.skip("checked variant not built")
    root = str(Path(__file__).resolve().parents[1])
    env = dict(os.environ, KAFKA_CHECKED="1")
    r = subprocess.run([sys.executable, "-c", "import __graft_entry__ as g; g.smoke()"], env=env, cwd=root,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "smoke ok" in r.stdout and "_kafka_hip_checked" in r.stdout, r.stdout[-2000:]


@pytest.mark.parametrize("case", [dict(h=300, w=1000, omegas=(1.0, 1.3, 1.2, 1.25, 1.22, 1.21, 1.2, 1.2)),
                                  dict(h=130, w=257, omegas=(1.1, 1.2, 1.3), cheb=(True, True, False)),
                                  dict(h=7, w=5, omegas=(1.0,) * 8), dict(h=64, w=128, omegas=(1.0,), cheb=(False,))])
def test_reg_sweeps_tiled_equals_sequential_on_device(cuda, case):
    """The LDS-tiled multi-sweep kernel is bit-identical to one row-loop sweep
    launch per sweep (partial tiles, domain edges, Jacobi and Chebyshev steps)."""
    (zt, zpt), (zs, zps) = C.tiled_vs_sequential(cuda, **case)
    assert torch.equal(zt, zs) and torch.equal(zpt, zps)
    (ht, hpt), _ = C.tiled_vs_sequential("cpu", **case)
    assert torch.equal(zt, ht) and torch.equal(zpt, hpt)


@pytest.mark.parametrize("case", [dict(split=True), dict(r0=0, r1=90), dict(device_sched=True, split=True),
                                  dict(device_sched=True, rho=0.0), dict(h_total=1400, w=1000, r0=600, r1=1290,
                                                                         split=True, device_sched=True)])
def test_reg_sweeps_tiled_deep_halo_on_device(cuda, case):
    """Deep-halo pass of a strip (C2 once per pass) on gfx950: equal to the
    whole-raster pass's rows and to the host runner, bit for bit."""
    (zs, zps), (zf, zpf) = C.deep_halo_vs_full(cuda, **case)
    assert torch.equal(zs, zf) and torch.equal(zps, zpf)
    (hs, hps), _ = C.deep_halo_vs_full("cpu", **case)
    assert torch.equal(zs, hs) and torch.equal(zps, hps)


def test_reg_finish_rows_clears_stale_partials(cuda):
    """The row-loop finish launches fewer blocks than the partials buffer has
    entries (w > 256: rows < grid); stale values in the unused entries must not
    reach the convergence norm."""
    h, w, n, j0 = 10, 300, 7, 6
    N = h * w
    rng = np.random.default_rng(3)
    geo = {"w": w, "h": h, "halo": 0, "n_up": 0}
    res = []
    for dev in (cuda, "cpu"):
        t = lambda a: torch.tensor(a, dtype=torch.float32, device=dev)  # noqa: E731
        u = t(rng.normal(size=(n, N)))
        v = t(rng.uniform(0, 0.2, size=(n, N)))
        z = t(rng.normal(size=(1, N)))
        xr = t(rng.normal(size=(n, N)))
        xo = torch.zeros((n, N), device=dev)
        part = K.partials_buffer(N, dev)
        part.fill_(1e30)
        K.reg_finish(n, u, v, z, None, xr, xo, 0.9, 1 << j0, N, partials=part, geo=geo)
        res.append(float(K.reduce_partials(part).cpu()))
        rng = np.random.default_rng(3)
    assert res[0] < 1e20 and abs(res[0] - res[1]) <= 1e-5 * abs(res[1]), res


def test_reg_schedule_on_device_matches_host(cuda):
    """The device schedule kernel and the host runner agree (count and weights)."""
    for rho in (0.833, 0.5, 0.97, 0.0, 1.5):
        out = []
        for dev in (cuda, "cpu"):
            rs = K.RegSchedule(1000, 64, dev)
            rs.rho.fill_(rho)
            rs.schedule(1e-3)
            out.append((rs.info.cpu(), rs.sched.cpu(), rs.omega.cpu()))
        assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
        assert torch.equal(out[0][2], out[1][2])


def test_reg_rho_pass_on_device(cuda):
    """rho = gamma max v deg over a dense strip with halo rows (device = torch)."""
    h, w = 300, 257
    N = h * w
    v = torch.rand(N + 10, device=cuda)
    geo = {"w": w, "h": h, "halo": 1, "n_up": w}
    rs = K.RegSchedule(N, 64, cuda)
    rs.rho_pass(v, geo, N, 2.5)
    rr = torch.arange(N, device=cuda) // w
    cc = torch.arange(N, device=cuda) % w
    deg = (1 + (rr + 1 < h).int() + (cc > 0).int() + (cc + 1 < w).int()).float()
    ref = float(torch.amax(v[:N] * deg) * 2.5)
    assert float(rs.rho) == ref


def test_spatial_tiled_sweeps_equal_per_sweep_launches_on_device(cuda):
    from test_engine import _spatial_dense_run
    a, na = _spatial_dense_run(cuda, True, size=(200, 300))
    b, nb = _spatial_dense_run(cuda, False, size=(200, 300))
    assert na > 0 and nb == 0
    assert torch.equal(a, b)


@pytest.mark.parametrize("rank,out", [(0, True), (1, True), (2, False), (1, False), (1, "mean")])
def test_dense_finish_vectorised_equals_host(cuda, rank, out):
    """The 16-byte finish (4 pixels of a row per thread) equals the host's
    per-pixel finish bit for bit (x, output mean), halo rows included;
    the norm partials agree to rounding (different summation order)."""
    d = C.dense_finish(cuda, rank=rank, out=out)
    h = C.dense_finish("cpu", rank=rank, out=out)
    assert torch.equal(d[0], h[0]) and torch.equal(d[1], h[1])
    # 1/sqrt(diag A): the device's rsqrt differs from the host's in the last bit
    assert torch.allclose(d[2], h[2], rtol=2e-7, atol=0)
    assert abs(d[3] - h[3]) <= 1e-5 * abs(h[3])
    if out == "mean":
        assert torch.equal(d[1], d[0]) and not d[2].any()


@pytest.mark.gpu
def test_phase_timer_native_events_gpu():
    """PhaseTimer on the native event pool: nested and repeated phases, more
    phases in flight than the recycle threshold, non-blocking snapshots that
    leave unfinished phases for later, exact run totals."""
    from kafka_inferenceengine_amd.utils.metrics import PhaseTimer

    dev = torch.device("cuda", 0)
    x = torch.randn(2048, 2048, device=dev)
    for sync in (False, True):
        t = PhaseTimer(dev, sync=sync)
        for _ in range(80):
            with t.phase("outer"):
                with t.phase("mm"):
                    y = x @ x
                y.add_(1.0)
        t.snapshot(block=False)
        total = t.cumulative()
        assert t._ev.pending == 0
        assert set(total) == {"outer", "mm"}
        assert 0 < total["mm"] <= total["outer"]
