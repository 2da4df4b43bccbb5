"""Engine (host runner of the kernel code) against the float64 oracle of the
reference run loop, plus compatibility paths, checkpoint/resume and output."""
import datetime as dt

import numpy as np
import pytest
import torch

import kafka_inferenceengine_amd as k
from kafka_inferenceengine_amd.utils.blocks import interleaved_to_soa, sparse_to_blocks, pack_blocks

from oracle import oracle_run


def _grid(n, step=16, start=dt.datetime(2017, 1, 1)):
    return [start + dt.timedelta(days=step * i) for i in range(n)]


def _setup(shape=(24, 20), n_train=80, stream=False, seed=0):
    mask = np.ones(shape, bool)
    mask[:3, :4] = False
    obs = k.SyntheticBHRObservations(mask, n_train=n_train, stream=stream, n_pool=5, device="cpu", seed=seed,
                                     field_cell=8)
    prior = k.JRCPrior(k.TIP_PARAMETERS, mask)
    x0, Pinv = prior.process_prior(None)
    Q = np.zeros_like(x0)
    Q[6::7] = 0.04
    return mask, obs, prior, x0, Pinv, Q


def _engine(mask, obs, Q, out=None, prior=None, prop=None, **cfg):
    kf = k.LinearKalman(obs, out, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS,
                        state_propagation=k.propagate_information_filter_LAI if prop is None else prop,
                        prior=prior, device="cpu", config=k.EngineConfig(**cfg))
    kf.set_trajectory_model()
    kf.set_trajectory_uncertainty(Q)
    return kf


def _compare(st, x_ref, Pi_ref, n=7, xtol=2e-3, ptol=2e-3):
    xs, Ps = st.numpy()
    xr = interleaved_to_soa(x_ref, n)
    Pr = pack_blocks(sparse_to_blocks(Pi_ref, n, check=False))
    scale = np.abs(xr).max(axis=1, keepdims=True) + 1e-3
    assert np.max(np.abs(xs - xr) / scale) < xtol
    assert np.max(np.abs(Ps - Pr) / (np.abs(Pr).max(axis=1, keepdims=True) + 1e-6)) < ptol


def test_engine_matches_oracle_tip_lai():
    mask, obs, prior, x0, Pinv, Q = _setup()
    grid = _grid(5)
    kf = _engine(mask, obs, Q)
    st = kf.run(grid, x0, None, Pinv)
    xr, Pr, iters = oracle_run(obs, mask, k.create_nonlinear_observation_operator, 7, grid, x0, Pinv,
                               propagator=k.propagate_information_filter_LAI, Q=Q)
    _compare(st, xr, Pr)
    assert [r["gn_iterations"][0] for r in kf.history] == iters


def test_engine_matches_oracle_prior_blend_quirk():
    mask, obs, prior, x0, Pinv, Q = _setup(seed=1)
    grid = _grid(4)
    kf = _engine(mask, obs, Q, prior=prior, reference_quirks=True)
    st = kf.run(grid, x0, None, Pinv)
    xr, Pr, _ = oracle_run(obs, mask, k.create_nonlinear_observation_operator, 7, grid, x0, Pinv,
                           propagator=k.propagate_information_filter_LAI, prior=prior, Q=Q)
    _compare(st, xr, Pr)


def test_engine_host_propagator_and_precomputed_operator_paths():
    """A user propagator (no device_spec) and a user factory (no device_spec) run
    on the host and must give the same answer as the device-spec versions."""
    mask, obs, prior, x0, Pinv, Q = _setup(seed=2)
    grid = _grid(3)

    def user_prop(*a, **kw):
        return k.propagate_information_filter_LAI(*a, **kw)

    def user_factory(*a):
        return k.create_nonlinear_observation_operator(*a)

    ref = _engine(mask, obs, Q).run(grid, x0, None, Pinv)
    kf = k.LinearKalman(obs, None, mask, user_factory, k.TIP_PARAMETERS, state_propagation=user_prop, device="cpu")
    kf.set_trajectory_model()
    kf.set_trajectory_uncertainty(Q)
    st = kf.run(grid, x0, None, Pinv)
    # host f64 Jacobians vs in-kernel f32 ones may change the GN iteration count
    # near the tolerance: compare relative to each row's scale
    assert torch.allclose(st.x, ref.x, atol=2e-3, rtol=1e-2)
    rowmax = ref.P.abs().amax(dim=1, keepdim=True).clamp(min=1.0)
    assert ((st.P - ref.P).abs() / rowmax).max() < 2e-3


def test_gain_form_fused_forecast_and_output():
    """Gain form with the forecast evaluated inside the K1g kernel and the
    output rasters written by it, against the materialised forecast (invert +
    propagate + invert passes) and the unpack pass."""
    mask, obs, prior, x0, Pinv, Q = _setup(seed=5)
    grid = _grid(4)
    res = []
    for fuse in (False, True):
        out = k.DeviceOutput(k.TIP_PARAMETERS)
        kf = _engine(mask, obs, Q, out=out, analysis_form="gain", fuse_propagation=fuse, fuse_output=fuse)
        st = kf.run(grid, x0, None, Pinv)
        res.append((st.x.clone(), st.P.clone(), out.mean.clone(), out.unc.clone(),
                    [h.get("gn_iterations") for h in kf.history]))
    (x1, P1, m1, u1, g1), (x2, P2, m2, u2, g2) = res
    assert g1 == g2
    assert torch.allclose(x1, x2, atol=1e-5, rtol=1e-4)
    assert ((P1 - P2).abs() / P1.abs().amax(dim=1, keepdim=True).clamp(min=1e-6)).max() < 1e-4
    assert torch.allclose(m1, m2, atol=1e-5, rtol=1e-4) and torch.allclose(u1, u2, rtol=1e-4)


def test_gain_form_equals_information_form():
    mask, obs, prior, x0, Pinv, Q = _setup(seed=3)
    grid = _grid(4)
    a = _engine(mask, obs, Q).run(grid, x0, None, Pinv)
    kfg = _engine(mask, obs, Q, analysis_form="gain")
    b = kfg.run(grid, x0, None, Pinv)
    bp = kfg._as_kind(b, "precision")
    assert torch.allclose(a.x, bp.x, atol=5e-4, rtol=1e-3)
    assert torch.allclose(a.P, bp.P, rtol=5e-3, atol=1e-1)


def test_gain_form_fused_gn_order_and_stored_rows():
    """K1g with K1's launch features: GN 1 + 2 in one launch equals two
    launches bit for bit, the observed-first order changes no pixel, and the
    stored-rows policy (the LAI precision diagonal instead of the covariance,
    read by the next fused forecast) equals storing the full covariance."""
    mask, obs, prior, x0, Pinv, Q = _setup(seed=6)
    grid = _grid(5)

    def run(**cfg):
        out = k.DeviceOutput(k.TIP_PARAMETERS, keep_history=True)
        kf = _engine(mask, obs, Q, out=out, analysis_form="gain", **cfg)
        st = kf.run(grid, x0, None, Pinv)
        return st, out, [h.get("gn_iterations") for h in kf.history], kf

    base, ob, gb, kfb = run()
    assert kfb._visit is not None or not kfb.config.observed_first
    sep, os_, gs, _ = run(fuse_gn=False)
    assert gb == gs
    assert torch.equal(base.x, sep.x)
    for t in ob.history:
        assert torch.equal(ob.history[t][0], os_.history[t][0]) and torch.equal(ob.history[t][1], os_.history[t][1])
    nat, _, gn_, _ = run(observed_first=False)
    assert gn_ == gb and torch.equal(base.x, nat.x)
    full, of, gf, _ = run(store_precision="always")
    assert gf == gb
    assert torch.allclose(base.x, full.x, rtol=1e-5, atol=1e-6)
    for t in ob.history:
        assert torch.allclose(ob.history[t][1], of.history[t][1], rtol=1e-4)


def test_checkpoint_resume_bit_identical(tmp_path):
    mask, obs, prior, x0, Pinv, Q = _setup(seed=4)
    grid = _grid(6)
    full = _engine(mask, obs, Q).run(grid, x0, None, Pinv)
    kf = _engine(mask, obs, Q, checkpoint_dir=str(tmp_path), checkpoint_every=1)
    kf.run(grid[:4], x0, None, Pinv)
    latest = k.CheckpointManager.latest(tmp_path)
    assert latest is not None and latest.name == grid[3].strftime("A%Y%j")
    kf2 = _engine(mask, obs, Q)
    st = kf2.run(grid, None, None, None, resume_from=latest)
    assert torch.equal(st.x, full.x) and torch.equal(st.P, full.P)


def test_checkpoint_every_other_step_with_partial_precision_dates(tmp_path):
    """store_precision="auto" keeps only the forecast's rows on dates that are
    not checkpointed; a checkpoint step stores the full precision, so resuming
    from it gives the uninterrupted run bit for bit."""
    mask, obs, prior, x0, Pinv, Q = _setup(seed=4)
    grid = _grid(7)
    full = _engine(mask, obs, Q).run(grid, x0, None, Pinv)
    kf = _engine(mask, obs, Q, checkpoint_dir=str(tmp_path), checkpoint_every=2)
    kf.run(grid[:6], x0, None, Pinv)
    latest = k.CheckpointManager.latest(tmp_path)
    assert latest is not None
    st = _engine(mask, obs, Q).run(grid, None, None, None, resume_from=latest)
    assert torch.equal(st.x, full.x) and torch.equal(st.P, full.P)


def test_checkpoint_retention_keeps_newest(tmp_path):
    mask, obs, prior, x0, Pinv, Q = _setup(seed=4)
    grid = _grid(5)
    kf = _engine(mask, obs, Q, checkpoint_dir=str(tmp_path), checkpoint_every=1, checkpoint_keep=2)
    kf.run(grid, x0, None, Pinv)
    kept = sorted(p.name for p in tmp_path.iterdir())
    assert kept == [g.strftime("A%Y%j") for g in grid[-2:]]
    assert k.CheckpointManager.latest(tmp_path).name == grid[-1].strftime("A%Y%j")
    assert kf.checkpointer.stats["bytes"] and len(kf.checkpointer.stats["write_s"]) == 4


def test_checkpoint_write_failure_is_not_committed(tmp_path, monkeypatch):
    """A writer that fails (disk full, EIO) must not get a manifest, must not
    prune the older good checkpoints, and must surface as an error."""
    from kafka_inferenceengine_amd.input_output import checkpoint as ck
    mask, obs, prior, x0, Pinv, Q = _setup(seed=4)
    grid = _grid(6)
    bad = grid[3].strftime("A%Y%j")
    real = ck._atomic_write

    def flaky(path, data):
        if path.parent.name == bad and path.name.startswith("state.rank0.P"):
            raise OSError(28, "No space left on device")
        return real(path, data)

    monkeypatch.setattr(ck, "_atomic_write", flaky)
    kf = _engine(mask, obs, Q, checkpoint_dir=str(tmp_path), checkpoint_every=1, checkpoint_keep=2)
    with pytest.raises(ck.CheckpointWriteError, match="not committed"):
        kf.run(grid, x0, None, Pinv)
    committed = sorted(p.name for p in tmp_path.iterdir() if (p / "manifest.json").exists())
    assert committed == [g.strftime("A%Y%j") for g in grid[1:3]]
    assert not (tmp_path / bad / "manifest.json").exists()
    assert k.CheckpointManager.latest(tmp_path).name == grid[2].strftime("A%Y%j")


def test_kafka_output_tiff_roundtrip(tmp_path):
    mask, obs, prior, x0, Pinv, Q = _setup(seed=5)
    grid = _grid(3)
    out = k.KafkaOutput(k.TIP_PARAMETERS, [500000., 10., 0., 4000000., 0., -10.], "EPSG:32630", str(tmp_path))
    kf = _engine(mask, obs, Q, out=out)
    st = kf.run(grid, x0, None, Pinv)
    out.flush()
    arr, info = k.read_tiff(tmp_path / f"TeLAI_{grid[-1].strftime('A%Y%j')}.tif")
    assert arr.shape == mask.shape and arr.dtype == np.float32
    assert np.allclose(arr[mask], st.x[6].numpy())
    unc, _ = k.read_tiff(tmp_path / f"TeLAI_{grid[-1].strftime('A%Y%j')}_unc.tif")
    assert np.allclose(unc[mask], kf.unc(st)[6].numpy(), rtol=1e-6)
    assert info["geotransform"][1] == 10.0 and info["projection"] == "EPSG:32630"
    # native tiled DEFLATE with a ProjectedCSType GeoKey (GDAL / QGIS recognise the CRS)
    hdr = k.tiff_info(tmp_path / f"TeLAI_{grid[-1].strftime('A%Y%j')}.tif")
    assert hdr["tiled"] and hdr["compression"] == 8 and hdr["epsg"] == 32630
    assert len(out.write_s) == len(grid) - 1 and len(out.written) == 14 * (len(grid) - 1)


def test_kafka_output_writer_telemetry_and_rolling_files(tmp_path):
    """The granule writer's telemetry (per timestep in the metrics record and
    writer_stats): queue depth at each submit, waits of the time loop on the
    writer, encode time, raster and file bytes; keep_timesteps leaves only the
    newest timesteps' files on disk.  Uncompressed output is written as strips
    straight from the planes and reads back exactly."""
    mask, obs, prior, x0, Pinv, Q = _setup(seed=5)
    grid = _grid(4)
    out = k.KafkaOutput(k.TIP_PARAMETERS, [500000., 10., 0., 4000000., 0., -10.], "EPSG:32630", str(tmp_path),
                        level=0, keep_timesteps=1)
    kf = _engine(mask, obs, Q, out=out)
    st = kf.run(grid, x0, None, Pinv)
    out.flush()
    ws = out.writer_stats()
    n_ts = len(grid) - 1
    assert ws["timesteps_written"] == n_ts and ws["queue_depth_max"] >= 0
    assert ws["raster_bytes"] == n_ts * 14 * mask.size * 4 and ws["file_bytes"] >= ws["raster_bytes"]
    assert ws["queue_wait_s"] >= 0 and ws["slot_wait_s"] >= 0 and ws["write_s_max"] > 0
    recs = [h for h in kf.history if "output" in h]
    assert len(recs) == n_ts and all("queue_depth_last" in h["output"] for h in recs)
    files = sorted(p.name for p in tmp_path.iterdir())
    assert len(files) == 14 and all(grid[-1].strftime("A%Y%j") in f for f in files)
    arr, _ = k.read_tiff(tmp_path / f"TeLAI_{grid[-1].strftime('A%Y%j')}.tif")
    assert np.array_equal(arr[mask], st.x[6].numpy())
    assert not k.tiff_info(tmp_path / f"TeLAI_{grid[-1].strftime('A%Y%j')}.tif")["tiled"]


def test_memory_output_reference_signature():
    mask, obs, prior, x0, Pinv, Q = _setup(seed=6)
    out = k.KafkaOutputMemory(k.TIP_PARAMETERS)
    kf = _engine(mask, obs, Q, out=out)
    st = kf.run(_grid(3), x0, None, Pinv)
    last = out.output[max(out.output)]
    assert np.allclose(last["TeLAI"], st.x[6].numpy())


def test_streaming_equals_resident():
    mask, obs_s, prior, x0, Pinv, Q = _setup(stream=True, seed=7)
    _, obs_r, _, _, _, _ = _setup(stream=False, seed=7)
    grid = _grid(5)
    a = _engine(mask, obs_s, Q).run(grid, x0, None, Pinv)
    b = _engine(mask, obs_r, Q).run(grid, x0, None, Pinv)
    assert torch.equal(a.x, b.x)
    assert obs_s.ingest_bytes() > 0


def test_band_sequential_mode_runs():
    mask, obs, prior, x0, Pinv, Q = _setup(seed=8)
    st = _engine(mask, obs, Q, band_sequential=True).run(_grid(3), x0, None, Pinv)
    assert torch.isfinite(st.x).all() and torch.isfinite(st.P).all()


def test_spatial_regulariser_smooths():
    mask, obs, prior, x0, Pinv, Q = _setup(seed=9)
    grid = _grid(3)
    a = _engine(mask, obs, Q).run(grid, x0, None, Pinv)
    b = _engine(mask, obs, Q, spatial_gamma=50.0, spatial_params=[6], jacobi_sweeps=8).run(grid, x0, None, Pinv)

    def rough(st):
        img = np.zeros(mask.shape)
        img[mask] = st.x[6].numpy()
        dx = np.abs(np.diff(img, axis=1))[mask[:, 1:] & mask[:, :-1]]
        return dx.mean()
    assert rough(b) < 0.8 * rough(a)
    assert (a.x[0] - b.x[0]).abs().mean() < 0.02  # unsmoothed parameter moves only through coupling


def test_sar_engine_runs_and_recovers():
    mask = np.ones((16, 16), bool)
    obs = k.SyntheticS1Observations(mask, device="cpu", stream=False, field_cell=4, cloud_fraction=0.0)
    prior = k.GaussianPrior(["lai", "sm"], mask, [2.0, 0.25], np.diag([1.0, 0.1 ** 2]))
    kf = k.LinearKalman(obs, None, mask, k.create_sar_observation_operator, ["lai", "sm"],
                        state_propagation=None, prior=prior, device="cpu")
    x0, Pinv = prior.process_prior(None)
    st = kf.run(_grid(4, 6, obs.dates[0]), x0, None, Pinv)
    assert torch.isfinite(st.x).all()


def test_invalid_n_params_rejected():
    with pytest.raises(ValueError):
        k.LinearKalman(None, None, np.ones((2, 2), bool), None, ["a"] * 11)


@pytest.mark.parametrize("chunk", [10, 3])
def test_split_gp_operator_path_equals_fused(chunk):
    """Split path (operator kernel -> HBM -> band-chunked accumulation) == fused kernel."""
    mask = np.ones((10, 9), bool)
    obs = k.SyntheticS2Observations(mask, n_bands=10, n_train=30, device="cpu", stream=False, n_pool=2,
                                    field_cell=4)
    prior = k.SAILPrior(k.SAIL_PARAMETERS, mask)
    x0, Pinv = prior.process_prior(None)
    grid = [obs.dates[0] - dt.timedelta(days=1), obs.dates[1] + dt.timedelta(days=1)]
    res = []
    for mode in ("never", "always"):
        kf = k.LinearKalman(obs, None, mask, k.create_prosail_observation_operator, k.SAIL_PARAMETERS,
                            state_propagation=None, prior=prior, device="cpu",
                            config=k.EngineConfig(gp_split=mode, band_chunk=chunk, return_innovations=True))
        res.append(kf.run(grid, x0, None, Pinv))
    assert torch.allclose(res[0].x, res[1].x, rtol=1e-4, atol=1e-5)
    assert torch.allclose(res[0].P, res[1].P, rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("with_prior", [False, True])
def test_fused_propagation_engine_equals_materialized(with_prior):
    """EngineConfig.fuse_propagation: the forecast evaluated inside the analysis
    kernel gives the same run as the propagate pass + analysis (blend => the
    engine falls back to materialising)."""
    mask, obs, prior, x0, Pinv, Q = _setup(seed=5)
    grid = _grid(4)
    runs = []
    for fuse in (False, True):
        kf = _engine(mask, obs, Q, prior=prior if with_prior else None, fuse_propagation=fuse)
        runs.append((kf.run(grid, x0, None, Pinv), [h["gn_iterations"] for h in kf.history]))
    (a, ia), (b, ib) = runs
    assert ia == ib
    assert torch.allclose(a.x, b.x, rtol=1e-6, atol=1e-7)
    assert torch.allclose(a.P, b.P, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("spatial", [False, True])
def test_fused_output_equals_unpack(spatial):
    """EngineConfig.fuse_output: DeviceOutput rasters written by the final
    analysis iteration (spatial prior: by the regulariser's finish pass) equal
    the separate unpack pass."""
    mask, obs, prior, x0, Pinv, Q = _setup(seed=6)
    grid = _grid(4)
    reg = dict(spatial_gamma=50.0, spatial_params=[6], jacobi_sweeps=4) if spatial else {}
    res = []
    for fuse in (False, True):
        out = k.DeviceOutput(k.TIP_PARAMETERS, keep_history=True)
        kf = _engine(mask, obs, Q, out=out, fuse_output=fuse, **reg)
        kf.run(grid, x0, None, Pinv)
        res.append(out)
    a, b = res
    assert sorted(a.history) == sorted(b.history) and len(a.history) == 3
    for t in a.history:
        assert torch.allclose(a.history[t][0], b.history[t][0], rtol=1e-6, atol=1e-7)
        assert torch.allclose(a.history[t][1], b.history[t][1], rtol=1e-5, atol=1e-7)


def test_structured_metrics_and_summary(tmp_path):
    import json
    mask, obs, prior, x0, Pinv, Q = _setup(seed=7)
    path = tmp_path / "m.jsonl"
    kf = _engine(mask, obs, Q, metrics_path=str(path))
    kf.run(_grid(4), x0, None, Pinv)
    recs = [json.loads(line) for line in open(path)]
    dates = [r for r in recs if r["event"] == "date"]
    assert dates and all("status" in r and "pixel_updates_per_s_local" in r and "phases_ms" in r for r in dates)
    assert all(0.0 <= r["masked_fraction"] <= 1.0 for r in dates)
    summary = json.load(open(tmp_path / "m.summary.json"))
    assert summary["n_pixels"] == kf.n_total and summary["pixel_updates_per_s"] > 0
    assert len(summary["ranks"]) == 1 and summary["ranks"][0]["n_dates"] == len(dates)


@pytest.mark.parametrize("encoding", ["bf16y", "bf16"])
def test_identity_operator_engine_matches_oracle(encoding):
    """BASELINE config 2 semantics: 7 direct (identity) observations of the TIP
    state, bf16 ingest (y only with the weight derived in-kernel, or (y, w)
    pairs), LAI propagator — engine (host runner) vs the float64 oracle driving
    the reference-API linear operator factory."""
    mask = np.ones((16, 12), bool)
    mask[:2, :3] = False
    obs = k.SyntheticIdentityObservations(mask, device="cpu", stream=False, n_pool=4, field_cell=8,
                                          encoding=encoding)
    prior = k.JRCPrior(k.TIP_PARAMETERS, mask)
    x0, Pinv = prior.process_prior(None)
    Q = np.zeros_like(x0)
    Q[6::7] = 0.04
    grid = _grid(4)
    kf = k.LinearKalman(obs, None, mask, k.create_linear_observation_operator, k.TIP_PARAMETERS,
                        state_propagation=k.propagate_information_filter_LAI, device="cpu")
    kf.set_trajectory_model()
    kf.set_trajectory_uncertainty(Q)
    st = kf.run(grid, x0, None, Pinv)
    xr, Pr, iters = oracle_run(obs, mask, k.create_linear_observation_operator, 7, grid, x0, Pinv,
                               propagator=k.propagate_information_filter_LAI, Q=Q)
    _compare(st, xr, Pr)
    # several observation dates per 16-day step (the source observes every 5 days)
    assert [n for r in kf.history for n in r.get("gn_iterations", [])] == iters


@pytest.mark.parametrize("tol", [1e-3, 1e-9])
def test_fused_gn_iterations_equal_separate_launches(tol):
    """EngineConfig.fuse_gn: Gauss-Newton iterations 1 and 2 in one launch
    (iteration 1 kept in registers) give bit-identical states, outputs,
    iteration counts and norms to one launch per iteration -- also when the
    tolerance forces more iterations after the fused pair."""
    mask, obs, prior, x0, Pinv, Q = _setup(seed=7)
    grid = _grid(6)
    res = []
    for fuse in (False, True):
        out = k.DeviceOutput(k.TIP_PARAMETERS, keep_history=True)
        kf = _engine(mask, obs, Q, out=out, fuse_gn=fuse, convergence_tolerance=tol,
                     max_iterations=4)
        st = kf.run(grid, x0, None, Pinv)
        res.append((st, out, [h["gn_iterations"] for h in kf.history], [h["norms"] for h in kf.history]))
    (a, oa, ia, na), (b, ob, ib, nb) = res
    assert ia == ib and na == nb
    assert torch.equal(a.x, b.x) and torch.equal(a.P, b.P)
    for t in oa.history:
        assert torch.equal(oa.history[t][0], ob.history[t][0]) and torch.equal(oa.history[t][1], ob.history[t][1])


@pytest.mark.parametrize("spatial", [False, True])
def test_observed_first_order_keeps_every_pixel(spatial):
    """EngineConfig.observed_first: the pixels with an observation are visited
    first (obs_order, a stable partition), so cloudy pixels fill whole waves
    that skip the GP.  Every pixel's analysis is unchanged: states and output
    rasters equal the natural order's bit for bit, and the GN counts match
    (the norms sum the per-workgroup partials of other pixel sets)."""
    mask, obs, prior, x0, Pinv, Q = _setup(seed=11)
    grid = _grid(5)
    reg = dict(spatial_gamma=5.0, spatial_params=[6]) if spatial else {}
    res = []
    for on in (False, True):
        out = k.DeviceOutput(k.TIP_PARAMETERS, keep_history=True)
        kf = _engine(mask, obs, Q, out=out, observed_first=on, **reg)
        st = kf.run(grid, x0, None, Pinv)
        res.append((st, out, [h["gn_iterations"] for h in kf.history], kf._visit))
    (a, oa, ia, va), (b, ob, ib, vb) = res
    assert va is None and vb is not None
    assert ia == ib
    assert torch.equal(a.x, b.x) and torch.equal(a.P, b.P)
    for t in oa.history:
        assert torch.equal(oa.history[t][0], ob.history[t][0]) and torch.equal(oa.history[t][1], ob.history[t][1])


def test_obs_order_is_a_stable_partition():
    """obs_order on the host: observed pixels (any band w > 0) first, each
    group in increasing pixel order, a permutation of 0..N-1."""
    from kafka_inferenceengine_amd.ops import kernels as K
    mask, obs, prior, x0, Pinv, Q = _setup(seed=12)
    kf = _engine(mask, obs, Q)
    date = obs.dates[0]
    bands = kf._device_bands(date)
    from kafka_inferenceengine_amd.engine.bands import build_table
    table = build_table([s for s, _ in bands], [d for _, d in bands], kf.n_params, kf._cache, kf.device)
    order, _ = K.obs_order(table, kf.N, kf.device)
    o = order.numpy()
    seen = np.zeros(kf.N, bool)
    for db in (d for _, d in bands):
        y, w = db.decode()
        seen |= (w[:kf.N] > 0).numpy()
    n_obs = int(seen.sum())
    assert sorted(o.tolist()) == list(range(kf.N))
    assert seen[o[:n_obs]].all() and not seen[o[n_obs:]].any()
    assert (np.diff(o[:n_obs]) > 0).all() and (np.diff(o[n_obs:]) > 0).all()
    assert 0 < n_obs < kf.N


@pytest.mark.parametrize("groups", [None, [0, 1]])
def test_obs_order_local_partitions_each_chunk(groups):
    """obs_order(local=True) (EngineConfig.observed_first_local): every
    4096-pixel chunk is a stable partition of its own pixels by class
    (chunk-aligned, so a wave never mixes chunks); the default global partition
    orders the same classes over the whole tile."""
    from kafka_inferenceengine_amd.engine.bands import build_table
    from kafka_inferenceengine_amd.ops import kernels as K
    mask = np.ones((150, 131), bool)
    mask[40:60, :] = False
    obs = k.SyntheticBHRObservations(mask, n_train=20, device="cpu", stream=True, n_pool=1, field_cell=8)
    kf = k.LinearKalman(obs, None, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS, device="cpu")
    bands = kf._device_bands(obs.dates[0])
    table = build_table([s for s, _ in bands], [d for _, d in bands], kf.n_params, kf._cache, kf.device)
    seen = np.zeros((2, kf.N), bool)
    for b, (_, db) in enumerate(bands):
        seen[b if groups else 0] |= (db.decode()[1][:kf.N] > 0).numpy()
    cls = (3 - (seen[0] * 1 + seen[1] * 2)) if groups else (1 - seen[0] * 1)
    o = K.obs_order(table, kf.N, kf.device, groups=groups, local=True)[0].numpy()
    C = 4096
    assert kf.N > 3 * C
    for c0 in range(0, kf.N, C):
        blk = o[c0:c0 + C]
        assert sorted(blk.tolist()) == list(range(c0, min(kf.N, c0 + C)))
        kc = cls[blk]
        assert (np.diff(kc) >= 0).all()
        for c in np.unique(kc):
            assert (np.diff(blk[kc == c]) > 0).all()
    og = K.obs_order(table, kf.N, kf.device, groups=groups, local=False)[0].numpy()
    assert (np.diff(cls[og]) >= 0).all() and sorted(og.tolist()) == list(range(kf.N))


def test_obs_order_classes_of_two_sensors():
    """obs_order with band groups (multi-sensor: one group per sensor): a
    stable partition into the classes observed by both / the first only / the
    second only / neither, in that order; the engine's multi-sensor states do
    not depend on the order."""
    import datetime as dt
    from kafka_inferenceengine_amd.engine.bands import build_table
    from kafka_inferenceengine_amd.ops import kernels as K
    mask = np.ones((30, 26), bool)
    dates = [dt.datetime(2017, 7, 3) + dt.timedelta(days=2 * i) for i in range(3)]
    res = []
    for on in (False, True):
        s2 = k.SyntheticS2Observations(mask, dates=dates, n_bands=3, n_train=30, device="cpu", n_pool=3,
                                       stream=False, cloud_fraction=0.3, seed=1)
        olci = k.SyntheticOLCIObservations(mask, dates=dates, n_bands=2, n_train=30, device="cpu", n_pool=3,
                                           stream=False, cloud_fraction=0.3, seed=22)
        obs = k.MultiSensorObservations([s2, olci])
        prior = k.SAILPrior(k.SAIL_PARAMETERS, mask)
        kf = k.LinearKalman(obs, None, mask, k.create_prosail_observation_operator, k.SAIL_PARAMETERS,
                            state_propagation=None, prior=prior, device="cpu",
                            config=k.EngineConfig(observed_first=on))
        st = kf.run([dates[0] - dt.timedelta(days=1)] + [d + dt.timedelta(days=1) for d in dates],
                    kf.state_from_prior(prior), None, None)
        res.append((st, [h["gn_iterations"] for h in kf.history]))
        if on:
            bands = kf._device_bands(dates[0])
            table = build_table([sp for sp, _ in bands], [d for _, d in bands], kf.n_params, kf._cache, kf.device)
            groups = obs.band_groups(dates[0])
            assert groups == [0, 0, 0, 1, 1]
            order, _ = K.obs_order(table, kf.N, kf.device, groups=groups)
            o = order.numpy()
            seen = np.zeros((2, kf.N), bool)
            for g, (_, db) in zip(groups, bands):
                seen[g] |= (db.decode()[1][:kf.N] > 0).numpy()
            cls = 3 - (seen[0] * 1 + seen[1] * 2)
            assert sorted(o.tolist()) == list(range(kf.N))
            c = cls[o]
            assert (np.diff(c) >= 0).all()
            for v in range(4):
                sel = o[c == v]
                assert (np.diff(sel) > 0).all()
            assert len(set(c.tolist())) >= 3
    (a, ia), (b, ib) = res
    assert ia == ib and torch.equal(a.x, b.x) and torch.equal(a.P, b.P)


@pytest.mark.parametrize("tol", [1e-3, 1e-9])
def test_fused_spatial_first_iteration_equals_separate_launches(tol):
    """Spatial prior with spatial_first_plain: the plain first Gauss-Newton
    iteration fused with the regularised prepare of the second (one launch)
    is bit-identical to a plain launch followed by the prepare launch --
    states, output rasters, iteration counts and norms, also when the
    tolerance forces more (regularised) iterations after the fused pair."""
    mask, obs, prior, x0, Pinv, Q = _setup(seed=9)
    grid = _grid(5)
    res = []
    for fuse in (False, True):
        out = k.DeviceOutput(k.TIP_PARAMETERS, keep_history=True)
        kf = _engine(mask, obs, Q, out=out, fuse_gn=fuse, convergence_tolerance=tol, max_iterations=4,
                     spatial_gamma=5.0, spatial_params=[6], metrics_path=None)
        st = kf.run(grid, x0, None, Pinv)
        res.append((st, out, [h["gn_iterations"] for h in kf.history], [h["norms"] for h in kf.history]))
    (a, oa, ia, na), (b, ob, ib, nb) = res
    assert ia == ib and na == nb
    if tol < 1e-6:
        assert max(n for g in ib for n in g) > 2
    assert torch.equal(a.x, b.x) and torch.equal(a.P, b.P)
    for t in oa.history:
        assert torch.equal(oa.history[t][0], ob.history[t][0]) and torch.equal(oa.history[t][1], ob.history[t][1])


def test_linear_operator_converges_statically():
    """Identity operator: y' = y - offset does not depend on the linearisation
    point, so the fused second iteration reproduces the first exactly (norm 0)
    and the date ends after 2 iterations without a norm read-back; the first
    norm is filled in afterwards and equals the separate-launch run's."""
    import datetime as dt
    mask = np.ones((20, 24), bool)
    dates = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(5)]
    res = []
    for fuse in (False, True):
        obs = k.SyntheticIdentityObservations(mask, dates=dates, device="cpu", seed=3, stream=False)
        kf = k.LinearKalman(obs, None, mask, k.create_linear_observation_operator, k.TIP_PARAMETERS,
                            state_propagation=k.propagate_information_filter_LAI, device="cpu",
                            config=k.EngineConfig(fuse_gn=fuse))
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
        prior = k.JRCPrior(k.TIP_PARAMETERS, mask)
        x0, Pi = prior.process_prior(None)
        grid = [dates[0] - dt.timedelta(days=1)] + [d + dt.timedelta(days=1) for d in dates]
        st = kf.run(grid, x0, None, Pi)
        res.append((st, [h["gn_iterations"] for h in kf.history], [h["norms"] for h in kf.history], kf))
    (a, ia, na, _), (b, ib, nb, kfb) = res
    assert torch.equal(a.x, b.x) and torch.equal(a.P, b.P)
    assert ia == ib and all(g == [2] for g in ib)
    assert na == nb
    assert all(n[-1] == 0.0 for n in nb) and not kfb._lazy_norms


class _HostOnlyPrior:
    """A reference-style prior object: only ``process_prior`` (no device fast path)."""

    def __init__(self, inner):
        self.inner = inner

    def process_prior(self, date, inv_cov=True):
        return self.inner.process_prior(date, inv_cov=inv_cov)


@pytest.mark.parametrize("quirks", [False, True], ids=["gaussian-product", "reference-swap"])
def test_prior_blend_same_on_host_and_device_paths(quirks):
    """EngineConfig.reference_quirks drives both the device blend (K5) and the
    host ``propagate_and_blend_prior`` used for reference prior objects."""
    import datetime as dt
    import kafka_inferenceengine_amd as k

    mask = np.ones((6, 5), bool)
    grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(4)]
    out = []
    for wrap in (False, True):
        obs = k.SyntheticBHRObservations(mask, n_train=30, device="cpu", stream=False, n_pool=2, seed=5)
        prior = k.JRCPrior(k.TIP_PARAMETERS, mask)
        kf = k.LinearKalman(obs, None, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS,
                            state_propagation=k.propagate_information_filter_LAI,
                            prior=_HostOnlyPrior(prior) if wrap else prior, device="cpu",
                            config=k.EngineConfig(reference_quirks=quirks))
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
        x0, Pinv = prior.process_prior(None)
        st = kf.run(grid, x0, None, Pinv)
        out.append(st.x[:, :st.N].numpy().copy())
    assert np.allclose(out[0], out[1], rtol=1e-4, atol=1e-5)


def test_streamer_copies_every_date_with_three_buffers():
    """Host entries are recycled across dates (pool of 3), but every date is
    streamed: device buffers are keyed by the date, so a resident copy of the
    same host entry is never reused for another date; three buffers allow two
    dates in flight beyond the one being consumed."""
    from kafka_inferenceengine_amd.input_output.streaming import DateStreamer
    s = DateStreamer(3, (2, 64), torch.int16, "cpu", n_bufs=3)
    for kk in range(3):
        s.host_view(kk).fill_(kk + 1)
    assert s.max_ahead == 2
    per = s.entry_bytes
    for day in range(9):
        b = s.acquire(day % 3, key=("d", day))
        s.prefetch((day + 1) % 3, ("d", day + 1))
        s.prefetch((day + 2) % 3, ("d", day + 2))
        assert int(b[0, 0]) == day % 3 + 1
    assert s.bytes_h2d == per * 11          # dates 0..10 each copied exactly once
    # engine-level: a 3-entry pool over 6 dates streams 6 copies
    mask = np.ones((8, 8), bool)
    obs = k.SyntheticIdentityObservations(mask, device="cpu", stream=True, n_pool=3)
    for d in obs.dates[:6]:
        obs.get_device_bands(d)
    assert obs.ingest_bytes() == 6 * obs._streamer.entry_bytes


def test_jacobian_blocks_matches_fancy_indexing():
    """_jacobian_blocks (vectorised triplet read) equals the per-parameter CSR
    fancy indexing it replaces, with unsummed duplicates and explicit zeros."""
    import scipy.sparse as sp
    from kafka_inferenceengine_amd.engine.linear_kf import _jacobian_blocks
    rng = np.random.default_rng(0)
    N, n = 300, 7
    rows = np.repeat(np.arange(N), 4)
    cols = rows * n + np.tile([0, 1, 6, 2], N)
    vals = rng.normal(size=rows.size)
    vals[::17] = 0.0
    H = sp.coo_matrix((np.r_[vals, vals[:50]], (np.r_[rows, rows[:50]], np.r_[cols, cols[:50]])), shape=(N, n * N))
    Hc = sp.csr_matrix(H)
    r = np.arange(N)
    ref = np.stack([np.asarray(Hc[r, r * n + j]).ravel() for j in range(n)])
    assert np.allclose(_jacobian_blocks(H, N, n), ref) and np.allclose(_jacobian_blocks(Hc, N, n), ref)
    bad = sp.csr_matrix(([1.0], ([0], [n * 5])), shape=(N, n * N))
    with pytest.raises(ValueError, match="couples pixels"):
        _jacobian_blocks(bad, N, n)


def test_reference_protocol_factory_at_1024_squared_is_fast():
    """A reference-style factory (returns (H0, H) with H an [N, 7N] sparse
    matrix, utils.py:181-219 protocol) on a 1024^2 tile: the host precompute
    path reads the Jacobian blocks in one vectorised pass (seconds, not the
    per-parameter fancy indexing), and the step equals the same operator run
    through a device spec."""
    import time
    import scipy.sparse as sp
    mask = np.ones((1024, 1024), bool)
    N, n = mask.size, 7
    w = np.array([0.3, -0.2, 0.1, 0.25, 0.0, -0.15, 0.4])

    def factory(n_params, emulator, metadata, obs_mask, state_mask, x_lin, band):
        X = x_lin.reshape(-1, n_params)
        H0 = np.tanh(X) @ w + 0.1 * band
        g = (1.0 - np.tanh(X) ** 2) * w[None, :]
        g[~obs_mask[state_mask]] = 0.0
        rows = np.repeat(np.arange(X.shape[0]), n_params)
        cols = np.arange(X.shape[0] * n_params)
        return H0, sp.csr_matrix((g.ravel(), (rows, cols)), shape=(X.shape[0], n_params * X.shape[0]))

    from kafka_inferenceengine_amd.models.operators import OP_PRECOMP, OperatorSpec
    obs = k.SyntheticIdentityObservations(mask, device="cpu", stream=False, n_pool=1, seed=2)
    kf = k.LinearKalman(obs, None, mask, factory, k.TIP_PARAMETERS, device="cpu",
                        state_propagation=k.propagate_information_filter_LAI)
    st = kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask))
    dbs = [obs.get_device_band_data(obs.dates[0], b) for b in range(2)]
    specs = [OperatorSpec(OP_PRECOMP, list(range(n)), [0.0] * n) for _ in dbs]
    t0 = time.perf_counter()
    pre = kf._precompute_host(specs, dbs, st.x)
    dt_pre = time.perf_counter() - t0
    assert dt_pre < 20.0, dt_pre
    h = pre[0][1].numpy()
    X = st.x[:, :N].numpy().T.astype(np.float64)
    valid = dbs[0].decode()[1].numpy() > 0
    gref = ((1.0 - np.tanh(X) ** 2) * w[None, :]).T
    assert np.allclose(h[:, valid], gref[:, valid], rtol=1e-5, atol=1e-6)
    assert np.all(h[:, ~valid] == 0)


def _spatial_dense_run(device, tiled, size=(40, 36)):
    mask = np.ones(size, bool)
    grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(3)]
    obs = k.SyntheticBHRObservations(mask, n_train=40, device=device, stream=False, n_pool=2, field_cell=8)
    kf = k.LinearKalman(obs, None, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS, device=device,
                        config=k.EngineConfig(spatial_gamma=20.0, spatial_params=[6], spatial_tiled=tiled,
                                              spatial_tol=1e-6))
    kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
    st = kf.run(grid, kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask)), None, None)
    return st.x.cpu(), kf.reg_tiled_launches


def test_spatial_tiled_sweeps_equal_per_sweep_launches():
    """K9 temporal blocking (several sweeps per launch) changes nothing: the
    same states bit for bit as one launch per sweep (dense tile, one rank)."""
    a, na = _spatial_dense_run("cpu", True)
    b, nb = _spatial_dense_run("cpu", False)
    assert na > 0 and nb == 0
    assert torch.equal(a, b)


@pytest.mark.parametrize("mode", ["lai", "spatial", "prior_reset", "info_approx"])
def test_store_precision_auto_equals_always(mode):
    """EngineConfig.store_precision="auto": a date whose analysis only feeds
    the next forecast stores the precision rows that forecast reads (LAI
    propagator: A[6,6]; prior reset: none; approximate information filter: the
    diagonal).  Nothing else reads them, so every date's state, GN iterations
    and output rasters equal the full store's bit for bit, and the run's final
    state carries the full precision."""
    mask, obs, prior, x0, Pinv, Q = _setup(seed=12)
    grid = _grid(6)
    kw, prop, pri = {}, None, None
    if mode == "spatial":
        kw = dict(spatial_gamma=5.0, spatial_params=[6])
    elif mode == "prior_reset":
        pri = prior
    elif mode == "info_approx":
        prop = k.propagate_information_filter_approx_SLOW
    res = []
    for store in ("always", "auto"):
        out = k.DeviceOutput(k.TIP_PARAMETERS, keep_history=True)
        if pri is not None:   # no propagator: the prior resets every date's forecast
            kf = k.LinearKalman(obs, out, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS,
                                state_propagation=None, prior=pri, device="cpu",
                                config=k.EngineConfig(store_precision=store))
            st = kf.run(grid, kf.state_from_prior(pri), None, None)
        else:
            kf = _engine(mask, obs, Q, out=out, prop=prop, store_precision=store, **kw)
            st = kf.run(grid, x0, None, Pinv)
        assert st.full
        res.append((st, out, [h["gn_iterations"] for h in kf.history]))
    (a, oa, ia), (b, ob, ib) = res
    assert ia == ib
    assert torch.equal(a.x, b.x) and torch.equal(a.P, b.P)
    for t in oa.history:
        assert torch.equal(oa.history[t][0], ob.history[t][0]) and torch.equal(oa.history[t][1], ob.history[t][1])


def test_partial_precision_refuses_full_readers():
    """A state stored with only some precision rows (KFState.p_valid) refuses
    every reader of the full precision instead of returning stale rows."""
    mask, obs, prior, x0, Pinv, Q = _setup(seed=13)
    grid = _grid(4)
    kf = _engine(mask, obs, Q, store_precision="auto")
    from kafka_inferenceengine_amd.inference import iterate_time_grid
    dates = list(obs.dates)
    t, loc, _ = next(s_ for s_ in iterate_time_grid(grid, dates) if len(s_[1]))
    st = kf.step(t, loc, kf.state_from_prior(prior), advance=False, all_dates=dates)
    assert not st.full and st.p_valid is not None
    with pytest.raises(RuntimeError):
        st.to_reference()
    with pytest.raises(RuntimeError):
        st.numpy()
    assert st.clone().p_valid == st.p_valid     # a copy keeps the marker


@pytest.mark.parametrize("spatial", [False, True])
def test_aliased_mean_raster_equals_written_one(spatial):
    """DeviceOutput(alias_state=True): on dense strips the state's x is the
    mean raster (the kernels write only the uncertainty); the rasters and the
    states equal those of an output that has the mean written, bit for bit."""
    mask = np.ones((24, 20), bool)
    obs = k.SyntheticBHRObservations(mask, n_train=80, n_pool=5, device="cpu", seed=14, field_cell=8)
    prior = k.JRCPrior(k.TIP_PARAMETERS, mask)
    x0, Pinv = prior.process_prior(None)
    Q = np.zeros_like(x0)
    Q[6::7] = 0.04
    grid = _grid(5)
    kw = dict(spatial_gamma=5.0, spatial_params=[6]) if spatial else {}
    res = []
    for alias in (False, True):
        out = k.DeviceOutput(k.TIP_PARAMETERS, keep_history=True, alias_state=alias)
        kf = _engine(mask, obs, Q, out=out, **kw)
        st = kf.run(grid, x0, None, Pinv)
        res.append((st, out))
    (a, oa), (b, ob) = res
    assert torch.equal(a.x, b.x) and torch.equal(a.P, b.P)
    assert list(oa.history) == list(ob.history)
    for t in oa.history:
        assert torch.equal(oa.history[t][0], ob.history[t][0]) and torch.equal(oa.history[t][1], ob.history[t][1])


def test_band_lists_memoised_per_pool_slot():
    """A synthetic source hands out one band list per pool slot (same buffers,
    same operators); the engine derives its (spec, band) pairs and band table
    once per list, and a changed source setting gives a new list."""
    mask = np.ones((12, 10), bool)
    dates = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(4)]
    obs = k.SyntheticBHRObservations(mask, dates=dates, n_train=20, device="cpu", stream=False, n_pool=2)
    kf = k.LinearKalman(obs, k.DeviceOutput(k.TIP_PARAMETERS), mask, k.create_nonlinear_observation_operator,
                        k.TIP_PARAMETERS, device="cpu")
    a, b, c = obs.get_device_bands(dates[0]), obs.get_device_bands(dates[1]), obs.get_device_bands(dates[2])
    assert a is c and a is not b                      # dates 0 and 2 share pool slot 0
    pa, pc = kf._device_bands(dates[0]), kf._device_bands(dates[2])
    assert pa is pc and [db for _, db in pa] == a
    specs, dbs = [s for s, _ in pa], [d for _, d in pa]
    t1 = kf._band_table(pa, specs, dbs)
    assert kf._band_table(pc, specs, dbs) is t1
    assert kf._tables.key(specs, dbs, 7, "cpu") == kf._tables.key(specs, [d for _, d in pc], 7, "cpu")
    obs.rel_unc = 0.1
    assert obs.get_device_bands(dates[0]) is not a
