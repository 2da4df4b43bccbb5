"""File-based readers (S2 granules, S1 sigma0, MCD43 BHR), TIFF IO and the
safe emulator format, exercised end to end through the engine on the CPU."""
import datetime as dt
import os

import numpy as np
import pytest
import torch

import kafka_inferenceengine_amd as k
from kafka_inferenceengine_amd.input_output import sentinel as S


def test_tiff_roundtrip_dtypes(tmp_path):
    rng = np.random.default_rng(0)
    for dtype in (np.float32, np.uint16, np.uint8, np.int16, np.float64):
        a = (rng.random((37, 23)) * 100).astype(dtype)
        for comp in (None, "deflate"):
            p = tmp_path / f"a_{np.dtype(dtype).name}_{comp}.tif"
            k.write_tiff(p, a, [10.0, 2.0, 0.0, 20.0, 0.0, -2.0], "EPSG:4326", comp, rows_per_strip=8)
            b, info = k.read_tiff(p)
            assert b.dtype == a.dtype and np.array_equal(a, b)
            assert info["geotransform"] == [10.0, 2.0, 0.0, 20.0, 0.0, -2.0]


def test_native_uncompressed_stack_is_striped_zero_copy(tmp_path):
    """Uncompressed native output: whole-row strips written straight from the
    planes (several strips per plane, a short last strip), read back exactly."""
    rng = np.random.default_rng(1)
    a = rng.random((3, 300, 5000)).astype(np.float32)       # 20 KB rows -> 209-row strips
    p = tmp_path / "stack_raw.tif"
    k.write_tiff(p, a, [0.0, 10.0, 0.0, 0.0, 0.0, -10.0], "EPSG:32630", None)
    b, info = k.read_tiff(p)
    assert np.array_equal(b, a)
    assert not info.get("tiled", False) and info.get("compression", 1) == 1


def test_deflate_backends_write_the_same_rasters(tmp_path):
    """Tile DEFLATE through libdeflate (when the system has it) and through
    zlib: both standard zlib streams (TIFF compression 8), both read back exactly."""
    from kafka_inferenceengine_amd.ops import kernels as K
    rng = np.random.default_rng(2)
    a = (rng.random((2, 300, 517)) + np.linspace(0, 1, 517)).astype(np.float32)
    out = {}
    try:
        for backend in ("zlib", "auto"):
            K.ext().tiff_deflate_backend(backend)
            p = tmp_path / f"d_{backend}.tif"
            k.write_tiff(p, a, level=1, predictor=3, tile=128)
            b, info = k.read_tiff(p)
            assert np.array_equal(a, b) and k.tiff_info(p)["compression"] == 8
            out[backend] = p.stat().st_size
    finally:
        K.ext().tiff_deflate_backend("auto")
    assert all(v < a.nbytes for v in out.values())


def test_reads_reference_mask_tiff():
    path = "/root/reference/Barrax_pivots.tif"
    if not os.path.exists(path):
        return
    m, info = k.read_tiff(path)
    assert m.shape == (204, 235)
    assert int((m > 0).sum()) == 13027  # 13,027 active pixels
    assert "geotransform" in info


def test_emulator_npz_roundtrip(tmp_path):
    em = k.make_tip_emulators(n_train=30)[0]
    S.save_emulator(tmp_path / "e.npz", em)
    em2 = S.load_emulator(tmp_path / "e.npz")
    x = np.random.default_rng(1).uniform(0, 0.5, (10, 4))
    assert np.allclose(em.predict(x)[0], em2.predict(x)[0])


def _make_s2_archive(root, shape, dates, emulators, consistent=False):
    """consistent=True: reflectance = emulator(truth near the SAIL prior mean),
    so the Gauss-Newton loop converges (random reflectances never do)."""
    rng = np.random.default_rng(2)
    truth = None
    if consistent:
        mu, _, _ = k.sail_prior()
        truth = mu[None, :] + rng.normal(0, 0.03, (shape[0] * shape[1], mu.size))
    emu_dir = root / "emus"
    emu_dir.mkdir()
    S.save_emulator_set(emu_dir / "sail_10_30_120.npz",
                        {f"S2A_MSI_{S.S2_EMULATOR_BANDS[b]:02d}": emulators[b] for b in range(10)})
    S.save_emulator_set(emu_dir / "sail_40_60_0.npz",
                        {f"S2A_MSI_{S.S2_EMULATOR_BANDS[b]:02d}": emulators[b] for b in range(10)})
    for d in dates:
        g = root / "data" / f"{d.year}" / f"{d.month}" / f"{d.day}" / "G1"
        g.mkdir(parents=True)
        k.write_tiff(g / "aot.tif", np.zeros(shape, np.float32))
        S.write_s2_metadata(g / "metadata.xml", 31.0, 0.0, 8.0, 118.0)
        for b, name in enumerate(S.S2_BAND_MAP):
            if truth is not None:
                rho = np.clip(emulators[b].predict(truth)[0].reshape(shape) + rng.normal(0, 0.002, shape), 0.01, 0.8)
            else:
                rho = np.clip(rng.normal(0.15 + 0.02 * b, 0.02, shape), 0.01, 0.8)
            dn = np.round(rho * 1e4).astype(np.uint16)
            dn[:2, :3] = 0  # no data
            k.write_tiff(g / f"B{name}_sur.tif", dn, compress="deflate")
    return root / "data", emu_dir


def test_sentinel2_reader_feeds_engine(tmp_path):
    shape = (12, 10)
    dates = [dt.datetime(2017, 7, 3) + dt.timedelta(days=2 * i) for i in range(3)]
    ems = k.make_prosail_emulators(10, n_train=40)
    data, emu = _make_s2_archive(tmp_path, shape, dates, ems, consistent=True)
    mask = np.ones(shape, bool)
    obs = S.Sentinel2Observations(str(data), str(emu), mask)
    assert obs.dates == dates and obs.bands_per_observation[dates[0]] == 10
    assert obs._find_emulator(31.0, 0.0, 8.0, 118.0).endswith("sail_10_30_120.npz")
    rec = obs.get_band_data(dates[0], 3)
    assert rec.mask.sum() == mask.sum() - 6 and rec.emulator is not None
    prior = k.SAILPrior(k.SAIL_PARAMETERS, mask)
    grid = [dates[0] - dt.timedelta(days=1)] + [d + dt.timedelta(days=1) for d in dates]
    states = []
    for ingest in (False, True):   # reference records (host) vs native decode -> DN16 device ingest
        obs = S.Sentinel2Observations(str(data), str(emu), mask, device_ingest=ingest)
        kf = k.LinearKalman(obs, None, mask, k.create_prosail_observation_operator, k.SAIL_PARAMETERS,
                            state_propagation=None, prior=prior, device="cpu")
        assert hasattr(obs, "get_device_band_data") == ingest
        x0, Pinv = prior.process_prior(None)
        st = kf.run(grid, x0, None, Pinv)
        assert torch.isfinite(st.x).all()
        assert all(h["gn_iterations"][0] < 25 for h in kf.history)
        states.append(st.x.numpy().copy())
    assert np.allclose(states[0], states[1], rtol=1e-4, atol=1e-5)
    assert obs._ingest.bytes_read == 3 * 10 * shape[0] * shape[1] * 2


def test_sentinel2_device_ingest_masked_strips(tmp_path):
    """Masked state grid, two strips: the native window decode + gather onto
    each strip's active pixels equals the host records."""
    from kafka_inferenceengine_amd.parallel import StripPartition
    shape = (14, 9)
    dates = [dt.datetime(2017, 7, 3)]
    ems = k.make_prosail_emulators(10, n_train=30)
    data, emu = _make_s2_archive(tmp_path, shape, dates, ems)
    mask = np.ones(shape, bool)
    mask[3:6, 2:7] = False
    for rank in range(2):
        part = StripPartition(mask, rank, 2)

        class _E:   # the two attributes bind_engine reads
            partition, device = part, torch.device("cpu")
        obs = S.Sentinel2Observations(str(data), str(emu), mask)
        obs.bind_engine(_E)
        for b in (0, 7):
            db = obs.get_device_band_data(dates[0], b)
            rec = obs.get_band_data(dates[0], b)
            y, w = db.decode()
            yr = rec.observations[part.r0:part.r1][part.local_mask]
            assert np.allclose(y.numpy(), yr, atol=1e-7)
            assert np.array_equal(w.numpy() > 0, rec.mask[part.r0:part.r1][part.local_mask])


def test_sentinel1_reader(tmp_path):
    shape = (8, 9)
    d = tmp_path / "S1_A_IW_GRDH_1SDV_20170405T060000_x"
    d.mkdir()
    rng = np.random.default_rng(3)
    for pol in ("VV", "VH"):
        s0 = rng.uniform(0.02, 0.2, shape).astype(np.float32)
        s0[0, 0] = S.WRONG_VALUE
        k.write_tiff(d / f"sigma0_{pol}.tif", s0)
    k.write_tiff(d / "theta.tif", np.full(shape, 37.0, np.float32))
    obs = S.S1Observations(str(tmp_path), np.ones(shape, bool))
    assert obs.dates == [dt.datetime(2017, 4, 5, 6, 0, 0)]
    r = obs.get_band_data(obs.dates[0], 1)
    assert not r.mask[0, 0] and r.mask.sum() == 71
    assert np.allclose(r.metadata["incidence_angle"], 37.0)
    mask = np.ones(shape, bool)
    prior = k.GaussianPrior(["lai", "sm"], mask, [2.0, 0.25], np.diag([1.0, 0.01]))
    kf = k.LinearKalman(obs, None, mask, k.create_sar_observation_operator, ["lai", "sm"], state_propagation=None,
                        prior=prior, device="cpu")
    x0, Pinv = prior.process_prior(None)
    st = kf.run([dt.datetime(2017, 4, 1), dt.datetime(2017, 4, 10)], x0, None, Pinv)
    assert torch.isfinite(st.x).all()


def test_bhr_reader_qa_uncertainty(tmp_path):
    shape = (6, 5)
    ems = k.make_tip_emulators(n_train=30)
    for day in (1, 17):
        tag = dt.datetime(2017, 1, day).strftime("A%Y%j")
        for band in (0, 1):
            for kk, v in enumerate((0.2, 0.05, 0.02)):
                k.write_tiff(tmp_path / f"{tag}_kernels_b{band}_k{kk}.tif", np.full(shape, v, np.float32))
        qa = np.zeros(shape, np.uint8)
        qa[0] = 1
        qa[1, 1] = 3  # bad
        k.write_tiff(tmp_path / f"{tag}_qa.tif", qa)
    obs = S.BHRObservations(ems, str(tmp_path), period=1)
    assert len(obs.dates) == 2
    r = obs.get_band_data(obs.dates[0], 0)
    bhr = 0.2 + 0.05 * 0.189184 - 0.02 * 1.377622
    assert np.isclose(r.observations[3, 3], bhr) and not r.mask[1, 1]
    w = r.uncertainty.diagonal().reshape(shape)
    assert np.isclose(w[0, 0], 1 / max(2.5e-3, 0.07 * bhr) ** 2)
    assert np.isclose(w[3, 3], 1 / max(2.5e-3, 0.05 * bhr) ** 2)


def test_ross_li_kernels_nadir():
    k0, kv, kg = S.ross_li_kernels(0.0, 0.0, 0.0)
    assert np.isclose(k0, 1.0)
    assert np.isclose(kv, -np.pi / 4 + np.pi / 4, atol=1e-12) or np.isfinite(kv)
    assert np.isfinite(kg)


# ---------------------------------------------------------------- footprints
REF_TIF = "/root/reference/Barrax_pivots.tif"
REF_JSON = "/root/reference/Barrax_pivots.json"


def test_utm_roundtrip_and_crs_parsing():
    from kafka_inferenceengine_amd.input_output import geo
    lon, lat = np.array([-2.1, -3.0, 0.5]), np.array([39.05, 41.2, 38.0])
    e, n = geo.lonlat_to_utm(lon, lat, 30)
    lo2, la2 = geo.utm_to_lonlat(e, n, 30)
    assert np.allclose(lo2, lon, atol=1e-8) and np.allclose(la2, lat, atol=1e-8)
    # central meridian of zone 30 is -3 deg: easting 500 km exactly, northing = k0 * meridian arc
    e0, _ = geo.lonlat_to_utm(-3.0, 40.0, 30)
    assert abs(e0 - 500000.0) < 1e-6
    assert geo.parse_crs("urn:ogc:def:crs:EPSG::32630") == geo.CRS("utm", 30, True)
    assert geo.parse_crs("WGS 84 / UTM zone 30N|WGS 84") == geo.CRS("utm", 30, True)
    assert geo.parse_crs(32731) == geo.CRS("utm", 31, False)
    assert geo.parse_crs("EPSG:4326") == geo.WGS84


def test_rasterized_pivots_reproduce_reference_mask():
    """The drivers' cutline mask: the 5 pivot polygons of Barrax_pivots.json
    rasterised on the grid of Barrax_pivots.tif give exactly its 13,027 pixels."""
    if not (os.path.exists(REF_TIF) and os.path.exists(REF_JSON)):
        return
    m, info = k.read_tiff(REF_TIF)
    polys = k.read_geojson_polygons(REF_JSON)
    assert len(polys) == 5
    r = k.rasterize_polygons(polys, info["geotransform"], info["shape"], info["projection"])
    assert np.array_equal(r, m > 0)


def test_raster_extent_feature_and_overlap(tmp_path):
    if not (os.path.exists(REF_TIF) and os.path.exists(REF_JSON)):
        return
    ext = k.raster_extent_feature(REF_TIF)
    x0, y0, x1, y1 = ext.bounds()
    assert -2.12 < x0 < x1 < -2.08 and 39.04 < y0 < y1 < 39.07       # Barrax, Spain
    assert all(k.find_overlap_raster_feature(REF_TIF, p) for p in k.read_geojson_polygons(REF_JSON))
    assert not k.find_overlap_raster_feature(REF_TIF, k.Polygon([[0, 0], [1, 0], [1, 1], [0, 1]], 4326))
    # a polygon containing the whole raster (no edge crossings) still intersects
    big = k.Polygon([[-3, 38], [-1, 38], [-1, 40], [-3, 40]], "EPSG:4326")
    assert k.find_overlap_raster_feature(REF_TIF, big)


# ---------------------------------------------------------------- MODIS
def test_mod09_reader_npz(tmp_path):
    rng = np.random.default_rng(3)
    f = tmp_path / "MOD09GA.A2017001.h17v05.npz"
    sds = {f"sur_refl_b0{b}_1": rng.integers(0, 5000, (8, 8)).astype(np.int16) for b in range(1, 8)}
    qa = np.full((4, 4), 8, np.uint16)
    qa[0, 0] = 9                                      # not in the QA whitelist
    sds.update(state_1km_1=qa, SolarZenith_1=np.full((4, 4), 3000), SolarAzimuth_1=np.full((4, 4), 1000),
               SensorZenith_1=np.full((4, 4), 1500), SensorAzimuth_1=np.full((4, 4), 4000))
    np.savez(f, **sds)
    d = dt.datetime(2017, 1, 1)
    obs = k.MOD09_ObservationsKernels([d], [str(f)])
    r = obs.get_band_data(d, 2)
    assert np.allclose(r.reflectance, sds["sur_refl_b02_1"] / 1e4)
    assert r.mask.shape == (8, 8) and not r.mask[:2, :2].any() and r.mask[2:, :].all()
    assert np.allclose(r.uncertainty, 0.015) and np.allclose(r.raa, 30.0) and np.allclose(r.sza, 30.0)
    _, kv, kg = S.ross_li_kernels(15.0, 30.0, 30.0)
    assert np.allclose(r.obs_op.Ross, kv) and np.allclose(r.obs_op.Li, kg)
    # kernels are reciprocal in (sza, vza) and vanish at nadir/nadir
    _, kv2, kg2 = S.ross_li_kernels(30.0, 15.0, 30.0)
    assert np.isclose(kv, kv2) and np.isclose(kg, kg2)
    _, kv0, kg0 = S.ross_li_kernels(0.0, 0.0, 0.0)
    assert abs(kv0) < 1e-12 and abs(kg0) < 1e-12
    assert obs.get_band_data(dt.datetime(2018, 1, 1), 1) is None
    with np.testing.assert_raises(IOError):
        k.MOD09_ObservationsKernels([d], ["x.hdf"]).get_band_data(d, 1)


def test_synergy_kernels_broadband(tmp_path):
    from kafka_inferenceengine_amd.input_output import modis as M
    shape = (5, 4)
    rng = np.random.default_rng(4)
    K = {}
    for day in (10, 40):
        stem = tmp_path / f"Synergy.A2017{day:03d}.h17v05"
        for b in range(7):
            K[(day, b)] = rng.uniform(0.0, 0.3, (3, *shape)).astype(np.float32)
            k.write_tiff(f"{stem}_b{b}_kernel_weights.tif", K[(day, b)])
        m = np.ones(shape, np.uint8)
        m[0, 0] = 0
        k.write_tiff(f"{stem}mask.tif", m)
    start = dt.datetime(2017, 1, 5)
    obs = k.SynergyKernels(str(tmp_path), "h17v05", start)
    assert sorted(obs.dates) == [dt.datetime(2017, 1, 10), dt.datetime(2017, 2, 9)]
    assert k.SynergyKernels(str(tmp_path), "h17v05", start, reference_quirks=True).dates == []
    d = dt.datetime(2017, 1, 10)
    for band, (coef, off) in enumerate(((M.TO_VIS, M.A_TO_VIS), (M.TO_NIR, M.A_TO_NIR))):
        r = obs.get_band_data(d, band)
        bhr = np.array([np.tensordot(M.TO_BHR, K[(10, b)].astype(np.float64), 1) for b in range(7)])
        want = np.tensordot(coef, bhr, 1) + off
        assert not r.mask[0, 0] and r.mask.sum() == shape[0] * shape[1] - 1
        assert np.allclose(r.observations[r.mask], want[r.mask])
        w = r.uncertainty.diagonal().reshape(shape)
        assert w[0, 0] == 0 and np.allclose(w[1:, 1:], 1 / np.maximum(2.5e-3, 0.05 * np.abs(want[1:, 1:])) ** 2)


def test_native_tiff_predictors_and_strategies(tmp_path):
    """Native tiled writer with the horizontal / floating-point predictors and
    the RLE / Huffman-only zlib strategies, decoded by the native reader and by
    the independent pure-Python decoder."""
    from kafka_inferenceengine_amd.input_output.tiff import _read_tiff_py, tiff_info
    rng = np.random.default_rng(3)
    f = (2.0 + np.cumsum(0.01 * rng.standard_normal((300, 517)), 1)).astype(np.float32)
    u = rng.integers(0, 4000, (300, 517)).astype(np.uint16)
    for a, pred, strat in ((f, 3, "rle"), (f, 3, "huffman"), (f, 1, "rle"), (f, 3, None), (u, 2, None),
                           (u, 2, "rle"), (u, 1, None)):
        p = tmp_path / f"p{pred}_{strat}_{a.dtype.name}.tif"
        k.write_tiff(p, a, [0.0, 10.0, 0.0, 0.0, 0.0, -10.0], "EPSG:32630", level=1, tile=128,
                     predictor=pred, strategy=strat)
        assert tiff_info(p)["predictor"] == pred
        b, _ = k.read_tiff(p)
        c, _ = _read_tiff_py(p)
        assert np.array_equal(a, b) and np.array_equal(a, c), (pred, strat, a.dtype)
    # python decoder also covers striped planar stacks from the fallback writer
    st = rng.random((3, 40, 33)).astype(np.float32)
    p = tmp_path / "stack.tif"
    k.write_tiff(p, st, tile=None, rows_per_strip=7)
    assert np.array_equal(_read_tiff_py(p)[0], st)


def test_reproject_utm_to_wgs84_golden(tmp_path):
    """CRS-aware warp (reference utils.py:43-64): Barrax_pivots.tif (UTM 30N)
    warped onto a WGS84 grid agrees with the pivot polygons rasterised straight
    on that WGS84 grid (an independent path: point-in-polygon after the
    polygon transform), and warping back onto the UTM grid restores the mask."""
    if not (os.path.exists(REF_TIF) and os.path.exists(REF_JSON)):
        return
    from kafka_inferenceengine_amd.input_output.utils import reproject_image
    m, info = k.read_tiff(REF_TIF)
    x0, y0, x1, y1 = k.raster_extent_feature(REF_TIF).bounds()
    res = 5e-5                                           # ~4.3 x 5.6 m at 39 N: finer than the 10 m source
    W, H = int(np.ceil((x1 - x0) / res)), int(np.ceil((y1 - y0) / res))
    gt = [x0, res, 0.0, y1, 0.0, -res]
    warped = reproject_image(m, info["geotransform"], (H, W), gt, 0, src_crs=info["projection"], dst_crs=4326)
    direct = k.rasterize_polygons(k.read_geojson_polygons(REF_JSON), gt, (H, W), "EPSG:4326")
    w = warped > 0
    assert w.sum() > 40000
    # disagreement only along the polygon edges: < 2 % of the pivot area
    assert (w ^ direct).sum() < 0.025 * direct.sum()
    assert abs(int(w.sum()) - int(direct.sum())) < 0.002 * direct.sum()          # no systematic shrink/grow
    cw, cd = np.argwhere(w).mean(0), np.argwhere(direct).mean(0)
    assert np.abs(cw - cd).max() < 0.25                                         # no shift (target pixels)
    back = reproject_image(warped, gt, m.shape, info["geotransform"], 0, src_crs=4326, dst_crs=info["projection"])
    assert ((back > 0) ^ (m > 0)).sum() < 0.005 * (m > 0).sum()
    # reference call form: file paths, target raster gives grid and CRS
    tgt = tmp_path / "wgs84_grid.tif"
    k.write_tiff(tgt, np.zeros((H, W), np.uint8), gt, "EPSG:4326")
    assert np.array_equal(reproject_image(REF_TIF, str(tgt)), warped)
    # same-CRS bilinear on a linear ramp is exact away from the edges
    ramp = np.add.outer(np.arange(50.0), 2 * np.arange(60.0)).astype(np.float32)
    out = reproject_image(ramp, [0, 1, 0, 0, 0, -1], (40, 40), [5.25, 1, 0, -5.5, 0, -1], resampling="bilinear")
    rr, cc = np.meshgrid(np.arange(40) + 5.5 + 0.5 - 0.5, np.arange(40) + 5.25 + 0.5 - 0.5, indexing="ij")
    assert np.allclose(out[:-2, :-2], (rr + 2 * cc)[:-2, :-2], atol=1e-4)


def _ifd_entries(b):
    """{tag: (entry offset, type, count, value-or-offset)} of a classic little-endian TIFF."""
    import struct
    assert b[:2] == b"II" and struct.unpack("<H", b[2:4])[0] == 42
    ifd = struct.unpack("<I", b[4:8])[0]
    n = struct.unpack("<H", b[ifd:ifd + 2])[0]
    out = {}
    for i in range(n):
        o = ifd + 2 + 12 * i
        tag, typ, cnt, val = struct.unpack("<HHII", b[o:o + 12])
        out[tag] = (o, typ, cnt, val)
    return out


def _strip_tiff(path, img, rps, pad_last=True):
    """A hand-made DEFLATE strip TIFF (float32) whose last strip, when
    ``pad_last``, is compressed padded to a full RowsPerStrip (as some writers
    do)."""
    import struct
    import zlib
    H, W = img.shape
    strips = []
    for r in range(0, H, rps):
        blk = img[r:r + rps]
        if pad_last and blk.shape[0] < rps:
            blk = np.vstack([blk, np.zeros((rps - blk.shape[0], W), np.float32)])
        strips.append(zlib.compress(np.ascontiguousarray(blk, "<f4").tobytes()))
    n = len(strips)
    entries = [(256, 4, 1, W), (257, 4, 1, H), (258, 3, 1, 32), (259, 3, 1, 8), (262, 3, 1, 1),
               (273, 4, n, None), (277, 3, 1, 1), (278, 4, 1, rps), (279, 4, n, None), (339, 3, 1, 3)]
    ifd_size = 2 + 12 * len(entries) + 4
    arr_off = 8 + ifd_size
    data_off = arr_off + 8 * n
    offs, o = [], data_off
    for s in strips:
        offs.append(o)
        o += len(s)
    out = bytearray(b"II*\x00" + struct.pack("<I", 8) + struct.pack("<H", len(entries)))
    for tag, typ, cnt, val in entries:
        if tag == 273:
            val = arr_off if n > 1 else offs[0]
        elif tag == 279:
            val = arr_off + 4 * n if n > 1 else len(strips[0])
        if typ == 3 and cnt == 1:
            out += struct.pack("<HHIHH", tag, typ, cnt, val, 0)
        else:
            out += struct.pack("<HHII", tag, typ, cnt, val)
    out += struct.pack("<I", 0)
    out += b"".join(struct.pack("<I", v) for v in offs) + b"".join(struct.pack("<I", len(s)) for s in strips)
    out += b"".join(strips)
    path.write_bytes(bytes(out))


def test_native_reader_accepts_padded_last_strip(tmp_path):
    """a compressed last strip padded to the full RowsPerStrip
    decodes (libtiff reads such files); one that stops short is refused."""
    from kafka_inferenceengine_amd.input_output.tiff import read_tiff_window
    img = np.random.default_rng(2).random((7, 10)).astype(np.float32)
    for pad in (True, False):
        p = tmp_path / f"s{int(pad)}.tif"
        _strip_tiff(p, img, 4, pad_last=pad)
        got = read_tiff_window(p, out=np.zeros((7, 10), np.float32))
        assert np.array_equal(got, img), pad
    # a last strip short of the raster's rows: refused
    p = tmp_path / "short.tif"
    _strip_tiff(p, img[:6], 4, pad_last=False)
    b = bytearray(p.read_bytes())
    import struct
    b[8 + 2 + 12 * 1 + 8:8 + 2 + 12 * 1 + 12] = struct.pack("<I", 7)   # ImageLength 6 -> 7
    (tmp_path / "short7.tif").write_bytes(bytes(b))
    with pytest.raises(RuntimeError, match="inflate failed"):
        read_tiff_window(tmp_path / "short7.tif", out=np.zeros((7, 10), np.float32))


def test_native_reader_rejects_bad_inputs(tmp_path):
    """the native reader must refuse (not overflow, zero-fill or
    index out of range on) a sample-size mismatch, a truncated DEFLATE stream,
    a chunk outside the file and a scalar tag without a value."""
    import struct
    from kafka_inferenceengine_amd.input_output.streaming import RasterIngest
    rng = np.random.default_rng(5)
    f32 = rng.random((64, 80)).astype(np.float32)
    p = tmp_path / "f32.tif"
    k.write_tiff(p, f32, compress="deflate")
    # 1. float32 file into an int16 ingest plane: refused, not a 2x overflow
    ing = RasterIngest(1, (64, 80), torch.int16, "cpu")
    with pytest.raises(RuntimeError, match="32-bit.*16-bit"):
        ing.acquire("d0", [(p, 0, (0, 64, 0, 80))])
    assert np.array_equal(k.read_tiff(p)[0], f32)
    b = bytearray(p.read_bytes())
    ent = _ifd_entries(bytes(b))
    cnt_tag = 325 if 325 in ent else 279
    o, typ, cnt, val = ent[cnt_tag]
    # 2. first chunk's byte count cut in half: inflate stops short (Z_BUF_ERROR)
    bc_off = o + 8 if cnt == 1 else val
    first = struct.unpack("<I", b[bc_off:bc_off + 4])[0]
    bad = bytearray(b)
    bad[bc_off:bc_off + 4] = struct.pack("<I", first // 2)
    (tmp_path / "trunc.tif").write_bytes(bytes(bad))
    with pytest.raises(RuntimeError, match="inflate failed"):
        k.read_tiff(tmp_path / "trunc.tif")
    # 3. a chunk that runs past the end of the file
    bad = bytearray(b)
    bad[bc_off:bc_off + 4] = struct.pack("<I", len(b) + 10)
    (tmp_path / "past.tif").write_bytes(bytes(bad))
    from kafka_inferenceengine_amd.input_output.tiff import tiff_info
    with pytest.raises(RuntimeError, match="outside the file"):
        tiff_info(tmp_path / "past.tif")
    # 4. a scalar tag (Compression) with count 0
    o, typ, cnt, val = ent[259]
    bad = bytearray(b)
    bad[o + 4:o + 8] = struct.pack("<I", 0)
    (tmp_path / "nocount.tif").write_bytes(bytes(bad))
    with pytest.raises(RuntimeError, match="no value"):
        tiff_info(tmp_path / "nocount.tif")


def test_record_types_defined_once():
    """each reference record type is one class, whichever
    reader module it is imported from (isinstance / pickling agree)."""
    from kafka_inferenceengine_amd.input_output import modis, observations, records, sentinel, synthetic

    assert sentinel.S2MSIdata is synthetic.S2MSIdata is records.S2MSIdata
    assert sentinel.BHR_data is observations.BHR_data is records.BHR_data
    assert sentinel.MOD09_data is modis.MOD09_data is records.MOD09_data
    assert sentinel.SARdata is records.SARdata
