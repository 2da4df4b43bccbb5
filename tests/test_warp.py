"""Observations warped onto the state-mask grid (reference
``Sentinel2_Observations.py:100-113,166``, ``Sentinel1_Observations.py:178,194``,
driver ``kafka_test_S2.py:155-162``): a granule on its own 20 m grid, offset
from the 10 m Barrax_pivots.tif state mask (235 x 204, EPSG:32630) and not
covering all of it, is read onto the mask grid — host path bit-identical to
``reproject_image``, device path (window decode + one gather) equal to the host
records, outputs on the mask's geotransform."""
import datetime as dt
import json
import os

import numpy as np
import pytest
import torch

import kafka_inferenceengine_amd as k
from kafka_inferenceengine_amd.input_output import sentinel as S
from kafka_inferenceengine_amd.input_output.tiff import read_tiff, tiff_info
from kafka_inferenceengine_amd.input_output.utils import GridWarp, reproject_image

REF_MASK = "/root/reference/Barrax_pivots.tif"
UTM30N = "WGS 84 / UTM zone 30N|WGS 84"
BARRAX_GT = [576452.584549, 10.0, 0.0, 4324696.153353, 0.0, -10.0]


def _mask_file():
    """The reference's Barrax_pivots.tif where the reference tree exists (this
    container); on a GPU box a stand-in on the same grid (235 x 204, 10 m,
    EPSG:32630) with five disc-shaped pivots."""
    if os.path.exists(REF_MASK):
        return REF_MASK
    import tempfile
    p = os.path.join(tempfile.gettempdir(), "kafka_barrax_grid_mask.tif")
    if not os.path.exists(p):
        yy, xx = np.mgrid[0:204, 0:235]
        m = np.zeros((204, 235), np.uint8)
        for cy, cx in ((50, 60), (60, 170), (150, 50), (140, 150), (100, 110)):
            m[(yy - cy) ** 2 + (xx - cx) ** 2 < 40 ** 2] = 1
        k.write_tiff(p, m, BARRAX_GT, UTM30N)
    return p


MASK = _mask_file()


def _granule_grid():
    """20 m grid, origin 100 m west / 60 m north of the mask's, 110 x 120 px:
    the mask's eastern 250 m are not covered."""
    mgt = tiff_info(MASK)["geotransform"]
    return (120, 110), [mgt[0] - 100.0, 20.0, 0.0, mgt[3] + 60.0, 0.0, -20.0]


def _s2_archive(root, n_dates=2, seed=0):
    shape, gt = _granule_grid()
    ems = k.make_prosail_emulators(10, n_train=30)
    rng = np.random.default_rng(seed)
    mu, _, _ = k.sail_prior()
    dates = [dt.datetime(2017, 7, 3) + dt.timedelta(days=2 * i) for i in range(n_dates)]
    dn_by_date = {}
    for d in dates:
        truth = mu[None, :] + rng.normal(0, 0.03, (shape[0] * shape[1], mu.size))
        dn = np.stack([np.round(np.clip(ems[b].predict(truth)[0], 0.01, 0.8) * 1e4).reshape(shape)
                       for b in range(10)]).astype(np.uint16)
        dn[:, :3, :5] = 0                          # no data inside the covered area
        dn_by_date[d] = dn
    keys = {f"S2A_MSI_{S.S2_EMULATOR_BANDS[b]:02d}": ems[b] for b in range(10)}
    data, emus = S.write_s2_archive(str(root), dn_by_date, keys, gt, UTM30N, emulator_angles=((8.0, 31.0, 118.0),))
    return data, emus, dates


def test_gridwarp_read_equals_reproject_image(tmp_path):
    shape, gt = _granule_grid()
    src = np.random.default_rng(1).integers(1, 9000, shape).astype(np.uint16)
    p = tmp_path / "b.tif"
    k.write_tiff(p, src, gt, UTM30N)
    minfo = tiff_info(MASK)
    w = GridWarp.from_files(p, minfo["shape"], minfo["geotransform"], minfo["epsg"])
    assert not w.identity
    ref = reproject_image(str(p), MASK)                  # the reference signature, whole band
    got = w.read(p)
    assert got.dtype == ref.dtype and np.array_equal(got, ref)
    assert (ref[:, -20:] == 0).all() and (ref[:, :200] > 0).all()   # eastern strip uncovered
    # only the bounding window is decoded
    r0, r1, c0, c1 = w.window(w.full_index())
    assert (r0, c0) == (3, 5) and r1 <= 120 and c1 == 110
    # identity grids map onto themselves
    wi = GridWarp(minfo["shape"], minfo["geotransform"], minfo["shape"], minfo["geotransform"], 32630, 32630)
    assert wi.identity and np.array_equal(wi.full_index(), np.arange(235 * 204))


def test_s2_reader_warps_onto_state_mask(tmp_path):
    data, emus, dates = _s2_archive(tmp_path)
    obs = S.Sentinel2Observations(data, emus, MASK)
    proj, gt = obs.define_output()
    assert gt == tiff_info(MASK)["geotransform"] and "UTM zone 30N" in proj
    mask = read_tiff(MASK)[0].astype(bool)
    folder = obs.date_data[dates[0]]
    for b in (0, 7):
        rec = obs.get_band_data(dates[0], b)
        assert rec.observations.shape == mask.shape
        ref = reproject_image(os.path.join(folder, f"B{S.S2_BAND_MAP[b]}_sur.tif"), MASK)
        assert np.array_equal(rec.mask, ref > 0)
        assert np.array_equal(rec.observations, np.where(ref > 0, ref / 10000., 0.0))
    # device protocol, two strips: window decode + gather == host records
    from kafka_inferenceengine_amd.parallel import StripPartition
    for rank in range(2):
        part = StripPartition(mask, rank, 2)

        class _E:   # the two attributes bind_engine reads
            partition, device = part, torch.device("cpu")
        o = S.Sentinel2Observations(data, emus, MASK)
        o.bind_engine(_E)
        assert o._warp_plan is not None
        for b in (0, 9):
            db = o.get_device_band_data(dates[1], b)
            ref = reproject_image(os.path.join(obs.date_data[dates[1]], f"B{S.S2_BAND_MAP[b]}_sur.tif"), MASK)
            assert np.array_equal(db.dn.numpy().view(np.uint16), ref[part.r0:part.r1][part.local_mask])
            y, wt = db.decode()
            rec = obs.get_band_data(dates[1], b)
            yr = rec.observations[part.r0:part.r1][part.local_mask]
            assert np.allclose(y.numpy(), yr, rtol=1e-6, atol=0)
            assert np.array_equal(wt.numpy() > 0, rec.mask[part.r0:part.r1][part.local_mask])
        win = next(iter(o._warp_plan["windows"].values()))
        assert o._ingest.bytes_read == 10 * (win[1] - win[0]) * (win[3] - win[2]) * 2


def test_s2_reader_refuses_roi_with_geo_mask(tmp_path):
    data, emus, _ = _s2_archive(tmp_path, n_dates=1)
    with pytest.raises(ValueError):
        S.Sentinel2Observations(data, emus, MASK, roi=[0, 0, 10, 10])


def test_cli_s2_run_on_reference_mask(tmp_path, capsys):
    """The reference S2 driver's workflow: granule folder + Barrax_pivots.tif
    as the state mask; outputs land on the mask's grid."""
    from kafka_inferenceengine_amd.cli import main
    data, emus, dates = _s2_archive(tmp_path / "arch")
    out = tmp_path / "out"
    main(["run", "--sensor", "s2", "--s2-folder", data, "--emulator-folder", emus, "--mask", MASK,
          "--out", str(out), "--steps", "2", "--device", "cpu"])
    rec = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert rec["timesteps"] == 2 and rec["finite"] and rec["pixels"] == int(read_tiff(MASK)[0].astype(bool).sum())
    files = sorted(p for p in os.listdir(out) if p.endswith(".tif"))
    assert files
    arr, info = read_tiff(out / files[0])
    assert arr.shape == (204, 235)
    assert info["geotransform"] == tiff_info(MASK)["geotransform"]


def test_s1_reader_warps_onto_state_mask(tmp_path):
    shape, gt = _granule_grid()
    d = tmp_path / "S1_A_IW_GRDH_1SDV_20170405T060000_x"
    d.mkdir()
    rng = np.random.default_rng(3)
    src = {}
    for pol in ("VV", "VH"):
        s0 = rng.uniform(0.02, 0.2, shape).astype(np.float32)
        s0[5, 7] = S.WRONG_VALUE
        src[pol] = s0
        k.write_tiff(d / f"sigma0_{pol}.tif", s0, gt, UTM30N)
    k.write_tiff(d / "theta.tif", rng.uniform(30, 45, shape).astype(np.float32), gt, UTM30N)
    obs = S.S1Observations(str(tmp_path), MASK)
    assert obs.define_output()[1] == tiff_info(MASK)["geotransform"]
    r = obs.get_band_data(obs.dates[0], 0)
    ref = reproject_image(str(d / "sigma0_VV.tif"), MASK)     # gdal.Warp's MEM raster: 0 where uncovered
    covered = GridWarp.from_files(d / "sigma0_VV.tif", (204, 235), tiff_info(MASK)["geotransform"],
                                  32630).full_index().reshape(204, 235) >= 0
    assert np.array_equal(r.mask, covered & (ref != S.WRONG_VALUE))
    assert np.array_equal(r.observations[r.mask], ref[r.mask].astype(np.float64))
    th = reproject_image(str(d / "theta.tif"), MASK)
    assert np.array_equal(r.metadata["incidence_angle"][covered], th[covered].astype(np.float64))


@pytest.mark.gpu
def test_s2_warp_device_ingest_gpu(tmp_path):
    """On the GPU: pinned window decode + H2D + the warp gather kernel equal
    the host reproject_image records bit for bit, both strips."""
    from kafka_inferenceengine_amd.parallel import StripPartition
    data, emus, dates = _s2_archive(tmp_path, n_dates=1)
    mask = read_tiff(MASK)[0].astype(bool)
    host = S.Sentinel2Observations(data, emus, MASK)
    folder = host.date_data[dates[0]]
    for rank in range(2):
        part = StripPartition(mask, rank, 2)

        class _E:
            partition, device = part, torch.device("cuda", 0)
        o = S.Sentinel2Observations(data, emus, MASK)
        o.bind_engine(_E)
        for b in range(10):
            db = o.get_device_band_data(dates[0], b)
            dn = db.dn.cpu().numpy().view(np.uint16)
            ref = reproject_image(os.path.join(folder, f"B{S.S2_BAND_MAP[b]}_sur.tif"), MASK)
            assert np.array_equal(dn, ref[part.r0:part.r1][part.local_mask])


@pytest.mark.gpu
def test_cli_s2_run_on_mask_gpu(cuda, tmp_path, capsys):
    """The S2 driver workflow on the GPU: warped device ingest, per-128^2-chunk
    convergence (the CLI default for S2), outputs on the mask's grid, and the
    same states as the CPU run."""
    from kafka_inferenceengine_amd.cli import main
    data, emus, dates = _s2_archive(tmp_path / "arch")
    recs = []
    for dev in ("cpu", "cuda"):
        out = tmp_path / f"out_{dev}"
        main(["run", "--sensor", "s2", "--s2-folder", data, "--emulator-folder", emus, "--mask", MASK,
              "--out", str(out), "--steps", "2", "--device", dev])
        recs.append(json.loads(capsys.readouterr().out.strip().splitlines()[-1]))
        name = sorted(p for p in os.listdir(out) if p.endswith(".tif") and "_unc" not in p)[0]
        arr, info = read_tiff(out / name)
        assert arr.shape == (204, 235) and info["geotransform"] == tiff_info(MASK)["geotransform"]
        recs[-1]["first"] = arr
    assert recs[0]["gn_iterations"] == recs[1]["gn_iterations"] and recs[1]["finite"]
    m = read_tiff(MASK)[0].astype(bool)
    a, b = recs[0]["first"][m], recs[1]["first"][m]
    assert np.allclose(a, b, rtol=2e-3, atol=2e-3), float(np.abs(a - b).max())
