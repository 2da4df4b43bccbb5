"""CLI drivers and chunk farming (reference driver scripts)."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=600):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="4")
    r = subprocess.run([sys.executable, "-m", "kafka_inferenceengine_amd", *args], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout


def test_cli_run_bhr_and_resume(tmp_path):
    out = _run("run", "--sensor", "bhr", "--size", "24", "20", "--steps", "4", "--n-train", "40", "--device", "cpu",
               "--checkpoint-dir", str(tmp_path / "ck"), "--checkpoint-every", "1", "--out", str(tmp_path / "tif"))
    rec = json.loads(out.strip().splitlines()[-1])
    assert rec["timesteps"] == 4 and rec["finite"]
    assert len(os.listdir(tmp_path / "tif")) == 4 * 2 * 7
    out = _run("run", "--sensor", "bhr", "--size", "24", "20", "--steps", "6", "--n-train", "40", "--device", "cpu",
               "--resume", str(tmp_path / "ck"))
    assert json.loads(out.strip().splitlines()[-1])["timesteps"] == 2
    # an explicit checkpoint directory and its manifest.json resume the same way
    ck = sorted(p for p in (tmp_path / "ck").iterdir() if (p / "manifest.json").exists())
    for target in (ck[1], ck[1] / "manifest.json"):
        out = _run("run", "--sensor", "bhr", "--size", "24", "20", "--steps", "4", "--n-train", "40", "--device",
                   "cpu", "--resume", str(target))
        assert json.loads(out.strip().splitlines()[-1])["timesteps"] == 2


def test_cli_run_per_chunk_convergence_with_output_telemetry(tmp_path):
    """cli run with the reference drivers' per-chunk exit test and GeoTIFF
    output: the record carries the end-to-end wall, per-timestep wall and the
    writer's telemetry (queue depth, waits, encode time)."""
    out = _run("run", "--sensor", "s2", "--size", "40", "36", "--steps", "2", "--n-train", "30", "--device", "cpu",
               "--convergence-chunk", "16", "--domain-history", "--out", str(tmp_path / "tif"), "--out-level", "1",
               "--out-keep", "1")
    rec = json.loads(out.strip().splitlines()[-1])
    assert rec["timesteps"] == 2 and rec["finite"] and rec["wall_s"] > 0
    assert len(rec["timestep_wall_ms"]) == 2
    o = rec["output"]
    assert o["timesteps_written"] == 2 and o["queue_depth_max"] >= 0 and o["raster_bytes"] > 0
    assert len(os.listdir(tmp_path / "tif")) == 2 * 10        # newest timestep only: 10 params x (mean, unc)


def test_cli_resume_without_checkpoint_fails_clearly(tmp_path):
    (tmp_path / "empty").mkdir()
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "kafka_inferenceengine_amd", "run", "--sensor", "bhr", "--size", "8",
                        "8", "--steps", "2", "--n-train", "20", "--device", "cpu", "--resume",
                        str(tmp_path / "empty")], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode != 0 and "no committed checkpoint" in r.stderr


def test_cli_chunks_matches_reference_golden():
    out = _run("chunks", "235", "204", "--block", "128", "128")
    assert out.split("\n")[:4] == ["0 0 128 128 1", "0 128 128 76 2", "128 0 107 128 3", "128 128 107 76 4"]


def test_farm_single_process_skips_empty_chunks():
    from kafka_inferenceengine_amd.parallel.farm import assign, run_chunks

    mask = np.zeros((100, 90), bool)
    mask[:40, :50] = True
    seen = []
    res = run_chunks(90, 100, [64, 64], lambda c: seen.append(c) or c[4], None, skip_empty_mask=mask)
    assert sorted(res) == [1, 2, 3, 4]
    assert [c[4] for c in seen] == [1]            # only chunk 1 overlaps the mask
    assert assign(10, 1, 4) == [1, 5, 9]


def test_cli_run_bhr_and_s1_folders(tmp_path):
    """File readers reachable from the CLI (kafka_test.py:156-217): MCD43
    kernel rasters with an ROI, and Sentinel-1 sigma0 folders."""
    import datetime as dt

    import kafka_inferenceengine_amd as k

    shape = (14, 12)
    rng = np.random.default_rng(0)
    bhr = tmp_path / "mcd43"
    bhr.mkdir()
    for i in range(4):
        tag = (dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i)).strftime("A%Y%j")
        for band in (0, 1):
            for kk, v in enumerate((0.2, 0.05, 0.02) if band == 0 else (0.35, 0.1, 0.03)):
                k.write_tiff(bhr / f"{tag}_kernels_b{band}_k{kk}.tif",
                             (v * (1 + 0.05 * rng.standard_normal(shape))).astype(np.float32),
                             [500000.0, 500.0, 0.0, 4400000.0, 0.0, -500.0], "EPSG:32630")
        k.write_tiff(bhr / f"{tag}_qa.tif", rng.integers(0, 2, shape).astype(np.uint8))
    out = _run("run", "--sensor", "bhr", "--bhr-folder", str(bhr), "--period", "1", "--roi", "2", "3", "10", "13",
               "--n-train", "40", "--device", "cpu", "--out", str(tmp_path / "o"))
    rec = json.loads(out.strip().splitlines()[-1])
    assert rec["timesteps"] == 4 and rec["finite"] and rec["pixels"] == 80
    m, info = k.read_tiff(sorted((tmp_path / "o").iterdir())[0])
    assert m.shape == (10, 8) and info["geotransform"][0] == 501000.0 and info["epsg"] == 32630
    s1 = tmp_path / "s1"
    for day in ("20170405", "20170411"):
        d = s1 / f"S1_A_IW_GRDH_1SDV_{day}T060000_x"
        d.mkdir(parents=True)
        for pol in ("VV", "VH"):
            k.write_tiff(d / f"sigma0_{pol}.tif", rng.uniform(0.02, 0.2, shape).astype(np.float32))
        k.write_tiff(d / "theta.tif", np.full(shape, 37.0, np.float32))
    out = _run("run", "--sensor", "s1", "--s1-folder", str(s1), "--device", "cpu")
    rec = json.loads(out.strip().splitlines()[-1])
    assert rec["timesteps"] == 2 and rec["finite"] and rec["pixels"] == shape[0] * shape[1]
