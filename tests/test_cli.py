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
