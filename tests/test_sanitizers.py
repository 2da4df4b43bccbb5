"""Host-code sanitizers.  GPU ASan / xnack+ runs are not
available on the MI355X pool, so the per-pixel code shared with the gfx950
kernels is run under AddressSanitizer + UBSan through the host runner with
exactly-sized buffers (tests/native/sanitize_host.cpp)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_runner_under_asan_ubsan(tmp_path):
    exe = tmp_path / "sanitize_host"
    cmd = ["g++", "-std=c++17", "-O0", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           "-fno-omit-frame-pointer", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", f"-I{ROOT}/csrc", "-fopenmp",
           f"{ROOT}/tests/native/sanitize_host.cpp", f"{ROOT}/csrc/kf_host.cpp", "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, OMP_NUM_THREADS="2", ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "sanitize_host ok" in r.stdout


_CHECKED_SCRIPT = r"""
import sys, numpy as np, torch
from kafka_inferenceengine_amd.ops import _ext, kernels as K
assert _ext.CHECKED and _ext.ext is not None and _ext.ext.__name__.endswith("_kafka_hip_checked")
N, n = 16, 4
rng = np.random.default_rng(0)
L = rng.normal(size=(N, n, n)) * 0.1
A = np.einsum("pij,pkj->pik", L, L) + np.eye(n)
iu = np.triu_indices(n)
a = torch.tensor(A[:, iu[0], iu[1]].T.copy(), dtype=torch.float32)
b = torch.randn(n, N); x = torch.randn(n, N); out = torch.zeros(n, N)
nbr = torch.full((4, N), -1, dtype=torch.int32)
nbr[0, 1:] = torch.arange(N - 1, dtype=torch.int32)
if sys.argv[1] == "bad":
    nbr[1, 3] = N + 5          # neighbour index past x_ext
K.jacobi(n, a, b, x, nbr, x, out, 2.0, 0b1111, N)
assert torch.isfinite(out).all()
print("ok")
"""


def test_checked_build_traps_out_of_range_neighbour(tmp_path):
    """Debug build (``_build.py --checked``): KF_DCHECK index
    assertions are live in the host runner of the same per-pixel code and abort
    on an out-of-range neighbour; valid input runs unchanged."""
    import os
    import subprocess
    import sys
    from pathlib import Path

    import pytest

    from kafka_inferenceengine_amd import _build

    if not _build.CHECKED_EXT_PATH.exists():
        pytest.skip("checked variant not built (python -m kafka_inferenceengine_amd._build --checked)")
    script = tmp_path / "checked.py"
    script.write_text(_CHECKED_SCRIPT)
    env = dict(os.environ, KAFKA_CHECKED="1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    root = str(Path(__file__).resolve().parents[1])
    env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
    good = subprocess.run([sys.executable, str(script), "good"], env=env, capture_output=True, text=True,
                          timeout=300, cwd=root)
    assert good.returncode == 0 and "ok" in good.stdout, good.stderr[-2000:]
    bad = subprocess.run([sys.executable, str(script), "bad"], env=env, capture_output=True, text=True,
                         timeout=300, cwd=root)
    assert bad.returncode != 0
    assert "KF_DCHECK failed" in bad.stderr and "ld_ext" in bad.stderr, bad.stderr[-2000:]
