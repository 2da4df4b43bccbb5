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
