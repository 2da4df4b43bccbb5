"""In-tree build of the native extension ``_kafka_hip`` for gfx950.

Drives ``hipcc --offload-arch=gfx950`` for the device kernels and ``g++``
(OpenMP) for the host runner, then links one pybind11 module next to this
file so it travels with the repository snapshot to the GPU box.  No hipify,
no JIT cache: the object files live under ``build/`` and are rebuilt only
when a source is newer.

Usage: ``python -m kafka_inferenceengine_amd._build [--force] [--verbose] [--checked]``.

``--checked`` builds the debug variant ``_kafka_hip_checked`` (``-DKF_CHECKED``:
device/host index assertions, csrc/kf_core.h ``KF_DCHECK``) into its own build
directory; ``KAFKA_CHECKED=1`` makes ``ops/_ext.py`` load it instead of the release
module.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
ROOT = PKG_DIR.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "kafka_hip"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("KAFKA_OFFLOAD_ARCH", "gfx950")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
EXT_PATH = PKG_DIR / f"_kafka_hip{EXT_SUFFIX}"
CHECKED_EXT_PATH = PKG_DIR / f"_kafka_hip_checked{EXT_SUFFIX}"
PROF_EXT_PATH = PKG_DIR / f"_kafka_hip_prof{EXT_SUFFIX}"

HEADERS = ["kf_core.h", "kf_launch.h", "kf_stream.h", "kf_device.h", "kf_gp_mfma.h", "kf_tiff.h", "kf_deflate.h"]
# device translation units (compiled concurrently: the NP = 7 / 10 analysis
# instantiations dominate the build)
HIP_SOURCES = ["kf_kernels.hip", "kf_analysis7.hip", "kf_analysis10.hip", "kf_reg_tiled.hip", "kf_deflate.hip"]


def _pybind_includes() -> list[str]:
    import pybind11

    return [f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]


def _hipcc() -> str:
    exe = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    if not Path(exe).exists():
        raise RuntimeError("hipcc not found; set ROCM_PATH")
    return exe


def _stale(obj: Path, srcs: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(s.stat().st_mtime > t for s in srcs)


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=not verbose, text=True)
    if r.returncode != 0:
        msg = (r.stderr or "") + (r.stdout or "")
        raise RuntimeError(f"build step failed ({r.returncode}): {' '.join(cmd)}\n{msg[-8000:]}")


def build(force: bool = False, verbose: bool = False, checked: bool = False, prof: bool = False,
          exp: str | None = None, exp_csrc: str | None = None) -> Path:
    """``prof``: the phase-clock variant ``_kafka_hip_prof`` (``-DKF_PHASE_CLOCKS``,
    loaded with ``KAFKA_PROF=1``): the fused analysis kernels add each phase's
    shader cycles per wave to a device counter (``ext.phase_clocks``); a
    measuring tool, not built by ``__graft_entry__.build``.

    ``exp``: an A/B experiment module ``_kafka_hip_<exp>`` built from the
    sources in ``exp_csrc`` (a patched copy of ``csrc/``), loaded with
    ``KAFKA_EXT=<exp>``; never part of the release build."""
    from concurrent.futures import ThreadPoolExecutor

    if sum(map(bool, (checked, prof, exp))) > 1:
        raise ValueError("checked, prof and exp are separate variants")
    csrc = Path(exp_csrc) if exp else CSRC
    build_dir = BUILD.with_name("kafka_hip_checked") if checked else BUILD.with_name("kafka_hip_prof") if prof \
        else BUILD.with_name(f"kafka_hip_{exp}") if exp else BUILD
    ext_path = CHECKED_EXT_PATH if checked else PROF_EXT_PATH if prof else \
        PKG_DIR / f"_kafka_hip_{exp}{EXT_SUFFIX}" if exp else EXT_PATH
    build_dir.mkdir(parents=True, exist_ok=True)
    hdrs = [csrc / h for h in HEADERS]
    common = ["-O3", "-fPIC", "-std=c++17", f"-I{csrc}"]
    if checked:
        common += ["-DKF_CHECKED", "-DKF_MODULE_NAME=_kafka_hip_checked"]
    if prof:
        common += ["-DKF_PHASE_CLOCKS", "-DKF_MODULE_NAME=_kafka_hip_prof"]
    if exp:
        common += [f"-DKF_MODULE_NAME=_kafka_hip_{exp}"]
    hip_defs = ["-D__HIP_PLATFORM_AMD__", f"-I{ROCM / 'include'}"]
    hipcc = _hipcc()
    jobs, objs = [], []

    # 1. device kernels (gfx950 code objects embedded in the host objects)
    for name in HIP_SOURCES:
        src, obj = csrc / name, build_dir / (Path(name).stem + ".o")
        if force or _stale(obj, [src] + hdrs):
            # MFMA results straight into VGPRs (no v_accvgpr_read per exponent in kf_gp_mfma.h)
            # -fno-slp-vectorize: keeps the GP hi/lo split scalar so hipcc selects
            # v_fma_mix (kf_gp_mfma.h:gpm_exp_split) instead of v_pk_fma_f32 + conversions
            jobs.append([hipcc, f"--offload-arch={ARCH}", *common, "-munsafe-fp-atomics", "-fno-slp-vectorize", "-mllvm",
                         "-amdgpu-mfma-vgpr-form", "-c", str(src), "-o", str(obj)])
        objs.append(obj)

    # 2. host runner of the same per-pixel code (g++, OpenMP)
    src, obj = csrc / "kf_host.cpp", build_dir / "kf_host.o"
    if force or _stale(obj, [src] + hdrs):
        jobs.append(["g++", *common, *hip_defs, "-fopenmp", "-mavx2", "-mfma", "-ffp-contract=fast", "-c", str(src),
                     "-o", str(obj)])
    objs.append(obj)

    # 3. bindings + ingest runtime (host code, HIP runtime API)
    for name in ("kf_bindings.cpp", "kf_stream.cpp", "kf_tiff.cpp"):
        src, obj = csrc / name, build_dir / (Path(name).stem + ".o")
        if force or _stale(obj, [src] + hdrs):
            jobs.append(["g++", *common, *hip_defs, *_pybind_includes(), "-fvisibility=hidden", "-c", str(src),
                         "-o", str(obj)])
        objs.append(obj)

    if jobs:
        workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
        with ThreadPoolExecutor(workers) as pool:
            for f in [pool.submit(_run, cmd, verbose) for cmd in jobs]:
                f.result()

    if force or _stale(ext_path, objs):
        _run([hipcc, "-shared", "-fPIC", *map(str, objs), "-o", str(ext_path), "-lgomp", "-lpthread", "-lz",
              f"-L{ROCM / 'lib'}", "-lamdhip64"], verbose)
    return ext_path


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--checked", action="store_true", help="debug build with index assertions")
    ap.add_argument("--prof", action="store_true", help="phase-clock build (KAFKA_PROF=1)")
    ap.add_argument("--exp", default=None, help="A/B experiment module _kafka_hip_<EXP> (KAFKA_EXT=<EXP>)")
    ap.add_argument("--exp-csrc", default=None, help="patched copy of csrc/ for --exp")
    a = ap.parse_args()
    if bool(a.exp) != bool(a.exp_csrc):
        ap.error("--exp and --exp-csrc go together")
    p = build(force=a.force, verbose=a.verbose, checked=a.checked, prof=a.prof, exp=a.exp, exp_csrc=a.exp_csrc)
    print(f"built {p}")


if __name__ == "__main__":
    sys.exit(main())
