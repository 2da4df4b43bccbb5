"""Loader for the native module ``_kafka_hip``.

``torch`` is imported first on purpose: the extension links
``libamdhip64.so.7``, and with torch already loaded the dynamic linker binds
it to torch's HIP runtime (same soname), so tensors, streams and events are
shared with PyTorch.  There is no Python fallback for device tensors: if the
module is missing on a GPU box every device op raises.
"""
from __future__ import annotations

import os

import torch  # noqa: F401  (must precede the extension import)

_err = None
CHECKED = os.environ.get("KAFKA_CHECKED", "0") not in ("", "0")
PROF = os.environ.get("KAFKA_PROF", "0") not in ("", "0")
EXP = os.environ.get("KAFKA_EXT", "")   # A/B experiment module (_build.py --exp)
try:
    if EXP:
        import importlib

        ext = importlib.import_module(f"kafka_inferenceengine_amd._kafka_hip_{EXP}")
    elif CHECKED:  # debug build with index assertions (_build.py --checked)
        from .. import _kafka_hip_checked as ext  # type: ignore
    elif PROF:  # phase-clock build of the JRC-TIP analysis kernel (_build.py --prof)
        from .. import _kafka_hip_prof as ext  # type: ignore
    else:
        from .. import _kafka_hip as ext  # type: ignore
except ImportError as e:  # pragma: no cover - exercised only when unbuilt
    ext = None
    _err = e


def require_ext():
    if ext is None:
        raise RuntimeError(
            "kafka_inferenceengine_amd native extension `_kafka_hip` is not built "
            f"({_err}); run `python -m kafka_inferenceengine_amd._build`")
    return ext


def ext_path() -> str | None:
    return None if ext is None else os.path.abspath(ext.__file__)


def ensure_built(verbose: bool = False):
    """Build in-tree if missing (used by tests / build())."""
    global ext, _err
    if ext is not None:
        return ext
    from .. import _build

    _build.build(verbose=verbose, checked=CHECKED)
    import importlib

    ext = importlib.import_module("kafka_inferenceengine_amd._kafka_hip" + ("_checked" if CHECKED else ""))
    _err = None
    return ext
