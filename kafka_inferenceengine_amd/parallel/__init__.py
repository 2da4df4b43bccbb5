"""Tile data parallelism over row strips with RCCL collectives (one process per GPU)."""
from .comm import Comm  # noqa: F401
from .partition import StripPartition, strip_bounds  # noqa: F401
from .farm import assign, run_chunks  # noqa: F401
