"""KaFKA on MI355X — Kalman-filter land-surface inference engine for gfx950.

Public names mirror the reference package (``kafka/__init__.py``): the engine
``LinearKalman``, the inference helpers, observation operators and the
input/output classes.
"""
__version__ = "0.1.0"

from .engine.config import EngineConfig  # noqa: F401,E402
from .engine.linear_kf import LinearKalman, Metadata, Previous_State  # noqa: F401,E402
from .engine.state import KFState  # noqa: F401,E402
from .inference import *  # noqa: F401,F403,E402
from .input_output import *  # noqa: F401,F403,E402
from .models import *  # noqa: F401,F403,E402
from .parallel import Comm, StripPartition  # noqa: F401,E402
