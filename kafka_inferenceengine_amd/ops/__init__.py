"""Device ops: gfx950 kernels (and the host runner of the same code) on torch tensors."""
from ._ext import ensure_built, ext_path, require_ext  # noqa: F401
from .kernels import (OBS_DN16, OBS_F32, OBS_NONE, ST_BAD_OP, ST_FALLBACK, ST_NO_OBS, ST_NONFINITE,  # noqa: F401
                      ST_NONSPD, SUPPORTED_NP, BandTable, analysis, check_np, gain, gather, grid_for, hessian,
                      invert, jacobi, lut_nearest, make_band_table, operator_eval, partials_buffer, prop_args, propagate,
                      reduce_partials, unpack)
