"""Inference utilities — reference API (``kafka/inference/utils.py``).

``iterate_time_grid`` keeps the exact semantics of utils.py:44-65 (dates in
[t_{k-1}, t_k), first yield flagged); the operator factories live in
``models.operators`` and are re-exported here under the reference names.
"""
from __future__ import annotations

import logging

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spl

from ..models.operators import (create_linear_observation_operator, create_nonlinear_observation_operator,  # noqa
                                create_prosail_observation_operator, create_sar_observation_operator,
                                create_uncertainty, locate_in_lut, run_emulator)
from ..utils.blocks import blocks_to_sparse

LOG = logging.getLogger(__name__)


def iterate_time_grid(time_grid, the_dates):
    """Yield ``(t_k, observation dates in [t_{k-1}, t_k), is_first)`` for k >= 1."""
    dates = np.array(list(the_dates))
    istart = time_grid[0]
    first = True
    for timestep in list(time_grid)[1:]:
        if dates.size:
            sel = np.logical_and(dates >= istart, dates < timestep)
            locate_times = dates[sel]
        else:
            locate_times = dates
        LOG.info("Doing timestep from {} -> {}".format(istart.strftime("%Y-%m-%d"), timestep.strftime("%Y-%m-%d")))
        LOG.info("# of Observations: %d" % len(locate_times))
        for iobs in locate_times:
            LOG.info("\t->{}".format(iobs.strftime("%Y-%m-%d")))
        istart = timestep
        yield timestep, locate_times, first
        first = False


def block_diag(mats, format=None, dtype=None):
    """Block-diagonal sparse matrix from equal-sized blocks (utils.py:240-339),
    rebuilt on ``bsr_matrix`` (the vendored SciPy-PR code breaks on SciPy>=1.8)."""
    mats = [np.asarray(m) for m in mats]
    if not mats:
        return sp.csr_matrix((0, 0))
    shapes = {m.shape for m in mats}
    if len(shapes) == 1 and mats[0].ndim == 2 and mats[0].shape[0] == mats[0].shape[1]:
        out = blocks_to_sparse(np.stack(mats), format or "coo", dtype)
        return out
    return sp.block_diag(mats, format=format, dtype=dtype)


def spsolve2(a, b):
    """Diagonal of a^-1 b column by column (utils.py:342-349)."""
    a_lu = spl.splu(sp.csc_matrix(a))
    out = np.zeros(a.shape[1])
    for j in range(a.shape[1]):
        bb = np.asarray(b[:, j].todense()).ravel() if sp.issparse(b) else np.asarray(b)[:, j]
        out[j] = a_lu.solve(bb)[j]
    return out
