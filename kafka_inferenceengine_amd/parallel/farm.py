"""Chunk farming — the reference's distribution model, kept for compatibility.

``kafka_test_Py36.py:241-255`` cuts the raster with ``get_chunks`` and maps an
independent ``LinearKalman`` per chunk over dask workers (``client.map`` +
``client.gather``), writing one file set per chunk (``prefix=hex(chunk)``).
``run_chunks`` does the same over ``torch.distributed`` ranks (static
round-robin, deterministic), returning every chunk's result on rank 0.
Tile-DP with a strip per GPU (``StripPartition``) is the preferred mode on
MI355X; farming remains useful for sparse masks and independent AOIs.
"""
from __future__ import annotations

import torch.distributed as dist

from ..input_output.utils import get_chunks


def assign(n_chunks: int, rank: int, world: int) -> list[int]:
    return [i for i in range(n_chunks) if i % world == rank]


def run_chunks(nx, ny, block_size, fn, comm=None, skip_empty_mask=None):
    """Run ``fn(chunk)`` for every ``(x_off, y_off, nx_valid, ny_valid, chunk_no)``
    of ``get_chunks(nx, ny, block_size)``; chunks whose window of
    ``skip_empty_mask`` is empty are skipped (kafka_test_Py36.py:154).
    Returns {chunk_no: result} on rank 0 (None elsewhere)."""
    chunks = list(get_chunks(nx, ny, block_size))
    rank = comm.rank if comm is not None else 0
    world = comm.world if comm is not None else 1
    mine = {}
    for i in assign(len(chunks), rank, world):
        x0, y0, w, h, no = chunks[i]
        if skip_empty_mask is not None and not skip_empty_mask[y0:y0 + h, x0:x0 + w].any():
            mine[no] = None
            continue
        mine[no] = fn(chunks[i])
    if world == 1:
        return mine
    out = [None] * world if rank == 0 else None
    dist.gather_object(mine, out, dst=0, group=comm.group)
    if rank != 0:
        return None
    merged = {}
    for part in out:
        merged.update(part)
    return dict(sorted(merged.items()))
