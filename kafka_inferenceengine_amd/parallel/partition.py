"""Tile-DP partition of the raster into row strips, one per rank.

Replaces the reference's chunk farming (``get_chunks`` + dask ``client.map``,
``kafka_test_Py36.py:241-255``): rank r owns rows [r0, r1) chosen so every
rank holds about the same number of *active* pixels (state_mask True).  The
active pixels of a strip, in C order, are a contiguous slice of the global
active-pixel numbering, so global interleaved vectors slice trivially.

For the spatial regulariser the partition also builds the 4-neighbour table
of every local active pixel, indexing an extended state
``[local pixels | halo row above | halo row below]``.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def strip_bounds(state_mask: np.ndarray, world: int, balance: str = "active") -> list[tuple[int, int]]:
    """Row ranges [r0, r1) per rank; every rank gets >= 1 row."""
    H = state_mask.shape[0]
    if world > H:
        raise ValueError(f"cannot split {H} rows over {world} ranks")
    if balance == "rows":
        edges = [round(k * H / world) for k in range(world + 1)]
    else:
        counts = state_mask.sum(1).astype(np.float64)
        if counts.sum() == 0:
            counts = np.ones(H)
        cum = np.concatenate([[0.0], np.cumsum(counts)])
        total = cum[-1]
        edges = [0]
        for k in range(1, world):
            target = total * k / world
            r = int(np.searchsorted(cum, target, side="left"))
            r = max(r, edges[-1] + 1)
            r = min(r, H - (world - k))
            edges.append(r)
        edges.append(H)
    return [(edges[k], edges[k + 1]) for k in range(world)]


@dataclass
class StripPartition:
    state_mask: np.ndarray
    rank: int = 0
    world: int = 1
    balance: str = "active"

    def __post_init__(self):
        self.state_mask = np.asarray(self.state_mask).astype(bool)
        self.shape = self.state_mask.shape
        self.bounds = strip_bounds(self.state_mask, self.world, self.balance)
        self.r0, self.r1 = self.bounds[self.rank]
        self.local_mask = self.state_mask[self.r0:self.r1]
        self.local_idx = np.flatnonzero(self.local_mask.ravel()).astype(np.int64)   # raster index in strip
        self.N = int(self.local_idx.size)
        counts = [int(self.state_mask[a:b].sum()) for a, b in self.bounds]
        self.counts = counts
        self.offset = int(sum(counts[:self.rank]))
        self.N_total = int(sum(counts))

    @property
    def pixel_slice(self) -> slice:
        return slice(self.offset, self.offset + self.N)

    @property
    def strip_shape(self):
        return (self.r1 - self.r0, self.shape[1])

    def global_index(self) -> np.ndarray:
        """Global raster (flat) index of each local active pixel."""
        return self.local_idx + self.r0 * self.shape[1]

    # -------------------------------------------------- regulariser
    def halo_layout(self):
        """Active pixels of the boundary rows: what I send and receive.

        Returns dict with send_up/send_down (local indices of my first/last row's
        active pixels) and n_up/n_down (halo sizes = neighbours' boundary rows)."""
        W = self.shape[1]
        first = self.local_idx[self.local_idx < W]
        last_row = self.r1 - self.r0 - 1
        last = np.nonzero(self.local_idx // W == last_row)[0]
        send_up = np.nonzero(self.local_idx < W)[0]
        n_up = int(self.state_mask[self.r0 - 1].sum()) if self.r0 > 0 else 0
        n_down = int(self.state_mask[self.r1].sum()) if self.r1 < self.shape[0] else 0
        del first
        return {"send_up": send_up.astype(np.int64), "send_down": last.astype(np.int64), "n_up": n_up,
                "n_down": n_down}

    def dense_geometry(self):
        """``{"w", "h", "halo", "n_up"}`` when the strip and its halo rows are fully
        active (the kernels then derive neighbours from the pixel index instead of
        reading the [4, N] table — kf_core.h:StripGeo), else None."""
        H, W = self.shape
        lo, hi = max(self.r0 - 1, 0), min(self.r1 + 1, H)
        if self.N == 0 or not self.state_mask[lo:hi].all() or self.N >= 2 ** 31:
            return None
        halo = (1 if self.r0 > 0 else 0) | (2 if self.r1 < H else 0)
        return {"w": W, "h": self.r1 - self.r0, "halo": halo, "n_up": W if self.r0 > 0 else 0}

    def neighbour_table(self) -> np.ndarray:
        """int32 [4, N]: index of the up/down/left/right active neighbour in the
        extended state (local 0..N-1, halo-up N.., halo-down N+n_up..), -1 if none."""
        H, W = self.shape
        h = self.r1 - self.r0
        lid = np.full((h + 2, W), -1, dtype=np.int64)       # rows r0-1 .. r1
        lid[1:h + 1].ravel()[self.local_idx] = np.arange(self.N)
        lay = self.halo_layout()
        if self.r0 > 0:
            cols = np.flatnonzero(self.state_mask[self.r0 - 1])
            lid[0, cols] = self.N + np.arange(cols.size)
        if self.r1 < H:
            cols = np.flatnonzero(self.state_mask[self.r1])
            lid[h + 1, cols] = self.N + lay["n_up"] + np.arange(cols.size)
        rr = self.local_idx // W + 1
        cc = self.local_idx % W
        up = lid[rr - 1, cc]
        down = lid[rr + 1, cc]
        left = np.where(cc > 0, lid[rr, np.maximum(cc - 1, 0)], -1)
        right = np.where(cc < W - 1, lid[rr, np.minimum(cc + 1, W - 1)], -1)
        return np.ascontiguousarray(np.stack([up, down, left, right]).astype(np.int32))
