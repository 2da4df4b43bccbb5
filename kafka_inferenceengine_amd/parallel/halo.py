"""Halo exchange for the GMRF spatial regulariser (K9 + C2).

The regularised fields live in extended buffers ``z_ext = [local pixels | halo
row above | halo row below]`` ([k, N + n_up + n_down]); the neighbour table
(or the dense strip geometry) indexes into them.  Each Jacobi sweep packs my
first / last row (gather kernel) and swaps them with strip rank -1 / +1 by
point-to-point RCCL: one xGMI link per direction, k floats per boundary pixel
(~43 KB per 10980-px row and field).

Overlap (C2): ``start_fill`` posts the exchange and returns at once;
``finish_fill`` makes the compute stream wait for it and unpacks the halo
columns.  The engine computes a sweep's boundary rows first, starts their
exchange, computes the interior rows while the rows are on the wire, and only
then finishes the exchange (``LinearKalman._regularised_iteration``).
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import kernels as K


class HaloExchanger:
    def __init__(self, partition, comm, n_params, device, spatial_params=None):
        self.partition = partition
        self.comm = comm
        self.n = n_params
        self.N = partition.N
        lay = partition.halo_layout()
        self.n_up, self.n_down = lay["n_up"], lay["n_down"]
        self.send_up_idx = torch.from_numpy(lay["send_up"]).to(device)
        self.send_down_idx = torch.from_numpy(lay["send_down"]).to(device)
        # C2 overlap split, dense or masked: local pixels are in row-major order,
        # so the rows the neighbours need are the index ranges [0, a) and
        # [N - b, N); everything between is interior (reads no halo of the next
        # iterate).  None when the boundary rows are not such ranges.
        a, b = int(lay["send_up"].size), int(lay["send_down"].size)
        N = self.N
        ok = (np.array_equal(lay["send_up"], np.arange(a)) and np.array_equal(lay["send_down"], np.arange(N - b, N))
              and a + b < N)
        self.split = (a, b) if ok else None
        self._nbr = None
        self._device = torch.device(device)
        self._z = None
        params = range(n_params) if spatial_params is None else spatial_params
        self.reg_mask = 0
        for j in params:
            self.reg_mask |= 1 << int(j)
        self.bytes_sent = 0
        self.exchanges = 0

    @property
    def nbr(self) -> torch.Tensor:
        """int32 [4, N] neighbour table (built on first use: dense strips use
        the index geometry instead, StripPartition.dense_geometry)."""
        if self._nbr is None:
            self._nbr = torch.from_numpy(self.partition.neighbour_table()).to(self._device)
        return self._nbr

    @property
    def degrees(self) -> torch.Tensor:
        """float32 [N]: active 4-neighbours of each local pixel (halo rows included)."""
        if getattr(self, "_deg", None) is None:
            nt = self.partition.neighbour_table()
            self._deg = torch.from_numpy((nt >= 0).sum(0).astype("float32")).to(self._device)
        return self._deg

    def z_buffers(self, k: int):
        """Three extended [k, N + n_up + n_down] buffers for the regularised fields
        (Chebyshev keeps the previous iterate besides the current and next)."""
        if self._z is None or self._z[0].shape[0] != k:
            cols = self.N + self.n_up + self.n_down
            self._z = [torch.zeros((k, cols), dtype=torch.float32, device=self._device) for _ in range(3)]
            self._z_recv = (torch.zeros((k, self.n_up), dtype=torch.float32, device=self._device),
                            torch.zeros((k, self.n_down), dtype=torch.float32, device=self._device))
        return self._z

    def reg_rows(self) -> list[int]:
        return [j for j in range(self.n) if (self.reg_mask >> j) & 1]

    # ------------------------------------------------------------------ C2
    def start_fill(self, z_ext: torch.Tensor):
        """Pack my boundary rows of ``z_ext`` (whose local part is current) and
        post their exchange with strip rank -1 / +1; returns a handle for
        ``finish_fill`` (None on one rank)."""
        if not self.comm.distributed:
            return None
        ru, rd = self._z_recv
        su = K.gather(z_ext, self.send_up_idx) if self.send_up_idx.numel() else None
        sd = K.gather(z_ext, self.send_down_idx) if self.send_down_idx.numel() else None
        pending = self.comm.exchange_halo_async(su, sd, ru, rd)
        self.bytes_sent += 4 * z_ext.shape[0] * (self.send_up_idx.numel() + self.send_down_idx.numel())
        self.exchanges += 1
        return pending, (su, sd)

    def finish_fill(self, handle, z_ext: torch.Tensor) -> torch.Tensor:
        """Wait (stream-ordered) for the exchange and write the received rows
        into the halo columns of ``z_ext``."""
        if handle is None:
            return z_ext
        pending, _keep = handle
        pending.wait()
        N = self.N
        ru, rd = self._z_recv
        if self.n_up:
            z_ext[:, N:N + self.n_up].copy_(ru)
        if self.n_down:
            z_ext[:, N + self.n_up:].copy_(rd)
        return z_ext

    def fill_halo(self, z_ext: torch.Tensor) -> torch.Tensor:
        """Blocking C2 (start + finish)."""
        return self.finish_fill(self.start_fill(z_ext), z_ext)

    # --------------------------------------------------------- deep halo
    # The tiled sweeps (kf_reg_tiled.hip) run up to `depth` sweeps per pass on
    # a dense strip; the ring of the edge tiles reads `depth` rows of each
    # neighbour -- u and v once per GN iteration, the iterate and the one
    # before it once per pass -- instead of one row per sweep.  A neighbour's
    # rows are contiguous slices of its row-major local arrays, so nothing is
    # packed: its first / last `depth` rows go straight on the wire into this
    # rank's planes.
    def deep_setup(self, depth: int):
        """Allocate the [4, depth * w] planes (u, v, z, zp) of each neighbour
        side; ``depth`` <= every strip's height (rank-uniform)."""
        geo = self.partition.dense_geometry()
        if geo is None:
            raise ValueError("deep halo: dense strips only")
        w, h = int(geo["w"]), int(geo["h"])
        if not 1 <= depth <= h:
            raise ValueError(f"deep halo depth {depth} outside [1, {h}]")
        self.deep_w, self.deep_h, self.depth = w, h, int(depth)
        up = bool(int(geo["halo"]) & 1)
        dn = bool(int(geo["halo"]) & 2)
        mk = lambda: torch.zeros((4, depth * w), dtype=torch.float32, device=self._device)  # noqa: E731
        self.deep_up = mk() if up else None
        self.deep_dn = mk() if dn else None
        self.deep_exchanges = 0
        return self

    def deep_halo(self):
        """``(hu, hd, up, dn)`` for :func:`ops.kernels.reg_sweeps_tiled`."""
        return (self.depth if self.deep_up is not None else 0, self.depth if self.deep_dn is not None else 0,
                self.deep_up, self.deep_dn)

    def _edge_rows(self, t: torch.Tensor):
        """My first / last ``depth`` rows of a local row-major field (views)."""
        d, w, h = self.depth, self.deep_w, self.deep_h
        return t[:d * w], t[(h - d) * w:h * w]

    def deep_start(self, fields: dict):
        """Post the exchange of ``{plane: local field [>= N]}`` (plane 0 u, 1 v,
        2 z, 3 zp): my first rows go to rank - 1's lower planes, my last rows to
        rank + 1's upper planes, theirs come into mine.  Returns a handle for
        :meth:`deep_finish` (None on one rank)."""
        if not self.comm.distributed:
            return None
        keys = sorted(fields)
        su, sd, ru, rd = [], [], [], []
        for kp in keys:
            first, last = self._edge_rows(fields[kp].reshape(-1))
            su.append(first if self.deep_up is not None else None)
            sd.append(last if self.deep_dn is not None else None)
            ru.append(self.deep_up[kp] if self.deep_up is not None else None)
            rd.append(self.deep_dn[kp] if self.deep_dn is not None else None)
        pending = self.comm.exchange_fields_async(su, sd, ru, rd)
        self.bytes_sent += 4 * sum(t.numel() for t in su + sd if t is not None)
        self.exchanges += 1
        self.deep_exchanges += 1
        return pending

    def deep_finish(self, handle):
        """The compute stream waits for the posted deep exchange (no host block on RCCL)."""
        if handle is not None:
            handle.wait()
