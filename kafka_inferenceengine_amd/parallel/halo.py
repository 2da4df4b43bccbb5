"""Halo exchange for the GMRF spatial regulariser (K9 + C2).

The extended state is ``x_ext = [local pixels | halo row above | halo row
below]`` ([n_p, N + n_up + n_down]); ``neighbour_table`` indexes into it.
Each Jacobi sweep refreshes the local part, packs my first/last rows
(gather kernel), and swaps them with rank-1 / rank+1 by point-to-point RCCL
(one xGMI link per direction; ≈307 KB per 10980-px row of a 7-parameter
state).
"""
from __future__ import annotations

import torch

from ..ops import kernels as K
from ..utils.blocks import tri_pos


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
        self._nbr = None
        self._device = device
        self.x_ext = torch.zeros((n_params, self.N + self.n_up + self.n_down), dtype=torch.float32, device=device)
        self.recv_up = torch.zeros((n_params, self.n_up), dtype=torch.float32, device=device)
        self.recv_down = torch.zeros((n_params, self.n_down), dtype=torch.float32, device=device)
        params = range(n_params) if spatial_params is None else spatial_params
        self.reg_mask = 0
        for j in params:
            self.reg_mask |= 1 << int(j)
        self._scratch = []
        self.bytes_sent = 0

    @property
    def nbr(self) -> torch.Tensor:
        """int32 [4, N] neighbour table (built on first use: dense strips use
        the index geometry instead, StripPartition.dense_geometry)."""
        if self._nbr is None:
            self._nbr = torch.from_numpy(self.partition.neighbour_table()).to(self._device)
        return self._nbr

    @property
    def deg(self) -> torch.Tensor:
        return (self.nbr >= 0).sum(0).to(torch.float32)

    def extend(self, x: torch.Tensor) -> torch.Tensor:
        N = self.N
        self.x_ext[:, :N].copy_(x[:, :N])
        if self.comm.distributed:
            su = K.gather(x, self.send_up_idx) if self.send_up_idx.numel() else None
            sd = K.gather(x, self.send_down_idx) if self.send_down_idx.numel() else None
            self.comm.exchange_halo(su, sd, self.recv_up, self.recv_down)
            if self.n_up:
                self.x_ext[:, N:N + self.n_up].copy_(self.recv_up)
            if self.n_down:
                self.x_ext[:, N + self.n_up:].copy_(self.recv_down)
            self.bytes_sent += 4 * self.n * (self.send_up_idx.numel() + self.send_down_idx.numel())
        return self.x_ext

    # --------------------------------------------- affine form (k regularised fields)
    def z_buffers(self, k: int):
        """Two extended [k, N + n_up + n_down] buffers for the regularised fields."""
        if getattr(self, "_z", None) is None or self._z[0].shape[0] != k:
            cols = self.N + self.n_up + self.n_down
            dev = self.x_ext.device
            self._z = [torch.zeros((k, cols), dtype=torch.float32, device=dev) for _ in range(2)]
            self._z_recv = (torch.zeros((k, self.n_up), dtype=torch.float32, device=dev),
                            torch.zeros((k, self.n_down), dtype=torch.float32, device=dev))
        return self._z

    def fill_halo(self, z_ext: torch.Tensor) -> torch.Tensor:
        """C2 for an extended buffer whose local part is current: send my boundary
        rows of its k fields to rank -1 / +1 and write theirs into the halo columns
        (k floats per boundary pixel instead of n_params)."""
        if self.comm.distributed:
            N = self.N
            ru, rd = self._z_recv
            su = K.gather(z_ext, self.send_up_idx) if self.send_up_idx.numel() else None
            sd = K.gather(z_ext, self.send_down_idx) if self.send_down_idx.numel() else None
            self.comm.exchange_halo(su, sd, ru, rd)
            if self.n_up:
                z_ext[:, N:N + self.n_up].copy_(ru)
            if self.n_down:
                z_ext[:, N + self.n_up:].copy_(rd)
            self.bytes_sent += 4 * z_ext.shape[0] * (self.send_up_idx.numel() + self.send_down_idx.numel())
        return z_ext

    def reg_rows(self) -> list[int]:
        return [j for j in range(self.n) if (self.reg_mask >> j) & 1]

    def scratch(self, avoid: torch.Tensor) -> torch.Tensor:
        if not self._scratch:
            self._scratch = [torch.empty_like(avoid), torch.empty_like(avoid)]
        for s in self._scratch:
            if s.data_ptr() != avoid.data_ptr():
                return s
        return self._scratch[0]

    def add_regulariser_diagonal(self, A: torch.Tensor, gamma: float):
        for j in range(self.n):
            if (self.reg_mask >> j) & 1:
                A[tri_pos(self.n, j, j), :self.N] += gamma * self.deg
