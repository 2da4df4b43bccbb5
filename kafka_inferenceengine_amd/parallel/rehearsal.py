"""Multi-rank rehearsal on one GPU: gloo for device tensors.

The production communicator (``parallel/comm.py:Comm``) runs RCCL for device
tensors and refuses anything else (no second backend in
production).  Several ranks sharing the one GPU of a test box cannot run RCCL
(one communicator rank per device), so the rehearsals of the multi-GPU paths
(``bench.py --rehearse-gloo``, ``scripts/gpu_rehearse_dist.sh``) inject this
subclass: gloo over the same collectives, with the two transfers gloo cannot
order against the device stream staged through host memory.  It is a harness,
selected explicitly by the caller -- no environment variable switches the
production class.
"""
from __future__ import annotations

import torch

from .comm import Comm, PendingP2P


class RehearsalComm(Comm):
    @staticmethod
    def default_backend(device) -> str:
        return "gloo"

    @staticmethod
    def check_backend(backend: str, device):
        if backend != "gloo":
            raise ValueError("RehearsalComm runs gloo")

    def exchange_fields_async(self, send_up, send_down, recv_up, recv_down) -> PendingP2P:
        """C2 through host memory: gloo P2P has no device-stream ordering, so the
        sends must see the finished pack kernels and the device the received
        rows in stream order (no overlap -- a rehearsal of the logic)."""
        every = [t for ts in (send_up, send_down, recv_up, recv_down) for t in ts if t is not None and t.numel()]
        if not (self.distributed and every and every[0].is_cuda):
            return super().exchange_fields_async(send_up, send_down, recv_up, recv_down)
        h_up = [None if t is None else t.cpu() for t in send_up]
        h_dn = [None if t is None else t.cpu() for t in send_down]
        r_up = [None if t is None else torch.empty(t.shape, dtype=t.dtype) for t in recv_up]
        r_dn = [None if t is None else torch.empty(t.shape, dtype=t.dtype) for t in recv_down]
        super().exchange_fields_async(h_up, h_dn, r_up, r_dn).wait()
        for dst, src in zip(list(recv_up) + list(recv_down), r_up + r_dn):
            if dst is not None and dst.numel():
                dst.copy_(src)
        return PendingP2P([])

    def gather_to_root(self, t: torch.Tensor, sizes: list[int]):
        """C3 through host memory (gloo gathers host tensors only)."""
        if not (self.distributed and t.is_cuda):
            return super().gather_to_root(t, sizes)
        out = super().gather_to_root(t.cpu(), sizes)
        return None if out is None else out.to(t.device)
