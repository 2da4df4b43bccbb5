"""Communication layer: one process per GPU, ``torch.distributed`` over RCCL.

Collectives used by the engine (SURVEY.md §2.7 C1–C4):
  C1  deterministic global sum of the Gauss-Newton convergence partials —
      ``all_gather`` of one f64 per rank, summed in rank order on every rank
      (bit-identical decision everywhere; the reference's criterion is global
      over the chunk, ``linear_kf.py:293``);
  C2  halo exchange with the ±1 strip neighbours (``batch_isend_irecv``,
      point-to-point — one xGMI link per direction);
  C3  gather of output strips to rank 0 (optional);
  C4  broadcast of setup objects;
  C5  band-parallel (TP-like): all-reduce of the per-pixel
      packed normal equations (A, b) inside a band group.
Backend ``nccl`` is RCCL on ROCm; ``gloo`` is only the CPU test harness.

Layout with ``band_parallel = B``: world = S x B; global rank r is strip
``r // B`` and band slot ``r % B``.  The returned Comm spans the S strips that
share a band slot (C1-C4 run there; halo peers are neighbouring strips) and
``Comm.band`` spans the B ranks of one strip (C5).  Band groups are
consecutive ranks, i.e. neighbouring GPUs on the xGMI mesh.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


class _PinnedMailbox:
    """Pinned f64 slots for norm read-backs, allocated once: a per-iteration
    pinned allocation can stall the host (and the stream) for milliseconds when
    the host runs ahead of the device.  A slot is reused after its copy ran."""

    SLOTS = 256

    def __init__(self, width: int):
        self.buf = torch.zeros((self.SLOTS, max(1, width)), dtype=torch.float64, pin_memory=True)
        self.events = [None] * self.SLOTS
        self.pool = [None] * self.SLOTS      # one reusable event per slot (no hipEventCreate per read-back)
        self.i = 0

    def take(self, n: int):
        j = self.i
        self.i = (self.i + 1) % self.SLOTS
        if self.events[j] is not None:
            self.events[j].synchronize()
            self.events[j] = None
        return j, self.buf[j, :n]


_MAILBOXES = {}


class PendingSum:
    """Deferred C1 result (``Comm.sum_f64_async``); ``k`` values per rank are
    summed column by column (``column(j)``), rank by rank in fixed order."""

    def __init__(self, vals: torch.Tensor, n: int, k: int = 1):
        self.n = n
        self.k = k
        self.event = None
        if vals.is_cuda:
            # async copy into a pinned mailbox slot + an event: result() waits for
            # THIS value only, not for work queued on the stream after it (the
            # next date's launches, the spatial prior's remaining sweep passes)
            key = (vals.device.index, vals.numel())
            box = _MAILBOXES.get(key)
            if box is None:
                box = _MAILBOXES[key] = _PinnedMailbox(vals.numel())
            j, self.vals = box.take(vals.numel())
            self.vals.copy_(vals.reshape(-1).to(torch.float64), non_blocking=True)
            ev = box.pool[j]
            if ev is None:
                ev = box.pool[j] = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(vals.device))
            self.event = box.events[j] = ev
        else:
            self.vals = vals

    def result(self, j: int = 0) -> float:
        if self.event is not None:
            self.event.synchronize()
            self.event = None
        total = 0.0
        for v in self.vals.tolist()[j::self.k]:  # fixed rank order
            total += v
        return total

    def column(self, j: int) -> "_PendingColumn":
        return _PendingColumn(self, j)


class _PendingColumn:
    def __init__(self, parent: PendingSum, j: int):
        self.parent, self.j = parent, j

    def result(self) -> float:
        return self.parent.result(self.j)


class PendingP2P:
    """Posted C2 transfers (``Comm.exchange_halo_async``)."""

    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()
        self.works = []


class Comm:
    def __init__(self, rank: int = 0, world: int = 1, device=None, group=None, ranks=None, band=None,
                 forced: bool = False):
        self.rank = rank
        self.world = world
        self.forced = forced   # KAFKA_FORCE_DIST: the collective code paths at world 1
        self.group = group
        self.ranks = list(ranks) if ranks is not None else list(range(world))   # global rank of each member
        self.band = band                                                       # band-parallel sub-comm (C5)
        self.device = torch.device(device) if device is not None else torch.device("cpu")

    # ------------------------------------------------------------ setup
    @classmethod
    def single(cls, device=None) -> "Comm":
        return cls(0, 1, device)

    @classmethod
    def from_env(cls, device=None, backend: str | None = None, timeout_s: float = 600.0,
                 band_parallel: int = 1) -> "Comm":
        """Initialise from torchrun env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*).
        ``band_parallel`` > 1 splits the world into strips x band groups."""
        world = int(os.environ.get("WORLD_SIZE", "1"))
        # KAFKA_FORCE_DIST=1: a one-rank job still initialises the process group
        # and runs every collective through it (RCCL on a one-GPU box: the
        # device code paths of C1/C3/C4 and the barrier, which several-rank
        # runs need and gloo rehearsals do not take)
        forced = os.environ.get("KAFKA_FORCE_DIST", "0") not in ("", "0")
        if world <= 1 and not dist.is_initialized() and not forced:
            return cls.single(device)
        rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if device is None:
            if torch.cuda.is_available():
                torch.cuda.set_device(local)
                device = torch.device("cuda", local)
            else:
                device = torch.device("cpu")
        device = torch.device(device)
        if not dist.is_initialized():
            # RCCL ("nccl") for device tensors, gloo for host tensors; gloo with
            # device tensors (several ranks rehearsed on one GPU) is the
            # RehearsalComm subclass (parallel/rehearsal.py), never this class
            backend = backend or cls.default_backend(device)
            cls.check_backend(backend, device)
            kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
            if backend == "nccl":
                kw["device_id"] = device
            dist.init_process_group(**kw)
        rank, world = dist.get_rank(), dist.get_world_size()
        B = int(band_parallel)
        if B <= 1:
            return cls(rank, world, device, forced=forced and world == 1)
        if world % B:
            raise ValueError(f"world size {world} is not a multiple of band_parallel={B}")
        S = world // B
        # every rank creates every group in the same order (torch.distributed contract)
        band_groups = [list(range(s * B, (s + 1) * B)) for s in range(S)]
        strip_groups = [list(range(b, world, B)) for b in range(B)]
        bg = [dist.new_group(r) for r in band_groups]
        sg = [dist.new_group(r) for r in strip_groups]
        s_idx, b_idx = rank // B, rank % B
        band = cls(b_idx, B, device, bg[s_idx], band_groups[s_idx])
        return cls(s_idx, S, device, sg[b_idx], strip_groups[b_idx], band=band)

    @staticmethod
    def default_backend(device) -> str:
        return "nccl" if torch.device(device).type == "cuda" else "gloo"

    @staticmethod
    def check_backend(backend: str, device):
        """Production: device tensors go over RCCL only."""
        if torch.device(device).type == "cuda" and backend != "nccl":
            raise ValueError(f"backend {backend!r} for device tensors: the production communicator runs RCCL; "
                             "multi-rank rehearsals on one GPU use parallel.rehearsal.RehearsalComm")

    @property
    def distributed(self) -> bool:
        return self.world > 1 or self.forced

    # ----------------------------------------------------- collectives
    def sum_f64(self, local: torch.Tensor) -> float:
        """C1: deterministic global sum of a 1-element f64 tensor."""
        if not self.distributed:
            return float(local.item())
        local = local.reshape(1).to(torch.float64)
        out = [torch.zeros_like(local) for _ in range(self.world)]
        dist.all_gather(out, local, group=self.group)
        vals = torch.cat(out).cpu().tolist()
        total = 0.0
        for v in vals:  # fixed rank order
            total += v
        return total

    def sum_f64_async(self, local: torch.Tensor) -> "PendingSum":
        """C1 without a host wait: the all-gather is queued on the stream (RCCL)
        and ``.result(j)`` reads the rank values of element j and sums them in
        rank order (``local`` holds k >= 1 values: one all-gather for all of
        them).  The values are copied to pinned host memory in stream order
        right away, so ``local`` may be overwritten by later queued work."""
        k = local.numel()
        if not self.distributed:
            return PendingSum(local.reshape(k), 1, k)
        local = local.reshape(k).to(torch.float64)
        out = torch.empty((self.world, k), dtype=torch.float64, device=local.device)
        dist.all_gather(list(out.unbind(0)), local, group=self.group)
        return PendingSum(out.reshape(-1), self.world, k)

    def all_gather_vec(self, t: torch.Tensor) -> torch.Tensor:
        """C1 for vectors (per-chunk norm partials): every rank's ``t`` in rank
        order, [world * k]; the local tensor itself on one rank."""
        if not self.distributed:
            return t
        k = t.numel()
        out = torch.empty((self.world, k), dtype=t.dtype, device=t.device)
        dist.all_gather(list(out.unbind(0)), t.reshape(k).contiguous(), group=self.group)
        return out.reshape(-1)

    def sum_int(self, v: int) -> int:
        if not self.distributed:
            return int(v)
        t = torch.tensor([int(v)], dtype=torch.int64, device=self.device)
        dist.all_reduce(t, group=self.group)
        return int(t.item())

    def max_float(self, v: float) -> float:
        """Max over every rank of the job (strips and band groups)."""
        if self.band is not None:
            v = self.band.max_float(v)
        if not self.distributed:
            return float(v)
        t = torch.tensor([float(v)], dtype=torch.float64, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return float(t.item())

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """C5: in-place all-reduce over this communicator (sum | max)."""
        if self.distributed:
            dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX, group=self.group)
        return t

    def barrier(self):
        """Barrier over every rank of the job (strips and band groups)."""
        if self.distributed:
            if self.device.type == "cuda" and dist.get_backend(self.group) == "nccl":
                dist.barrier(group=self.group, device_ids=[self.device.index])
            else:
                dist.barrier(group=self.group)
        if self.band is not None:
            self.band.barrier()

    def broadcast_object(self, obj, src: int = 0):
        """C4: broadcast a picklable setup object from ``src`` (objects created by
        this process only — never data read from untrusted files)."""
        if not self.distributed:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=self.ranks[src], group=self.group)
        return lst[0]

    def broadcast_packed(self, header, buf, src: int = 0):
        """C4 for setup data: a small header (plain lists / strings / numbers made
        by this process) as an object, the bulk as one float64 tensor broadcast
        (RCCL on device, gloo on host).  Returns (header, numpy buffer) on every
        rank; non-root ranks pass ``None, None``."""
        if not self.distributed:
            return header, buf
        meta = self.broadcast_object((header, None if buf is None else int(buf.size)), src)
        header, n = meta
        use_dev = self.device.type == "cuda" and dist.get_backend(self.group) == "nccl"
        dev = self.device if use_dev else torch.device("cpu")
        t = (torch.from_numpy(buf.astype("float64")).to(dev) if self.rank == src
             else torch.empty(n, dtype=torch.float64, device=dev))
        dist.broadcast(t, src=self.ranks[src], group=self.group)
        return header, t.cpu().numpy()

    def exchange_halo(self, send_up: torch.Tensor | None, send_down: torch.Tensor | None,
                      recv_up: torch.Tensor | None, recv_down: torch.Tensor | None):
        """C2 (blocking): send my first rows to rank-1 / last rows to rank+1 and
        receive their boundary rows.  Empty tensors are skipped consistently on
        both sides."""
        self.exchange_halo_async(send_up, send_down, recv_up, recv_down).wait()

    def exchange_halo_async(self, send_up: torch.Tensor | None, send_down: torch.Tensor | None,
                            recv_up: torch.Tensor | None, recv_down: torch.Tensor | None) -> "PendingP2P":
        """C2 posted without waiting.  On RCCL the transfers run on the process
        group's own stream, ordered after the work already queued on the current
        stream (the pack kernels); ``wait()`` makes the current stream wait for
        them (no host block), so kernels queued in between overlap the
        transfer."""
        return self.exchange_fields_async([send_up], [send_down], [recv_up], [recv_down])

    def exchange_fields_async(self, send_up, send_down, recv_up, recv_down) -> "PendingP2P":
        """C2 with several fields per direction in one batch (the deep halo of
        the tiled sweeps: u, v, z, zp rows).  Field i sent up is received by
        rank - 1 as its field i from below (same order on both sides); None or
        empty entries are skipped consistently on both sides."""
        if not self.distributed:
            return PendingP2P([])
        ops = []
        if self.rank > 0:
            peer = self.ranks[self.rank - 1]
            for s, r in zip(send_up, recv_up):
                if s is not None and s.numel():
                    ops.append(dist.P2POp(dist.isend, s.contiguous(), peer, group=self.group))
                if r is not None and r.numel():
                    ops.append(dist.P2POp(dist.irecv, r, peer, group=self.group))
        if self.rank < self.world - 1:
            peer = self.ranks[self.rank + 1]
            for s, r in zip(send_down, recv_down):
                if s is not None and s.numel():
                    ops.append(dist.P2POp(dist.isend, s.contiguous(), peer, group=self.group))
                if r is not None and r.numel():
                    ops.append(dist.P2POp(dist.irecv, r, peer, group=self.group))
        return PendingP2P(dist.batch_isend_irecv(ops) if ops else [])

    def gather_object(self, obj):
        """Gather a small picklable object (metrics) from every rank onto rank 0
        (list in rank order there, None elsewhere).  Objects are this process's own."""
        if not self.distributed:
            return [obj]
        out = [None] * self.world if self.rank == 0 else None
        dist.gather_object(obj, out, dst=self.ranks[0], group=self.group)
        return out if self.rank == 0 else None

    def gather_to_root(self, t: torch.Tensor, sizes: list[int]):
        """C3: gather variable-length pixel blocks [rows, n_i] onto rank 0."""
        if not self.distributed:
            return t
        rows = t.shape[0]
        maxn = max(sizes)
        pad = torch.zeros((rows, maxn), dtype=t.dtype, device=t.device)
        pad[:, :t.shape[1]] = t
        out = [torch.zeros_like(pad) for _ in range(self.world)] if self.rank == 0 else None
        dist.gather(pad, out, dst=self.ranks[0], group=self.group)
        if self.rank != 0:
            return None
        return torch.cat([o[:, :n] for o, n in zip(out, sizes)], dim=1)

    def destroy(self):
        if (self.distributed or self.band is not None) and dist.is_initialized():
            dist.destroy_process_group()
