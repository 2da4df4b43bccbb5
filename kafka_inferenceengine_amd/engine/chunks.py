"""Per-chunk Gauss-Newton convergence: the reference's driver semantics on one filter.

The reference never runs a whole tile as one filter.  Its drivers cut the
raster with ``get_chunks`` (256² in ``kafka_test_Py36.py:241``, 128² in
``kafka_test_S2.py:202``) and give every chunk its own ``LinearKalman``
(``kafka_test_Py36.py:147-187``), so the Gauss-Newton exit test
``||x_a - x_prev||_2 / len(x_a) < tol`` (``linear_kf.py:293-304``) is taken over
ONE chunk: each chunk runs its own number of iterations.  Over a whole tile
the same test is vacuous (the norm scales like rms(dx) / sqrt(n_p N)).

``ChunkConvergence`` keeps the engine's one device state per rank and applies
the test per chunk (``EngineConfig.convergence_chunk``):

* the analysis writes each pixel's |x - x0|^2 (``AnalysisArgs.dn_out``);
* ``chunk_partials`` sums them per chunk over this rank's pixels as integer
  quanta of the chunk's squared norm (:meth:`ChunkConvergence.quantum`): the
  sums are exact, so they do not depend on the order of the adds, on the
  device, or on where strip boundaries cut a chunk;
* the per-chunk partials of every rank are all-gathered (C1: one int64 per
  chunk, ~15 KB for a 10980² granule in 256² chunks) and added by
  ``chunk_decide`` -- the same decision on every rank and for any rank count
  -- which marks the chunks that stop now;
* ``chunk_compact`` removes the stopped chunks' pixels from the visiting
  order (stable, so the observed-first order of ``obs_order`` survives) and
  copies their final x into the next launch's output buffer: later launches
  visit only the chunks still iterating, and the loop ends when none is left.

Chunk ids follow ``get_chunks`` (X-major; ``chunk_no`` - 1); chunks without
active pixels are never tested (the reference's farm skips them,
``kafka_test_Py36.py:154``).
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import kernels as K


def chunk_grid(shape, block):
    """(nxb, nyb) chunk counts of ``get_chunks(W, H, block)`` over a raster of
    ``shape`` = (H, W); ``block`` = (x size, y size) as in get_chunks."""
    H, W = shape
    bx, by = int(block[0]), int(block[1])
    if bx < 1 or by < 1:
        raise ValueError(f"convergence_chunk {block}: sizes must be >= 1")
    return -(-W // bx), -(-H // by)


def chunk_counts(state_mask, block) -> np.ndarray:
    """Active pixels per chunk, indexed by get_chunks order (chunk_no - 1)."""
    m = np.asarray(state_mask).astype(bool)
    H, W = m.shape
    bx, by = int(block[0]), int(block[1])
    nxb, nyb = chunk_grid(m.shape, block)
    pad = np.zeros((nyb * by, nxb * bx), dtype=np.int64)
    pad[:H, :W] = m
    cnt = pad.reshape(nyb, by, nxb, bx).sum(axis=(1, 3))      # [Y, X]
    return np.ascontiguousarray(cnt.T).reshape(-1)              # X-major: X * nyb + Y


class ChunkConvergence:
    """Device state of the per-chunk Gauss-Newton test for one rank's strip."""

    def __init__(self, partition, block, n_params: int, device, comm):
        self.block = (int(block[0]), int(block[1]))
        self.comm = comm
        self.device = torch.device(device)
        self.n_params = int(n_params)
        H, W = partition.shape
        bx, by = self.block
        self.nxb, self.nyb = chunk_grid((H, W), self.block)
        self.nc = self.nxb * self.nyb
        counts = chunk_counts(partition.state_mask, self.block)
        N = partition.N
        self.N = N
        idx = np.asarray(partition.local_idx, dtype=np.int64)
        r_loc = idx // W
        col = idx % W
        gid = (col // bx) * self.nyb + (r_loc + partition.r0) // by
        # runs of consecutive local pixels within one (raster row, chunk column)
        key = r_loc * self.nxb + col // bx
        starts = np.flatnonzero(np.r_[True, np.diff(key) != 0]) if N else np.zeros(0, np.int64)
        lens = np.diff(np.r_[starts, N]) if N else np.zeros(0, np.int64)
        seg_g, seg_row = gid[starts], r_loc[starts]
        o = np.lexsort((seg_row, seg_g))
        seg_start, seg_len, sg = starts[o], lens[o], seg_g[o]
        lc_gid, first = np.unique(sg, return_index=True)
        lc_ptr = np.r_[first, sg.size]
        local_count = np.bincount(gid, minlength=self.nc) if N else np.zeros(self.nc, np.int64)
        i32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(self.device)  # noqa: E731
        self.seg_start, self.seg_len = i32(seg_start), i32(seg_len)
        self.lc_ptr, self.lc_gid = i32(lc_ptr), i32(lc_gid)
        self.groups = K.chunk_groups(lc_ptr)
        self.gpart = torch.zeros(max(lc_gid.size, 1) * self.groups, dtype=torch.int64, device=self.device)
        self.chunk_of = i32(gid) if N else torch.zeros(1, dtype=torch.int32, device=self.device)
        self.local_count = i32(local_count)
        self.counts = counts
        self.len_x = torch.from_numpy(np.maximum(counts, 1) * float(self.n_params)).to(self.device)
        self.active0 = torch.from_numpy((counts > 0).astype(np.uint8)).to(self.device)
        self.active = self.active0.clone()
        self.newly = torch.zeros(self.nc, dtype=torch.uint8, device=self.device)
        self._iters = torch.zeros(self.nc, dtype=torch.int32, device=self.device)
        self._static = None   # set_static(): every tested chunk stopped at this iteration (filled lazily)
        self.part = torch.zeros(self.nc, dtype=torch.int64, device=self.device)
        self._quanta = {}
        self.info = torch.zeros(4, dtype=torch.float64, device=self.device)
        # this rank's active pixels after the decisions of odd / even iterations
        # (int32): the device counts of launches queued before the host reads them
        self.px = torch.zeros(2, dtype=torch.int32, device=self.device)
        self.dn = torch.zeros(max(N, 1), dtype=torch.float32, device=self.device)
        self.orders = [torch.empty(max(N, 1), dtype=torch.int32, device=self.device) for _ in range(2)]
        self.scratch = K.chunk_compact_scratch(max(N, 1), self.device)
        self.tested = int((counts > 0).sum())   # chunks with active pixels (all ranks)

    @property
    def iters(self) -> torch.Tensor:
        """Gauss-Newton iterations of every chunk on the last date (0: untested)."""
        if self._static is not None:
            self._iters.copy_(self.active0.to(torch.int32) * self._static)
            self._static = None
        return self._iters

    @property
    def ready(self) -> bool:
        """begin() was queued after the last date (the next date may start)."""
        return getattr(self, "_ready", False)

    def begin(self):
        """A new date: every chunk with active pixels iterates.  (The per-chunk
        iteration counts need no reset: every chunk that iterates stops on some
        iteration, bailing out past max_iterations at the latest, and chunk_decide
        records it then; chunks without pixels keep 0.)"""
        if self._static is not None:
            self.iters        # a static date's counts (read before they would be overwritten)
        self.active.copy_(self.active0)
        self._ready = True

    def set_static(self, n_iter: int) -> dict:
        """A date whose every chunk stops at ``n_iter`` by construction (linear
        operators: iteration 2 repeats iteration 1 exactly): no device work,
        the per-chunk counts are filled in only if read.  Returns the histogram."""
        self._static = int(n_iter)
        self._ready = False
        return {int(n_iter): self.tested} if self.tested else {}

    def px_slot(self, n_iter: int) -> torch.Tensor:
        """int32 [1] that iteration ``n_iter``'s decision writes this rank's
        active pixel count to (two slots alternate: a decision never overwrites
        a count a queued launch or compaction has still to read)."""
        return self.px[n_iter % 2:n_iter % 2 + 1]

    def quantum(self, tol: float):
        """(qinv [nc], clamp, unit) of the integer norm sums for exit tolerance
        ``tol``.  A chunk's squared norm ||dx||^2 / len_x^2 is counted in quanta
        of ``unit`` = tol^2 / 2^(61 - B) (B: bits of the largest chunk's pixel
        count), so the threshold tol^2 is 2^(61 - B) quanta -- 2^44 for 256²
        chunks, a resolution far below float32 |dx|^2 rounding -- and one pixel
        contributes at most ``clamp`` = twice that: no chunk total can overflow
        int64, and a clamped pixel still keeps its chunk iterating.  tol <= 0
        (stop at max_iterations only) quantises against 1e-3."""
        hit = self._quanta.get(float(tol))
        if hit is None:
            B = int(max(int(self.counts.max()) if self.counts.size else 1, 1)).bit_length()
            thr = 2 ** (61 - B)
            t = float(tol) if tol > 0 else 1e-3
            unit = t * t / thr
            lx = np.maximum(self.counts, 1) * float(self.n_params)
            qinv = torch.from_numpy(1.0 / (lx * lx * unit)).to(self.device)
            hit = self._quanta[float(tol)] = (qinv, 2 * thr, unit)
        return hit

    def decide(self, n_iter: int, tol: float, min_iter: int, max_iter: int):
        """Per-chunk norms of the last launch's dn and the exit test; returns
        a pending read-back of (active chunks, largest norm, this rank's
        active pixels, chunks stopped now), and leaves the pixel count in
        :meth:`px_slot` too.

        The decision is rank-uniform and rank-count invariant by
        construction: the partials are exact integer sums of per-pixel quanta
        (:meth:`quantum`), so 1, 4 and 8 ranks add up the same totals
        whatever the strip cuts."""
        from ..parallel.comm import PendingSum

        self._ready = False
        qinv, clamp, unit = self.quantum(tol)
        if self.N:
            K.chunk_partials(self.dn, self.seg_start, self.seg_len, self.lc_ptr, self.lc_gid, self.active, self.part,
                             self.gpart, self.groups, qinv, clamp)
        part_all = self.comm.all_gather_vec(self.part)
        K.chunk_decide(part_all, self.comm.world, self.len_x, self.local_count, tol, n_iter, min_iter, max_iter,
                       self.active, self.newly, self._iters, self.info, px_out=self.px_slot(n_iter), unit=unit)
        # (a device result goes to its own pinned mailbox slot; the host runner's
        # is copied, the next decision may run before this one is read)
        return PendingSum(self.info if self.device.type == "cuda" else self.info.clone(), 1, 4)

    def compact(self, order_in, n_in: int, n_out, x_src, x_dst, n_in_dev=None):
        """Visiting order of the next launch (the active chunks' pixels of
        order_in[:n_in]); the stopped chunks' x copied x_src -> x_dst.
        ``n_in_dev``: order_in's slot count on the device (``n_in`` then only
        bounds it); ``n_out`` (None: not read yet) checks the host runner."""
        out = self.orders[0]
        if order_in is not None and order_in.data_ptr() == out.data_ptr():
            out = self.orders[1]
        if n_in:
            got = K.chunk_compact(order_in, n_in, self.chunk_of, self.active, self.newly, self.scratch, out,
                                  x_src, x_dst, n_in_dev=n_in_dev)
            if got is not None and n_out is not None and got != n_out:
                raise RuntimeError(f"chunk_compact kept {got} pixels, chunk_decide counted {n_out}")
        return out

    def histogram(self) -> dict:
        """{Gauss-Newton iterations: chunks} of the date (every rank's chunks)."""
        return self._hist(self.iters.cpu().numpy())

    def _hist(self, it) -> dict:
        vals, cnt = np.unique(it[self.counts > 0], return_counts=True)
        return {int(v): int(c) for v, c in zip(vals, cnt)}

    def histogram_async(self, on_resolve=None) -> dict:
        """The date's histogram without a host wait: the per-chunk counts go to
        pinned memory in stream order and the returned dict is filled in place
        by :meth:`resolve` (the next date, or the run's end), so the host does
        not drain the stream between dates.  ``on_resolve(hist)`` runs then."""
        if self._static is not None or self.device.type != "cuda":
            h = self.set_static(self._static) if self._static is not None else self.histogram()
            if on_resolve is not None:
                on_resolve(h)
            return h
        if not hasattr(self, "_pinned"):
            self._pinned = [torch.empty(self.nc, dtype=torch.int32, pin_memory=True) for _ in range(2)]
            self._pin_turn = 0
            self._pending = []
        if len(self._pending) >= 2:
            self.resolve()
        buf = self._pinned[self._pin_turn % 2]
        self._pin_turn += 1
        buf.copy_(self._iters, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        out = {}
        self._pending.append((out, buf, ev, on_resolve))
        return out

    def resolve(self):
        """Fill the histograms :meth:`histogram_async` handed out."""
        for out, buf, ev, cb in getattr(self, "_pending", []):
            ev.synchronize()
            out.update(self._hist(buf.numpy()))
            if cb is not None:
                cb(out)
        self._pending = []
