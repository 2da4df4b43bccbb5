"""Gauss-Newton iteration strategies of ``LinearKalman`` (reference:
``kafka/linear_kf.py:245-307``, the ``while not_converged`` loop of
``do_all_bands``).

``do_all_bands_state`` sets one date's problem up (:class:`_GNRun`) and hands
it to a strategy:

* :meth:`GaussNewtonMixin._gn_global` -- the reference's exit test
  ||x_a - x_prev||_2 / len(x_a) < tol over the engine's whole state (every
  rank's pixels, C1 all-gather), iterations that cannot end the loop queued
  without a host wait, GN 1 + 2 fused into one launch, static convergence of
  linear operators;
* :meth:`GaussNewtonMixin._gn_chunked` -- the same test per get_chunks tile
  (EngineConfig.convergence_chunk, engine/chunks.py), the reference drivers'
  one-LinearKalman-per-chunk semantics (kafka_test_Py36.py:147-187).

Each iteration's device work goes through :meth:`_launch_iteration` (gain
form, spatial prior, band-parallel, split GP path or the plain fused
analysis) or :meth:`_launch_fused2` (GN 1 + 2 in one launch).
"""
from __future__ import annotations

import logging
from dataclasses import dataclass

import numpy as np
import torch

from ..ops import kernels as K
from .bands import build_table

LOG = logging.getLogger(__name__.rsplit(".", 1)[0] + ".linear_kf.linear_kf")


@dataclass
class _GNRun:
    """One date's Gauss-Newton problem as set up by do_all_bands_state: the
    operators, the forecast (fused ``prop`` or materialised ``fc``), the
    state / precision / status buffers and the launch options the iteration
    strategies (_gn_global, _gn_chunked) and the per-mode launches share."""
    timestep: object
    specs: list
    dbs: list
    table: object
    precomp: bool
    gain: bool
    bp: bool
    split: object
    prop: object
    fc: object
    x_prev: object
    x_new: object
    P_out: object
    status: object
    order: object
    out_t: object
    h0_outs: object
    a_rows: int
    pdiag_rows: int
    len_x: float
    n_bands: int
    fuse2: bool
    fuse_sp: bool
    first_plain: bool
    static_conv: bool


class GaussNewtonMixin:
    """The Gauss-Newton loop strategies and their launches (mixed into LinearKalman)."""

    def _norms_needed_now(self) -> bool:
        """Per-date metrics report the norms as they happen.  Rank-uniform on
        purpose (the metrics path is part of the shared config): the answer
        decides whether this rank queues another collective, so a per-process
        setting such as the log level (INFO often on rank 0 only) must not
        enter it -- INFO lines of statically converged dates are logged when
        the deferred norms resolve."""
        return bool(self.metrics.enabled)

    def resolve_pending(self):
        """Every deferred read-back of the dates run so far: the norms of
        statically converged dates and the per-chunk iteration histograms."""
        self._resolve_lazy_norms()
        if self._chunks is not None:
            self._chunks.resolve()

    def _resolve_lazy_norms(self):
        """Fill in the deferred norms of statically converged dates (linear
        operators): iteration 1's norm, and a check that iteration 2's is 0."""
        while self._lazy_norms:
            norms, p1, p2, len_x, nb = self._lazy_norms.pop(0)
            norms[0] = self._log_norm(p1.result(), len_x, nb, 1)
            n2 = p2.result()
            if n2 != 0.0:
                LOG.warning("linear operator: second Gauss-Newton norm %g is not 0", n2)
                norms[1] = self._log_norm(n2, len_x, nb, 2)

    @staticmethod
    def _log_norm(total: float, len_x: float, n_bands: int, n_iter: int) -> float:
        """convergence_norm = ||x_a - x_prev||_2 / len(x_a) (linear_kf.py:293-296)."""
        convergence_norm = float(np.sqrt(max(total, 0.0)) / len_x)
        LOG.info("Band {:d}, Iteration # {:d}, convergence norm: {:g}".format(n_bands - 1, n_iter,
                                                                             convergence_norm))
        return convergence_norm

    def _gn_global(self, run: "_GNRun"):
        """Gauss-Newton loop with the reference's exit test over this engine's
        whole state (linear_kf.py:293-304: ||x_a - x_prev|| / len(x_a) over every
        rank's pixels, C1).  Iterations that cannot end the loop are queued
        without waiting for their norm; GN 1 + 2 run in one launch where the
        first cannot end it (fuse_gn); linear operators converge statically.
        Returns (x, iterations, norms)."""
        cfg = self.config
        N = self.N
        n_iter = 1
        norms, deferred = [], []
        x_prev, x_new = run.x_prev, run.x_new
        while True:
            # the analysis precision is only needed from the iteration that can
            # end the loop on: skip its 4*ntri B/px store before min_iterations
            A_keep = run.P_out if n_iter >= cfg.min_iterations else None
            out_now = run.out_t if n_iter >= cfg.min_iterations else None
            if run.precomp:
                pre = self._precompute_host(run.specs, run.dbs, x_prev)
                run.table = build_table(run.specs, run.dbs, self.n_params, self._cache, self.device, run.h0_outs, pre)
            if run.fuse2 or run.fuse_sp:
                # iterations 1 + 2 in one launch: outputs of iteration 2 (which can end the loop)
                red2 = self._red_hist[1:3]
                with self.timer.phase("analysis"):
                    if N:
                        self._launch_fused2(run, x_prev, x_new)
                        K.reduce_partials(self._partials1, red2[0:1])
                        K.reduce_partials(self._partials, red2[1:2])
                    else:
                        red2.zero_()
                with self.timer.phase("converge"):
                    pend2 = self.comm.sum_f64_async(red2)
                run.fuse2 = run.fuse_sp = False
                deferred.append((1, pend2.column(0)))
                pend = pend2.column(1)
                n_iter = 2
                x_prev, x_new = x_new, (x_prev if x_prev is not None else torch.empty_like(x_new))
                if run.static_conv and not self._norms_needed_now():
                    # norm 2 is exactly 0: converged.  Norm 1 is read after the
                    # next launch is queued (no host wait between the steps)
                    if self._lookahead_fn is not None:
                        self._lookahead_fn()
                        self._lookahead_fn = None
                    self._resolve_lazy_norms()
                    norms = [None, 0.0]
                    self._lazy_norms.append((norms, deferred[0][1], pend, run.len_x, run.n_bands))
                    return x_prev, n_iter, norms
            else:
                with self.timer.phase("analysis"):
                    if N:
                        self._launch_iteration(run, n_iter, x_prev, x_new, A_keep, out_now)
                red = self._red_hist[min(n_iter, self._red_hist.numel() - 1):][:1]
                with self.timer.phase("analysis"):
                    if N:
                        K.reduce_partials(self._partials, red)
                    else:
                        red.zero_()
                with self.timer.phase("converge"):
                    pend = self.comm.sum_f64_async(red)
                x_prev, x_new = x_new, (x_prev if x_prev is not None else torch.empty_like(x_new))
            if n_iter < cfg.min_iterations:
                # this iteration cannot end the loop (n_iter <= max_iterations too):
                # queue the next one without waiting for the norm
                deferred.append((n_iter, pend))
                n_iter += 1
                continue
            if self._lookahead_fn is not None:
                # host preparation of the next date runs under this iteration's kernels
                self._lookahead_fn()
                self._lookahead_fn = None
            self._resolve_lazy_norms()
            for it, pd in deferred:
                norms.append(self._log_norm(pd.result(), run.len_x, run.n_bands, it))
            deferred = []
            convergence_norm = self._log_norm(pend.result(), run.len_x, run.n_bands, n_iter)
            norms.append(convergence_norm)
            if convergence_norm < cfg.convergence_tolerance and n_iter >= cfg.min_iterations:
                return x_prev, n_iter, norms
            if n_iter > cfg.max_iterations:
                LOG.warning("Bailing out after 25 iterations!!!!!!")
                return x_prev, n_iter, norms
            n_iter += 1

    def _launch_fused2(self, run: "_GNRun", x_prev, x_new):
        """GN iterations 1 and 2 in one launch (the plain analysis, or the plain
        first iteration with the regularised prepare of the second)."""
        n, N, prop, fc = self.n_params, self.N, run.prop, run.fc
        if run.gain:
            fx, fP = (None, None) if prop is not None else (fc.x, fc.P)
            K.gain(n, run.table, x_prev, fx, fP, x_new, run.P_out, run.status, self._partials, N=N,
                   joseph=self.config.joseph, prop=prop, out=run.out_t, gn_fused=2, partials_first=self._partials1,
                   order=run.order, pdiag_rows=run.pdiag_rows, line=self._line_opt)
        elif run.fuse_sp:
            self._regularised_iteration(run.table, x_prev, fc, x_new, run.P_out, run.status, prop, run.out_t,
                                        final=True, partials_first=self._partials1, a_rows=run.a_rows)
        else:
            K.analysis(n, run.table, x_prev, None if prop is not None else fc.x, None if prop is not None else fc.P,
                       x_new, run.P_out, None, run.status, self._partials, N=N, prop=prop, out=run.out_t,
                       gn_fused=2, partials_first=self._partials1, order=run.order, a_rows=run.a_rows,
                       line=self._line_opt)

    def _launch_iteration(self, run: "_GNRun", n_iter, x_prev, x_new, A_keep, out_now):
        """One Gauss-Newton iteration's device work, by mode: the gain form
        (K1g), the spatial prior's plain first iteration or regularised solve
        (K9 + C2), band-parallel (C5), the split GP path, or the plain fused
        analysis (K1)."""
        cfg = self.config
        n, N, prop, fc, table = self.n_params, self.N, run.prop, run.fc, run.table
        fx, fP = (None, None) if prop is not None else (fc.x, fc.P)
        if run.gain:
            K.gain(n, table, x_prev, fx, fP, x_new, A_keep, run.status, self._partials, N=N, joseph=cfg.joseph,
                   prop=prop, out=out_now, order=run.order, pdiag_rows=run.pdiag_rows if A_keep is not None else 0,
                   line=self._line_opt)
        elif run.first_plain and n_iter == 1:
            # the unfused form of fuse_sp's first iteration (same kernel path)
            K.analysis(n, table, x_prev, fx, fP, x_new, None, None, run.status, self._partials, N=N, prop=prop,
                       order=run.order, line=self._line_opt)
            self._reg_log.append({"solver": "plain", "rho": 0.0, "sweeps": 0, "r2": None, "count": 0})
        elif cfg.spatial_gamma > 0:
            self._regularised_iteration(table, x_prev, fc, x_new, A_keep, run.status, prop, out_now,
                                        final=n_iter >= cfg.min_iterations, a_rows=run.a_rows)
        elif run.bp:
            self._band_parallel_iteration(table, x_prev, fc, x_new, A_keep, run.status)
        elif run.split is not None:
            self._split_iteration(run.split, x_prev, fc, x_new, A_keep, run.status)
        else:
            K.analysis(n, table, x_prev, fx, fP, x_new, A_keep, None, run.status, self._partials, N=N, prop=prop,
                       out=out_now, order=run.order, a_rows=run.a_rows, line=self._line_opt)

    def _chunk_state(self):
        from .chunks import ChunkConvergence

        cc = self._chunks
        block = tuple(int(v) for v in self.config.convergence_chunk)
        if cc is None or cc.block != block:
            cc = self._chunks = ChunkConvergence(self.partition, block, self.n_params, self.device, self.comm)
        return cc

    def _gn_chunked(self, run: "_GNRun"):
        """Gauss-Newton loop with the exit test per chunk (engine/chunks.py;
        reference: one LinearKalman per get_chunks tile, kafka_test_Py36.py:147-187,
        each testing ||x_a - x_prev|| / len(x_a) < tol, linear_kf.py:293-304).

        Every launch writes each visited pixel's |dx|^2; after each iteration
        that can end the loop the chunks are tested (one C1 all-gather of the
        per-chunk partials), and the next launch visits only the pixels of the
        chunks still iterating (the stopped chunks' x, precision, outputs and
        status stay as their last iteration wrote them).  Returns (x, the
        largest chunk's iteration count, the largest tested norm per
        iteration)."""
        cfg = self.config
        n, N = self.n_params, self.N
        table, specs, dbs, precomp, prop, fc = run.table, run.specs, run.dbs, run.precomp, run.prop, run.fc
        x_prev, x_new, P_out, status, order, out_t = run.x_prev, run.x_new, run.P_out, run.status, run.order, run.out_t
        h0_outs, a_rows, gain = run.h0_outs, run.a_rows, run.gain
        cc = self._chunk_state()
        fx, fP = (None, None) if prop is not None else (fc.x, fc.P)
        fuse = (cfg.fuse_gn and not precomp and not run.bp and cfg.min_iterations >= 2 and cfg.max_iterations >= 1
                and not (prop is None and fc is None))
        # linear operators: iteration 2 repeats iteration 1 exactly, so every
        # chunk's norm is 0 and every chunk stops at iteration 2 -- the decision
        # is known without the per-chunk norms' read-back
        static = fuse and run.static_conv and not self._norms_needed_now()
        if not static and not cc.ready:
            cc.begin()          # (normally queued at the end of the previous date, off this date's host path)
        n_iter, n_visit, vis, full = 1, N, order, True
        norms = []
        # the tail past the first decision that keeps chunks iterating: up to
        # ``gn_lookahead`` iterations queued ahead of the read-backs, each
        # launch / compaction reading its pixel count on the device (n_dev);
        # n_visit stays a host bound (the last count read: counts only shrink)
        depth = cfg.gn_lookahead if not (run.bp or precomp) else 0
        pending = []            # (iteration, its decision) not read yet
        tail, n_dev, n_end = False, None, None
        while True:
            A_keep = P_out if n_iter >= cfg.min_iterations else None
            out_now = out_t if n_iter >= cfg.min_iterations else None
            if precomp:
                pre = self._precompute_host(specs, dbs, x_prev)
                table = build_table(specs, dbs, n, self._cache, self.device, h0_outs, pre)
            kw = dict(prop=prop, order=vis, dn_out=None if static else cc.dn)
            if not full:
                kw["n_visit"] = n_visit
                if n_dev is not None:
                    kw["n_visit_dev"] = n_dev
            with self.timer.phase("analysis"):
                if N and n_visit:
                    first2 = fuse and n_iter == 1
                    if run.bp:      # C5 band groups: the all-reduced normal equations, same subset and norms
                        self._band_parallel_iteration(table, x_prev, fc, x_new, A_keep, status, order=vis,
                                                      n_visit=kw.get("n_visit"), dn_out=cc.dn)
                    elif gain:      # K1g: the same visiting, subset and per-pixel norms
                        K.gain(n, table, x_prev, fx, fP, x_new, P_out if first2 else A_keep, status, None, N=N,
                               joseph=cfg.joseph, out=out_t if first2 else out_now, gn_fused=2 if first2 else 1,
                               pdiag_rows=run.pdiag_rows if (first2 or A_keep is not None) else 0, **kw,
                               line=self._line_opt)
                    elif first2:
                        K.analysis(n, table, x_prev, fx, fP, x_new, P_out, None, status, None, N=N, out=out_t,
                                   gn_fused=2, a_rows=a_rows, **kw, line=self._line_opt)
                    else:
                        K.analysis(n, table, x_prev, fx, fP, x_new, A_keep, None, status, None, N=N, out=out_now,
                                   a_rows=a_rows, **kw, line=self._line_opt)
            if n_iter == 1:
                cc.resolve()    # the previous dates' histograms, under this launch (read-backs done long ago)
            if fuse and n_iter == 1:
                n_iter = 2
            x_prev, x_new = x_new, (x_prev if x_prev is not None else torch.empty_like(x_new))
            if static:
                self.last_chunk_iters = cc.set_static(n_iter)
                return x_prev, n_iter, [0.0]
            if n_iter < cfg.min_iterations:
                n_iter += 1
                continue
            with self.timer.phase("converge"):
                pending.append((n_iter, cc.decide(n_iter, cfg.convergence_tolerance, cfg.min_iterations,
                                                  cfg.max_iterations)))
            if self._lookahead_fn is not None:
                self._lookahead_fn()
                self._lookahead_fn = None
            read = None
            # read the oldest decision unless the tail may queue one more iteration first
            while pending and not (tail and len(pending) <= depth and n_iter <= cfg.max_iterations):
                k, pend = pending.pop(0)
                n_act, mx, px, n_new = (pend.result(j) for j in range(4))
                n_act, px = int(n_act), int(px)
                norms.append(float(mx))
                LOG.info("Iteration # %d: %d of %d chunks converged, %d still iterating, largest chunk norm %g",
                         k, int(n_new), cc.tested, n_act, mx)
                if n_act == 0:
                    n_end = k           # the later queued iterations (if any) visit nothing
                    break
                if k > cfg.max_iterations:      # chunk_decide bails every chunk out past max_iterations
                    raise RuntimeError("per-chunk loop past max_iterations with active chunks")
                read = (k, px)
                tail = depth > 0
            if n_end is not None:
                break
            # queue iteration n_iter + 1: its pixel count is exact when this
            # iteration's decision was just read, else on the device only
            exact = read is not None and read[0] == n_iter
            with self.timer.phase("converge"):
                vis = cc.compact(vis, n_visit if N else 0, read[1] if exact else None, x_prev, x_new, n_in_dev=n_dev)
            if read is not None:
                n_visit = min(n_visit, read[1])
            n_dev = None if exact else cc.px_slot(n_iter)
            full = False
            n_iter += 1
        n_iter = n_end
        def bail(hist, max_it=cfg.max_iterations):
            if max(hist or {0: 0}) > max_it:
                LOG.warning("Bailing out after 25 iterations!!!!!!")
        # per-date metrics serialise the record now; otherwise the histogram is
        # read back without draining the stream (filled in by the next date)
        self.last_chunk_iters = cc.histogram() if self._norms_needed_now() else cc.histogram_async(bail)
        if self._norms_needed_now():
            bail(self.last_chunk_iters)
        cc.begin()              # the next date's reset, queued behind this date's read-backs
        return x_prev, n_iter, norms
