"""GMRF spatial prior of ``LinearKalman`` (K9 + C2; new capability, no
reference equivalent -- the reference has no spatial coupling).

Per Gauss-Newton iteration the analysis kernel prepares the affine
block-Jacobi form (A_reg = A + g deg E_R, u = A_reg^-1 b, V = A_reg^-1 E_R),
a Chebyshev-accelerated Jacobi solve couples the regularised fields (one
launch per sweep on masked strips, LDS-tiled passes of up to 8 sweeps with a
device schedule on dense strips; halo rows exchanged by C2 under the interior
rows) and ``reg_finish`` forms x with the convergence partials.
"""
from __future__ import annotations

import logging
import math

import torch

from ..ops import kernels as K

LOG = logging.getLogger(__name__.rsplit(".", 1)[0] + ".linear_kf.linear_kf")


class SpatialPriorMixin:
    """The coupled solve of the spatial prior (mixed into LinearKalman)."""

    def _spatial_record(self) -> list:
        """Per GN iteration of the date: solver, Jacobi bound rho, sweeps and --
        with metrics on (one read-back + C1 sum) -- the RMS residual of the
        coupled GMRF system after the sweeps."""
        out = []
        for r in self._reg_log:
            e = {"solver": r["solver"], "rho": round(r["rho"], 6), "sweeps": r["sweeps"]}
            if self.metrics.enabled and r["r2"] is not None:
                tot = self.comm.sum_f64(r["r2"].reshape(1))
                e["residual_rms"] = math.sqrt(max(tot, 0.0) / max(1, r["count"]))
            out.append(e)
        self._reg_log = []
        return out

    def _regularised_iteration(self, table, x_prev, fc: KFState | None, x_out, A_out, status, prop=None, out=None,
                               final=True, partials_first=None, a_rows=0):
        """GMRF spatial prior (K9 + C2), affine block-Jacobi form (kf_core.h):
        the analysis kernel assembles (A, b) and, instead of solving, factors
        A_reg = A + g deg E_R once and writes u = A_reg^-1 b and V = A_reg^-1 E_R;
        each sweep then iterates only the k regularised fields z <- u_R + g V_RR
        s(z) (s: neighbour sums, halo rows exchanged by C2), and the last one forms
        x = u + g V s(z) with the convergence partials.  Identical to ``sweeps``
        block-Jacobi sweeps of (A_reg) x = b + g E_R sum_q x_q.  The analysis
        precision includes the smoother's diagonal.  With ``prop`` the forecast
        is fused as in the plain path (first iteration: x0 = forecast, written
        for the norm and the first sweep).  ``a_rows``: the precision rows
        stored (0: all; EngineConfig.store_precision).  ``partials_first``: the launch runs
        the plain first Gauss-Newton iteration in registers (its norm there)
        and prepares the regularised second, linearised at x_1 (written to the
        x0 buffer, the finish's reference for the norm)."""
        from ..parallel.halo import HaloExchanger

        if self._reg is None:
            self._reg = HaloExchanger(self.partition, self.comm, self.n_params, self.device,
                                      self.config.spatial_params)
            self._reg_geo = self.partition.dense_geometry()
        reg, geo = self._reg, self._reg_geo
        n, N = self.n_params, self.N
        gamma = self.config.spatial_gamma
        sweeps = max(1, int(self.config.jacobi_sweeps))
        rows = reg.reg_rows()
        fx, fP = (fc.x, fc.P) if fc is not None else (None, None)
        fused = partials_first is not None
        if not rows:   # nothing regularised: plain analysis
            K.analysis(n, table, x_prev, fx, fP, x_out, A_out, None, status, self._partials, N=N, prop=prop, out=out,
                       gn_fused=2 if fused else 1, partials_first=partials_first, order=self._visit, a_rows=a_rows,
                       line=self._line_opt)
            return
        k = len(rows)
        ld = x_out.shape[1]
        if self._reg_uv is None or self._reg_uv[0].shape[1] != ld or self._reg_uv[1].shape[0] != k * n:
            self._reg_uv = tuple(torch.empty((r, ld), dtype=torch.float32, device=self.device)
                                 for r in (n, k * n, n))
        u, v, x0_buf = self._reg_uv
        x_ref = x_prev if (x_prev is not None and not fused) else x0_buf
        # the final iteration's uncertainty raster comes from the prepare (diag of
        # the regularised precision in registers), the mean from reg_finish
        K.analysis(n, table, x_prev, fx, fP, u, A_out, None, status, None, N=N, prop=prop,
                   reg=dict(gamma=gamma, mask=reg.reg_mask, v_out=v, nbr=None if geo else reg.nbr, geo=geo),
                   x0_out=None if x_ref is x_prev else x0_buf,
                   out=None if out is None else (None, out[1], out[2]),
                   gn_fused=2 if fused else 1, partials_first=partials_first, order=self._visit, a_rows=a_rows,
                   line=self._line_opt)
        if fused:
            self._reg_log.append({"solver": "plain", "rho": 0.0, "sweeps": 0, "r2": None, "count": 0})
        nbr = None if geo else reg.nbr
        tol = self.config.spatial_tol if final else self.config.spatial_tol_first
        depth = self._reg_tiled_depth(k)
        if depth:
            cur, rho, sweeps = self._reg_tiled_solve(reg, geo, u, v, x_ref, rows[0], gamma, tol, depth, sweeps)
        else:
            cur, rho, sweeps = self._reg_sweep_solve(reg, geo, nbr, u, v, x_ref, rows, gamma, tol, sweeps)
        # mean raster: written by the finish, or (DeviceOutput alias, out[0] None) x_out itself
        K.reg_finish(n, u, v, cur, nbr, x_ref, x_out, gamma, reg.reg_mask, N, partials=self._partials, geo=geo,
                     out=None if (out is None or out[0] is None) else (out[0], None, out[2]))
        # residual of the coupled solve (metrics only): the finish applied one more
        # Jacobi update to the last iterate, x_R - z = J z + f - z (device, read lazily)
        r2 = None
        if self.metrics.enabled:
            r2 = sum(((x_out[r, :N] - cur[i, :N]).double().pow(2).sum() for i, r in enumerate(rows)),
                     torch.zeros((), dtype=torch.float64, device=self.device))
        self._reg_log.append({"solver": self.config.spatial_solver, "rho": rho, "sweeps": sweeps, "r2": r2,
                              "count": k * self.n_total})

    def _reg_tiled_depth(self, k: int) -> int:
        """Sweeps per temporal-blocking pass of the coupled solve, 0 for the
        per-sweep path.  Rank-uniform (every rank sees the whole state mask and
        the strip bounds): one regularised field on a fully active raster, a
        pass as deep as the shallowest strip (its deep halo comes from one
        neighbour) and at most REG_TILE_MAX_SWEEPS."""
        if not self.config.spatial_tiled or k != 1:
            return 0
        dense = getattr(self, "_mask_dense", None)
        if dense is None:
            dense = self._mask_dense = bool(self.state_mask.size) and bool(self.state_mask.all())
        if not dense:
            return 0
        h_min = min(b - a for a, b in self.partition.bounds)
        return int(min(K.REG_TILE_MAX_SWEEPS, h_min))

    def _reg_rho_async(self, reg, v, rows, k, gamma):
        """Chebyshev bound rho = max over pixels of g deg ||V_RR||_inf, a
        Gershgorin bound of the Jacobi matrix's spectral radius (its spectrum is
        real: J is similar to a symmetric matrix), max-reduced over the ranks
        on the stream; returns a pending read-back (PendingSum, element 0)."""
        from ..parallel.comm import PendingSum

        n, N = self.n_params, self.N
        if N and k == 1:
            # V row (c * n + r_j): component r_j of column c (kf_core.h JacobiArgs); one
            # field: V_RR >= 0 is the row itself (a view), one fused multiply + max
            rho_t = (torch.amax(v[rows[0], :N] * reg.degrees) * gamma).reshape(1).double()
        elif N:
            blk = torch.stack([v[[c * n + r for c in range(k)], :N].abs().sum(0) for r in rows])   # [k, N]
            rho_t = (gamma * blk.amax(0) * reg.degrees).amax().reshape(1).double()
        else:
            rho_t = torch.zeros(1, dtype=torch.float64, device=self.device)
        return PendingSum(self.comm.all_reduce_(rho_t, op="max"), 1, 1)

    def _reg_sweeps_for(self, rho: float, tol: float):
        """(rho, sweeps) of the coupled solve: the sweeps (the finish included)
        cut the error by ``tol`` at the Chebyshev rate sigma = rho / (1 + sqrt(1
        - rho^2)); the same expressions as the device schedule
        (kf_core.h:reg_cheb_schedule).  ``tol``: spatial_tol for an iteration
        that can end the GN loop, spatial_tol_first before."""
        cfg = self.config
        if not rho < 1.0:
            LOG.warning("spatial prior: Jacobi bound rho=%.4f >= 1, plain Jacobi sweeps", rho)
            return 0.0, max(1, int(cfg.spatial_max_sweeps))
        if rho <= 0.0:
            return 0.0, 1
        sigma = rho / (1.0 + math.sqrt(max(0.0, 1.0 - rho * rho)))
        need = math.ceil(math.log(2.0 / tol) / math.log(1.0 / sigma))
        return rho, int(min(max(1, need), int(cfg.spatial_max_sweeps)))

    @staticmethod
    def _cheb_weights(rho: float, n_sweeps: int):
        """Chebyshev semi-iterative weights of the sweeps before the finish:
        (omega, Chebyshev step?) -- the first step is plain Jacobi."""
        sched, omega = [], 1.0
        for it in range(n_sweeps):
            if rho > 0 and it > 0:
                omega = 1.0 / (1.0 - 0.5 * rho * rho) if it == 1 else 1.0 / (1.0 - 0.25 * rho * rho * omega)
            sched.append((omega, rho > 0 and it > 0))
        return sched

    def _reg_sweep_solve(self, reg, geo, nbr, u, v, x_ref, rows, gamma, tol, sweeps):
        """Coupled solve, one launch per sweep (masked strips, several fields).
        The first sweep is plain Jacobi whatever rho is, so it is queued before
        rho is read back: the host waits while the GPU runs it.  (With rho <= 0
        the schedule has no sweep before the finish; V_RR deg = 0 everywhere
        then, so that extra sweep leaves z = u and the finish unchanged.)  C2
        overlap on distributed strips: each sweep's boundary rows, their
        exchange posted, the interior rows under it."""
        cfg = self.config
        n, N = self.n_params, self.N
        k = len(rows)
        cheb = cfg.spatial_solver == "chebyshev"
        pend = self._reg_rho_async(reg, v, rows, k, gamma) if cheb else None
        rho = 0.0
        z = reg.z_buffers(k)
        for i, r in enumerate(rows):
            z[0][i, :N].copy_(x_ref[r, :N])
        cur = reg.fill_halo(z[0])
        prev = None
        overlap = self.comm.distributed and reg.split is not None
        sa, sb = reg.split if overlap else (0, 0)
        sched = [(1.0, False)] if cheb else self._cheb_weights(0.0, sweeps - 1)
        it = 0
        while it < len(sched):
            omega, use_prev = sched[it]
            nxt = next(b for b in z if b is not cur and b is not prev)
            zp = prev if use_prev else None
            if overlap:
                with self.timer.phase("reg_boundary"):
                    K.reg_sweep(n, u, v, cur, nbr, nxt, gamma, reg.reg_mask, N, geo=geo, rows=(0, sa), z_prev=zp,
                                omega=omega)
                    K.reg_sweep(n, u, v, cur, nbr, nxt, gamma, reg.reg_mask, N, geo=geo, rows=(N - sb, sb),
                                z_prev=zp, omega=omega)
                with self.timer.phase("halo"):
                    hp = reg.start_fill(nxt)
                with self.timer.phase("reg_interior"):
                    K.reg_sweep(n, u, v, cur, nbr, nxt, gamma, reg.reg_mask, N, geo=geo, rows=(sa, N - sa - sb),
                                z_prev=zp, omega=omega)
                with self.timer.phase("halo"):
                    nxt = reg.finish_fill(hp, nxt)
                self.reg_overlapped_sweeps += 1
            else:
                K.reg_sweep(n, u, v, cur, nbr, nxt, gamma, reg.reg_mask, N, geo=geo, z_prev=zp, omega=omega)
                nxt = reg.fill_halo(nxt)
            prev, cur = cur, nxt
            it += 1
            if pend is not None:
                # the first sweep is queued: read rho while the GPU runs it
                rho, sweeps = self._reg_sweeps_for(pend.result(0), tol)
                pend = None
                sched = self._cheb_weights(rho, max(sweeps - 1, 1))
        return cur, rho, sweeps

    def _reg_tiled_solve(self, reg, geo, u, v, x_ref, j0, gamma, tol, depth, sweeps):
        """Coupled solve of one regularised field on dense strips, `depth`
        sweeps per pass out of LDS (kf_reg_tiled.hip).

        * The schedule lives on the device: rho (one max pass over V_RR deg),
          its all-rank max, then the sweep count and Chebyshev weights
          (RegSchedule).  The first pass is queued at once and reads them; the
          host reads the sweep count back while the GPU runs that pass, then
          queues the rest (no host wait between the prepare and the sweeps).
        * Tile-DP (C2): once per GN iteration the neighbours' u, v and initial
          iterate rows, then once per pass the last two iterates -- `depth`
          rows each -- instead of one row per sweep.  A pass runs its boundary
          tile rows, posts their exchange and runs the interior under it.  The
          finish reads the neighbours' adjacent row of the final iterate from
          the last pass's exchange (no extra exchange).
        Bit-identical to one launch per sweep, at any rank count."""
        from ..parallel.comm import PendingSum

        cfg = self.config
        n, N = self.n_params, self.N
        dist_ = self.comm.distributed
        z = reg.z_buffers(1)
        if self._reg_z4 is None or self._reg_z4.shape != z[0].shape:
            self._reg_z4 = torch.zeros_like(z[0])
        bufs = [z[0], z[1], z[2], self._reg_z4]
        cur, prev = bufs[0], bufs[1]
        cur[0, :N].copy_(x_ref[j0, :N])
        cheb = cfg.spatial_solver == "chebyshev"
        pend, rs, rho = None, None, 0.0
        if cheb:
            rs = getattr(self, "_reg_sched", None)
            if rs is None or rs.max_sweeps != int(cfg.spatial_max_sweeps):
                rs = self._reg_sched = K.RegSchedule(N, cfg.spatial_max_sweeps, self.device)
            with self.timer.phase("reg_schedule"):
                rs.rho_pass(v[j0], geo, N, gamma)
                self.comm.all_reduce_(rs.rho, op="max")
                rs.schedule(tol)
                pend = PendingSum(rs.info, 1, 2)
            n_sched = None
        else:
            n_sched = max(1, int(sweeps)) - 1
            if n_sched == 0:
                return reg.fill_halo(cur), 0.0, 1
        halo, rows_b = None, None
        if dist_:
            if getattr(reg, "depth", None) != depth:
                reg.deep_setup(depth)
            with self.timer.phase("halo"):
                reg.deep_finish(reg.deep_start({0: u[j0], 1: v[j0], 2: cur[0]}))
            halo = reg.deep_halo()
            T = K.reg_tile_rows(geo["h"])
            ta, tb = K.reg_boundary_tile_rows(geo["h"], depth, halo[0] > 0, halo[1] > 0)
            rows_b = ((0, ta), (tb, T), (ta, tb))
        s_base = 0
        while True:
            o_cur, o_prev = [b for b in bufs if b is not cur and b is not prev]
            if cheb:
                kw = dict(sched=(rs.sched, rs.omega), s_base=s_base, nsweep=depth)
            else:
                ns = min(depth, n_sched - s_base)
                part = self._cheb_weights(0.0, n_sched)[s_base:s_base + ns]
                kw = dict(omegas=[o for o, _ in part], chebyshev=[c for _, c in part])

            def launch(tr):
                K.reg_sweeps_tiled(n, u, v, cur, prev, o_cur, o_prev, gamma, reg.reg_mask, N, geo, halo=halo,
                                   tile_rows=tr, **kw)
            if dist_:
                with self.timer.phase("reg_boundary"):
                    launch(rows_b[0])
                    launch(rows_b[1])
                with self.timer.phase("halo"):
                    hp = reg.deep_start({2: o_cur[0], 3: o_prev[0]})
                with self.timer.phase("reg_interior"):
                    launch(rows_b[2])
                with self.timer.phase("halo"):
                    reg.deep_finish(hp)
                self.reg_overlapped_sweeps += 1
            else:
                launch(None)
            self.reg_tiled_launches += 1
            cur, prev = o_cur, o_prev
            s_base += depth
            if n_sched is None:
                # the first pass is queued: read the schedule while the GPU runs it
                rho = pend.result(0)
                sweeps = int(pend.result(1))
                n_sched = sweeps - 1
                if not rho < 1.0:
                    LOG.warning("spatial prior: Jacobi bound rho=%.4f >= 1, plain Jacobi sweeps", rho)
            if s_base >= n_sched:
                break
        if dist_:
            # the finish's one-row halo: the neighbours' adjacent rows of the final iterate
            w = int(geo["w"])
            if halo[2] is not None:
                cur[0, N:N + w].copy_(halo[2][2, (depth - 1) * w:depth * w])
            if halo[3] is not None:
                off = N + reg.n_up
                cur[0, off:off + w].copy_(halo[3][2, :w])
        return cur, rho, sweeps
