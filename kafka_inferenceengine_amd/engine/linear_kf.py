"""LinearKalman — the engine driver (reference: ``kafka/linear_kf.py``).

Same constructor, ``set_trajectory_model``, ``set_trajectory_uncertainty``,
``run``, ``advance``, ``assimilate_multiple_bands``, ``do_all_bands``,
``assimilate``/``assimilate_band``, ``solver``/``solver_multiband`` as
``linear_kf.py:59-452``, but the state lives on the GPU as SoA tensors and each
Gauss-Newton iteration is ONE fused gfx950 kernel (operator + Jacobian +
normal equations + Cholesky + convergence partial) followed by a fixed-order
reduction and — under tile-DP — a deterministic all-gather of one f64 per rank.

Host loops that remain: the time grid, the observation
dates of a step, and the Gauss-Newton iteration (one 8-byte D2H per
iteration).  Objects that only speak the reference protocol (a user's
observation class, operator factory, propagator or prior) are still accepted:
the engine converts at the boundary and runs that piece on the host.
"""
from __future__ import annotations

import bisect
import logging
import time
from collections import namedtuple

import numpy as np
import scipy.sparse as sp
import torch

from ..inference.kf_tools import (PROP_IDENTITY, PROP_PRIOR, PROP_STANDARD, PropagatorSpec,
                                  propagate_and_blend_prior, propagate_information_filter_LAI)
from ..inference.solvers import variational_kalman, variational_kalman_multiband
from ..inference.utils import iterate_time_grid
from ..models.operators import OP_GP, OP_LINEAR, OP_PRECOMP, OperatorSpec
from ..ops import kernels as K
from ..parallel.comm import Comm
from ..parallel.partition import StripPartition
from ..utils.blocks import ntri, pack_matrix, soa_to_interleaved, tri_pos
from ..utils.metrics import MetricsLogger, PhaseTimer
from .bands import DeviceBand, RecordCache, TableCache, build_table
from .config import EngineConfig
from .gn import GaussNewtonMixin, _GNRun
from .spatial import SpatialPriorMixin
from .state import COVARIANCE, PRECISION, KFState, LazyForecast

LOG = logging.getLogger(__name__ + ".linear_kf")

Metadata = namedtuple("Metadata", "mask uncertainty")
Previous_State = namedtuple("Previous_State", "timestamp x_vect cov_m icov_mv")
AssimilationResult = namedtuple("AssimilationResult", "state n_iter norms innovations")



def _resolve_device(device):
    if device is not None:
        d = torch.device(device)
        if d.type == "cuda" and d.index is None:
            d = torch.device("cuda", torch.cuda.current_device())
        return d
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


def _jacobian_blocks(Hm, N: int, n: int) -> np.ndarray:
    """SoA Jacobian rows h [n, N] of a reference-protocol operator matrix
    (``utils.py:197-215``: row i holds pixel i's gradient in columns n*i ..
    n*i + n - 1), read straight from the sparse triplets -- one vectorised
    pass instead of per-parameter CSR fancy indexing (which is O(N) Python-
    level work per parameter and unusable at granule scale).  An entry outside
    its row's block would couple pixels, which the reference never does
    (SURVEY.md §0): refused."""
    if sp.issparse(Hm):
        coo = Hm.tocoo()
        r, c, v = coo.row, coo.col, coo.data
    else:
        Hd = np.asarray(Hm)
        r, c = np.nonzero(Hd)
        v = Hd[r, c]
    if Hm.shape[0] != N or Hm.shape[1] != N * n:
        raise ValueError(f"operator matrix {Hm.shape} is not [N, n*N] = [{N}, {N * n}]")
    pix, par = np.divmod(c.astype(np.int64), n)
    off = pix != r
    if off.any() and np.any(v[off] != 0):
        raise ValueError("operator matrix couples pixels (entries outside the per-pixel blocks)")
    h = np.zeros((n, N), dtype=np.float64)
    keep = ~off
    np.add.at(h, (par[keep], r[keep]), v[keep])   # duplicates (unsummed COO) add up
    return h


class LinearKalman(GaussNewtonMixin, SpatialPriorMixin):
    """Iterated (Gauss-Newton) information-form Kalman filter over rasters."""

    def __init__(self, observations, output, state_mask, create_observation_operator, parameters_list,
                 state_propagation=propagate_information_filter_LAI, band_mapper=None, linear=True,
                 diagnostics=True, prior=None, *, config: EngineConfig | None = None, device=None,
                 comm: Comm | None = None, partition: StripPartition | None = None):
        self.parameters_list = list(parameters_list)
        self.n_params = len(self.parameters_list)
        K.check_np(self.n_params)
        self.observations = observations
        self.output = output
        self.diagnostics = diagnostics
        self.linear = linear
        if isinstance(state_mask, (str, bytes)):
            from ..input_output.tiff import read_tiff
            state_mask = read_tiff(state_mask)[0]
        self.state_mask = np.asarray(state_mask).astype(bool)
        self._state_propagator = state_propagation
        self._advance = propagate_and_blend_prior
        self.prior = prior
        self.band_mapper = band_mapper
        self._create_observation_operator = create_observation_operator
        self.config = (config or EngineConfig()).validate()
        self.comm = comm or Comm.single(_resolve_device(device or self.config.device))
        self.device = _resolve_device(device or self.config.device) if comm is None else comm.device
        self.partition = partition or getattr(observations, "partition", None) or \
            StripPartition(self.state_mask, self.comm.rank, self.comm.world)
        if self.partition.world != self.comm.world or self.partition.rank != self.comm.rank:
            raise ValueError("partition does not match the communicator")
        self.N = self.partition.N
        self.n_state_elems = self.N
        self.n_total = self.partition.N_total
        self._m = np.ones(self.n_params)
        self._q = np.zeros(self.n_params)
        self._q_pix = None
        self.trajectory_model = None
        self.trajectory_uncertainty = None
        self.current_timestep = None
        self.previous_state = None
        self._cache = RecordCache()
        self._tables = TableCache()
        # per-date band lists a source hands out again for every date of a pool
        # slot (``band_specs_static`` sources): id -> [list, (spec, band) pairs, table]
        self._bands_memo = {}
        self._prop_bufs = {}            # fused-propagation argument blocks on the device, by content
        self._prop_dicts = {}           # propagation argument dicts by (propagator, prior, Q) identity
        self._partials = K.partials_buffer(max(self.N, 1), self.device)
        # one reduction slot per GN iteration: norms of iterations that cannot end
        # the loop (n_iter < min_iterations) are read after the loop, not waited on
        self._red_hist = torch.zeros(self.config.max_iterations + 3, dtype=torch.float64, device=self.device)
        self._partials1 = K.partials_buffer(max(self.N, 1), self.device)   # first fused GN iteration
        self._red = self._red_hist[:1]
        self.metrics = MetricsLogger(self.config.metrics_path, rank=self.comm.rank)
        self.timer = PhaseTimer(self.device, sync=self.config.sync_timing,
                                enabled=self.metrics.enabled or self.config.phase_timing)
        self._lookahead_fn = None       # host prep of the next date, run under the last GN iteration
        self._prepared = None           # (date, bands, table) made by it
        self._lazy_norms = []           # (norms, pending 1, pending 2, len_x, n_bands) of static convergence
        self._reg_log = []              # per GN iteration of the spatial prior: rho, sweeps, residual
        self._order_bufs = [None, None]  # (order, scratch) of obs_order: two sets, alternating dates
        self._order_turn = 0
        self._visit = None              # this date's pixel visiting order (config.observed_first)
        self._split_chunk = {}          # split path: bands per chunk, per band count
        self._reg = None
        self._reg_uv = None             # affine regulariser: u = A_reg^-1 b, V = A_reg^-1 E_R, x0
        self._reg_geo = None
        self._reg_z4 = None               # 4th regularised-field buffer of the tiled sweeps
        self.reg_tiled_launches = 0       # K9 temporal-blocking launches (kf_reg_tiled.hip)
        self.reg_overlapped_sweeps = 0    # C2 sweeps whose halo exchange ran under the interior rows
        self._output_written = None
        self._chunks = None               # per-chunk convergence state (config.convergence_chunk)
        self.last_chunk_iters = None      # {GN iterations: chunks} of the last date (chunked test)
        self.ood_history = None           # config.domain_history: ST_OUT_OF_DOMAIN on any date so far
        self._full_precision_step = False
        band = getattr(self.comm, "band", None)
        self.band_comm = band if (band is not None and band.world > 1) else None
        self._bp_buf = None
        self.history = []
        if hasattr(observations, "bind_engine"):
            # file readers learn the strip / device here and switch to the
            # device ingest path (pinned native decode -> async H2D)
            observations.bind_engine(self)
        LOG.info("Starting KaFKA run!!!")

    # ------------------------------------------------------------ model
    def set_trajectory_model(self, m=None):
        """Identity trajectory model (linear_kf.py:123-129); optional per-parameter diagonal."""
        self._m = np.ones(self.n_params) if m is None else np.broadcast_to(np.asarray(m, float), (self.n_params,))
        self.trajectory_model = "identity" if m is None else self._m.copy()

    def set_trajectory_uncertainty(self, Q):
        """Diagonal model error Q (linear_kf.py:131-146).  Accepts the reference's
        interleaved vector over all pixels, or one value per parameter."""
        Q = np.asarray(Q, dtype=np.float64).ravel()
        n = self.n_params
        if Q.size == n:
            self._q, self._q_pix = Q.copy(), None
        elif Q.size == n * self.n_total:
            rows = Q.reshape(self.n_total, n)
            if np.all(rows == rows[0]):
                self._q, self._q_pix = rows[0].copy(), None
            else:
                loc = rows[self.partition.pixel_slice].T
                self._q_pix = torch.from_numpy(np.ascontiguousarray(loc, dtype=np.float32)).to(self.device)
        else:
            raise ValueError(f"Q has {Q.size} entries; expected {n} or {n * self.n_total}")
        self.trajectory_uncertainty = Q

    # ------------------------------------------------------- overrides
    def _set_plot_view(self, diag_string, timestep, obs):
        pass

    def _plotter_iteration_start(self, plot_obj, x, obs, mask):
        pass

    def _plotter_iteration_end(self, plot_obj, x, P, innovation, mask):
        pass

    def _get_observations_timestep(self, timestep, band=None):
        """Override point (reference ``linear_kf.py:148-169``, unused by ``run``):
        ``(observations, uncertainty, mask, metadata, emulator)`` of one band."""
        data = self.observations.get_band_data(timestep, band)
        return data.observations, data.uncertainty, data.mask, data.metadata, data.emulator

    # ------------------------------------------------------ conversion
    def initial_state(self, x_forecast, P_forecast=None, P_forecast_inverse=None) -> KFState:
        """Reference inputs (interleaved x over ALL active pixels, block-diagonal
        P or P^-1) or a KFState / DevicePrior -> this rank's device state."""
        if isinstance(x_forecast, KFState):
            return x_forecast
        want = COVARIANCE if self.config.analysis_form == "gain" else PRECISION
        if P_forecast_inverse is not None:
            st = KFState.from_reference(x_forecast, P_forecast_inverse, self.n_params, PRECISION, self.device,
                                        self._pixel_slice_for(x_forecast))
        elif P_forecast is not None:
            st = KFState.from_reference(x_forecast, P_forecast, self.n_params, COVARIANCE, self.device,
                                        self._pixel_slice_for(x_forecast))
        else:
            raise ValueError("need P_forecast or P_forecast_inverse")
        return self._as_kind(st, want)

    def _pixel_slice_for(self, x):
        n = np.asarray(x).size // self.n_params
        if n == self.n_total:
            return self.partition.pixel_slice
        if n == self.N:
            return None
        raise ValueError(f"state has {n} pixels; expected {self.n_total} (global) or {self.N} (local)")

    def state_from_prior(self, prior=None) -> KFState:
        """Initial state straight from a prior's per-pixel constants (no N² objects)."""
        pr = (prior or self.prior).device_prior(None)
        if not pr.constant:
            raise ValueError("state_from_prior needs a per-pixel constant prior")
        st = KFState.constant(pr.mean, pr.cinv, self.N, self.device, PRECISION)
        return self._as_kind(st, COVARIANCE if self.config.analysis_form == "gain" else PRECISION)

    @staticmethod
    def _materialize(st):
        return st.materialize() if isinstance(st, LazyForecast) else st

    def _as_kind(self, st: KFState, kind: str) -> KFState:
        st = self._materialize(st)
        if st.kind == kind:
            return st
        st.require_full("the precision / covariance conversion")
        out = torch.empty_like(st.P)
        K.invert(self.n_params, st.P, out, N=st.N)
        return KFState(st.x, out, kind, st.N)

    # ------------------------------------------------------------ run
    def run(self, time_grid, x_forecast, P_forecast, P_forecast_inverse, diag_str="diagnostics", band=None,
            approx_diagonal=True, refine_diag=True, iter_obs_op=False, is_robust=False, dates=None,
            resume_from=None):
        """Full assimilation over ``time_grid`` (linear_kf.py:171-212).  Returns the
        final analysis state (device).  ``resume_from`` restarts from a checkpoint."""
        from ..input_output.checkpoint import CheckpointManager

        ckpt = CheckpointManager(self.config.checkpoint_dir, self) if self.config.checkpoint_dir else None
        self.checkpointer = ckpt
        if self.config.gc_freeze:
            # long-lived setup objects out of the collector's full passes (which
            # otherwise stall sub-millisecond time steps by milliseconds)
            import gc
            gc.freeze()
        resume_t = None
        analysis = None
        if resume_from is not None:
            analysis, resume_t = CheckpointManager.load(resume_from, self)
            forecast = None
        else:
            forecast = self.initial_state(x_forecast, P_forecast, P_forecast_inverse)
        all_dates = list(self.observations.dates)
        steps = list(iterate_time_grid(time_grid, all_dates))
        for step_i, (timestep, locate_times, is_first) in enumerate(steps):
            if resume_t is not None and timestep <= resume_t:
                continue
            advance = analysis is not None and (not is_first or resume_t is not None)
            # the precision policy (store_precision="auto") keeps the full analysis
            # precision where it is read: the returned final state, checkpoints
            self._full_precision_step = (step_i == len(steps) - 1 or (
                ckpt is not None and bool(self.config.checkpoint_every)
                and (step_i + 1) % self.config.checkpoint_every == 0))
            try:
                analysis = self.step(timestep, locate_times, analysis if advance else forecast, advance, all_dates)
            finally:
                self._full_precision_step = False
            if ckpt is not None and self.config.checkpoint_every and (step_i + 1) % self.config.checkpoint_every == 0:
                with self.timer.phase("checkpoint"):
                    ckpt.save(timestep, analysis)
        if ckpt is not None:
            with self.timer.phase("checkpoint"):
                ckpt.finish()
        self.resolve_pending()
        self.final_state = analysis
        if self.metrics.enabled:
            self.metrics_summary()
        return analysis

    def _upcoming(self, all_dates, first):
        """Dates >= first (a slice when the list is sorted: O(log n) per step)."""
        key = (id(all_dates), len(all_dates))
        if getattr(self, "_dates_sorted", (None,))[0] != key:
            self._dates_sorted = (key, all(a <= b for a, b in zip(all_dates, all_dates[1:])))
        if self._dates_sorted[1]:
            return all_dates[bisect.bisect_left(all_dates, first):]
        return [d for d in all_dates if d >= first]

    def step(self, timestep, locate_times, state: KFState, advance: bool = True, all_dates=None) -> KFState:
        """One time-grid step: advance (unless ``advance`` is False, i.e. ``state``
        already is the forecast), assimilate every date in ``locate_times``,
        dump.  Returns the analysis state."""
        self.current_timestep = timestep
        t0 = time.perf_counter()
        forecast = state
        if advance:
            if LOG.isEnabledFor(logging.INFO):
                LOG.info("Advancing state, %s" % timestep.strftime("%Y-%m-%d"))
            forecast = self.advance_state(state, timestep, lazy=self.config.fuse_propagation)
        if len(locate_times) == 0:
            analysis = self._materialize(forecast)
            LOG.info("No observations in this time")
            info = {"n_dates": 0}
        else:
            all_dates = list(self.observations.dates) if all_dates is None else all_dates
            upcoming = self._upcoming(all_dates, locate_times[0])
            analysis, info = self._assimilate_dates(locate_times, forecast, upcoming)
        LOG.info("Dumping results to disk")
        self._dump(timestep, analysis)
        rec = {"event": "timestep", "timestep": timestep.isoformat(), "wall_s": time.perf_counter() - t0,
               "n_pixels": self.n_total, **info}
        if hasattr(self.output, "writer_stats"):
            rec["output"] = self.output.writer_stats()     # granule writer: queue depth / waits / encode time
        self.metrics.log(rec)
        self.history.append(rec)
        return analysis

    # --------------------------------------------------------- advance
    def advance(self, x_analysis, P_analysis, P_analysis_inverse, trajectory_model=None, trajectory_uncertainty=None):
        """Reference-signature advance (linear_kf.py:99-108) on reference objects."""
        if isinstance(x_analysis, KFState):
            return self.advance_state(x_analysis, self.current_timestep)
        P = P_analysis_inverse if P_analysis_inverse is not None else P_analysis
        kind = PRECISION if P_analysis_inverse is not None else COVARIANCE
        st = KFState.from_reference(x_analysis, P, self.n_params, kind, self.device, self._pixel_slice_for(x_analysis))
        f = self.advance_state(st, self.current_timestep)
        x, Pl = f.to_reference()
        return (x, None, Pl) if f.kind == PRECISION else (x, Pl, None)

    def advance_state(self, analysis: KFState, date, lazy: bool = False):
        """Propagation + prior blend on device (kf_tools.py:136-171 semantics).

        ``lazy``: when the propagation is a single propagate pass producing a
        precision-form forecast, return a :class:`LazyForecast` instead; the
        fused analysis kernel then computes the forecast per pixel and it is
        never written to memory."""
        # device passes are timed in _run_propagate / _advance_host ("propagate")
        prop = self._state_propagator
        spec = getattr(prop, "device_spec", None) if prop is not None else None
        prior_dev = self.prior.device_prior(date) if (self.prior is not None and
                                                      hasattr(self.prior, "device_prior")) else None
        if (prop is not None and spec is None) or (self.prior is not None and prior_dev is None):
            with self.timer.phase("propagate"):
                return self._advance_host(analysis, date)
        n = self.n_params
        memo_key = (id(spec), id(prior_dev) if prior_dev is not None else None, id(self._m), id(self._q),
                    bool(self.config.reference_quirks), self._analysis_kind(), analysis.kind)
        memo = self._prop_dicts.get(memo_key)
        if memo is not None and lazy:
            # same propagator / prior / Q objects as an earlier step: reuse the
            # (immutable) argument dict, so the fused argument block is reused too
            kind, d = memo[0], memo[1]
            if kind == "lazy":
                return self._lazy(d, self._as_kind(analysis, PRECISION), None)
            if kind == "lazy_cov":
                return self._lazy_cov(d, analysis)
        d = {"m": self._m, "q": self._q}
        d["_key"] = memo_key
        keep = (spec, prior_dev, self._m, self._q)
        if prop is None and self.prior is None:
            spec = PropagatorSpec(PROP_IDENTITY)
        elif prop is None and prior_dev.constant:
            # prior only (kf_tools.py:165-166): reset to the prior, no blend needed
            d.update(mode=PROP_PRIOR, prop_mask=0, reset_mean=np.asarray(prior_dev.mean),
                     reset_cinv=pack_matrix(np.asarray(prior_dev.cinv)))
            if lazy and self._analysis_kind() == PRECISION and analysis.kind == PRECISION:
                self._remember_prop(memo_key, "lazy", d, keep)
                return self._lazy(d, analysis, None)
            if lazy and analysis.kind == COVARIANCE:
                self._remember_prop(memo_key, "lazy_cov", d, keep)
                return self._lazy_cov(d, analysis)
            out = self._run_propagate(d, analysis, None, PRECISION)
            return self._as_kind(out, self._analysis_kind())
        elif prop is None:
            spec = PropagatorSpec(PROP_PRIOR, reset_mean=np.zeros(n), reset_cinv=np.zeros((n, n)))
        d["mode"] = spec.mode
        mask = 0
        for k in spec.propagated:
            mask |= 1 << int(k)
        d["prop_mask"] = mask
        if spec.reset_mean is not None:
            d["reset_mean"] = np.asarray(spec.reset_mean)
            d["reset_cinv"] = pack_matrix(np.asarray(spec.reset_cinv))
        in_kind = COVARIANCE if spec.mode == PROP_STANDARD else PRECISION
        out_kind = COVARIANCE if spec.output == "covariance" else PRECISION
        if (lazy and self.prior is None and in_kind == PRECISION and out_kind == PRECISION
                and analysis.kind == COVARIANCE and self._analysis_kind() == COVARIANCE):
            # gain form: the K1g kernel evaluates this forecast from the analysis covariance
            self._remember_prop(memo_key, "lazy_cov", d, keep)
            return self._lazy_cov(d, analysis)
        src = self._as_kind(analysis, in_kind)
        blend_pix = (None, None)
        if self.prior is not None:
            if out_kind == COVARIANCE:
                # covariance-form propagator + prior: blend in precision form afterwards
                fc = self._run_propagate(d, src, None, COVARIANCE)
                fc = self._as_kind(fc, PRECISION)
                d2 = {"mode": PROP_IDENTITY, "m": np.ones(n), "q": np.zeros(n)}
                self._fill_blend(d2, prior_dev)
                out = self._run_propagate(d2, fc, self._blend_pix(prior_dev), PRECISION)
                return self._as_kind(out, self._analysis_kind())
            self._fill_blend(d, prior_dev)
            blend_pix = self._blend_pix(prior_dev)
        if lazy and out_kind == PRECISION and self._analysis_kind() == PRECISION:
            if blend_pix == (None, None) and src.kind == PRECISION:
                self._remember_prop(memo_key, "lazy", d, keep)
            return self._lazy(d, src, blend_pix)
        out = self._run_propagate(d, src, blend_pix, out_kind)
        return self._as_kind(out, self._analysis_kind())

    def cache_stats(self) -> dict:
        """Host-side reuse counters (band tables, fused-argument blocks)."""
        return {"table_hits": self._tables.hits, "table_misses": self._tables.misses,
                "prop_hits": self._prop_bufs.get("_hits", 0), "prop_misses": self._prop_bufs.get("_misses", 0)}

    def _remember_prop(self, key, kind, d, keep):
        if len(self._prop_dicts) > 32:
            self._prop_dicts.clear()
        self._prop_dicts[key] = (kind, d, keep)

    def _lazy(self, d, src: KFState, blend_pix):
        def materialize():
            return self._run_propagate(d, src, blend_pix, PRECISION)
        if not K.prop_is_light(d["mode"], d.get("blend", False)):
            return materialize()
        return LazyForecast(src, d, blend_pix, self._q_pix, materialize, cache=self._prop_bufs)

    def _lazy_cov(self, d, src: KFState):
        """Gain-form twin of :meth:`_lazy`: a light propagation of an analysis
        held as a covariance, evaluated per pixel by the K1g kernel
        (kf_core.h:forecast_partial_cov) instead of invert + propagate + invert
        passes; other consumers materialise it through those passes."""
        def materialize():
            out = self._run_propagate(d, self._as_kind(src, PRECISION), None, PRECISION)
            return self._as_kind(out, COVARIANCE)
        if not K.prop_is_light(d["mode"], d.get("blend", False)):
            return materialize()
        return LazyForecast(src, d, None, self._q_pix, materialize, kind=COVARIANCE, cache=self._prop_bufs)

    @property
    def _line_opt(self):
        """The launches' ``line`` option: EngineConfig.line_tables False turns the
        line tables off; True leaves them to ops.kernels.LINE_TABLES (on)."""
        return None if self.config.line_tables else False

    def _analysis_kind(self):
        return COVARIANCE if self.config.analysis_form == "gain" else PRECISION

    def _fill_blend(self, d, prior_dev):
        d["blend"] = True
        d["quirk_blend"] = bool(self.config.reference_quirks)
        if prior_dev.constant:
            d["blend_mean"] = np.asarray(prior_dev.mean)
            d["blend_cinv"] = pack_matrix(np.asarray(prior_dev.cinv))

    def _blend_pix(self, prior_dev):
        if prior_dev.constant:
            return (None, None)
        return (prior_dev.mean_soa, prior_dev.cinv_packed)

    def _run_propagate(self, d, src: KFState, blend_pix, out_kind) -> KFState:
        out = KFState.empty(self.n_params, self.N, self.device, out_kind, ld=src.x.shape[1])
        bm, bc = blend_pix if blend_pix else (None, None)
        if self.N:
            with self.timer.phase("propagate"):
                K.propagate(self.n_params, d, src.x, src.P, out.x, out.P, N=self.N, q_pix=self._q_pix,
                            blend_mean_pix=bm, blend_cinv_pix=bc)
        return out

    def _advance_host(self, analysis: KFState, date) -> KFState:
        """Reference propagator/prior objects: run them on the host."""
        x, P = analysis.to_reference()
        n = self.n_params * self.N
        M = sp.eye(n, n, format="csr") * 1.0
        if not np.all(self._m == 1):
            M = sp.diags(np.tile(self._m, self.N)).tocsr()
        if self._q_pix is not None:
            qv = soa_to_interleaved(self._q_pix.cpu().numpy().astype(np.float64))
        else:
            qv = np.tile(self._q, self.N)
        Q = sp.diags(qv).tocsr()
        kw = dict(prior=self.prior, date=date, state_propagator=self._state_propagator)
        if self._advance is propagate_and_blend_prior:
            kw["reference_quirks"] = bool(self.config.reference_quirks)   # same blend as the device path
        if analysis.kind == PRECISION:
            xf, Pf, Pfi = self._advance(x, None, P.tocsr(), M, Q, **kw)
        else:
            xf, Pf, Pfi = self._advance(x, P.tocsr(), None, M, Q, **kw)
        if xf is None:
            return analysis
        if Pfi is not None:
            st = KFState.from_reference(xf, Pfi, self.n_params, PRECISION, self.device)
        else:
            st = KFState.from_reference(xf, Pf, self.n_params, COVARIANCE, self.device)
        return self._as_kind(st, self._analysis_kind())

    # ------------------------------------------------------ assimilate
    def assimilate_multiple_bands(self, locate_times, x_forecast, P_forecast, P_forecast_inverse,
                                  approx_diagonal=True, refine_diag=False, iter_obs_op=False, is_robust=False,
                                  diag_str="diag"):
        """All bands of each date jointly (linear_kf.py:214-242); reference objects in/out."""
        st = self.initial_state(x_forecast, P_forecast, P_forecast_inverse)
        out, _ = self._assimilate_dates(locate_times, st, list(locate_times))
        x, P = out.to_reference()
        return (x, None, P) if out.kind == PRECISION else (x, P, None)

    def _assimilate_dates(self, locate_times, forecast: KFState, upcoming):
        info = {"n_dates": len(locate_times), "gn_iterations": [], "norms": []}
        for i, step in enumerate(locate_times):
            if LOG.isEnabledFor(logging.INFO):
                LOG.info("Assimilating %s..." % step.strftime("%Y-%m-%d"))
            t0 = time.perf_counter()
            if self.config.band_sequential:
                res = self._assimilate_sequential(step, self._materialize(forecast))
            else:
                prep = self._prepared
                self._prepared = None
                bands = prep[1] if (prep is not None and prep[0] == step) else self._device_bands(step)
                if getattr(self, "_dates_sorted", (None, False))[1]:
                    nxt = upcoming[bisect.bisect_right(upcoming, step):]
                else:
                    nxt = [d for d in upcoming if d > step]
                if nxt and self.config.prefetch and hasattr(self.observations, "prefetch"):
                    # as many dates ahead as the source has buffers for (one copy
                    # per step stays on the DMA engine back to back)
                    for d_ahead in nxt[:max(1, int(getattr(self.observations, "max_prefetch", 1)))]:
                        self.observations.prefetch(d_ahead)
                if nxt and self.config.lookahead:
                    self._lookahead_fn = lambda d=nxt[0]: self._prepare_date(d)
                rows = self._precision_rows(last_of_step=i == len(locate_times) - 1, more_dates=bool(nxt))
                try:
                    ready = prep is not None and prep[1] is bands
                    res = self.do_all_bands_state(step, bands, forecast, table=prep[2] if ready else None,
                                                  store_rows=rows,
                                                  order=prep[3] if ready and prep[3] is not None else False)
                finally:
                    self._lookahead_fn = None
            forecast = res.state
            if self.config.domain_history and getattr(self, "last_status", None) is not None and self.N:
                # pixels whose GP inputs left an emulator's domain on any date of the run
                ood = self.last_status[:self.N] & K.ST_OUT_OF_DOMAIN
                self.ood_history = ood if self.ood_history is None else (self.ood_history | ood)
            info["gn_iterations"].append(res.n_iter)
            info["norms"].append(res.norms[-1] if res.norms else None)
            rec = {"event": "date", "date": step.isoformat(), "n_iter": res.n_iter, "norms": res.norms,
                   "wall_s": time.perf_counter() - t0,
                   # exact per-date phases only when per-date metrics are asked for
                   "phases_ms": self.timer.snapshot(block=self.metrics.enabled)}
            if self.last_chunk_iters is not None:
                rec["chunk_iters"] = self.last_chunk_iters
                info.setdefault("chunk_iters", []).append(self.last_chunk_iters)
            if self._reg_log:
                rec["spatial"] = self._spatial_record()
            if self.metrics.enabled:
                rec.update(self._health_metrics(rec["wall_s"]))
            self.metrics.log(rec)
        return forecast, info

    def _prepare_date(self, date):
        """Lookahead: acquire the next date's device bands and build its band
        table while the current date's last Gauss-Newton iteration runs (the
        host work otherwise sits between two dates with the GPU idle).  Only the
        fused single-kernel path reuses the table; the bands serve every path."""
        bands = self._device_bands(date)
        table = None
        specs = [sp for sp, _ in bands]
        cfg = self.config
        order = None
        if not (cfg.return_innovations or cfg.spatial_gamma > 0 or
                self.band_comm is not None or any(sp.kind == OP_PRECOMP for sp in specs)) and \
                self._split_plan_kind(specs) is None:
            table = self._band_table(bands, specs, [d for _, d in bands])
            # the next date's observed-first order too: its passes run on the
            # device after this date's launches, under the host's norm wait and
            # step bookkeeping, instead of between the two dates' analyses
            order = self._visit_order(date, specs, table)
        self._prepared = (date, bands, table, order)

    def _visit_order(self, timestep, specs, table):
        """Observed-first visiting order of one date (config.observed_first; GP
        bands on the fused kernels), or None.  The two buffer sets alternate by
        date: a date's order is computed ahead (lookahead) while the previous
        date's launches may still read theirs."""
        cfg = self.config
        N = self.N
        if not (cfg.observed_first and table is not None and N and any(s.kind == OP_GP for s in specs)):
            return None
        slot = self._order_turn % 2
        self._order_turn += 1
        buf, scratch = self._order_bufs[slot] if self._order_bufs[slot] is not None else (None, None)
        # band groups: the bands of one sensor share its clouds (multi-sensor sources)
        groups = self.observations.band_groups(timestep) if hasattr(self.observations, "band_groups") else None
        if groups is not None and (len(groups) != len(specs) or max(groups) > 2):
            groups = None
        order, scratch = K.obs_order(table, N, self.device, buf, scratch, groups=groups,
                                     local=cfg.observed_first_local)
        self._order_bufs[slot] = (order if buf is None or buf.numel() < N else buf, scratch)
        return order

    def _health_metrics(self, wall_s: float) -> dict:
        """Per-date structured metrics: rank-local pixel updates/s,
        per-pixel status counts (masked, fallback, non-SPD, bad operator) and
        host-to-device ingest bytes.  One device reduction + sync, only when
        metrics are enabled."""
        out = {"n_pixels_local": self.N, "pixel_updates_per_s_local": self.N / max(wall_s, 1e-9)}
        st = getattr(self, "last_status", None)
        if st is not None and self.N:
            s = st[:self.N]
            bits = torch.stack([(s & b) > 0 for b in (K.ST_NO_OBS, K.ST_FALLBACK, K.ST_NONSPD, K.ST_NONFINITE,
                                                      K.ST_BAD_OP, K.ST_OUT_OF_DOMAIN)]).sum(1).cpu().tolist()
            out["status"] = dict(zip(("no_obs", "fallback", "non_spd", "non_finite", "bad_operator",
                                      "out_of_domain"), bits))
            out["masked_fraction"] = bits[0] / self.N
        if hasattr(self.observations, "ingest_bytes"):
            total = int(self.observations.ingest_bytes())
            out["h2d_bytes"] = total - getattr(self, "_h2d_seen", 0)
            self._h2d_seen = total
        return out

    def metrics_summary(self) -> dict | None:
        """Aggregate this run's per-date metrics over every rank onto rank 0
        (written next to the JSONL as ``*.summary.json``); None on other ranks."""
        dates = [r for r in self.metrics.records if r.get("event") == "date"]
        mine = {"rank": self.comm.rank, "n_pixels": self.N, "n_dates": len(dates),
                "wall_s": sum(r["wall_s"] for r in dates),
                "gn_iterations": [r["n_iter"] for r in dates],
                "phases_ms": {}, "status": {}, "h2d_bytes": sum(r.get("h2d_bytes", 0) for r in dates)}
        for r in dates:
            for k2, v in r.get("phases_ms", {}).items():
                mine["phases_ms"][k2] = mine["phases_ms"].get(k2, 0.0) + v
            for k2, v in r.get("status", {}).items():
                mine["status"][k2] = mine["status"].get(k2, 0) + v
        per_rank = self.comm.gather_object(mine)
        if per_rank is None:
            return None
        summary = {"ranks": per_rank, "n_pixels": sum(p["n_pixels"] for p in per_rank),
                   "n_dates": max(p["n_dates"] for p in per_rank),
                   "wall_s_max": max(p["wall_s"] for p in per_rank),
                   "h2d_bytes": sum(p["h2d_bytes"] for p in per_rank)}
        if summary["wall_s_max"] > 0:
            summary["pixel_updates_per_s"] = summary["n_pixels"] * summary["n_dates"] / summary["wall_s_max"]
        self.metrics.write_summary(summary)
        return summary

    # ----------------------------------------------------- observations
    def _device_bands(self, date):
        """-> list of (OperatorSpec, DeviceBand) for every band of ``date``."""
        obs = self.observations
        nb = obs.bands_per_observation[date]
        out = []
        mine = range(nb)
        if self.band_comm is not None and not self.config.band_sequential:
            # band-parallel: this rank owns bands b = slot, slot + B, ...
            mine = range(self.band_comm.rank, nb, self.band_comm.world)
        with self.timer.phase("ingest"):
            if hasattr(obs, "get_device_bands") and len(mine) == nb:
                dbs = obs.get_device_bands(date)     # one acquire of the date's buffers
                if not getattr(obs, "band_specs_static", False):
                    return [(self._operator_spec(db, b, date), db) for b, db in enumerate(dbs)]
                # the source hands out the same band list for every date of a
                # pool slot and its operators do not depend on the date: the
                # (spec, band) pairs and their band table are built once per list
                hit = self._bands_memo.get(id(dbs))
                if hit is None or hit[0] is not dbs:
                    if len(self._bands_memo) >= 32:
                        self._bands_memo.clear()
                    hit = self._bands_memo[id(dbs)] = [dbs, [(self._operator_spec(db, b, date), db)
                                                             for b, db in enumerate(dbs)], None]
                return hit[1]
            for b in mine:
                if hasattr(obs, "get_device_band_data"):
                    db = obs.get_device_band_data(date, b)
                else:
                    db = self._band_from_reference(obs.get_band_data(date, b))
                spec = self._operator_spec(db, b, date)
                out.append((spec, db))
        return out

    def _band_table(self, bands, specs, dbs) -> K.BandTable:
        """The band table of ``bands`` (TableCache); memoised with the pairs
        list of a ``band_specs_static`` source (:meth:`_device_bands`)."""
        for hit in self._bands_memo.values():
            if hit[1] is bands:
                if hit[2] is None:
                    hit[2] = self._tables.get(specs, dbs, self.n_params, self._cache, self.device)
                return hit[2]
        return self._tables.get(specs, dbs, self.n_params, self._cache, self.device)

    def _band_from_reference(self, data) -> DeviceBand:
        """Reference record (full strip rasters, sparse diagonal inverse variance)."""
        part = self.partition
        sm = part.local_mask
        y = np.asarray(data.observations, dtype=np.float64)
        unc = data.uncertainty
        if sp.issparse(unc):
            w = np.asarray(unc.diagonal(), dtype=np.float64)
        else:
            u = np.asarray(unc, dtype=np.float64)
            w = u.ravel() if u.shape == sm.shape else np.diag(u)
        m = np.asarray(data.mask).astype(bool)
        if y.shape != sm.shape:
            raise ValueError(f"observation raster {y.shape} does not match the strip {sm.shape}")
        yl, wl, ml = y[sm], w[sm.ravel()], m[sm]
        wl = np.where(ml & np.isfinite(wl), wl, 0.0)
        dev = self.device
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
        aux = None
        meta = data.metadata if isinstance(data.metadata, dict) else {}
        if meta.get("incidence_angle") is not None:
            a = np.asarray(meta["incidence_angle"], dtype=np.float32)
            aux = t(a[sm] if a.shape == sm.shape else np.broadcast_to(a.ravel(), (self.N,)), np.float32)
        return DeviceBand(K.OBS_F32, y=t(np.where(ml, yl, 0.0), np.float32), w=t(wl, np.float32),
                          mask=t(ml, np.uint8), metadata=meta, emulator=data.emulator, aux=aux)

    def _operator_spec(self, db: DeviceBand, band, date) -> OperatorSpec:
        spec_fn = getattr(self._create_observation_operator, "device_spec", None)
        spec = None
        if hasattr(self.observations, "band_spec"):
            spec = self.observations.band_spec(date, band)
        if spec is None and spec_fn is not None:
            spec = spec_fn(self.n_params, db.emulator, db.metadata, band, self.band_mapper)
        if spec is None:
            spec = OperatorSpec(OP_PRECOMP, list(range(self.n_params)), [0.0] * self.n_params)
        return spec

    def _precompute_host(self, specs, bands, x_prev: torch.Tensor):
        """Host evaluation of reference-protocol factories (OP_PRECOMP bands)."""
        pre = []
        x_flat = None
        for b, (spec, db) in enumerate(zip(specs, bands)):
            if spec.kind != OP_PRECOMP:
                pre.append(None)
                continue
            if x_flat is None:
                x_flat = soa_to_interleaved(x_prev[:, :self.N].cpu().numpy().astype(np.float64))
            mask = np.zeros(self.partition.local_mask.shape, dtype=bool)
            mask[self.partition.local_mask] = db.decode()[1].cpu().numpy() > 0
            H = self._create_observation_operator(self.n_params, db.emulator, db.metadata, mask,
                                                  self.partition.local_mask, x_flat, b)
            if isinstance(H, (tuple, list)) and len(H) == 2:
                H0, Hm = H
                H0 = np.broadcast_to(np.asarray(H0, dtype=np.float64), (self.N,))
            else:
                Hm = H
                H0 = np.asarray(Hm.dot(x_flat)).ravel()
            h = _jacobian_blocks(Hm, self.N, self.n_params)
            dev = self.device
            pre.append((torch.from_numpy(np.ascontiguousarray(H0, dtype=np.float32)).to(dev),
                        torch.from_numpy(np.ascontiguousarray(h, dtype=np.float32)).to(dev)))
        return pre

    # ------------------------------------------------------ GN solver
    def do_all_bands(self, timestep, current_data, x_forecast, P_forecast, P_forecast_inverse,
                     convergence_tolerance=1e-3, min_iterations=2):
        """Reference-signature joint analysis (linear_kf.py:245-323); ``current_data``
        are reference band records.  Returns (x_a, P_a, P_a^-1, innovations)."""
        st = self.initial_state(x_forecast, P_forecast, P_forecast_inverse)
        bands = []
        for b, data in enumerate(current_data):
            db = self._band_from_reference(data)
            bands.append((self._operator_spec(db, b, timestep), db))
        old = (self.config.convergence_tolerance, self.config.min_iterations)
        self.config.convergence_tolerance, self.config.min_iterations = convergence_tolerance, min_iterations
        try:
            res = self.do_all_bands_state(timestep, bands, st, innovations=True)
        finally:
            self.config.convergence_tolerance, self.config.min_iterations = old
        x, P = res.state.to_reference()
        inn = np.hstack([i.cpu().numpy() for i in res.innovations]) if res.innovations else None
        return (x, None, P, inn) if res.state.kind == PRECISION else (x, P, None, inn)

    def do_all_bands_state(self, timestep, bands, forecast: KFState, innovations=None,
                           table=None, store_rows=None, order=False) -> AssimilationResult:
        """Gauss-Newton loop on device (linear_kf.py:245-307).

        ``store_rows``: the packed precision rows the caller needs of the
        analysis (None: all; a set of row indices otherwise, see
        :meth:`_precision_rows`); the returned state marks the others invalid.
        With ``EngineConfig.convergence_chunk`` the exit test runs per chunk
        (:meth:`_gn_chunked`).  ``order``: the date's visiting order computed
        ahead with ``table`` (:meth:`_prepare_date`; False: compute it here)."""
        cfg = self.config
        n = self.n_params
        N = self.N
        self.last_chunk_iters = None
        specs = [s for s, _ in bands]
        dbs = [d for _, d in bands]
        need_inn = cfg.return_innovations if innovations is None else innovations
        h0_outs = [torch.zeros(max(N, 1), dtype=torch.float32, device=self.device) for _ in bands] \
            if need_inn else None
        gain = cfg.analysis_form == "gain"
        precomp = any(s.kind == OP_PRECOMP for s in specs)
        bp = self.band_comm is not None
        if bp and (gain or cfg.spatial_gamma > 0 or cfg.hessian_correction):
            raise ValueError("band_parallel runs the information form without regulariser / Hessian correction")
        if bp and not getattr(self, "_bp_checked", False):
            nb_all = getattr(self.observations, "bands_per_observation", {}).get(timestep) \
                if hasattr(self.observations, "bands_per_observation") else None
            self._band_parallel_check(specs, nb_all)
        chunked = bool(cfg.convergence_chunk)
        if chunked and (cfg.spatial_gamma > 0 or (gain and precomp) or (bp and gain)):
            raise ValueError("convergence_chunk runs without the spatial prior (which couples the chunks)")
        split = None if (precomp or gain or bp or cfg.spatial_gamma > 0 or chunked) else \
            self._split_plan(specs, dbs, h0_outs)
        if precomp or split:
            table = None
        elif h0_outs is not None:
            table = build_table(specs, dbs, n, self._cache, self.device, h0_outs)
        elif table is None:
            table = self._band_table(bands, specs, dbs)
        prop = None
        if (isinstance(forecast, LazyForecast) and forecast.kind == (COVARIANCE if gain else PRECISION)
                and not (precomp or split or bp) and N):
            # fused propagation: the kernel computes the forecast per pixel from
            # the previous analysis; the first iteration linearises at it
            prop = forecast.handle()
            src = forecast.src
            fc = None
            x_prev = None
            x_new = torch.empty_like(src.x)
            P_out = torch.empty_like(src.P)
            ld = src.x.shape[1]
        else:
            fc = self._as_kind(forecast, COVARIANCE if gain else PRECISION)
            ld = fc.x.shape[1]
            x_prev = fc.x.clone()
            x_new = torch.empty_like(fc.x)
            P_out = torch.empty_like(fc.P)
        # every analysis / gain kernel writes the status of each of its N pixels
        status = torch.empty(max(N, 1), dtype=torch.uint8, device=self.device)
        len_x = float(n * self.n_total)
        # fused output: an output with device rasters is written by the analysis
        # kernel itself in every iteration that can end the loop (the last one wins)
        plain = not (gain or precomp or split or bp or cfg.spatial_gamma > 0 or cfg.hessian_correction)
        spatial = cfg.spatial_gamma > 0 and not (gain or precomp or bp or cfg.hessian_correction)
        out_t = None
        if ((plain or spatial or (gain and not precomp)) and N and cfg.fuse_output
                and hasattr(self.output, "device_targets")):
            # plain and spatial paths: the final state's x doubles as the mean raster (dense strips)
            out_t = self.output.device_targets(self, self.device, alias=plain or spatial or gain)
        # analysis precision rows stored (EngineConfig.store_precision): a mask of
        # the rows the caller reads (0: all); no row at all -> no precision store.
        # Paths whose output is dumped from the state afterwards keep every row
        a_rows, p_valid, pdiag_rows = 0, None, 0
        diag_pos = {tri_pos(n, j, j): j for j in range(n)}
        if (store_rows is not None and not cfg.hessian_correction
                and (out_t is not None or self.output is None)
                and not (gain and (precomp or any(r not in diag_pos for r in store_rows)))):
            p_valid = 0
            for r in store_rows:
                p_valid |= 1 << int(r)
                if gain:            # the gain form stores those rows as precision diagonal entries
                    pdiag_rows |= 1 << diag_pos[int(r)]
            a_rows = 0 if gain else p_valid
            if p_valid == 0:
                P_out = None
        # GN iterations 1 and 2 in one launch (the first never ends the loop): rank-
        # independent test, so every rank queues the same collectives
        fuse2 = ((plain or (gain and not precomp)) and cfg.fuse_gn and cfg.min_iterations >= 2
                 and cfg.max_iterations >= 1 and not (prop is None and fc is None))
        # linear / identity operators: y' = y - offset does not depend on the
        # linearisation point (kf_core.h FD_LINEAR), so iteration 2 repeats
        # iteration 1 exactly and its norm is 0 -- converged without a read-back
        static_conv = (fuse2 and plain and cfg.convergence_tolerance > 0 and bool(specs)
                       and all(s.kind == OP_LINEAR for s in specs))
        # observed pixels first (config.observed_first): one order per date for
        # every analysis launch of it (GP bands on the fused kernels only)
        if order is False or table is None or not N or precomp or split or bp:
            order = None if (precomp or split or bp) else self._visit_order(timestep, specs, table)
        self._visit = order
        # spatial prior: a plain first iteration (config.spatial_first_plain; it
        # cannot end the loop), fused with the regularised prepare of the second
        first_plain = spatial and cfg.spatial_first_plain and cfg.min_iterations >= 2 and cfg.max_iterations >= 1
        fuse_sp = first_plain and cfg.fuse_gn
        run = _GNRun(timestep=timestep, specs=specs, dbs=dbs, table=table, precomp=precomp, gain=gain, bp=bp,
                     split=split, prop=prop, fc=fc, x_prev=x_prev, x_new=x_new, P_out=P_out, status=status,
                     order=order, out_t=out_t, h0_outs=h0_outs, a_rows=a_rows, pdiag_rows=pdiag_rows, len_x=len_x,
                     n_bands=len(bands),
                     fuse2=fuse2, fuse_sp=fuse_sp, first_plain=first_plain, static_conv=static_conv)
        # the iteration strategy: the reference's exit test per chunk or over the tile
        x_prev, n_iter, norms = (self._gn_chunked if chunked else self._gn_global)(run)
        if ld != x_prev.shape[1]:
            raise RuntimeError("leading dimension changed")
        if P_out is None:
            # no precision row needed: a buffer of the forecast's shape with nothing
            # valid (p_valid = 0), never written -- one shared by every such date
            pu = getattr(self, "_p_unused", None)
            if pu is None or pu.shape != (ntri(n), ld) or pu.device != self.device:
                pu = self._p_unused = torch.empty((ntri(n), ld), dtype=torch.float32, device=self.device)
            P_out = pu
        state = KFState(x_prev, P_out, COVARIANCE if gain else PRECISION, N, p_valid=p_valid,
                        p_diag_precision=gain and p_valid is not None)
        self._output_written = state if out_t is not None else None
        if cfg.hessian_correction and not gain and N:
            with self.timer.phase("hessian"):
                K.hessian(n, run.table, state.x, state.P, N=N)
        if bp:
            status = self._band_parallel_status(status)
        self.last_status = status
        inn = None
        if need_inn:
            inn = []
            for db, h0 in zip(dbs, h0_outs):
                y, w = db.decode()
                inn.append(torch.where(w > 0, y - h0[:N], torch.zeros_like(y)))
        return AssimilationResult(state, n_iter, norms, inn)

    # --------------------------------------------- precision store policy
    def _precision_rows(self, last_of_step: bool, more_dates: bool):
        """Packed precision rows of this date's analysis that anything reads
        (None: all).  Under ``store_precision="auto"`` the analysis of a date
        whose state only feeds the next step's forecast stores what that
        forecast reads -- the propagated parameters' diagonal entries for the
        LAI propagator (kf_tools.py:292-314: [6, 6] only), nothing for a prior
        reset (no_propagation / prior only, kf_tools.py:316-353, 165-166), the
        diagonal for the approximate information filter -- instead of the full
        4 ntri B/px.  Full where the state is read otherwise: the run's last
        step or a checkpoint step, the last observation date, a date whose
        analysis is the next date's forecast within one step, a non-fused
        output, reference-protocol propagators; the gain form keeps the rows as
        precision diagonal entries when its next forecast is fused (a light
        propagator, no prior blend), the full covariance otherwise."""
        cfg = self.config
        if (cfg.store_precision == "always" or self._full_precision_step or not last_of_step or not more_dates
                or cfg.band_sequential or cfg.hessian_correction or cfg.return_innovations):
            return None
        if not (cfg.fuse_output and hasattr(self.output, "device_targets")) and self.output is not None:
            return None            # the dump reads the precision diagonal (observations.py:392-393)
        if cfg.analysis_form == "gain":
            # the gain form stores the rows as precision diagonal entries, which only
            # its fused forecast reads (a light propagator without a prior blend:
            # advance_state's lazy_cov); other forecasts invert the full covariance
            prop = self._state_propagator
            spec = getattr(prop, "device_spec", None) if prop is not None else None
            if self.prior is not None or spec is None or not K.prop_is_light(spec.mode):
                return None
        return self._next_forecast_rows()

    def _next_forecast_rows(self):
        """Packed rows of the analysis precision the next forecast reads (None:
        all), from the configured propagator / prior (advance_state)."""
        from ..inference.kf_tools import PROP_PRIOR_PARTIAL, PROP_INFO_APPROX

        n = self.n_params
        prop = self._state_propagator
        spec = getattr(prop, "device_spec", None) if prop is not None else None
        if prop is not None and spec is None:
            return None                       # host (reference-protocol) propagator
        if self.prior is not None and not hasattr(self.prior, "device_prior"):
            return None
        if prop is None:
            # no propagator: the prior alone resets the state (nothing read); neither: identity
            return set() if self.prior is not None else None
        if spec.mode == PROP_PRIOR:
            return set()
        if spec.mode == PROP_PRIOR_PARTIAL:
            return {tri_pos(n, int(j), int(j)) for j in spec.propagated}
        if spec.mode == PROP_INFO_APPROX:
            return {tri_pos(n, j, j) for j in range(n)}
        return None

    # ------------------------------------------------ split GP operator path
    def _split_plan_kind(self, specs):
        """GP input count d when these bands take the split path, else None."""

        cfg = self.config
        if cfg.gp_split == "never" or not specs or any(s.kind != OP_GP for s in specs):
            return None
        ds = {s.d for s in specs}
        if len(ds) != 1:
            return None
        d = ds.pop()
        on_dev = self.device.type == "cuda"
        if on_dev and not K.gp_operator_supported(self.n_params, d):
            return None
        if cfg.gp_split == "auto" and d < cfg.gp_split_min_d and len(specs) < cfg.gp_split_min_bands:
            return None
        if (cfg.gp_split == "auto" and on_dev and d == self.n_params and d in K.GPM_GLOBAL_D
                and K.DEFAULT_VARIANT != K.Variant.VALU_ORACLE and all(self._cache.get_mfma(s, self.device) is not None for s in specs)):
            # many full-state GP bands: the fused matrix-core kernel with the
            # tables in global memory beats the split path (34 bands: 631 vs
            # 1064 ms/step, profiles/r2_v10_prosail_mfma_g_ab.log)
            return None
        return d

    def _split_plan(self, specs, dbs, h0_outs):
        """Band chunks for the split path, or None for the fused kernel."""
        d = self._split_plan_kind(specs)
        if d is None:
            return None
        cfg = self.config
        n, N = self.n_params, self.N
        C = int(cfg.band_chunk)
        if C <= 0:
            # as many bands per chunk as fit in the free HBM (h0 + h: 4 (1 + n) B/px/band) after
            # the iteration's own state buffers (x_prev, x_new, P_out, the forecast and the (A, b)
            # accumulators of a multi-chunk plan) and 2 GiB of slack: one chunk = one operator
            # pass and no (A, b) round trip.  Sized once per band count (later dates see the
            # allocator's cached blocks as used).
            C = self._split_chunk.get(len(specs))
            if C is None:
                C = 10
                if self.device.type == "cuda":
                    free, _ = torch.cuda.mem_get_info(self.device)
                    nt = ntri(n)
                    reserve = 4 * max(N, 1) * (4 * n + 2 * nt + 2 * (nt + n)) + (2 << 30)
                    C = max(1, int((free - reserve) // (4 * (1 + n) * max(N, 1))))
                self._split_chunk[len(specs)] = C
        C = max(1, min(C, len(specs)))
        ldh = max(N, 1)
        h0_buf = torch.empty((C, ldh), dtype=torch.float32, device=self.device)
        h_buf = torch.empty((C * n, ldh), dtype=torch.float32, device=self.device)
        chunks = []
        for c0 in range(0, len(specs), C):
            idx = list(range(c0, min(c0 + C, len(specs))))
            op_tab = build_table([specs[i] for i in idx], [dbs[i] for i in idx], n, self._cache, self.device)
            pre_specs = [OperatorSpec(OP_PRECOMP, list(range(n)), [0.0] * n) for _ in idx]
            pre = [(h0_buf[j], h_buf[j * n:(j + 1) * n]) for j in range(len(idx))]
            h0s = None if h0_outs is None else [h0_outs[i] for i in idx]
            an_tab = build_table(pre_specs, [dbs[i] for i in idx], n, self._cache, self.device, h0s, pre)
            chunks.append((op_tab, an_tab, len(idx)))
        acc = None
        if len(chunks) > 1:
            acc = [(torch.empty((ntri(n), ldh), dtype=torch.float32, device=self.device),
                    torch.empty((n, ldh), dtype=torch.float32, device=self.device)) for _ in range(2)]
        return {"d": d, "chunks": chunks, "h0": h0_buf, "h": h_buf, "acc": acc}

    def _split_iteration(self, plan, x_prev, fc: KFState, x_out, A_out, status):
        n, N = self.n_params, self.N
        chunks = plan["chunks"]
        prev = None
        for ci, (op_tab, an_tab, nb) in enumerate(chunks):
            K.gp_operator(n, op_tab, x_prev, plan["h0"][:nb], plan["h"][:nb * n], N=N, d=plan["d"])
            last = ci == len(chunks) - 1
            a_in, b_in = prev if prev is not None else (None, None)
            if last:
                K.analysis(n, an_tab, x_prev, fc.x, fc.P, x_out, A_out, None, status, self._partials, N=N,
                           a_in=a_in, b_in=b_in)
            else:
                A_c, b_c = plan["acc"][ci % 2]
                K.analysis(n, an_tab, x_prev, fc.x, fc.P, None, A_c, b_c, status, None, N=N, solve=False,
                           a_in=a_in, b_in=b_in)
                prev = (A_c, b_c)

    # ------------------------------------------------ band-parallel (TP-like)
    def _band_parallel_iteration(self, table, x_prev, fc: KFState, x_out, A_out, status, order=None, n_visit=None,
                                 dn_out=None):
        """C5: this rank accumulates sum_b w h h^T and sum_b w h y' over its own
        bands (band slot 0 also adds the forecast precision), one RCCL
        all-reduce of the packed [A | b] per pixel within the band group, then
        every member solves redundantly (identical x on the group).  ``order`` /
        ``n_visit`` / ``dn_out``: the per-chunk loop's visiting subset and
        per-pixel norms (both launches visit the same pixels; the all-reduced
        entries of the others are never read)."""
        vis = dict(order=order, n_visit=n_visit)
        n, N = self.n_params, self.N
        nt = ntri(n)
        ld = fc.x.shape[1]
        if self._bp_buf is None or self._bp_buf.shape[1] != ld:
            self._bp_buf = torch.zeros((nt + n, ld), dtype=torch.float32, device=self.device)
            self._bp_solve_tab = build_table([], [], n, self._cache, self.device)
            self._bp_status = torch.zeros(max(N, 1), dtype=torch.uint8, device=self.device)
        A_part, b_part = self._bp_buf[:nt], self._bp_buf[nt:]
        if N:
            if self.band_comm.rank == 0:
                K.analysis(n, table, x_prev, fc.x, fc.P, None, A_part, b_part, status, None, N=N, solve=False, **vis)
            else:
                self._bp_buf.zero_()
                K.analysis(n, table, x_prev, fc.x, fc.P, None, A_part, b_part, status, None, N=N, solve=False,
                           a_in=A_part, b_in=b_part, **vis)
        with self.timer.phase("band_allreduce"):
            self.band_comm.all_reduce_(self._bp_buf)
        if N:
            K.analysis(n, self._bp_solve_tab, x_prev, fc.x, fc.P, x_out, A_out, None, self._bp_status,
                       None if dn_out is not None else self._partials, N=N, a_in=A_part, b_in=b_part,
                       dn_out=dn_out, **vis)

    def _band_parallel_check(self, specs, n_bands=None):
        """Refuse band-parallel where its C5 all-reduce dwarfs the analysis it
        splits (parallel/policy.py).  ``specs``: this rank's bands; ``n_bands``:
        the date's full band count.  Rank-uniform by construction: bands are
        dealt round-robin, so the ranks of a group can hold different band
        counts and emulators (34 bands over 4 ranks: 9/9/8/8) -- the decision
        uses the full band count and the group-wide largest training set (one
        max all-reduce over the band group), so every rank raises or none does
        (a split decision would leave the others waiting in the band
        all-reduce)."""
        from ..parallel.policy import band_parallel_decision

        self._bp_checked = True
        B = self.band_comm.world
        if n_bands is None:
            n_bands = len(specs) * B
        n_train_local = max([int(getattr(s.emulator, "n_train", 0) or 0) for s in specs] or [0])
        n_train = int(self.band_comm.max_float(float(n_train_local)))
        B_eff, why = band_parallel_decision(self.n_params, int(n_bands), n_train, B, self.device.type,
                                            force=self.config.band_parallel_force)
        if B_eff != B:
            raise ValueError(why + " (set band_parallel_force to run it anyway)")

    def _band_parallel_status(self, status):
        """Combine per-rank band flags (BAD_OP any, NO_OBS all) with the solve flags."""
        N = self.N
        flags = torch.stack([(status & K.ST_BAD_OP) > 0, (status & K.ST_NO_OBS) == 0]).to(torch.int32)
        self.band_comm.all_reduce_(flags, op="max")
        out = self._bp_status & ~torch.tensor(K.ST_NO_OBS, dtype=torch.uint8, device=status.device)
        out = out | torch.where(flags[0] > 0, K.ST_BAD_OP, 0).to(torch.uint8)
        out = out | torch.where(flags[1] > 0, 0, K.ST_NO_OBS).to(torch.uint8)
        return out[:max(N, 1)]

    # --------------------------------------------------- band-sequential
    def _assimilate_sequential(self, step, forecast: KFState) -> AssimilationResult:
        bands = self._device_bands(step)
        total_iter, norms = 0, []
        st = forecast
        for b, band in enumerate(bands):
            cfg = self.config
            old = cfg.min_iterations
            cfg.min_iterations = 1
            try:
                res = self._band_gn_masked(step, band, st)
            finally:
                cfg.min_iterations = old
            st = res.state
            total_iter += res.n_iter
            norms += res.norms
        self.previous_state = Previous_State(step, st.x, None, st.P)
        return AssimilationResult(st, total_iter, norms, None)

    def _band_gn_masked(self, step, band, st):
        """Single band with the masked convergence norm (linear_kf.py:356-425)."""
        spec, db = band
        _, w = db.decode()
        n_valid = self.comm.sum_int(int((w > 0).sum().item()))
        scale = (self.n_params * self.n_total) / max(self.n_params * n_valid, 1)
        old_tol = self.config.convergence_tolerance
        self.config.convergence_tolerance = old_tol / scale
        try:
            res = self.do_all_bands_state(step, [band], st)
        finally:
            self.config.convergence_tolerance = old_tol
        if self.config.hessian_correction is False and spec.kind != OP_PRECOMP and self.N:
            table = build_table([spec], [db], self.n_params, self._cache, self.device)
            K.hessian(self.n_params, table, res.state.x, res.state.P, N=self.N)
        return res

    def assimilate(self, locate_times, x_forecast, P_forecast, P_forecast_inverse, approx_diagonal=True,
                   refine_diag=False, iter_obs_op=False, is_robust=False, diag_str="diag"):
        """Band-sequential assimilation (linear_kf.py:325-354)."""
        st = self.initial_state(x_forecast, P_forecast, P_forecast_inverse)
        for step in locate_times:
            st = self._assimilate_sequential(step, st).state
        x, P = st.to_reference()
        return (x, None, P) if st.kind == PRECISION else (x, P, None)

    def assimilate_band(self, band, timestep, x_forecast, P_forecast, P_forecast_inverse,
                        convergence_tolerance=1e-3, min_iterations=1):
        st = self.initial_state(x_forecast, P_forecast, P_forecast_inverse)
        bands = self._device_bands(timestep)
        res = self._band_gn_masked(timestep, bands[band], st)
        x, P = res.state.to_reference()
        return x, None, P, None

    # ------------------------------------------------- reference shims
    def solver(self, observations, mask, H_matrix, x_forecast, P_forecast, P_forecast_inv, R_mat, the_metadata):
        return variational_kalman(observations, mask, self.state_mask, R_mat, H_matrix, self.n_params, x_forecast,
                                  P_forecast, P_forecast_inv, the_metadata)

    def solver_multiband(self, observations, mask, H_matrix, x0, x_forecast, P_forecast, P_forecast_inv, R_mat,
                         the_metadata):
        return variational_kalman_multiband(observations, mask, self.state_mask, R_mat, H_matrix, self.n_params, x0,
                                            x_forecast, P_forecast, P_forecast_inv, the_metadata)

    # ------------------------------------------------------------ output
    def _dump(self, timestep, state: KFState):
        if self.output is None:
            return
        if getattr(self, "_output_written", None) is state:
            # written by the analysis kernel: bookkeeping only (no device work to time)
            self.output.mark_written(timestep, state, self)
            return
        state.require_full("the output dump")
        with self.timer.phase("output"):
            if hasattr(self.output, "dump_state"):
                self.output.dump_state(timestep, state, self)
                return
            x, P = state.to_reference()
            if state.kind == PRECISION:
                self.output.dump_data(timestep, x, None, P, self.partition.local_mask, self.n_params)
            else:
                prec = self._as_kind(state, PRECISION)
                self.output.dump_data(timestep, x, P, prec.to_reference()[1], self.partition.local_mask,
                                      self.n_params)

    def unc(self, state: KFState) -> torch.Tensor:
        """1/sqrt(diag(P^-1)) per parameter, [n_p, N] (observations.py:392-393)."""
        prec = self._as_kind(state, PRECISION)
        prec.require_full("unc")
        idx = [tri_pos(self.n_params, j, j) for j in range(self.n_params)]
        return 1.0 / torch.sqrt(prec.P[idx, :self.N])
