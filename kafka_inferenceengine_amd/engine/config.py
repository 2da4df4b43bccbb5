"""EngineConfig: every hard-coded constant of the reference as a named default.

Reference constants: GN tolerance 1e-3, min iterations 2,
bail-out after 25 (``linear_kf.py:246-247,297-304``); S2 uncertainty 5 %
(``Sentinel2_Observations.py:174``), scale 1e-4 (:169); BHR 5 %/7 %, floor
2.5e-3 (``observations.py:301-302``).
"""
from __future__ import annotations

import argparse
import dataclasses
from dataclasses import dataclass, field

import yaml


@dataclass
class EngineConfig:
    # Gauss-Newton loop (linear_kf.py:245-307)
    convergence_tolerance: float = 1e-3
    min_iterations: int = 2
    max_iterations: int = 25
    # per-chunk exit test (reference driver semantics, engine/chunks.py): [x size,
    # y size] of get_chunks tiles (kafka_test_Py36.py:241: 256^2; kafka_test_S2.py:202:
    # 128^2) whose ||dx|| / len(x) is tested on its own, converged chunks frozen;
    # None: one test over the whole tile / strip set (the norm of one filter)
    convergence_chunk: list | None = None
    # per-chunk loop past the first decision that keeps chunks iterating: up to
    # this many further iterations are queued before their exit decisions are
    # read (each launch reads its pixel count on the device; the launches past
    # the real end visit nothing), so the host's read-back leaves the
    # critical path of long tails (prosail10_hard: up to 26 iterations).  0: read
    # every decision before the next launch
    gn_lookahead: int = 2
    # analysis precision stored per date: "auto" keeps what the next forecast
    # reads (LAI propagator: the TLAI diagonal; prior reset: nothing) unless a
    # checkpoint is due, the date is the run's last, the output is not fused or
    # another consumer needs it; "always": every packed row, every date
    store_precision: str = "auto"
    # keep a per-pixel record of every date's ST_OUT_OF_DOMAIN (LinearKalman.
    # ood_history): a state that left an emulator's domain carries the
    # extrapolation forward through the propagated parameters (one uint8 OR per date)
    domain_history: bool = False
    # analysis
    analysis_form: str = "information"        # 'information' (K1) | 'gain' (K1g)
    joseph: bool = False                      # Joseph-form covariance update (gain form)
    hessian_correction: bool = False          # K6 after convergence (off: linear_kf.py:313-319)
    reference_quirks: bool = False            # swapped prior blend (kf_tools.py:90)
    band_sequential: bool = False             # legacy per-band assimilation (linear_kf.py:325-425)
    # spatial regulariser (new capability, off by default => reference results)
    spatial_gamma: float = 0.0
    spatial_params: list | None = None        # parameter indices smoothed (None: all)
    # coupled GMRF solve per Gauss-Newton iteration: "chebyshev" (Chebyshev-
    # accelerated block Jacobi, sweeps chosen from a Gershgorin bound of the
    # Jacobi spectral radius to cut the error by spatial_tol) or "jacobi"
    # (exactly jacobi_sweeps plain sweeps, the round-2 smoother)
    spatial_solver: str = "chebyshev"
    spatial_tol: float = 1e-3
    # inexact Newton: a Gauss-Newton iteration that cannot end the loop
    # (n_iter < min_iterations) only needs a linearisation point, so its coupled
    # solve stops at this looser tolerance (the final iteration uses spatial_tol)
    spatial_tol_first: float = 1e-1
    # with fuse_gn: the first Gauss-Newton iteration (which only supplies the
    # second's linearisation point) is the plain per-pixel solve, fused into
    # the launch that prepares the regularised second iteration -- one analysis
    # pass and no coupled solve saved per date (False: both iterations coupled,
    # the first to spatial_tol_first)
    spatial_first_plain: bool = True
    # visit the pixels with an observation first (obs_order): cloudy pixels then
    # fill whole waves that skip the GP emulator (the reference runs it on the
    # observed pixels only); each pixel's analysis is unchanged
    observed_first: bool = True
    # one global partition (default) or each 4096-pixel chunk in place (True,
    # A/B: +2.5 % tip7, +7.6 % prosail10, r4_v31 -- the grid stride is a whole
    # number of chunks, so a wave meets the same in-chunk position, and class,
    # on every sweep: waves of only observed pixels set the kernel's length)
    observed_first_local: bool = False
    spatial_max_sweeps: int = 64
    # one field on a dense strip without halo rows (one rank, or no strip
    # neighbours): up to 8 sweeps per launch out of LDS (kf_reg_tiled.hip),
    # bit-identical to one launch per sweep
    spatial_tiled: bool = True
    jacobi_sweeps: int = 4
    # GP operator placement: fused into the analysis kernel, or "split" (high-
    # occupancy operator kernel -> HBM -> analysis over band chunks)
    gp_split: str = "auto"                    # 'auto' | 'always' | 'never'
    # auto: split when a GP band has >= gp_split_min_d inputs or a date has >= gp_split_min_bands
    # GP bands.  Measured (profiles/r1_v8_split_vs_fused.log, compact records): PROSAIL 10 bands
    # x D=10 fused 300 ms vs split 306 ms/step; 34 bands split (one chunk) 133 vs fused 142 ms.
    # On a GPU, full-state GP bands with matrix-core tables (D = n_params in 7, 10) stay fused
    # under 'auto' at any band count (global-table kernel: 34 bands 631 vs 1064 ms/step split).
    gp_split_min_d: int = 99
    gp_split_min_bands: int = 13
    band_chunk: int = 0                       # bands per split chunk; 0 = as many as fit in half the free HBM
    # band-parallel (TP-like) decomposition: ranks = strips x band_parallel;
    # the B ranks of a strip split the bands and all-reduce the normal equations
    band_parallel: int = 1
    # band-parallel costs one all-reduce of the per-pixel [A | b] per GN iteration;
    # on a GPU the engine refuses it when that costs > 25 % of the per-rank analysis
    # (parallel/policy.py) unless forced
    band_parallel_force: bool = False
    # runtime
    device: str | None = None                 # 'cuda', 'cuda:1', 'cpu' (default: cuda if present)
    prefetch: bool = True                     # overlap next date's ingest with compute
    lookahead: bool = True                    # prepare the next date's bands under the last GN iteration
    fuse_propagation: bool = True             # evaluate the forecast inside the analysis kernel
    fuse_gn: bool = True                      # GN iterations 1 and 2 in one launch (iteration 1 can never
                                              # end the loop, linear_kf.py:297-304); plain fused path only
    fuse_output: bool = True                  # device outputs written by the final analysis iteration
    line_tables: bool = True                  # first GN iteration at a fused partial-reset forecast from
                                              # float64 cubic line tables instead of the GP sums (the
                                              # forecast varies in one parameter only; models/gp.py)
    return_innovations: bool = False
    metrics_path: str | None = None           # JSONL metrics (per date / timestep)
    checkpoint_dir: str | None = None
    checkpoint_every: int = 0                 # timesteps between checkpoints (0: off)
    checkpoint_keep: int = 0                  # committed checkpoints kept (older ones pruned; 0: all)
    gc_freeze: bool = True                    # run(): move setup objects to the permanent GC generation
    comm_timeout_s: float = 600.0
    phase_timing: bool = False                # per-phase hipEvent timers without metrics_path
    sync_timing: bool = False                 # device-synchronising per-phase timers
    extra: dict = field(default_factory=dict)

    def validate(self):
        if self.analysis_form not in ("information", "gain"):
            raise ValueError("analysis_form must be 'information' or 'gain'")
        if self.spatial_gamma < 0:
            raise ValueError("spatial_gamma must be >= 0")
        if self.spatial_solver not in ("chebyshev", "jacobi"):
            raise ValueError("spatial_solver must be 'chebyshev' or 'jacobi'")
        if not 0 < self.spatial_tol < 1 or not 0 < self.spatial_tol_first < 1 or self.spatial_max_sweeps < 1:
            raise ValueError("spatial_tol must be in (0, 1) and spatial_max_sweeps >= 1")
        if self.spatial_gamma > 0 and self.analysis_form != "information":
            raise ValueError("the spatial regulariser runs in information form")
        if self.band_parallel < 1:
            raise ValueError("band_parallel must be >= 1")
        if self.min_iterations < 1 or self.max_iterations < self.min_iterations:
            raise ValueError("bad iteration limits")
        if int(self.gn_lookahead) < 0:
            raise ValueError("gn_lookahead must be >= 0")
        self.gn_lookahead = int(self.gn_lookahead)
        if self.store_precision not in ("auto", "always"):
            raise ValueError("store_precision must be 'auto' or 'always'")
        if isinstance(self.convergence_chunk, str) and self.convergence_chunk.strip().lower() in ("", "0", "tile",
                                                                                                 "none", "off"):
            self.convergence_chunk = None      # the exit test over the engine's whole state
        if self.convergence_chunk is not None:
            cc = self.convergence_chunk
            if isinstance(cc, (int, float)):
                cc = [int(cc), int(cc)]
            if isinstance(cc, str):
                cc = [int(v) for v in cc.replace("x", ",").split(",")]
            cc = [int(v) for v in cc]
            if len(cc) == 1:
                cc = cc * 2
            if len(cc) != 2 or min(cc) < 1:
                raise ValueError("convergence_chunk must be [x size, y size] >= 1 (or one size)")
            self.convergence_chunk = cc
            if self.spatial_gamma > 0:
                raise ValueError("convergence_chunk runs without the spatial prior (which couples the chunks)")
        return self

    # ------------------------------------------------------------- IO
    @classmethod
    def from_dict(cls, d: dict) -> "EngineConfig":
        names = {f.name for f in dataclasses.fields(cls)}
        known = {k: v for k, v in (d or {}).items() if k in names}
        extra = {k: v for k, v in (d or {}).items() if k not in names}
        cfg = cls(**known)
        cfg.extra.update(extra)
        return cfg.validate()

    @classmethod
    def from_yaml(cls, path) -> "EngineConfig":
        with open(path) as f:
            return cls.from_dict(yaml.safe_load(f) or {})

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)

    @classmethod
    def add_arguments(cls, ap: argparse.ArgumentParser):
        for f in dataclasses.fields(cls):
            if f.name == "extra":
                continue
            flag = "--" + f.name.replace("_", "-")
            if f.type in ("bool", bool):
                ap.add_argument(flag, dest=f.name, action=argparse.BooleanOptionalAction, default=None)
            elif f.type in ("int", int):
                ap.add_argument(flag, dest=f.name, type=int, default=None)
            elif f.type in ("float", float):
                ap.add_argument(flag, dest=f.name, type=float, default=None)
            else:
                ap.add_argument(flag, dest=f.name, default=None)
        ap.add_argument("--config", dest="config_file", default=None, help="YAML EngineConfig")
        return ap

    @classmethod
    def from_args(cls, ns) -> "EngineConfig":
        base = cls.from_yaml(ns.config_file).to_dict() if getattr(ns, "config_file", None) else {}
        for f in dataclasses.fields(cls):
            v = getattr(ns, f.name, None)
            if v is not None:
                base[f.name] = v
        if base.get("spatial_params") and isinstance(base["spatial_params"], str):
            base["spatial_params"] = [int(s) for s in base["spatial_params"].split(",")]
        return cls.from_dict(base)
