"""Metrics and timers.

* ``MetricsLogger`` — structured JSONL per date / timestep (GN iterations,
  convergence norms, per-phase ms, wall time, pixel updates/s, per-pixel status
  counts, ingest bytes), one file per rank, plus a rank-0 summary aggregated
  over the ranks (``LinearKalman.metrics_summary``).
* ``PhaseTimer`` — hipEvent-based per-phase timing on the compute stream
  (native event pool); host clock on CPU.  Non-synchronising by default: the
  event pairs are resolved lazily in ``snapshot()``.
"""
from __future__ import annotations

import contextlib
import json
import os
import time
from collections import defaultdict

import torch


class MetricsLogger:
    def __init__(self, path=None, rank: int = 0):
        self.path = None
        self.records = []
        if path:
            root, ext = os.path.splitext(str(path))
            self.path = f"{root}.rank{rank}{ext or '.jsonl'}" if rank else str(path)
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
        self.rank = rank

    @property
    def enabled(self) -> bool:
        return self.path is not None

    def write_summary(self, summary: dict):
        if self.path:
            root, _ = os.path.splitext(self.path)
            with open(root + ".summary.json", "w") as f:
                json.dump(summary, f, indent=1, default=str)

    def log(self, rec: dict):
        rec = {"rank": self.rank, "t": time.time(), **rec}
        self.records.append(rec)
        if self.path:
            with open(self.path, "a") as f:
                f.write(json.dumps(rec, default=str) + "\n")


_NULL = contextlib.nullcontext()


class PhaseTimer:
    """``enabled=False`` makes ``phase()`` a shared null context: nothing reads
    the totals unless metrics or phase timing are on.  On the GPU each phase
    edge is one call into the native event pool (``PhaseEvents``,
    ``csrc/kf_stream.cpp``): hipEvent pairs recorded on the current stream and
    resolved in completion order."""

    def __init__(self, device, sync: bool = False, enabled: bool = True):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.sync = sync
        self.enabled = bool(enabled or sync)
        self._ids = {}                         # phase name -> id in the native pool
        self._names = []
        self._ev = None
        if self.cuda and self.enabled:
            from ..ops import _ext
            from ..ops.kernels import current_raw_stream

            self._ev = _ext.require_ext().PhaseEvents()
            self._cur = current_raw_stream
        self.totals = defaultdict(float)
        self.run_totals = defaultdict(float)   # over the whole run (snapshots reset `totals`)

    def phase(self, name: str):
        if not self.enabled:
            return _NULL
        return self._phase(name)

    @contextlib.contextmanager
    def _phase(self, name: str):
        if self.cuda:
            pid = self._ids.get(name)
            if pid is None:
                pid = self._ids[name] = len(self._names)
                self._names.append(name)
            stream = self._cur(self.device)
            token = self._ev.begin(pid, stream)
            try:
                yield
            finally:
                self._ev.end(token, stream)
                if self.sync:
                    self._absorb(self._ev.collect(True))
                elif self._ev.pending > 64:
                    self._absorb(self._ev.collect(False))   # recycle finished pairs
        else:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self.totals[name] += 1e3 * (time.perf_counter() - t0)

    def _absorb(self, done):
        for pid, ms in done:
            self.totals[self._names[pid]] += ms

    def cumulative(self) -> dict:
        """Per-phase ms over the whole run (pending events included)."""
        cur = self.snapshot(reset=True)
        del cur
        return {k: round(v, 3) for k, v in self.run_totals.items()}

    def snapshot(self, reset: bool = True, block: bool = True) -> dict:
        """Phase totals since the last snapshot.  ``block=False`` accounts only
        the phases that have finished (no host wait: a per-date wait would
        serialise the host's next date behind the device's work when nothing
        else waits, e.g. statically converged linear operators); the rest are
        counted by a later snapshot, so run totals stay exact."""
        if self._ev is not None and self._ev.pending:
            self._absorb(self._ev.collect(bool(block)))
        out = {k: round(v, 3) for k, v in self.totals.items()}
        if reset:
            for k, v in self.totals.items():
                self.run_totals[k] += v
            self.totals = defaultdict(float)
        return out
