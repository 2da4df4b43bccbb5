"""Metrics and timers.

* ``MetricsLogger`` — structured JSONL per date / timestep (GN iterations,
  convergence norms, per-phase ms, wall time, pixel updates/s, per-pixel status
  counts, ingest bytes), one file per rank, plus a rank-0 summary aggregated
  over the ranks (``LinearKalman.metrics_summary``).
* ``PhaseTimer`` — hipEvent-based (``torch.cuda.Event``) per-phase timing on
  the compute stream; host clock on CPU.  Non-synchronising by default: the
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
    """``enabled=False`` makes ``phase()`` a shared null context: two hipEvent
    records and two stream lookups per phase are ~25 % of the engine's host
    time per step, and nothing reads the totals unless metrics are on."""

    def __init__(self, device, sync: bool = False, enabled: bool = True):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.sync = sync
        self.enabled = bool(enabled or sync)
        self._pending = []
        self._free = []                        # resolved event pairs, re-recorded (no hipEventCreate per phase)
        self.totals = defaultdict(float)
        self.run_totals = defaultdict(float)   # over the whole run (snapshots reset `totals`)

    def phase(self, name: str):
        if not self.enabled:
            return _NULL
        return self._phase(name)

    @contextlib.contextmanager
    def _phase(self, name: str):
        if self.cuda:
            if not self._free and len(self._pending) > 32:
                self._reap()
            if self._free:
                s, e = self._free.pop()
            else:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            # one stream lookup per phase (Event.record() without a stream looks
            # the current one up again)
            cur = torch.cuda.current_stream(self.device)
            s.record(cur)
            try:
                yield
            finally:
                e.record(cur)
                self._pending.append((name, s, e))
                if self.sync:
                    e.synchronize()
        else:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self.totals[name] += 1e3 * (time.perf_counter() - t0)

    def _reap(self):
        """Account the oldest pending phases whose end event has completed
        (non-blocking query) and recycle their event pairs."""
        done = 0
        while done < len(self._pending) and done < 32 and self._pending[done][2].query():
            name, s, e = self._pending[done]
            self.totals[name] += s.elapsed_time(e)
            self._free.append((s, e))
            done += 1
        del self._pending[:done]

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
        if self._pending and not block:
            done = 0
            while done < len(self._pending) and self._pending[done][2].query():
                name, s, e = self._pending[done]
                self.totals[name] += s.elapsed_time(e)
                self._free.append((s, e))
                done += 1
            del self._pending[:done]
        elif self._pending:
            self._pending[-1][2].synchronize()
            for name, s, e in self._pending:
                self.totals[name] += s.elapsed_time(e)
                self._free.append((s, e))
            self._pending = []
        out = {k: round(v, 3) for k, v in self.totals.items()}
        if reset:
            for k, v in self.totals.items():
                self.run_totals[k] += v
            self.totals = defaultdict(float)
        return out
