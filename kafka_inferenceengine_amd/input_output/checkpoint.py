"""State/covariance checkpoint format and resume.

The reference has no resume: its GeoTIFFs keep only the mean and
1/sqrt(diag(P^-1)), losing the off-diagonal precision.  A checkpoint here is
one directory per timestep with, per rank:

  ``manifest.json``            format/version, n_params, parameter names, raster
                               shape, strip rows, timestep (ISO), kind, dtype,
                               world size, state_mask bitmap file
  ``state.rank{r}.x.f32``      x   as SoA [n_p, N_r]            (raw little-endian)
  ``state.rank{r}.P.f32``      P   packed upper triangle [ntri, N_r]
  ``state_mask.u8``            packed bits of the global state mask (rank 0)

Loading re-partitions if the world size differs (rank r reads the global
pixel range it owns under the new partition from the per-rank files).
"""
from __future__ import annotations

import datetime as dt
import json
import os
from pathlib import Path

import numpy as np
import torch

from ..engine.state import KFState
from ..utils.blocks import ntri

FORMAT = "kafka-amd-state"
VERSION = 1


class CheckpointWriteError(IOError):
    """A rank failed to write its checkpoint files; nothing was committed."""


class CheckpointManager:
    def __init__(self, root, engine):
        self.root = Path(root)
        self.engine = engine
        self.root.mkdir(parents=True, exist_ok=True)
        self._side = None       # D2H side stream
        self._pinned = None     # reused pinned host buffers (x, P)
        self._thread = None     # background file writer
        self._pending = None    # (dir, timestep, kind) awaiting commit
        self._err = None        # exception raised by the pending checkpoint's writer
        self.last_enqueue_s = 0.0
        self.last_commit_wait_s = 0.0
        self.stats = {"enqueue_s": [], "write_s": [], "commit_wait_s": [], "bytes": []}

    def path_for(self, timestep) -> Path:
        return self.root / timestep.strftime("A%Y%j")

    def save(self, timestep, state: KFState, block: bool = False) -> Path:
        """Checkpoint ``state`` at ``timestep``.  Device states are snapshotted
        with one device-to-device copy on the compute stream (milliseconds), then
        copied to reused pinned host buffers on a side stream and written by a
        background thread, so the next time step runs under the write.  The
        checkpoint is committed (barrier, rank 0 writes ``manifest.json``,
        barrier) by the next ``save`` or by :meth:`finish`; ``latest`` only sees
        committed checkpoints.  With band-parallel groups only band slot 0 of
        each strip writes (every member holds the same state)."""
        if hasattr(state, "require_full"):
            state.require_full("a checkpoint")
        import threading
        import time

        self.finish()
        e = self.engine
        d = self.path_for(timestep)
        t0 = time.perf_counter()
        writer = e.band_comm is None or e.band_comm.rank == 0
        if writer:
            d.mkdir(parents=True, exist_ok=True)
            r = e.comm.rank
            N = state.N
            if state.x.is_cuda:
                cur = torch.cuda.current_stream(state.x.device)
                snap = (state.x[:, :N].clone(), state.P[:, :N].clone())   # compute stream, HBM copy
                if self._side is None:
                    self._side = torch.cuda.Stream(state.x.device)
                if self._pinned is None or any(p.shape != s.shape for p, s in zip(self._pinned, snap)):
                    self._pinned = tuple(torch.empty(s.shape, dtype=s.dtype, pin_memory=True) for s in snap)
                ev = torch.cuda.Event()
                self._side.wait_stream(cur)
                with torch.cuda.stream(self._side):
                    for h, s in zip(self._pinned, snap):
                        h.copy_(s, non_blocking=True)
                    ev.record(self._side)
                host = self._pinned
            else:
                snap, ev = None, None
                host = (state.x[:, :N].detach().clone(), state.P[:, :N].detach().clone())

            def write(host=host, ev=ev, snap=snap):
                # any failure (disk full, EIO, fsync, the native writer) is kept
                # for finish(), which refuses to commit on every rank: an
                # exception left on this thread would only be printed and the
                # manifest of a checkpoint with missing files committed
                try:
                    t1 = time.perf_counter()
                    if ev is not None:
                        ev.synchronize()
                    nbytes = 0
                    for tag, h in zip(("x", "P"), host):
                        a = np.ascontiguousarray(h.numpy(), dtype="<f4")
                        _atomic_write(d / f"state.rank{r}.{tag}.f32", a)
                        nbytes += a.nbytes
                    if r == 0:
                        _atomic_write(d / "state_mask.u8", np.packbits(e.partition.state_mask.ravel()).tobytes())
                    self.stats["write_s"].append(time.perf_counter() - t1)
                    self.stats["bytes"].append(nbytes)
                except BaseException as exc:   # noqa: BLE001 -- re-raised by finish()
                    self._err = exc
                finally:
                    del snap

            if block or snap is None:
                write()
            else:
                self._thread = threading.Thread(target=write, name="kafka-ckpt", daemon=True)
                self._thread.start()
        self._pending = (d, timestep, state.kind)
        self.last_enqueue_s = time.perf_counter() - t0
        self.stats["enqueue_s"].append(self.last_enqueue_s)
        if block:
            self.finish()
        return d

    def finish(self):
        """Wait for the pending checkpoint's files and commit its manifest."""
        if self._pending is None:
            return
        import time

        t0 = time.perf_counter()
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        d, timestep, kind = self._pending
        self._pending = None
        err, self._err = self._err, None
        e = self.engine
        part = e.partition
        # commit only when every rank's files are complete: one failed writer
        # leaves the checkpoint uncommitted everywhere (no manifest, no prune of
        # the older good checkpoints) and raises on every rank
        n_failed = e.comm.sum_int(1 if err is not None else 0)
        if n_failed:
            self.last_commit_wait_s = time.perf_counter() - t0
            raise CheckpointWriteError(f"checkpoint {d} not committed: {n_failed} rank(s) failed to write"
                                       + (f" (this rank: {err!r})" if err is not None else "")) from err
        e.comm.barrier()
        if e.comm.rank == 0 and (e.band_comm is None or e.band_comm.rank == 0):
            man = {"format": FORMAT, "version": VERSION, "n_params": e.n_params,
                   "parameters": e.parameters_list, "shape": list(part.shape), "timestep": timestep.isoformat(),
                   "kind": kind, "dtype": "float32", "world": e.comm.world, "bounds": part.bounds,
                   "counts": part.counts, "layout": {"x": "soa[n_p,N]", "P": "packed_upper_rowmajor[ntri,N]"}}
            _atomic_write(d / "manifest.json", json.dumps(man, indent=1).encode())
            self._prune(int(getattr(e.config, "checkpoint_keep", 0) or 0))
        e.comm.barrier()
        self.last_commit_wait_s = time.perf_counter() - t0
        self.stats["commit_wait_s"].append(self.last_commit_wait_s)

    def _prune(self, keep: int):
        """Delete committed checkpoints older than the newest ``keep`` (rank 0,
        after the commit: a crash in between leaves one extra, never none)."""
        if keep <= 0:
            return
        import shutil
        done = sorted(p for p in self.root.glob("A*") if (p / "manifest.json").exists())
        for old in done[:-keep]:
            (old / "manifest.json").unlink()          # uncommit first: `latest` never sees a partial one
            shutil.rmtree(old, ignore_errors=True)

    @staticmethod
    def read_manifest(path) -> dict:
        with open(Path(path) / "manifest.json") as f:
            man = json.load(f)
        if man.get("format") != FORMAT or man.get("version") != VERSION:
            raise ValueError(f"not a {FORMAT} v{VERSION} checkpoint: {path}")
        return man

    @staticmethod
    def load(path, engine):
        """-> (KFState on this rank, timestep datetime)."""
        path = Path(path)
        man = CheckpointManager.read_manifest(path)
        n = int(man["n_params"])
        if n != engine.n_params:
            raise ValueError("checkpoint n_params differs from the engine")
        mask = np.unpackbits(np.frombuffer((path / "state_mask.u8").read_bytes(), dtype=np.uint8))
        mask = mask[:int(np.prod(man["shape"]))].reshape(man["shape"]).astype(bool)
        if not np.array_equal(mask, engine.partition.state_mask):
            raise ValueError("checkpoint state_mask differs from the engine's")
        nt = ntri(n)
        counts = man["counts"]
        offs = np.concatenate([[0], np.cumsum(counts)])
        lo, hi = engine.partition.offset, engine.partition.offset + engine.partition.N
        xs, Ps = [], []
        for r, (a, b) in enumerate(zip(offs[:-1], offs[1:])):
            s, t = max(a, lo), min(b, hi)
            if s >= t:
                continue
            Nr = int(b - a)
            x = np.fromfile(path / f"state.rank{r}.x.f32", dtype="<f4").reshape(n, Nr)
            P = np.fromfile(path / f"state.rank{r}.P.f32", dtype="<f4").reshape(nt, Nr)
            xs.append(x[:, s - a:t - a])
            Ps.append(P[:, s - a:t - a])
        x = np.concatenate(xs, 1) if xs else np.zeros((n, 0), "<f4")
        P = np.concatenate(Ps, 1) if Ps else np.zeros((nt, 0), "<f4")
        dev = engine.device
        st = KFState(torch.from_numpy(np.ascontiguousarray(x)).to(dev), torch.from_numpy(np.ascontiguousarray(P)).to(dev),
                     man["kind"], x.shape[1])
        st = engine._as_kind(st, engine._analysis_kind())
        return st, dt.datetime.fromisoformat(man["timestep"])

    @staticmethod
    def resolve(path) -> Path:
        """A checkpoint directory from ``path``: a ``manifest.json`` file (its
        directory), a checkpoint directory, or a checkpoint root (its latest
        committed checkpoint).  Raises FileNotFoundError when there is none."""
        p = Path(path)
        if p.is_file() and p.name == "manifest.json":
            return p.parent
        if (p / "manifest.json").is_file():
            return p
        last = CheckpointManager.latest(p) if p.is_dir() else None
        if last is None:
            raise FileNotFoundError(f"no committed checkpoint (manifest.json) at or under {path}")
        return last

    @staticmethod
    def latest(root):
        root = Path(root)
        cands = sorted(p for p in root.glob("A*") if (p / "manifest.json").exists())
        return cands[-1] if cands else None


def _atomic_write(path: Path, data):
    """Write ``data`` (bytes or a contiguous array) to ``path`` via a fsynced
    tmp file; arrays of 64 MiB and more go through the native parallel writer
    (``write_raw`` in csrc/kf_tiff.cpp)."""
    tmp = path.with_suffix(path.suffix + ".tmp")
    E = None
    if isinstance(data, np.ndarray) and data.nbytes >= (64 << 20):
        from .tiff import _native, _threads
        E = _native()
    if E is not None:
        E.write_raw(str(tmp), data.ctypes.data, int(data.nbytes), _threads(), True)
    else:
        with open(tmp, "wb") as f:
            f.write(data)
            f.flush()
            os.fsync(f.fileno())
    os.replace(tmp, path)
