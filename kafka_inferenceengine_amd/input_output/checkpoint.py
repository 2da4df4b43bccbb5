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


class CheckpointManager:
    def __init__(self, root, engine):
        self.root = Path(root)
        self.engine = engine
        self.root.mkdir(parents=True, exist_ok=True)

    def path_for(self, timestep) -> Path:
        return self.root / timestep.strftime("A%Y%j")

    def save(self, timestep, state: KFState) -> Path:
        e = self.engine
        part = e.partition
        d = self.path_for(timestep)
        d.mkdir(parents=True, exist_ok=True)
        r = e.comm.rank
        x = state.x[:, :state.N].detach().cpu().numpy().astype("<f4")
        P = state.P[:, :state.N].detach().cpu().numpy().astype("<f4")
        _atomic_write(d / f"state.rank{r}.x.f32", x.tobytes())
        _atomic_write(d / f"state.rank{r}.P.f32", P.tobytes())
        if r == 0:
            _atomic_write(d / "state_mask.u8", np.packbits(part.state_mask.ravel()).tobytes())
        e.comm.barrier()
        if r == 0:
            man = {"format": FORMAT, "version": VERSION, "n_params": e.n_params,
                   "parameters": e.parameters_list, "shape": list(part.shape), "timestep": timestep.isoformat(),
                   "kind": state.kind, "dtype": "float32", "world": e.comm.world, "bounds": part.bounds,
                   "counts": part.counts, "layout": {"x": "soa[n_p,N]", "P": "packed_upper_rowmajor[ntri,N]"}}
            _atomic_write(d / "manifest.json", json.dumps(man, indent=1).encode())
        e.comm.barrier()
        return d

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
    def latest(root):
        root = Path(root)
        cands = sorted(p for p in root.glob("A*") if (p / "manifest.json").exists())
        return cands[-1] if cands else None


def _atomic_write(path: Path, data: bytes):
    tmp = path.with_suffix(path.suffix + ".tmp")
    with open(tmp, "wb") as f:
        f.write(data)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)
