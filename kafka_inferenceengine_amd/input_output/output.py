"""Output writers (plug-in point L1: ``dump_data`` / device ``dump_state``).

* ``KafkaOutput`` — per parameter and timestep a Float32 GeoTIFF of the mean
  and one of 1/sqrt(diag(P^-1)) (the conditional std), file names
  ``{param}_A%Y%j[_{prefix}].tif`` / ``..._unc.tif`` (``observations.py:338-394``).
  Rasters are produced on the device by the unpack kernel and written by a
  background thread.
* ``KafkaOutputMemory`` — in-memory dict {timestep: {param: values}}
  (``kafka_test.py:135-145``; fixed to accept the engine's 6 arguments).
* ``DeviceOutput`` — keeps the latest mean/unc rasters on the device
  (the benchmark's writer: no host traffic in the timed loop).
"""
from __future__ import annotations

import os
import threading
import time
from queue import Queue

import numpy as np
import torch

from ..ops import kernels as K
from .tiff import write_tiff


def _fname(folder, param, timestep, prefix, suffix=""):
    core = f"{param}_{timestep.strftime('A%Y%j')}"
    if prefix is not None:
        core += f"_{prefix}"
    return os.path.join(folder, core + suffix + ".tif")


class _Writer:
    """One background thread draining a bounded job queue.  Telemetry:
    ``depth`` (jobs queued or running, sampled at each submit), ``wait_s``
    (seconds the producer -- the engine's host thread -- blocked on a full
    queue) and ``busy_s`` (seconds the thread spent in jobs)."""

    def __init__(self, maxsize: int = 4):
        self.q = Queue(maxsize=maxsize)
        self.err = None
        self.depth = []
        self.wait_s = 0.0
        self.busy_s = 0.0
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def _run(self):
        while True:
            job = self.q.get()
            if job is None:
                return
            t0 = time.perf_counter()
            try:
                job()
            except Exception as e:  # surfaced on flush()
                self.err = e
            finally:
                self.busy_s += time.perf_counter() - t0
                self.q.task_done()

    def submit(self, job):
        if self.err:
            raise self.err
        self.depth.append(self.q.unfinished_tasks)
        t0 = time.perf_counter()
        self.q.put(job)
        self.wait_s += time.perf_counter() - t0

    def flush(self):
        self.q.join()
        if self.err:
            raise self.err


def _device_rasters(state, engine, mean=True, unc=True):   # host copies (tests / tools)
    """(mean, unc) as [n_p, H_strip, W] float32 CPU arrays (inactive = 0)."""
    part = engine.partition
    n = engine.n_params
    H, W = part.strip_shape
    dev = state.x.device
    prec = engine._as_kind(state, "precision")
    m = torch.zeros((n, H * W), dtype=torch.float32, device=dev) if mean else None
    u = torch.zeros((n, H * W), dtype=torch.float32, device=dev) if unc else None
    idx = torch.from_numpy(part.local_idx).to(dev)
    if state.N:
        K.unpack(n, prec.x, prec.P, m, u, idx=idx, N=state.N)
    return (None if m is None else m.view(n, H, W).cpu().numpy(),
            None if u is None else u.view(n, H, W).cpu().numpy())


class KafkaOutput:
    """GeoTIFF writer (``observations.py:338-394``): per parameter and timestep a
    Float32 raster of the mean and one of 1/sqrt(diag(P^-1)).

    Device path: the final Gauss-Newton iteration writes the mean / unc rasters
    straight into device planes (``device_targets``, fused output); the planes
    go to pinned host memory by an async copy on a side stream, and a writer
    thread encodes tiled DEFLATE GeoTIFFs with the native parallel encoder
    (``csrc/kf_tiff.cpp``, EPSG GeoKeys from ``projection``) while the next
    timesteps run.  ``level`` trades size for speed; ``predictor=3,
    strategy="rle"`` (floating-point predictor, run-length zlib) encodes about
    3x faster than level 6 at a similar ratio.
    With ``gather=True`` and several ranks, strips are gathered to rank 0
    (C3, ``Comm.gather_to_root``) and written as one raster; otherwise every
    rank writes its strip with a per-rank prefix and a shifted geotransform.

    ``encoder``: "device" encodes the DEFLATE tiles on the GPU
    (``ops.kernels.TileEncoder``, csrc/kf_deflate.hip: predictor 3 and one
    fixed-Huffman zlib stream per 256 x 256 tile) on the side stream, so only
    the compressed tiles cross PCIe and the writer thread only writes files;
    "host" sends the raw planes to the native CPU encoder (``level``,
    ``strategy``, ``predictor``); "auto" (default): device for GPU planes with
    DEFLATE output in 256-pixel tiles."""

    def __init__(self, parameter_list, geotransform, projection, folder, prefix=None, fmt="GTiff",
                 compress="deflate", asynchronous=True, level: int = 6, tile: int = 256, gather: bool = False,
                 threads: int | None = None, predictor: int = 1, strategy: str | None = None,
                 keep_timesteps: int | None = None, encoder: str = "auto"):
        if encoder not in ("auto", "device", "host"):
            raise ValueError("encoder must be 'auto', 'device' or 'host'")
        self.encoder = encoder
        self._enc = None          # ops.kernels.TileEncoder (device encoder)
        self._copier = None       # device encoder: the thread bringing compressed tiles to pinned memory
        self._eslots = []         # device encoder: ring of 2 (packed device buffer, meta pinned, host pinned, done)
        self.geotransform = geotransform
        self.projection = projection
        self.folder = folder
        self.fmt = fmt
        self.parameter_list = list(parameter_list)
        self.prefix = prefix
        self.compress = compress
        self.level = int(level)
        self.tile = int(tile)
        self.gather = bool(gather)
        self.threads = threads
        self.predictor = int(predictor)
        self.strategy = strategy
        # rolling local buffer: keep only the newest ``keep_timesteps`` timesteps'
        # files on disk (a node that ships granules elsewhere; benchmarks)
        self.keep_timesteps = keep_timesteps
        self._by_step = []
        os.makedirs(folder, exist_ok=True)
        self._w = _Writer() if asynchronous else None
        self._dev = None          # DeviceOutput: device planes the analysis kernel writes
        self._host = []           # pinned host planes in flight (ring of 2)
        self._stream = None
        self.written = []
        self.write_s = []         # per timestep: encode + write wall seconds (writer thread)
        self.bytes_in = self.bytes_out = 0
        self.prune_s = 0.0        # keep_timesteps: removing the older timesteps' files
        self.slot_wait_s = 0.0    # engine thread blocked on a pinned slot still being written
        self.d2h_s = 0.0          # writer thread waiting for the planes' device->host copy

    def _geo(self, engine=None):
        gt = list(self.geotransform) if self.geotransform is not None else None
        if gt is not None and engine is not None and engine.partition.r0 and not self._gathering(engine):
            gt[3] = gt[3] + engine.partition.r0 * gt[5]
        return gt

    def _gathering(self, engine) -> bool:
        return self.gather and engine is not None and engine.comm.world > 1

    def _prefix(self, engine):
        if engine is not None and engine.comm.world > 1 and not self._gathering(engine):
            return f"{self.prefix}_r{engine.comm.rank}" if self.prefix is not None else f"r{engine.comm.rank}"
        return self.prefix

    def _write_all(self, timestep, mean, unc, gt, prefix):
        t0 = time.perf_counter()
        names = []
        for planes, suffix in ((mean, ""), (unc, "_unc")):
            for ii, param in enumerate(self.parameter_list):
                fn = _fname(self.folder, param, timestep, prefix, suffix)
                write_tiff(fn, planes[ii], gt, self.projection, self.compress, level=self.level, tile=self.tile,
                           threads=self.threads, predictor=self.predictor, strategy=self.strategy)
                self.written.append(fn)
                names.append(fn)
                self.bytes_in += planes[ii].nbytes
                self.bytes_out += os.path.getsize(fn)
        self.write_s.append(time.perf_counter() - t0)
        self._prune(names)

    def _prune(self, names):
        if self.keep_timesteps is not None:
            t1 = time.perf_counter()
            self._by_step.append(names)
            while len(self._by_step) > self.keep_timesteps:
                for fn in self._by_step.pop(0):
                    if os.path.exists(fn):
                        os.remove(fn)
            self.prune_s += time.perf_counter() - t1

    def writer_stats(self) -> dict:
        """Granule output telemetry (per-timestep and cumulative): encode+write
        seconds per timestep, raster bytes in / file bytes out, the writer
        queue's depth at each submit and the seconds the engine blocked on it
        (a full queue, or a pinned host slot still held by its writer job)."""
        w = self._w
        ws = self.write_s
        out = {"timesteps_written": len(ws), "write_s_last": ws[-1] if ws else None,
               "write_s_mean": sum(ws) / len(ws) if ws else None, "write_s_max": max(ws) if ws else None,
               "raster_bytes": self.bytes_in, "file_bytes": self.bytes_out,
               "ratio": round(self.bytes_in / self.bytes_out, 3) if self.bytes_out else None,
               "slot_wait_s": round(self.slot_wait_s, 6), "d2h_s": round(self.d2h_s, 6),
               "prune_s": round(self.prune_s, 6), "deflate_backend": self.deflate_backend()}
        if w is not None:
            out.update({"queue_depth_last": w.depth[-1] if w.depth else 0,
                        "queue_depth_max": max(w.depth) if w.depth else 0,
                        "queue_wait_s": round(w.wait_s, 6), "writer_busy_s": round(w.busy_s, 6)})
        return out

    def deflate_backend(self) -> str | None:
        """Encoder of the DEFLATE tiles: libdeflate (default strategy, when the
        host has it) or zlib (always for the rle / huffman strategies)."""
        if self.compress != "deflate":
            return None
        if self._eslots:
            return "device (fixed-Huffman run-length zlib streams, kf_deflate.hip)"
        from .tiff import _native
        E = _native()
        if E is None or not self.tile:
            return "zlib (python)"
        fast = hasattr(E, "tiff_fast_deflate") and bool(E.tiff_fast_deflate())
        return "libdeflate" if fast and self.strategy in (None, "default") else "zlib"

    # ------------------------------------------------------- device path
    def device_targets(self, engine, dev, alias: bool = True):
        if self._dev is None:
            self._dev = DeviceOutput(self.parameter_list)
        return self._dev.device_targets(engine, dev, alias)

    def mark_written(self, timestep, state, engine):
        self._dev.mark_written(timestep, state, engine)
        self._ship(timestep, engine)

    def dump_state(self, timestep, state, engine):
        if self._dev is None:
            self._dev = DeviceOutput(self.parameter_list)
        self._dev.dump_state(timestep, state, engine)
        self._ship(timestep, engine)

    def _device_encode(self, cuda: bool) -> bool:
        if self.encoder == "host" or not cuda or self.compress != "deflate":
            return False
        ok = self.tile == 256
        if self.encoder == "device" and not ok:
            raise ValueError("the device encoder writes 256-pixel tiles")
        return ok

    def _ship(self, timestep, engine):
        """Device planes -> pinned host (async, side stream) -> writer thread."""
        mean_d, unc_d = self._dev.mean, self._dev.unc
        n, HW = mean_d.shape
        H, W = engine.partition.strip_shape
        gt, pf = self._geo(engine), self._prefix(engine)
        if self._gathering(engine):
            both = torch.cat([mean_d, unc_d], 0)
            rows = [b - a for a, b in engine.partition.bounds]
            full = engine.comm.gather_to_root(both, [r * W for r in rows])
            if engine.comm.rank != 0:
                return
            mean_d, unc_d = full[:n], full[n:]
            H = sum(rows)
        cuda = mean_d.is_cuda
        if self._device_encode(cuda):
            self._ship_encoded(timestep, mean_d, unc_d, n, H, W, gt, pf, release=not self._gathering(engine))
            return
        if cuda and self._stream is None:
            self._stream = torch.cuda.Stream(mean_d.device)
        # ring of two pinned buffer pairs; a pair is reused once its writer job is done
        slot = self._next_slot(n, mean_d.shape[1], cuda)
        hm, hu, done = slot
        done.clear()
        ev = None
        if cuda:
            self._stream.wait_stream(torch.cuda.current_stream(mean_d.device))
            with torch.cuda.stream(self._stream):
                hm.copy_(mean_d, non_blocking=True)
                hu.copy_(unc_d, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self._stream)
            # the planes' next writer waits for this copy (DeviceOutput.release); an
            # aliased mean (the state's x) is not recycled by the allocator before it
            mean_d.record_stream(self._stream)
            if not self._gathering(engine):
                self._dev.release(ev)
        else:
            hm.copy_(mean_d)
            hu.copy_(unc_d)

        def job(hm=hm, hu=hu, ev=ev, done=done):
            try:
                if ev is not None:
                    t0 = time.perf_counter()
                    ev.synchronize()
                    self.d2h_s += time.perf_counter() - t0
                self._write_all(timestep, hm.numpy().reshape(n, H, W), hu.numpy().reshape(n, H, W), gt, pf)
            finally:
                done.set()

        if self._w is not None:
            self._w.submit(job)
        else:
            job()

    def _ship_encoded(self, timestep, mean_d, unc_d, n, H, W, gt, pf, release: bool):
        """Device encoder: both rasters' tiles encoded and packed into one device
        buffer on the side stream, their sizes / offsets to pinned host memory;
        the writer thread then copies exactly the compressed bytes and writes
        the files (no encode on the host)."""
        from ..ops.kernels import TileEncoder
        from ..ops import _ext
        dev = mean_d.device
        if self._stream is None:
            self._stream = torch.cuda.Stream(dev)
        if self._enc is None:
            self._enc = TileEncoder()
        tx, ty = TileEncoder.tiles(H, W)
        per = tx * ty
        nt = n * per
        bound = int(_ext.require_ext().DFL_BOUND)
        # pinned host bytes for the compressed tiles: allocated with the slot (a
        # multi-GB pinned allocation in the writer thread would stall a timed
        # date), sized for the raw planes plus the fixed-Huffman worst case
        host_bytes = int(2 * n * H * W * 4 * 1.13) + 2 * nt * 64 + (1 << 20)
        packed, meta_h, host_box, done = self._next_enc_slot(2 * nt * bound, 4 * nt, dev, host_bytes)
        done.clear()
        self._stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(self._stream):
            _, sm, om = self._enc.encode(mean_d, H, W, packed=packed)
            _, su, ou = self._enc.encode(unc_d, H, W, packed=packed, base=om[-1:] + sm[-1:])
            meta_h.copy_(torch.cat([sm, om, su, ou]), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._stream)
        mean_d.record_stream(self._stream)
        unc_d.record_stream(self._stream)
        if release:
            self._dev.release(ev)
        wstream = self._wstream = getattr(self, "_wstream", None) or torch.cuda.Stream(dev)

        # two stages on two threads: the copier brings date t + 1's compressed
        # tiles to pinned memory while the writer writes date t's files (the
        # slot -- device packed buffer and pinned bytes -- is released after the
        # write; the ring of two keeps the stages one date apart)
        def write(host, m, done=done):
            try:
                self._write_encoded(timestep, host, m, n, per, H, W, gt, pf)
            finally:
                done.set()

        def copy(packed=packed, meta_h=meta_h, host_box=host_box, ev=ev, done=done):
            try:
                t0 = time.perf_counter()
                ev.synchronize()
                m = meta_h.numpy().reshape(4, nt).copy()
                total = int(m[3, -1] + m[2, -1])
                host = host_box[0]
                if host is None or host.numel() < total:
                    host = host_box[0] = torch.empty(int(total * 1.25) + 4096, dtype=torch.uint8, pin_memory=True)
                with torch.cuda.stream(wstream):
                    host[:total].copy_(packed[:total], non_blocking=True)
                wstream.synchronize()
                self.d2h_s += time.perf_counter() - t0
            except BaseException:
                done.set()
                raise
            if self._w is not None:
                self._w.submit(lambda: write(host, m))
            else:
                write(host, m)

        if self._w is not None:
            if self._copier is None:
                self._copier = _Writer()
            self._copier.submit(copy)
        else:
            copy()

    def _write_encoded(self, timestep, host, meta, n, per, H, W, gt, prefix):
        from .tiff import write_tiff_tiles
        t0 = time.perf_counter()
        names = []
        sm, om, su, ou = meta
        for sizes, offs, suffix in ((sm, om, ""), (su, ou, "_unc")):
            for ii, param in enumerate(self.parameter_list):
                fn = _fname(self.folder, param, timestep, prefix, suffix)
                sl = slice(ii * per, (ii + 1) * per)
                write_tiff_tiles(fn, H, W, host, offs[sl], sizes[sl], gt, self.projection, predictor=3,
                                 threads=self.threads)
                self.written.append(fn)
                names.append(fn)
                self.bytes_in += H * W * 4
                self.bytes_out += os.path.getsize(fn)
        self.write_s.append(time.perf_counter() - t0)
        self._prune(names)

    def _next_enc_slot(self, packed_bytes, meta_n, dev, host_bytes):
        if not self._eslots or self._eslots[0][0].numel() < packed_bytes or self._eslots[0][1].numel() != meta_n:
            for sl in self._eslots:
                sl[3].wait()                # a writer job still reading a slot being replaced
            self._eslots = []
            for _ in range(2):
                ev = threading.Event()
                ev.set()
                self._eslots.append((torch.empty(packed_bytes, dtype=torch.uint8, device=dev),
                                     torch.empty(meta_n, dtype=torch.int64, pin_memory=True),
                                     [torch.empty(host_bytes, dtype=torch.uint8, pin_memory=True)], ev))
            self._eturn = 0
        slot = self._eslots[self._eturn % 2]
        self._eturn += 1
        t0 = time.perf_counter()
        slot[3].wait()                      # its previous writer job has copied its tiles out
        self.slot_wait_s += time.perf_counter() - t0
        return slot

    def _next_slot(self, n, cols, cuda):
        if not self._host or self._host[0][0].shape != (n, cols):
            pin = cuda and torch.cuda.is_available()
            self._host = []
            for _ in range(2):
                ev = threading.Event()
                ev.set()
                self._host.append((torch.empty((n, cols), dtype=torch.float32, pin_memory=pin),
                                   torch.empty((n, cols), dtype=torch.float32, pin_memory=pin), ev))
            self._turn = 0
        slot = self._host[self._turn % 2]
        self._turn += 1
        t0 = time.perf_counter()
        slot[2].wait()                      # its previous writer job has finished with it
        self.slot_wait_s += time.perf_counter() - t0
        return slot

    def dump_data(self, timestep, x_analysis, P_analysis, P_analysis_inv, state_mask, n_params):
        """Reference signature: interleaved x and block-diagonal P^-1."""
        sm = np.asarray(state_mask).astype(bool)
        mean = np.zeros((n_params,) + sm.shape, dtype=np.float32)
        unc = np.zeros_like(mean)
        d = P_analysis_inv.diagonal()
        for ii in range(n_params):
            mean[ii][sm] = x_analysis[ii::n_params]
            unc[ii][sm] = 1. / np.sqrt(d[ii::n_params])
        self._write_all(timestep, mean, unc, self.geotransform, self.prefix)

    def flush(self):
        if self._copier is not None:
            self._copier.flush()       # its jobs hand their writes to the writer thread
        if self._w is not None:
            self._w.flush()


class KafkaOutputMemory:
    """In-memory output (kafka_test.py:135-145)."""

    def __init__(self, parameter_list):
        self.parameter_list = list(parameter_list)
        self.output = {}

    def dump_data(self, timestep, x_analysis, P_analysis, P_analysis_inv, state_mask, n_params=None):
        n = n_params or len(self.parameter_list)
        sol = {p: np.asarray(x_analysis)[ii::n].copy() for ii, p in enumerate(self.parameter_list)}
        if P_analysis_inv is not None:
            d = P_analysis_inv.diagonal()
            for ii, p in enumerate(self.parameter_list):
                sol[p + "_unc"] = 1. / np.sqrt(d[ii::n])
        self.output[timestep] = sol


class DeviceOutput:
    """Keeps the latest analysis rasters on the device (mean and unc planes on
    the strip grid) — the analysis kernel writes them in its final iteration
    (fused output), nothing leaves the GPU unless ``to_host`` is called.

    On a dense strip (every pixel active: the identity raster map) the mean
    raster IS the analysis state's x ([n_p, N] with N = H W), so it is not
    written twice: ``mean`` then references the state's x (``alias_state``;
    a state's buffers are never rewritten -- each date allocates new ones).
    The planes the output owns (the uncertainty planes, and the mean planes of
    a masked strip, the gain form or ``dump_state``) alternate between two
    buffer pairs, so a reader of one date's planes (``KafkaOutput``'s
    device-to-host copy) runs under the next date's analysis;
    ``device_targets`` makes the analysis wait only for a reader of the pair it
    is about to overwrite (``release``)."""

    def __init__(self, parameter_list, keep_history: bool = False, alias_state: bool = True):
        self.parameter_list = list(parameter_list)
        self.keep_history = keep_history
        self.alias_state = bool(alias_state)
        self.mean = None
        self.unc = None
        self.timestep = None
        self.history = {}
        self._mean_bufs = [None, None]
        self._unc_bufs = None
        self._readers = [None, None]   # event of the last reader of each (mean, unc) buffer pair
        self._turn = 0
        self._alias = False

    def _ensure(self, engine, dev):
        part = engine.partition
        n = engine.n_params
        H, W = part.strip_shape
        if self._unc_bufs is None or self._unc_bufs[0].device != dev or self._unc_bufs[0].shape != (n, H * W):
            self._unc_bufs = [torch.zeros((n, H * W), dtype=torch.float32, device=dev) for _ in range(2)]
            self._mean_bufs = [None, None]
            self._readers = [None, None]
            idx = np.asarray(part.local_idx, dtype=np.int64)
            if idx.size and (idx.min() < 0 or idx.max() >= H * W):
                raise ValueError("partition raster index outside the strip")
            self._idx = torch.from_numpy(idx).to(dev)
            self._identity = part.N == H * W
            self._plane = H * W
        if self.unc is None:
            self.unc = self._unc_bufs[0]

    def _own_mean(self):
        """The mean planes of the current buffer pair (``_turn``): guarded by
        the same reader event as its uncertainty planes."""
        b = self._mean_bufs[self._turn]
        if b is None:
            b = self._mean_bufs[self._turn] = torch.zeros_like(self._unc_bufs[0])
        return b

    def _next_unc(self, dev):
        """The uncertainty buffer of the next date (the other pair than the
        latest), after the last reader of that pair."""
        self._turn ^= 1
        ev = self._readers[self._turn]
        if ev is not None and dev.type == "cuda":
            torch.cuda.current_stream(dev).wait_event(ev)
            self._readers[self._turn] = None
        return self._unc_bufs[self._turn]

    def release(self, event):
        """A reader of the latest planes (recorded after its copy): the
        buffer is not overwritten before it (next-but-one date)."""
        self._readers[self._turn] = event

    def device_targets(self, engine, dev, alias: bool = True):
        """(mean, unc, idx) rasters the analysis kernel can write directly
        (fused output, AnalysisArgs.out_*); followed by ``mark_written``.
        mean None: the state's x is the mean raster (dense strips; ``alias``:
        the caller's kernel writes the final x as the state, the plain
        information-form analysis)."""
        self._ensure(engine, dev)
        unc = self._next_unc(dev)
        self._alias = self.alias_state and self._identity and alias
        self._pending = unc
        return (None if self._alias else self._own_mean()), unc, None if self._identity else self._idx

    def mark_written(self, timestep, state, engine):
        self.timestep = timestep
        self.unc = getattr(self, "_pending", self.unc)
        if self._alias:
            self.mean = state.x[:, :self._plane]
        else:
            self.mean = self._own_mean()
        if self.keep_history:
            self.history[timestep] = (self.mean.clone(), self.unc.clone())

    def dump_state(self, timestep, state, engine):
        n = engine.n_params
        self._ensure(engine, state.x.device)
        prec = engine._as_kind(state, "precision")
        unc = self._next_unc(state.x.device)
        mean = self._own_mean()
        if state.N:
            K.unpack(n, prec.x, prec.P, mean, unc, idx=None if self._identity else self._idx, N=state.N)
        self._pending, self._alias = unc, False
        self.mark_written(timestep, state, engine)

    def to_host(self, shape=None):
        n = self.mean.shape[0]
        m = self.mean.cpu().numpy()
        u = self.unc.cpu().numpy()
        if shape is not None:
            m, u = m.reshape((n,) + tuple(shape)), u.reshape((n,) + tuple(shape))
        return m, u
