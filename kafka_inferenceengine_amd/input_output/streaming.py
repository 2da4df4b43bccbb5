"""Double-buffered observation ingest: pinned host pool -> device on a side stream.

A date's bands live contiguously in one pinned ``HostRing`` slot (native,
``csrc/kf_stream.cpp``).  ``prefetch(k)`` issues the H2D copy of pool entry k
into the idle device buffer on the ingest stream after that buffer's last
consumer finished; ``acquire(k)`` makes the compute stream wait on the copy's
event only.  H2D of date t+1 therefore overlaps the Gauss-Newton kernels of
date t.
"""
from __future__ import annotations

import torch

from ..ops import _ext
from ..ops.kernels import current_raw_stream


class DateStreamer:
    """``n_bufs`` device buffers: 2 double-buffer (date t+1 in flight under date
    t); 3 lets the caller prefetch two dates ahead, so a copy that takes longer
    than one step's kernels still streams back to back."""

    def __init__(self, n_pool: int, entry_shape, dtype, device, n_threads: int = 2, n_bufs: int = 2):
        self.device = torch.device(device)
        self.entry_shape = tuple(entry_shape)
        self.dtype = dtype
        numel = 1
        for s in self.entry_shape:
            numel *= s
        self.entry_bytes = numel * torch.empty((), dtype=dtype).element_size()
        self.ring = _ext.require_ext().HostRing(n_pool, self.entry_bytes, n_threads)
        self.n_pool = n_pool
        self.n_bufs = max(2, int(n_bufs))
        self.bufs = [torch.empty(self.entry_shape, dtype=dtype, device=self.device) for _ in range(self.n_bufs)]
        self.loaded = [None] * self.n_bufs  # pool index held by each device buffer
        self._stamp = [0] * self.n_bufs     # last load / acquire (eviction: oldest not in use)
        self._inflight = []                 # host slots of copies issued and not yet waited for
        self._clock = 0
        self.cuda = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(self.device) if self.cuda else None
        self.bytes_h2d = 0

    @property
    def pinned(self) -> bool:
        return bool(self.ring.pinned)

    def host_view(self, k: int) -> torch.Tensor:
        """Writable CPU tensor aliasing pool slot k (fill once at setup)."""
        import ctypes

        numel = self.entry_bytes // torch.empty((), dtype=self.dtype).element_size()
        buf = (ctypes.c_char * self.entry_bytes).from_address(self.ring.slot(k))
        return torch.frombuffer(buf, dtype=self.dtype, count=numel).view(self.entry_shape)

    def fill_from_file(self, k: int, path: str, offset: int = 0):
        """Background read of a raw file into slot k (native reader threads)."""
        self.ring.read_file_async(k, str(path), int(offset), self.entry_bytes, 0)

    def warm(self):
        """Issue one copy per device buffer back to back (overlapping on the DMA
        engines) and wait: the runtime sets up its extra copy queues the first
        time copies overlap (a one-off host stall of ~6 ms each on MI355X,
        measured), which belongs in setup, not in the first time steps."""
        if not self.cuda:
            return
        # the steady-state pattern: compute work in flight, the copy stream waiting
        # on the compute stream, copies back to back (prefetch)
        scratch = torch.empty(16 << 20, dtype=torch.float32, device=self.device)
        cur = torch.cuda.current_stream(self.device)
        for r in range(2 * max(4, self.n_bufs)):
            scratch.mul_(0.5)
            self.stream.wait_stream(cur)
            b = r % self.n_bufs
            self.ring.h2d(r % self.n_pool, self.bufs[b].data_ptr(), self.entry_bytes, 0, int(self.stream.cuda_stream))
            self.ring.stream_wait(r % self.n_pool, int(cur.cuda_stream))
        torch.cuda.synchronize(self.device)
        # then the steady-state cycle itself (acquire one date, prefetch the next
        # n_bufs - 1, a short kernel): the runtime stalls one hipMemcpyAsync of
        # this pattern for ~6 ms once per process, a few cycles in (probe:
        # scripts/probes/copy_stall_probe.py) -- here, not in the time steps
        for r in range(12):
            buf = self.acquire(r % self.n_pool, key=("warm", r))
            for j in range(1, self.n_bufs):
                self.prefetch((r + j) % self.n_pool, key=("warm", r + j))
            scratch.mul_(0.5)
            scratch[:1].add_(buf.reshape(-1)[:1].float())
        torch.cuda.synchronize(self.device)
        self._current = None
        del scratch
        self._inflight = []
        self.loaded = [None] * self.n_bufs

    @property
    def max_ahead(self) -> int:
        """Dates that can be in flight beyond the one being consumed."""
        return self.n_bufs - 1

    def _slot_for(self, key) -> int:
        for b, v in enumerate(self.loaded):
            if v == key:
                return b
        return -1

    def prefetch(self, k: int, key=None) -> int:
        """H2D of host entry ``k`` into a free device buffer, tagged ``key``
        (default k).  A key already resident is not copied again; callers that
        recycle host entries for distinct dates pass the date as the key, so
        every date is streamed."""
        key = k if key is None else key
        b = self._slot_for(key)
        self._clock += 1
        if b >= 0:
            return b
        # evict the least recently loaded / acquired buffer that is not being consumed
        cand = [i for i in range(self.n_bufs) if self.loaded[i] is None or self.loaded[i] != self._current]
        b = min(cand, key=lambda i: (self.loaded[i] is not None, self._stamp[i]))
        self._stamp[b] = self._clock
        dst = self.bufs[b]
        if self.cuda:
            # bound the host's run-ahead to n_bufs - 1 copies in flight: the host
            # waits (microseconds, on the oldest copy) instead of letting the
            # runtime's command backlog grow until it stalls for milliseconds
            while len(self._inflight) >= self.n_bufs - 1:
                self.ring.host_wait(self._inflight.pop(0))
            # the buffer's previous consumer is everything queued so far on the
            # compute stream; the copy itself is issued by the ring's submitter
            # thread (hipMemcpyAsync can stall its caller for milliseconds)
            self.ring.h2d_async(k, dst.data_ptr(), self.entry_bytes, 0, int(self.stream.cuda_stream),
                                current_raw_stream(self.device))
            self._inflight.append(k)
        else:
            self.ring.h2d(k, dst.data_ptr(), self.entry_bytes, 0, 0)
        self.loaded[b] = key
        self.bytes_h2d += self.entry_bytes
        return b

    _current = None

    def acquire(self, k: int, key=None) -> torch.Tensor:
        key = k if key is None else key
        b = self.prefetch(k, key)
        self._stamp[b] = self._clock
        if self.cuda:
            self.ring.stream_wait(k, current_raw_stream(self.device))
        self._current = key
        return self.bufs[b]


class RasterIngest:
    """Granule ingest from GeoTIFF files: every band of a date is decoded by the
    native reader (``csrc/kf_tiff.cpp``, thread pool, DEFLATE) straight into one
    pinned ``HostRing`` slot in the background, shipped with hipMemcpyAsync on
    a side stream into one of two device buffers, and the compute stream waits
    on that copy's event only.  ``prefetch(key, files)`` for date t + 1 runs
    under date t's Gauss-Newton kernels; replaces the per-band
    GDAL reads of Sentinel2_Observations.py:148-185.

    ``files``: list of ``(path, band_index_in_file, (r0, r1, c0, c1))`` of
    element type ``dtype``; each window is decoded row-major into the start of
    its plane, so windows of the shape ``plane`` fill it and smaller ones (a
    warp reader's per-grid windows, ``plane = (1, max elements)``) leave a
    tail the gather never reads."""

    def __init__(self, n_planes: int, plane, dtype, device, n_slots: int = 2, io_threads: int | None = None):
        import os

        self.device = torch.device(device)
        self.n_planes = int(n_planes)
        self.plane = tuple(int(v) for v in plane)
        self.dtype = dtype
        self.esize = torch.empty((), dtype=dtype).element_size()
        self.plane_bytes = self.plane[0] * self.plane[1] * self.esize
        self.slot_bytes = self.plane_bytes * self.n_planes
        self.ring = _ext.require_ext().HostRing(n_slots, self.slot_bytes, 2)
        self.slot_key = [None] * n_slots
        self.bufs = [torch.empty((self.n_planes,) + self.plane, dtype=dtype, device=self.device) for _ in range(2)]
        self.buf_key = [None, None]
        self.cuda = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(self.device) if self.cuda else None
        self.io_threads = io_threads or max(1, min(16, (os.cpu_count() or 4)))
        self._current = None
        self.bytes_h2d = 0
        self.bytes_read = 0

    @property
    def pinned(self) -> bool:
        return bool(self.ring.pinned)

    def prefetch(self, key, files) -> int:
        """Start decoding ``files`` into a free pinned slot (no wait)."""
        if key in self.slot_key:
            return self.slot_key.index(key)
        if len(files) != self.n_planes:
            raise ValueError(f"{len(files)} files for {self.n_planes} planes")
        cur = self.slot_key.index(self._current) if self._current in self.slot_key else -1
        s = next((i for i in range(len(self.slot_key)) if i != cur and self.slot_key[i] is None),
                 next(i for i in range(len(self.slot_key)) if i != cur))
        self.ring.host_wait(s)          # the slot's previous H2D has finished reading it
        for i, (path, band, (r0, r1, c0, c1)) in enumerate(files):
            if (r1 - r0, c1 - c0) != self.plane and (r1 - r0) * (c1 - c0) > self.plane[0] * self.plane[1]:
                raise ValueError(f"window {(r0, r1, c0, c1)} does not fit a {self.plane} plane")
            self.ring.read_tiff_async(s, str(path), int(band), r0, r1, c0, c1, self.esize, i * self.plane_bytes,
                                      self.io_threads)
            self.bytes_read += self.plane_bytes
        self.slot_key[s] = key
        return s

    def acquire(self, key, files) -> torch.Tensor:
        """Device planes ``[n_planes, *plane]`` of ``key``; the current stream
        waits for their copy."""
        s = self.prefetch(key, files)
        if key in self.buf_key:
            b = self.buf_key.index(key)
        else:
            b = 1 if (self._current is not None and self.buf_key[0] == self._current) else 0
            dst = self.bufs[b]
            if self.cuda:
                self.stream.wait_stream(torch.cuda.current_stream(self.device))
                self.ring.h2d(s, dst.data_ptr(), self.slot_bytes, 0, int(self.stream.cuda_stream))
            else:
                self.ring.h2d(s, dst.data_ptr(), self.slot_bytes, 0, 0)
            self.buf_key[b] = key
            self.bytes_h2d += self.slot_bytes
        if self.cuda:
            self.ring.stream_wait(s, current_raw_stream(self.device))
        self._current = key
        return self.bufs[b]
