"""GeoTIFF writer/reader (GDAL is not available in this stack).

The hot paths are native (``csrc/kf_tiff.cpp``, thread-pool DEFLATE of tiles /
strips straight into or out of caller buffers): ``write_tiff`` writes tiled
DEFLATE GeoTIFFs with EPSG GeoKeys, ``read_tiff`` / ``read_tiff_window`` decode
strips or tiles in parallel.  The pure-Python codec below is the fallback for
layouts the native reader does not take (big-endian, pixel-interleaved) and
for builds without the extension.

Writes single- or multi-band (planar, ``(bands, H, W)``) rasters (float32 / uint8 / uint16 / int16 / float64) as
classic or BigTIFF, striped, uncompressed or DEFLATE (the reference writes
DEFLATE/BIGTIFF/TILED Float32, ``observations.py:366-371``), with GeoTIFF
georeferencing: ModelPixelScale (33550), ModelTiepoint (33922), a
GeoKeyDirectory (34735) and the projection WKT in GTCitationGeoKey (34737).
The reader handles what the writer produces plus the uncompressed / DEFLATE
striped files of the reference (e.g. ``Barrax_pivots.tif``).
"""
from __future__ import annotations

import os
import re
import struct
import zlib

import numpy as np

_DT = {np.dtype("uint8"): (1, 8), np.dtype("uint16"): (1, 16), np.dtype("int16"): (2, 16),
       np.dtype("int32"): (2, 32), np.dtype("uint32"): (1, 32), np.dtype("float32"): (3, 32),
       np.dtype("float64"): (3, 64)}
# TIFF field types
SHORT, LONG, DOUBLE, ASCII, LONG8 = 3, 4, 12, 2, 16
_TSIZE = {1: 1, 2: 1, 3: 2, 4: 4, 5: 8, 11: 4, 12: 8, 16: 8}
_TFMT = {1: "B", 2: "c", 3: "H", 4: "I", 11: "f", 12: "d", 16: "Q"}


_NATIVE_FMT = {np.dtype("uint8"): (8, 1), np.dtype("uint16"): (16, 1), np.dtype("int16"): (16, 2),
               np.dtype("int32"): (32, 2), np.dtype("uint32"): (32, 1), np.dtype("float32"): (32, 3),
               np.dtype("float64"): (64, 3)}


def _native():
    try:
        from ..ops._ext import ext
    except Exception:  # pragma: no cover
        return None
    return ext if (ext is not None and hasattr(ext, "tiff_write")) else None


_STRATEGY = {None: 0, "default": 0, "filtered": 1, "huffman": 2, "rle": 3}


def _threads() -> int:
    """KAFKA_IO_THREADS, else the OMP_NUM_THREADS share of a batch box (whose
    affinity mask shows the whole machine), else the affinity mask."""
    n = int(os.environ.get("KAFKA_IO_THREADS", "0") or 0) or int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if not n:
        try:
            n = len(os.sched_getaffinity(0))
        except AttributeError:
            n = os.cpu_count() or 4
    return max(1, min(n, 64))


def epsg_of(projection) -> int:
    """EPSG code of a projection given as an int, ``"EPSG:32630"`` or a WKT
    with an ``AUTHORITY["EPSG", "..."]`` (the outermost, i.e. last, one); 0 if
    none is found."""
    if projection is None:
        return 0
    if isinstance(projection, (int, np.integer)):
        return int(projection)
    s = str(projection)
    m = re.findall(r'AUTHORITY\["EPSG",\s*"?(\d+)"?\]', s) or re.findall(r"EPSG:(\d+)", s)
    if m:
        return int(m[-1])
    m = re.search(r"UTM zone (\d+)\s*([NS])", s, re.I)      # a citation such as "WGS 84 / UTM zone 30N"
    if m and "WGS" in s.upper():
        return (32600 if m.group(2).upper() == "N" else 32700) + int(m.group(1))
    return 0


def write_tiff(path, array, geotransform=None, projection: str | None = None, compress: str | None = "deflate",
               rows_per_strip: int = 64, bigtiff: bool | None = None, nodata=None, tile: int | None = 256,
               level: int = 6, threads: int | None = None, predictor: int = 1, strategy: str | None = None):
    """Write a 2-D raster or a (bands, H, W) stack.  Native path: tiled
    (``tile`` px) DEFLATE, parallel compression, EPSG GeoKeys from
    ``projection``; ``tile=None`` (or no extension) writes the striped Python
    layout.  ``predictor`` 2 (integers) / 3 (floats) is the TIFF horizontal
    predictor; ``strategy`` "rle" / "huffman" selects the zlib strategy (about
    3x faster encoding of float rasters at a similar ratio)."""
    a = np.ascontiguousarray(np.asarray(array))
    if a.dtype == np.bool_:
        a = a.astype(np.uint8)
    E = _native() if tile else None
    if E is not None and a.ndim in (2, 3) and a.dtype in _NATIVE_FMT and a.dtype.byteorder in ("=", "<", "|"):
        planes = a[None] if a.ndim == 2 else a
        nb, H, W = planes.shape
        bits, fmt = _NATIVE_FMT[a.dtype]
        gt = [float(v) for v in geotransform] if geotransform is not None else []
        big = -1 if bigtiff is None else int(bool(bigtiff))
        E.tiff_write(str(path), planes.ctypes.data, nb, H, W, bits, fmt, int(tile),
                     level if compress == "deflate" else 0, threads or _threads(), gt, epsg_of(projection),
                     "" if projection is None else str(projection), "" if nodata is None else str(nodata), big,
                     int(predictor), _STRATEGY[strategy])
        return
    _write_tiff_py(path, a, geotransform, projection, compress, rows_per_strip, bigtiff, nodata)


def write_tiff_tiles(path, H: int, W: int, data, offsets, sizes, geotransform=None, projection: str | None = None,
                     nodata=None, predictor: int = 3, bigtiff: bool | None = None, threads: int | None = None,
                     tile: int = 256):
    """A float32 GeoTIFF from tiles already encoded as zlib streams
    (``ops.kernels.TileEncoder``: tile i's ``sizes[i]`` bytes at ``data`` +
    ``offsets[i]``, row-major tiles); only the file layout is written here."""
    E = _native()
    if E is None or not hasattr(E, "tiff_write_tiles"):
        raise RuntimeError("write_tiff_tiles needs the native extension")
    ptr = data.data_ptr() if hasattr(data, "data_ptr") else np.asarray(data).ctypes.data
    gt = [float(v) for v in geotransform] if geotransform is not None else []
    big = -1 if bigtiff is None else int(bool(bigtiff))
    E.tiff_write_tiles(str(path), ptr, int(H), int(W), 32, 3, int(tile), 8, int(predictor),
                       [int(v) for v in offsets], [int(v) for v in sizes], threads or _threads(), gt,
                       epsg_of(projection), "" if projection is None else str(projection),
                       "" if nodata is None else str(nodata), big)


def _write_tiff_py(path, array, geotransform=None, projection: str | None = None, compress: str | None = "deflate",
                   rows_per_strip: int = 64, bigtiff: bool | None = None, nodata=None):
    a = np.ascontiguousarray(np.asarray(array))
    if a.ndim not in (2, 3):
        raise ValueError("write_tiff writes 2-D rasters or (bands, H, W) stacks")
    if a.dtype == np.bool_:
        a = a.astype(np.uint8)
    if a.dtype not in _DT:
        raise TypeError(f"unsupported dtype {a.dtype}")
    fmt_code, bits = _DT[a.dtype]
    a = a.astype(a.dtype.newbyteorder("<"), copy=False)
    planes = a[None] if a.ndim == 2 else a
    nb, H, W = planes.shape
    rps = max(1, min(rows_per_strip, H))
    strips = []
    for plane in planes:     # PlanarConfiguration 2: all strips of band 0, then band 1, ...
        for r in range(0, H, rps):
            raw = plane[r:r + rps].tobytes()
            strips.append(zlib.compress(raw, 6) if compress == "deflate" else raw)
    total = sum(len(s) for s in strips)
    if bigtiff is None:
        bigtiff = total > 3_500_000_000
    tags = [(256, LONG, [W]), (257, LONG, [H]), (258, SHORT, [bits] * nb),
            (259, SHORT, [8 if compress == "deflate" else 1]), (262, SHORT, [1]), (277, SHORT, [nb]),
            (278, LONG, [rps]), (284, SHORT, [2 if nb > 1 else 1]), (339, SHORT, [fmt_code] * nb)]
    if geotransform is not None:
        gt = [float(v) for v in geotransform]
        tags.append((33550, DOUBLE, [gt[1], -gt[5], 0.0]))
        tags.append((33922, DOUBLE, [0.0, 0.0, 0.0, gt[0], gt[3], 0.0]))
        cit = (projection or "unknown") + "|"
        keys = [1, 1, 0, 3, 1024, 0, 1, 1, 1025, 0, 1, 1, 1026, 34737, len(cit), 0]
        tags.append((34735, SHORT, keys))
        tags.append((34737, ASCII, cit))
    if nodata is not None:
        tags.append((42113, ASCII, str(nodata)))
    # data first, IFD after
    hdr = 16 if bigtiff else 8
    body = bytearray()
    offsets = []
    for s in strips:
        offsets.append(hdr + len(body))
        body += s
        if len(body) % 2:
            body += b"\0"
    off_type = LONG8 if bigtiff else LONG
    tags.append((273, off_type, offsets))
    tags.append((279, off_type, [len(s) for s in strips]))
    tags.sort(key=lambda t: t[0])
    ifd_off = hdr + len(body)
    ent = 20 if bigtiff else 12
    cnt_sz = 8 if bigtiff else 2
    inline = 8 if bigtiff else 4
    ext = bytearray()
    ext_base = ifd_off + cnt_sz + ent * len(tags) + (8 if bigtiff else 4)
    entries = bytearray()
    for tag, typ, vals in tags:
        if typ == ASCII:
            payload = (vals if isinstance(vals, bytes) else vals.encode()) + b"\0"
            count = len(payload)
        else:
            payload = struct.pack("<" + _TFMT[typ] * len(vals), *vals)
            count = len(vals)
        if len(payload) <= inline:
            val = payload.ljust(inline, b"\0")
        else:
            val = struct.pack("<Q" if bigtiff else "<I", ext_base + len(ext))
            ext += payload
            if len(ext) % 2:
                ext += b"\0"
        entries += struct.pack("<HHQ" if bigtiff else "<HHI", tag, typ, count) + val
    with open(path, "wb") as f:
        if bigtiff:
            f.write(b"II" + struct.pack("<HHHQ", 43, 8, 0, ifd_off))
        else:
            f.write(b"II" + struct.pack("<HI", 42, ifd_off))
        f.write(body)
        f.write(struct.pack("<Q" if bigtiff else "<H", len(tags)))
        f.write(entries)
        f.write(struct.pack("<Q" if bigtiff else "<I", 0))
        f.write(ext)


def _geo_from_native(info) -> dict:
    out = {"shape": (int(info["height"]), int(info["width"])), "bands": int(info["bands"])}
    sc, tp = info["pixel_scale"], info["tiepoint"]
    if len(sc) >= 2 and len(tp) >= 5:
        out["geotransform"] = [tp[3] - tp[0] * sc[0], sc[0], 0.0, tp[4] + tp[1] * sc[1], 0.0, -sc[1]]
    if info["geo_ascii"]:
        out["projection"] = info["geo_ascii"].rstrip("|")
    keys = list(info["geokeys"])
    for i in range(4, len(keys) - 3, 4):
        if keys[i] in (3072, 2048) and keys[i + 1] == 0:
            out["epsg"] = int(keys[i + 3])
    if info["nodata"]:
        out["nodata"] = info["nodata"]
    return out


_NP_OF = {(8, 1): "u1", (16, 1): "u2", (16, 2): "i2", (32, 1): "u4", (32, 2): "i4", (32, 3): "f4", (64, 3): "f8"}


def tiff_info(path) -> dict:
    """Header of a GeoTIFF (native parser): size, bands, layout, georeferencing."""
    E = _native()
    if E is None:
        return read_tiff(path)[1]
    info = E.tiff_info(str(path))
    out = _geo_from_native(info)
    out.update({k: info[k] for k in ("bits", "sample_format", "compression", "predictor", "tiled", "tile",
                                     "rows_per_strip", "bigtiff", "planar")})
    out["dtype"] = np.dtype(_NP_OF[(int(info["bits"]), int(info["sample_format"]))])
    return out


def read_tiff_window(path, band: int = 0, window=None, out=None, threads: int | None = None):
    """Decode one band (rows r0:r1, columns c0:c1 of ``window = (r0, r1, c0,
    c1)``) into ``out`` (a C-contiguous numpy array or a pinned CPU tensor of
    the raster dtype) with the native thread pool; returns ``out``."""
    E = _native()
    info = E.tiff_info(str(path))
    H, W = int(info["height"]), int(info["width"])
    r0, r1, c0, c1 = window if window is not None else (0, H, 0, W)
    dt = np.dtype(_NP_OF[(int(info["bits"]), int(info["sample_format"]))])
    if out is None:
        out = np.empty((r1 - r0, c1 - c0), dtype=dt)
    ptr = out.data_ptr() if hasattr(out, "data_ptr") else out.ctypes.data
    nbytes = out.numel() * out.element_size() if hasattr(out, "data_ptr") else out.nbytes
    if nbytes != (r1 - r0) * (c1 - c0) * dt.itemsize:
        raise ValueError("out does not match the window")
    E.tiff_read(str(path), int(band), ptr, r0, r1, c0, c1, threads or _threads(), dt.itemsize)
    return out


def read_tiff(path):
    """-> (array, info dict with geotransform/projection)."""
    E = _native()
    if E is not None:
        try:
            info = E.tiff_info(str(path))
        except RuntimeError:
            info = None   # big-endian etc.: Python codec below
        if info is not None and (int(info["bands"]) == 1 or int(info["planar"]) == 2) and \
                (int(info["bits"]), int(info["sample_format"])) in _NP_OF and \
                int(info["compression"]) in (1, 8, 32946):
            H, W, nb = int(info["height"]), int(info["width"]), int(info["bands"])
            dt = np.dtype(_NP_OF[(int(info["bits"]), int(info["sample_format"]))])
            arr = np.empty((nb, H, W), dtype=dt)
            for b in range(nb):
                E.tiff_read(str(path), b, arr[b].ctypes.data, 0, H, 0, W, _threads(), dt.itemsize)
            return (arr[0] if nb == 1 else arr), _geo_from_native(info)
    return _read_tiff_py(path)


def _read_tiff_py(path):
    """Pure-Python reader (strips or tiles, uncompressed / DEFLATE, predictor
    1-3, either byte order) — the fallback and an independent decoder for tests."""
    with open(path, "rb") as f:
        b = f.read()
    bo = "<" if b[:2] == b"II" else ">"
    magic = struct.unpack(bo + "H", b[2:4])[0]
    big = magic == 43
    ifd = struct.unpack(bo + ("Q" if big else "I"), b[8:16] if big else b[4:8])[0]
    n = struct.unpack(bo + ("Q" if big else "H"), b[ifd:ifd + (8 if big else 2)])[0]
    p = ifd + (8 if big else 2)
    ent = 20 if big else 12
    tags = {}
    for i in range(n):
        e = b[p + i * ent:p + (i + 1) * ent]
        if big:
            tag, typ, cnt = struct.unpack(bo + "HHQ", e[:12])
            raw = e[12:20]
            inline = 8
        else:
            tag, typ, cnt = struct.unpack(bo + "HHI", e[:8])
            raw = e[8:12]
            inline = 4
        sz = _TSIZE.get(typ, 1) * cnt
        if sz > inline:
            off = struct.unpack(bo + ("Q" if big else "I"), raw)[0]
            data = b[off:off + sz]
        else:
            data = raw[:sz]
        if typ == ASCII:
            tags[tag] = data.rstrip(b"\0").decode(errors="replace")
        else:
            tags[tag] = list(struct.unpack(bo + _TFMT[typ] * cnt, data))
    W, H = tags[256][0], tags[257][0]
    bits = tags.get(258, [8])[0]
    fmt = tags.get(339, [1])[0]
    comp = tags.get(259, [1])[0]
    dt = {(1, 8): "u1", (1, 16): "u2", (2, 16): "i2", (1, 32): "u4", (2, 32): "i4", (3, 32): "f4",
          (3, 64): "f8"}[(fmt, bits)]
    dtype = np.dtype(bo + dt)
    nb = tags.get(277, [1])[0]
    planar = tags.get(284, [1])[0]
    pred = tags.get(317, [1])[0]
    spp = nb if planar == 1 else 1                 # samples per chunk pixel

    def decode(chunk, w):
        """-> rows of ``w * spp`` samples with the horizontal predictor undone."""
        if comp in (8, 32946):
            chunk = zlib.decompress(chunk)
        elif comp != 1:
            raise ValueError(f"unsupported TIFF compression {comp}")
        if pred == 1:
            return np.frombuffer(chunk, dtype=dtype)
        isz = dtype.itemsize
        rows = np.frombuffer(chunk, np.uint8)
        rows = rows[:len(rows) // (w * spp * isz) * (w * spp * isz)].reshape(-1, w * spp * isz)
        if pred == 2:
            ui = np.dtype(bo + f"u{isz}")
            v = rows.view(ui).reshape(rows.shape[0], w, spp)
            return np.cumsum(v, axis=1, dtype=ui).astype(ui).view(dtype).ravel()
        # 3: floating point — bytes differenced, MSB plane first (TIFF TN3)
        u = np.cumsum(rows, axis=1, dtype=np.uint8).reshape(rows.shape[0], isz, w * spp)
        u = u[:, ::-1, :] if bo == "<" else u
        return np.ascontiguousarray(u.transpose(0, 2, 1)).view(dtype).ravel()

    planes = nb if planar == 2 else 1
    full = np.zeros((planes, H, W * spp), dtype=dtype)
    if 322 in tags:                                 # tiled
        tw, th = tags[322][0], tags[323][0]
        across, down = -(-W // tw), -(-H // th)
        for i, (off, cnt) in enumerate(zip(tags[324], tags[325])):
            pl, t = divmod(i, across * down)
            ty, tx = divmod(t, across)
            tile = decode(b[off:off + cnt], tw).reshape(th, tw * spp)
            r, c = min(th, H - ty * th), min(tw, W - tx * tw)
            full[pl, ty * th:ty * th + r, tx * tw * spp:(tx * tw + c) * spp] = tile[:r, :c * spp]
    else:
        rps = tags.get(278, [H])[0]
        per = -(-H // rps)
        for i, (off, cnt) in enumerate(zip(tags[273], tags[279])):
            pl, s_ = divmod(i, per)
            rows = decode(b[off:off + cnt], W)
            n_r = min(rps, H - s_ * rps)
            full[pl, s_ * rps:s_ * rps + n_r] = rows[:n_r * W * spp].reshape(n_r, W * spp)
    if nb == 1:
        arr = full[0]
    elif planar == 2:
        arr = full
    else:                    # chunky (pixel-interleaved) -> (bands, H, W)
        arr = full[0].reshape(H, W, nb).transpose(2, 0, 1).copy()
    info = {"shape": (H, W), "bands": nb}
    if 33550 in tags and 33922 in tags:
        sx, sy = tags[33550][0], tags[33550][1]
        tp = tags[33922]
        info["geotransform"] = [tp[3] - tp[0] * sx, sx, 0.0, tp[4] + tp[1] * sy, 0.0, -sy]
    if 34737 in tags:
        info["projection"] = tags[34737].rstrip("|")
    return arr.astype(dtype.newbyteorder("=")), info
