"""Raster utilities (``kafka/input_output/utils.py``).

``get_chunks`` keeps the reference semantics exactly (X-major, 1-based chunk
numbers, ragged last tiles; utils.py:12-40).  ``reproject_image`` replaces the
reference's ``gdal.Warp`` onto a target raster's grid (utils.py:43-64) without
GDAL: target pixel centres are mapped into the source CRS with
``geo.transform_points`` (UTM <-> WGS84) and sampled nearest-neighbour (the
``gdal.Warp`` default) or bilinearly.
"""
from __future__ import annotations

import os

import numpy as np


def get_chunks(nx, ny, block_size=(256, 256)):
    """Yield (x_off, y_off, nx_valid, ny_valid, chunk_no)."""
    bx, by = int(block_size[0]), int(block_size[1])
    nxb = (nx + bx - 1) // bx
    nyb = (ny + by - 1) // by
    chunk = 0
    for X in range(nxb):
        nx_valid = nx - X * bx if X == nxb - 1 else bx
        for Y in range(nyb):
            ny_valid = ny - Y * by if Y == nyb - 1 else by
            chunk += 1
            yield X * bx, Y * by, nx_valid, ny_valid, chunk


def _inverse_gt(gt):
    a, b, c, d, e, f = gt
    det = b * f - c * e
    if det == 0:
        raise ValueError("singular geotransform")
    return a, d, f / det, -c / det, -e / det, b / det


def _crs_pair(src_crs, dst_crs):
    """(source CRS, target CRS) when a coordinate transform is needed, else None."""
    from .geo import parse_crs

    crs_s = parse_crs(src_crs) if src_crs not in (None, "", 0) else None
    crs_d = parse_crs(dst_crs) if dst_crs not in (None, "", 0) else None
    return (crs_s, crs_d) if crs_s is not None and crs_d is not None and crs_s != crs_d else None


def _source_coords(tgt_gt, inv, crs, rows, cols):
    """Continuous source (col, row) under the centres of target pixels (rows, cols)."""
    from .geo import transform_points

    R, C = rows + 0.5, cols + 0.5
    x = tgt_gt[0] + C * tgt_gt[1] + R * tgt_gt[2]
    y = tgt_gt[3] + C * tgt_gt[4] + R * tgt_gt[5]
    if crs is not None:
        xy = transform_points(np.stack([np.ravel(x), np.ravel(y)], 1), crs[1], crs[0])
        x, y = xy[:, 0].reshape(np.shape(x)), xy[:, 1].reshape(np.shape(y))
    dx, dy = x - inv[0], y - inv[1]
    return inv[2] * dx + inv[3] * dy, inv[4] * dx + inv[5] * dy


def _nearest_flat(col, row, src_shape):
    """Flat (row-major) index of the source pixel containing (col, row); -1 outside."""
    sh, sw = src_shape
    ci, ri = np.floor(col).astype(np.int64), np.floor(row).astype(np.int64)
    ok = (ci >= 0) & (ci < sw) & (ri >= 0) & (ri < sh)
    return np.where(ok, ri * sw + ci, -1)


class GridWarp:
    """Nearest-neighbour warp of one raster grid (the source: a granule band)
    onto another (the target: the state mask) — the pixel mapping the
    reference's ``gdal.Warp(source, outputBounds=<mask extent>, xRes/yRes=<mask
    resolution>, dstSRS=<mask CRS>)`` applies to every band it reads
    (``Sentinel2_Observations.py:56-79,166``, ``Sentinel1_Observations.py:178,194``).

    The mapping is computed once per (source grid, target grid) pair and then
    applied as an index gather: ``index(rows, cols)`` gives the flat source
    index under each target pixel centre (-1 where the source does not cover
    it, which reads as nodata 0 like GDAL's MEM output), ``window(flat)`` the
    bounding source window of a set of such indices, so a reader decodes only
    the part of the granule the state grid touches.  ``reproject_image``'s
    nearest branch uses the same index arithmetic, so warped host reads equal
    it bit for bit."""

    def __init__(self, src_shape, src_gt, dst_shape, dst_gt, src_crs=None, dst_crs=None):
        self.src_shape = tuple(int(v) for v in src_shape)
        self.dst_shape = tuple(int(v) for v in dst_shape)
        self.src_gt = [float(v) for v in src_gt]
        self.dst_gt = [float(v) for v in dst_gt]
        self.crs = _crs_pair(src_crs, dst_crs)
        self._inv = _inverse_gt(self.src_gt)
        self.identity = self.crs is None and self.src_shape == self.dst_shape and self.src_gt == self.dst_gt

    @classmethod
    def from_files(cls, source_path, dst_shape, dst_gt, dst_crs=None):
        from .tiff import tiff_info

        i = tiff_info(source_path)
        return cls(i["shape"], i.get("geotransform", [0, 1, 0, 0, 0, -1]), dst_shape, dst_gt,
                   i.get("epsg") or i.get("projection"), dst_crs)

    def key(self):
        return (self.src_shape, tuple(self.src_gt), self.dst_shape, tuple(self.dst_gt), repr(self.crs))

    def index(self, rows, cols) -> np.ndarray:
        """Flat source indices (int64, -1 = not covered) under target pixels."""
        rows, cols = np.asarray(rows, np.float64), np.asarray(cols, np.float64)
        col, row = _source_coords(self.dst_gt, self._inv, self.crs, rows, cols)
        return _nearest_flat(col, row, self.src_shape)

    def index_of_mask(self, mask, row0: int = 0, block_rows: int = 1024) -> np.ndarray:
        """Source index of every True pixel of ``mask`` (row-major order), whose
        first row is target row ``row0``."""
        mask = np.asarray(mask, bool)
        out = []
        for r in range(0, mask.shape[0], block_rows):
            rr, cc = np.nonzero(mask[r:r + block_rows])
            out.append(self.index(rr + (row0 + r), cc))
        return np.concatenate(out) if out else np.zeros(0, np.int64)

    def window(self, flat) -> tuple[int, int, int, int]:
        """(r0, r1, c0, c1) bounding the covered source pixels of ``flat``
        (a 1x1 window at the origin when none is covered)."""
        flat = np.asarray(flat)
        hit = flat[flat >= 0]
        if hit.size == 0:
            return 0, 1, 0, 1
        sw = self.src_shape[1]
        r, c = hit // sw, hit % sw
        return int(r.min()), int(r.max()) + 1, int(c.min()), int(c.max()) + 1

    def local(self, flat, window) -> np.ndarray:
        """Indices into the row-major ``window`` of the source (-1 kept)."""
        flat = np.asarray(flat, np.int64)
        r0, r1, c0, c1 = window
        sw = self.src_shape[1]
        r, c = flat // sw, flat % sw
        return np.where(flat >= 0, (r - r0) * (c1 - c0) + (c - c0), -1)

    def read(self, path, band: int = 0, nodata=0, mask=None):
        """Warped band of a GeoTIFF on the target grid: only the bounding source
        window is decoded.  ``mask``: compute only these target pixels (others
        nodata)."""
        from .tiff import read_tiff_window

        H, W = self.dst_shape
        if mask is None:
            flat = self.full_index()
        else:
            flat = np.full(H * W, -1, np.int64)
            flat[np.flatnonzero(np.asarray(mask, bool))] = self.index_of_mask(mask)
        win = self.window(flat)
        src = read_tiff_window(path, band, win)
        loc = self.local(flat, win)
        out = np.full(H * W, nodata, dtype=src.dtype)
        ok = loc >= 0
        out[ok] = src.reshape(-1)[loc[ok]]
        return out.reshape(H, W)

    _full = None

    def full_index(self) -> np.ndarray:
        if self._full is None:
            H, W = self.dst_shape
            self._full = self.index_of_mask(np.ones((H, W), bool))
        return self._full


def reproject_image(source, source_geotransform=None, target_shape=None, target_geotransform=None, nodata=0,
                    src_crs=None, dst_crs=None, resampling: str = "nearest", block_rows: int = 512):
    """Warp ``source`` onto a target grid, possibly in another CRS.

    Array form: ``reproject_image(array, src_gt, (H, W), dst_gt, nodata,
    src_crs=..., dst_crs=...)`` (CRSs as EPSG codes / WKT / names; both None
    means one shared CRS).  Reference form: ``reproject_image(source_img,
    target_img, dstSRSs=None)`` with GeoTIFF paths, where the target raster
    supplies extent, resolution and (unless ``dstSRSs`` is given) the CRS.
    Returns the warped array ((H, W) or (bands, H, W)); the reference returns
    a GDAL MEM dataset holding the same raster.
    """
    if isinstance(source_geotransform, (str, os.PathLike)):       # reference signature
        from .tiff import read_tiff, tiff_info
        tinfo = tiff_info(source_geotransform)
        dst = target_shape if target_shape is not None else tinfo.get("epsg") or tinfo.get("projection")
        src_arr, sinfo = read_tiff(source) if isinstance(source, (str, os.PathLike)) else (source, {})
        return reproject_image(src_arr, sinfo["geotransform"], tinfo["shape"], tinfo["geotransform"], nodata,
                               src_crs=sinfo.get("epsg") or sinfo.get("projection"), dst_crs=dst,
                               resampling=resampling, block_rows=block_rows)
    src = np.asarray(source)
    planes = src[None] if src.ndim == 2 else src
    nb, sh, sw = planes.shape
    H, W = target_shape
    tgt = [float(v) for v in target_geotransform]
    inv = _inverse_gt([float(v) for v in source_geotransform])
    crs = _crs_pair(src_crs, dst_crs)
    out = np.full((nb, H, W), nodata, dtype=src.dtype)
    flat_src = planes.reshape(nb, -1)
    cc = np.arange(W, dtype=np.float64)
    for r0 in range(0, H, block_rows):
        rr = np.arange(r0, min(H, r0 + block_rows), dtype=np.float64)
        R, C = np.meshgrid(rr, cc, indexing="ij")
        col, row = _source_coords(tgt, inv, crs, R, C)   # source pixel coordinates (continuous)
        blk = out[:, r0:r0 + R.shape[0]]
        if resampling == "nearest":                    # the GridWarp index arithmetic
            idx = _nearest_flat(col, row, (sh, sw))
            ok = idx >= 0
            blk[:, ok] = flat_src[:, idx[ok]]
        elif resampling == "bilinear":
            fc, fr = col - 0.5, row - 0.5
            c0, r0_ = np.floor(fc).astype(np.int64), np.floor(fr).astype(np.int64)
            ok = (c0 >= 0) & (c0 + 1 < sw) & (r0_ >= 0) & (r0_ + 1 < sh)
            a, b_ = (fc - c0)[ok], (fr - r0_)[ok]
            c0, r0_ = c0[ok], r0_[ok]
            v = ((1 - a) * (1 - b_) * planes[:, r0_, c0] + a * (1 - b_) * planes[:, r0_, c0 + 1]
                 + (1 - a) * b_ * planes[:, r0_ + 1, c0] + a * b_ * planes[:, r0_ + 1, c0 + 1])
            blk[:, ok] = v.astype(src.dtype) if np.issubdtype(src.dtype, np.floating) else np.rint(v).astype(src.dtype)
        else:
            raise ValueError(f"resampling {resampling!r}")
    return out[0] if src.ndim == 2 else out


def raster_extent(geotransform, shape):
    """(xmin, ymin, xmax, ymax) of a north-up raster (raster_extent_feature, :66-95)."""
    gt = geotransform
    H, W = shape
    x0, y0 = gt[0], gt[3]
    x1, y1 = x0 + W * gt[1], y0 + H * gt[5]
    return min(x0, x1), min(y0, y1), max(x0, x1), max(y0, y1)


def find_overlap(extent_a, extent_b):
    """Intersection of two extents or None (find_overlap_raster_feature, :98-108)."""
    xmin, ymin = max(extent_a[0], extent_b[0]), max(extent_a[1], extent_b[1])
    xmax, ymax = min(extent_a[2], extent_b[2]), min(extent_a[3], extent_b[3])
    if xmin >= xmax or ymin >= ymax:
        return None
    return xmin, ymin, xmax, ymax
