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
    from .geo import parse_crs, transform_points

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
    crs_s = parse_crs(src_crs) if src_crs not in (None, "") else None
    crs_d = parse_crs(dst_crs) if dst_crs not in (None, "") else None
    warp = crs_s is not None and crs_d is not None and crs_s != crs_d
    out = np.full((nb, H, W), nodata, dtype=src.dtype)
    cc = np.arange(W) + 0.5
    for r0 in range(0, H, block_rows):
        rr = np.arange(r0, min(H, r0 + block_rows)) + 0.5
        R, C = np.meshgrid(rr, cc, indexing="ij")
        x = tgt[0] + C * tgt[1] + R * tgt[2]
        y = tgt[3] + C * tgt[4] + R * tgt[5]
        if warp:
            xy = transform_points(np.stack([x.ravel(), y.ravel()], 1), crs_d, crs_s)
            x, y = xy[:, 0].reshape(R.shape), xy[:, 1].reshape(R.shape)
        dx, dy = x - inv[0], y - inv[1]
        col = inv[2] * dx + inv[3] * dy          # source pixel coordinates (continuous)
        row = inv[4] * dx + inv[5] * dy
        blk = out[:, r0:r0 + R.shape[0]]
        if resampling == "nearest":
            ci, ri = np.floor(col).astype(np.int64), np.floor(row).astype(np.int64)
            ok = (ci >= 0) & (ci < sw) & (ri >= 0) & (ri < sh)
            blk[:, ok] = planes[:, ri[ok], ci[ok]]
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
