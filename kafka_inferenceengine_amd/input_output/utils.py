"""Raster utilities (``kafka/input_output/utils.py``).

``get_chunks`` keeps the reference semantics exactly (X-major, 1-based chunk
numbers, ragged last tiles; utils.py:12-40).  ``reproject_image`` is a GDAL-free
nearest-neighbour resampler between north-up grids sharing one CRS (the
reference's GDAL warp, utils.py:43-64, is not available in this stack).
"""
from __future__ import annotations

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


def reproject_image(source, source_geotransform, target_shape, target_geotransform, nodata=0):
    """Nearest-neighbour resampling of ``source`` onto the target grid (same CRS)."""
    src = np.asarray(source)
    sgt, tgt = list(source_geotransform), list(target_geotransform)
    H, W = target_shape
    cols = tgt[0] + (np.arange(W) + 0.5) * tgt[1]
    rows = tgt[3] + (np.arange(H) + 0.5) * tgt[5]
    ci = np.floor((cols - sgt[0]) / sgt[1]).astype(np.int64)
    ri = np.floor((rows - sgt[3]) / sgt[5]).astype(np.int64)
    out = np.full((H, W), nodata, dtype=src.dtype)
    okc = (ci >= 0) & (ci < src.shape[1])
    okr = (ri >= 0) & (ri < src.shape[0])
    out[np.ix_(okr, okc)] = src[np.ix_(ri[okr], ci[okc])]
    return out


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
