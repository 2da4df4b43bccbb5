"""Vector/raster footprint helpers without GDAL/OGR/OSR.

Reference: ``kafka/input_output/utils.py:66-108`` (``raster_extent_feature``,
``find_overlap_raster_feature``) and the drivers' cutline masks
(``kafka_test.py:45-66``, ``kafka_test_Py36.py:190-206``), which go through
OGR geometries and an OSR transform to WGS84.  This stack has no GDAL, so the
pieces those functions need are implemented here directly:

* CRS parsing for the cases the reference data uses — geographic WGS84
  (EPSG:4326) and UTM north/south (EPSG:326zz / 327zz, or a WKT/name containing
  ``UTM zone zzN``; ``Barrax_pivots.tif`` and ``Barrax_pivots.json`` are
  EPSG:32630);
* the UTM <-> geographic transverse-Mercator series (Snyder, *Map Projections —
  A Working Manual*, USGS PP 1395, eqs. 8-9 .. 8-25), sub-millimetre over a zone;
* polygon intersection (edge crossings + containment) and point-in-polygon
  rasterisation of GeoJSON polygons onto a north-up grid (the cutline warp).

The reference builds its extent ring in the order TL, BL, TR, BR (a bow tie,
``utils.py:86-91``); here the ring is the raster's actual rectangle.
"""
from __future__ import annotations

import json
import math
import re

import numpy as np

_A = 6378137.0                      # WGS84 semi-major axis
_F = 1.0 / 298.257223563
_E2 = _F * (2.0 - _F)
_EP2 = _E2 / (1.0 - _E2)
_K0 = 0.9996


class CRS:
    """``kind`` is "geographic" or "utm"; UTM carries ``zone`` and ``north``."""

    def __init__(self, kind: str, zone: int | None = None, north: bool = True):
        self.kind, self.zone, self.north = kind, zone, north

    def __eq__(self, other):
        return isinstance(other, CRS) and (self.kind, self.zone, self.north) == (other.kind, other.zone, other.north)

    def __repr__(self):
        return "CRS(geographic)" if self.kind == "geographic" else \
            f"CRS(utm {self.zone}{'N' if self.north else 'S'})"


WGS84 = CRS("geographic")


def parse_crs(spec) -> CRS:
    """EPSG code (int or "EPSG:…"/URN string), UTM name/WKT, or a CRS."""
    if isinstance(spec, CRS):
        return spec
    if spec is None:
        raise ValueError("no CRS given")
    if isinstance(spec, (int, np.integer)):
        code = int(spec)
    else:
        s = str(spec)
        m = re.search(r"UTM zone (\d+)\s*([NS])", s, re.I)
        if m:
            return CRS("utm", int(m.group(1)), m.group(2).upper() == "N")
        m = re.search(r"EPSG[:]+(\d+)", s, re.I)
        if m:
            code = int(m.group(1))
        elif re.search(r"WGS\s*84", s, re.I) and "UTM" not in s.upper():
            return WGS84
        else:
            raise ValueError(f"unsupported CRS {s!r}")
    if code == 4326:
        return WGS84
    if 32601 <= code <= 32660:
        return CRS("utm", code - 32600, True)
    if 32701 <= code <= 32760:
        return CRS("utm", code - 32700, False)
    raise ValueError(f"unsupported EPSG code {code}")


def _meridian_arc(phi):
    e2, e4, e6 = _E2, _E2 ** 2, _E2 ** 3
    return _A * ((1 - e2 / 4 - 3 * e4 / 64 - 5 * e6 / 256) * phi
                 - (3 * e2 / 8 + 3 * e4 / 32 + 45 * e6 / 1024) * np.sin(2 * phi)
                 + (15 * e4 / 256 + 45 * e6 / 1024) * np.sin(4 * phi)
                 - (35 * e6 / 3072) * np.sin(6 * phi))


def lonlat_to_utm(lon, lat, zone: int, north: bool = True):
    """Geographic degrees -> UTM metres (Snyder 8-9 .. 8-10)."""
    lon, lat = np.asarray(lon, np.float64), np.asarray(lat, np.float64)
    phi = np.radians(lat)
    lam0 = math.radians(6.0 * zone - 183.0)
    n = _A / np.sqrt(1 - _E2 * np.sin(phi) ** 2)
    t = np.tan(phi) ** 2
    c = _EP2 * np.cos(phi) ** 2
    a = np.cos(phi) * (np.radians(lon) - lam0)
    m = _meridian_arc(phi)
    x = _K0 * n * (a + (1 - t + c) * a ** 3 / 6 + (5 - 18 * t + t * t + 72 * c - 58 * _EP2) * a ** 5 / 120)
    y = _K0 * (m + n * np.tan(phi) * (a * a / 2 + (5 - t + 9 * c + 4 * c * c) * a ** 4 / 24
                                      + (61 - 58 * t + t * t + 600 * c - 330 * _EP2) * a ** 6 / 720))
    return x + 500000.0, y + (0.0 if north else 10000000.0)


def utm_to_lonlat(easting, northing, zone: int, north: bool = True):
    """UTM metres -> geographic degrees (Snyder 8-18 .. 8-25, footpoint latitude)."""
    x = np.asarray(easting, np.float64) - 500000.0
    y = np.asarray(northing, np.float64) - (0.0 if north else 10000000.0)
    m = y / _K0
    mu = m / (_A * (1 - _E2 / 4 - 3 * _E2 ** 2 / 64 - 5 * _E2 ** 3 / 256))
    e1 = (1 - math.sqrt(1 - _E2)) / (1 + math.sqrt(1 - _E2))
    phi1 = (mu + (3 * e1 / 2 - 27 * e1 ** 3 / 32) * np.sin(2 * mu)
            + (21 * e1 ** 2 / 16 - 55 * e1 ** 4 / 32) * np.sin(4 * mu)
            + (151 * e1 ** 3 / 96) * np.sin(6 * mu) + (1097 * e1 ** 4 / 512) * np.sin(8 * mu))
    c1 = _EP2 * np.cos(phi1) ** 2
    t1 = np.tan(phi1) ** 2
    n1 = _A / np.sqrt(1 - _E2 * np.sin(phi1) ** 2)
    r1 = _A * (1 - _E2) / (1 - _E2 * np.sin(phi1) ** 2) ** 1.5
    d = x / (n1 * _K0)
    lat = phi1 - (n1 * np.tan(phi1) / r1) * (d * d / 2 - (5 + 3 * t1 + 10 * c1 - 4 * c1 * c1 - 9 * _EP2) * d ** 4 / 24
                                             + (61 + 90 * t1 + 298 * c1 + 45 * t1 * t1 - 252 * _EP2 - 3 * c1 * c1)
                                             * d ** 6 / 720)
    lon = (d - (1 + 2 * t1 + c1) * d ** 3 / 6 + (5 - 2 * c1 + 28 * t1 - 3 * c1 * c1 + 8 * _EP2 + 24 * t1 * t1)
           * d ** 5 / 120) / np.cos(phi1)
    return np.degrees(lon) + (6.0 * zone - 183.0), np.degrees(lat)


def transform_points(xy, src, dst):
    """(n, 2) coordinates from ``src`` CRS to ``dst`` CRS."""
    src, dst = parse_crs(src), parse_crs(dst)
    xy = np.asarray(xy, np.float64).reshape(-1, 2)
    if src == dst:
        return xy.copy()
    if src.kind == "utm":
        lon, lat = utm_to_lonlat(xy[:, 0], xy[:, 1], src.zone, src.north)
    else:
        lon, lat = xy[:, 0], xy[:, 1]
    if dst.kind == "geographic":
        return np.stack([lon, lat], 1)
    e, n = lonlat_to_utm(lon, lat, dst.zone, dst.north)
    return np.stack([e, n], 1)


class Polygon:
    """A polygon (exterior ring + optional holes) with its CRS — the subset of an
    OGR geometry the reference's footprint code uses."""

    def __init__(self, exterior, crs=WGS84, holes=()):
        self.exterior = np.asarray(exterior, np.float64)[:, :2]
        self.holes = [np.asarray(h, np.float64)[:, :2] for h in holes]
        self.crs = parse_crs(crs)

    def GetSpatialReference(self):
        return self.crs

    def Transform(self, dst) -> "Polygon":
        """In-place reprojection (OGR semantics); returns self."""
        dst = parse_crs(dst)
        self.exterior = transform_points(self.exterior, self.crs, dst)
        self.holes = [transform_points(h, self.crs, dst) for h in self.holes]
        self.crs = dst
        return self

    def transformed(self, dst) -> "Polygon":
        return Polygon(self.exterior, self.crs, self.holes).Transform(dst)

    def bounds(self):
        return (*self.exterior.min(0), *self.exterior.max(0))

    def contains_points(self, x, y):
        inside = points_in_ring(self.exterior, x, y)
        for h in self.holes:
            inside &= ~points_in_ring(h, x, y)
        return inside

    def Intersects(self, other: "Polygon") -> bool:
        return polygons_intersect(self, other.transformed(self.crs))

    def __repr__(self):
        return f"Polygon({len(self.exterior)} vertices, {self.crs})"


def points_in_ring(ring, x, y):
    """Even-odd rule, vectorised over points (boundary points count as inside
    on the lower/left edges, like a half-open pixel test)."""
    ring = np.asarray(ring, np.float64)
    x, y = np.asarray(x, np.float64), np.asarray(y, np.float64)
    inside = np.zeros(np.broadcast(x, y).shape, bool)
    xs, ys = ring[:, 0], ring[:, 1]
    xj, yj = np.roll(xs, 1), np.roll(ys, 1)
    for xa, ya, xb, yb in zip(xs, ys, xj, yj):
        if ya == yb:
            continue
        crosses = (ya > y) != (yb > y)
        xint = xa + (y - ya) * (xb - xa) / (yb - ya)
        inside ^= crosses & (x < xint)
    return inside


def _segments_cross(p1, p2, q1, q2):
    def orient(a, b, c):
        return np.sign((b[..., 0] - a[..., 0]) * (c[..., 1] - a[..., 1]) - (b[..., 1] - a[..., 1]) * (c[..., 0] - a[..., 0]))
    o1, o2 = orient(p1, p2, q1), orient(p1, p2, q2)
    o3, o4 = orient(q1, q2, p1), orient(q1, q2, p2)
    return (o1 != o2) & (o3 != o4)


def polygons_intersect(a: Polygon, b: Polygon) -> bool:
    """True when the exteriors overlap or touch (edge crossing or containment)."""
    ax0, ay0, ax1, ay1 = a.bounds()
    bx0, by0, bx1, by1 = b.bounds()
    if ax1 < bx0 or bx1 < ax0 or ay1 < by0 or by1 < ay0:
        return False
    ea, eb = a.exterior, b.exterior
    p1, p2 = ea[:, None, :], np.roll(ea, -1, 0)[:, None, :]
    q1, q2 = eb[None, :, :], np.roll(eb, -1, 0)[None, :, :]
    if np.any(_segments_cross(p1, p2, q1, q2)):
        return True
    return bool(points_in_ring(eb, ea[:1, 0], ea[:1, 1])[0] or points_in_ring(ea, eb[:1, 0], eb[:1, 1])[0])


def _raster_geo(raster):
    """(geotransform, (H, W), projection) from a TIFF path or a tuple."""
    if isinstance(raster, str):
        from .tiff import read_tiff
        arr, info = read_tiff(raster)
        if "geotransform" not in info:
            raise ValueError(f"{raster} has no georeferencing")
        return info["geotransform"], info["shape"], info.get("projection")
    gt, shape, proj = raster
    return list(gt), tuple(shape), proj


def raster_extent_feature(raster, crs=WGS84) -> Polygon:
    """Extent of a north-up raster as a polygon in ``crs`` (default WGS84)
    (``utils.py:66-95``).  ``raster`` is a GeoTIFF path or
    ``(geotransform, (H, W), projection)``; the edges are densified so the
    footprint stays accurate after reprojection."""
    gt, (H, W), proj = _raster_geo(raster)
    x0, y0 = gt[0], gt[3]
    x1, y1 = x0 + W * gt[1], y0 + H * gt[5]
    t = np.linspace(0.0, 1.0, 9)[:-1]
    ring = np.concatenate([
        np.stack([x0 + 0 * t, y0 + (y1 - y0) * t], 1),       # left edge, top -> bottom
        np.stack([x0 + (x1 - x0) * t, y1 + 0 * t], 1),       # bottom edge
        np.stack([x1 + 0 * t, y1 + (y0 - y1) * t], 1),       # right edge
        np.stack([x1 + (x0 - x1) * t, y0 + 0 * t], 1)])      # top edge
    poly = Polygon(ring, proj if proj else crs)
    return poly.Transform(crs)


def find_overlap_raster_feature(raster, feature: Polygon) -> bool:
    """Does ``feature`` (any supported CRS) intersect the raster footprint?
    (``utils.py:98-108``; like OGR's ``Transform`` the feature is reprojected to
    WGS84 in place.)"""
    feature.Transform(WGS84)
    return feature.Intersects(raster_extent_feature(raster, WGS84))


def read_geojson_polygons(path_or_obj) -> list[Polygon]:
    """Polygons / MultiPolygons of a GeoJSON FeatureCollection, in its CRS
    (``crs.properties.name``, default WGS84) — e.g. ``Barrax_pivots.json``."""
    obj = path_or_obj
    if isinstance(path_or_obj, str):
        with open(path_or_obj) as f:
            obj = json.load(f)
    crs = WGS84
    name = (obj.get("crs") or {}).get("properties", {}).get("name")
    if name:
        crs = parse_crs(name)
    feats = obj["features"] if obj.get("type") == "FeatureCollection" else [obj]
    out = []
    for ft in feats:
        g = ft["geometry"] if "geometry" in ft else ft
        polys = [g["coordinates"]] if g["type"] == "Polygon" else g["coordinates"] if g["type"] == "MultiPolygon" else []
        for rings in polys:
            out.append(Polygon(rings[0], crs, rings[1:]))
    return out


def rasterize_polygons(polygons, geotransform, shape, projection=None):
    """Boolean mask of the pixels whose centres fall inside any polygon — the
    reference drivers' GDAL cutline mask (``kafka_test.py:45-66``).  Polygons
    are reprojected to the raster CRS when it is given."""
    H, W = shape
    gt = list(geotransform)
    xc = gt[0] + (np.arange(W) + 0.5) * gt[1]
    yc = gt[3] + (np.arange(H) + 0.5) * gt[5]
    X, Y = np.meshgrid(xc, yc)
    mask = np.zeros((H, W), bool)
    for p in polygons:
        if projection is not None:
            p = p.transformed(parse_crs(projection))
        bx0, by0, bx1, by1 = p.bounds()
        sel = (X >= bx0) & (X <= bx1) & (Y >= by0) & (Y <= by1)
        if sel.any():
            mask[sel] |= p.contains_points(X[sel], Y[sel])
    return mask
