"""File-based sensor readers (Sentinel-2 L2A granules, Sentinel-1 sigma0,
MODIS MCD43 BRDF kernels) with the reference observation protocol.

GDAL/NetCDF/HDF4 are not available in this stack, so the readers consume
GeoTIFF rasters (``input_output.tiff``) laid out like the reference's inputs:

* Sentinel-2 (``Sentinel2_Observations.py:85-185``): a granule folder
  ``.../YYYY/MM/DD/<granule>/`` containing ``aot.tif`` (discovery marker),
  ``B{02..12}_sur.tif`` (uint16 surface reflectance x 1e4, 0 = no data) and
  ``metadata.xml`` (mean sun/view angles, ``parse_xml``).  The emulator is
  chosen per date by nearest (sza, vza, raa) from file names
  ``*_{vza}_{sza}_{raa}.npz`` (``_find_emulator``, :133-145) and loaded with
  ``numpy.load(allow_pickle=False)`` — never unpickled.
* Sentinel-1 (``Sentinel1_Observations.py:56-197``): ``S1_*_{YYYYmmddTHHMMSS}_*``
  folders with ``sigma0_VV.tif``, ``sigma0_VH.tif``, ``theta.tif``; -999 = no data;
  5 % uncertainty.
* MCD43 BHR (``observations.py:214-310``): per date ``{date}_kernels_b{band}.tif``
  3-band-as-3-files kernel weights + ``{date}_qa.tif``; BHR = K . [1, 0.189184,
  -1.377622]; sigma = max(2.5e-3, 5 %/7 % BHR) by QA level.
"""
from __future__ import annotations

import datetime
import glob
import os
import xml.etree.ElementTree as ET

import numpy as np
import scipy.sparse as sp

from ..models.gp import GaussianProcessEmulator, pack_emulator_set, unpack_emulator_set
from .tiff import read_tiff, write_tiff

from .records import BHR_data, MOD09_data, S2MSIdata, SARdata  # noqa: F401  (re-exports)

S2_BAND_MAP = ["02", "03", "04", "05", "06", "07", "08", "8A", "09", "12"]
S2_EMULATOR_BANDS = [2, 3, 4, 5, 6, 7, 8, 9, 12, 13]
TO_BHR = np.array([1.0, 0.189184, -1.377622])
WRONG_VALUE = -999.0


# ------------------------------------------------------------- emulators
def save_emulator(path, em: GaussianProcessEmulator, **extra):
    """Emulator -> .npz (plain arrays only; loadable without pickle)."""
    np.savez(path, inputs=em.inputs, alpha=em.alpha, lam=em.lam, signal=np.array(em.signal),
             mean=np.array(em.mean), name=np.array(em.name), **extra)


def load_emulator(path) -> GaussianProcessEmulator:
    with np.load(path, allow_pickle=False) as z:
        return GaussianProcessEmulator(z["inputs"], z["alpha"], z["lam"], float(z["signal"]), float(z["mean"]),
                                       name=str(z["name"]))


def load_emulator_set(path) -> dict:
    """Multi-band emulator file: keys ``{band}__inputs`` etc. -> {band: emulator}."""
    out = {}
    with np.load(path, allow_pickle=False) as z:
        bands = sorted({k.split("__")[0] for k in z.files if "__" in k})
        for b in bands:
            out[b] = GaussianProcessEmulator(z[f"{b}__inputs"], z[f"{b}__alpha"], z[f"{b}__lam"],
                                             float(z[f"{b}__signal"]), float(z[f"{b}__mean"]), name=b)
    return out


def save_emulator_set(path, ems: dict):
    arrs = {}
    for b, em in ems.items():
        arrs.update({f"{b}__inputs": em.inputs, f"{b}__alpha": em.alpha, f"{b}__lam": em.lam,
                     f"{b}__signal": np.array(em.signal), f"{b}__mean": np.array(em.mean)})
    np.savez(path, **arrs)


# ------------------------------------------------------------- helpers
def parse_xml(meta_file):
    """Mean sun/view zenith/azimuth from an S2 L1C tile metadata XML (:23-53)."""
    tree = ET.parse(meta_file)
    root = tree.getroot()

    def first(tag):
        for el in root.iter():
            if el.tag.split("}")[-1] == tag:
                return el
        return None
    sun = first("Mean_Sun_Angle")
    sza = float(sun.find("ZENITH_ANGLE").text)
    saa = float(sun.find("AZIMUTH_ANGLE").text)
    vzas, vaas = [], []
    for el in root.iter():
        if el.tag.split("}")[-1] == "Mean_Viewing_Incidence_Angle":
            vzas.append(float(el.find("ZENITH_ANGLE").text))
            vaas.append(float(el.find("AZIMUTH_ANGLE").text))
    return sza, saa, float(np.mean(vzas)), float(np.mean(vaas))


def write_s2_metadata(path, sza, saa, vza, vaa, n_bands=13):
    views = "".join(f'<Mean_Viewing_Incidence_Angle bandId="{b}"><ZENITH_ANGLE unit="deg">{vza}</ZENITH_ANGLE>'
                    f'<AZIMUTH_ANGLE unit="deg">{vaa}</AZIMUTH_ANGLE></Mean_Viewing_Incidence_Angle>'
                    for b in range(n_bands))
    xml = (f'<?xml version="1.0"?><Level-1C_Tile_ID><Geometric_Info><Tile_Angles><Mean_Sun_Angle>'
           f'<ZENITH_ANGLE unit="deg">{sza}</ZENITH_ANGLE><AZIMUTH_ANGLE unit="deg">{saa}</AZIMUTH_ANGLE>'
           f'</Mean_Sun_Angle><Mean_Viewing_Incidence_Angle_List>{views}</Mean_Viewing_Incidence_Angle_List>'
           f'</Tile_Angles></Geometric_Info></Level-1C_Tile_ID>')
    with open(path, "w") as f:
        f.write(xml)


def _weights(sigma, mask):
    with np.errstate(divide="ignore"):
        w = np.where(mask & (sigma > 0), 1.0 / np.where(sigma > 0, sigma, 1.0) ** 2, 0.0)
    return sp.dia_matrix((w.ravel(), 0), shape=(w.size, w.size)).tocsr()


def _crop(a, roi):
    if roi is None:
        return a
    ulx, uly, lrx, lry = roi
    return a[uly:lry, ulx:lrx]


class _StateGrid:
    """The state mask's raster grid, onto which every band is warped.

    ``state_mask`` is a GeoTIFF path (the reference's form: a file or VRT
    handed to ``gdal.Warp`` as the target, ``kafka_test_S2.py:155-160``) or an
    array with ``geotransform`` / ``projection``.  A bare array carries no
    geometry: the reader then keeps the granule grid (cropped to ``roi``)."""

    def __init__(self, state_mask, geotransform=None, projection=None):
        self.geo = False
        if isinstance(state_mask, (str, os.PathLike)):
            arr, info = read_tiff(state_mask)
            self.mask = np.asarray(arr).astype(bool)
            geotransform = info.get("geotransform")
            projection = info.get("epsg") or info.get("projection")
            self.projection = info.get("projection", "")
        else:
            self.mask = None if state_mask is None else np.asarray(state_mask).astype(bool)
            self.projection = "" if projection is None else projection
        self.crs = projection
        if geotransform is not None:
            self.geo = True
            self.gt = [float(v) for v in geotransform]
            self.shape = self.mask.shape
        self._warps = {}

    def warp_for(self, path):
        """GridWarp from the raster at ``path`` onto this grid (cached per source grid)."""
        from .tiff import tiff_info
        from .utils import GridWarp

        i = tiff_info(path)
        key = (i["shape"], tuple(i.get("geotransform", ())), i.get("epsg") or i.get("projection"))
        w = self._warps.get(key)
        if w is None:
            w = self._warps[key] = GridWarp(i["shape"], i.get("geotransform", [0, 1, 0, 0, 0, -1]), self.shape,
                                            self.gt, key[2], self.crs)
        return w

    def read(self, path, band=0, nodata=0):
        """A band warped onto the grid (host path); equals ``reproject_image``."""
        return self.warp_for(path).read(path, band, nodata)


# ------------------------------------------------------------- Sentinel-2
class Sentinel2Observations:
    """Sentinel-2 L2 surface-reflectance granules (``Sentinel2_Observations.py``).

    Host protocol: ``get_band_data`` returns the reference's ``S2MSIdata``
    record (reflectance, sparse inverse-variance diagonal, mask, angles,
    emulator).  Device protocol (after ``bind_engine``): every band of a date
    is decoded as raw uint16 DN by the native reader straight into a pinned
    slot, copied on the ingest stream, gathered onto the strip's active pixels
    and decoded inside the analysis kernel (``OBS_DN16``: reflectance = DN x
    1e-4, valid = DN > 0, sigma = rel_unc x reflectance, weight = 1 / sigma^2 —
    the reference's :163-179 without the N x N sparse weight matrix).
    ``prefetch(date)`` starts the next date's decode under the current
    kernels.

    Grids: with a georeferenced state mask (a GeoTIFF path, or an array plus
    ``mask_geotransform`` / ``mask_projection``) every band is warped onto the
    mask's grid, nearest neighbour, as the reference's ``reproject_image``
    call does (:166), and ``define_output`` returns the mask's geometry
    (:100-113).  The host path decodes the bounding source window and warps
    it (``GridWarp.read``, bit-identical to ``reproject_image``).  The device
    path computes once per (band grid, strip) the source pixel under every
    active state pixel; the pinned slot receives only the bounding source
    window and the warp is the one gather that compacts the strip anyway
    (uncovered pixels read as DN 0 = no data).  A mask without geometry
    keeps the granule grid, cropped to ``roi``."""

    def __init__(self, parent_folder, emulator_folder, state_mask, chunk=None, roi=None, rel_unc=0.05,
                 device_ingest: bool = True, mask_geotransform=None, mask_projection=None):
        if not os.path.exists(parent_folder):
            raise IOError("S2 data folder doesn't exist")
        self.device_ingest = device_ingest
        self.parent = parent_folder
        self.emulator_folder = emulator_folder
        self.state_mask = state_mask
        self.grid = _StateGrid(state_mask, mask_geotransform, mask_projection)
        if self.grid.geo and roi is not None:
            raise ValueError("roi crops the granule grid; with a georeferenced state mask the mask defines the grid")
        self.roi = roi
        self.rel_unc = rel_unc
        self.band_map = list(S2_BAND_MAP)
        self.emulator_files = sorted(glob.glob(os.path.join(emulator_folder, "*.npz")))
        self._find_granules(parent_folder)
        self._emu_cache = {}
        self._meta_cache = {}
        self.chunk = chunk
        self._ingest = None

    def _find_granules(self, parent_folder):
        self.dates, self.date_data = [], {}
        for root, dirs, files in os.walk(parent_folder):
            if "aot.tif" in files:
                parts = root.rstrip("/").split("/")
                y, m, d = (int(v) for v in parts[-4:-1])
                date = datetime.datetime(y, m, d)
                self.dates.append(date)
                self.date_data[date] = root
        self.dates.sort()
        self.bands_per_observation = {d: len(self.band_map) for d in self.dates}

    def define_output(self):
        if self.grid.geo:                  # the state mask's geometry (:100-113)
            return self.grid.projection, list(self.grid.gt)
        from .tiff import tiff_info
        ref = glob.glob(os.path.join(self.date_data[self.dates[0]], "B02_sur.tif"))
        info = tiff_info(ref[0]) if ref else {}
        gt = list(info.get("geotransform", [0, 1, 0, 0, 0, -1]))
        if self.roi is not None:
            gt[0] += self.roi[0] * gt[1]
            gt[3] += self.roi[1] * gt[5]
        return info.get("projection", ""), gt

    def _find_emulator(self, sza, saa, vza, vaa):
        raa = vaa - saa
        vzas = np.array([float(os.path.basename(s).split("_")[-3]) for s in self.emulator_files])
        szas = np.array([float(os.path.basename(s).split("_")[-2]) for s in self.emulator_files])
        raas = np.array([float(os.path.basename(s).split("_")[-1].rsplit(".", 1)[0]) for s in self.emulator_files])
        e1 = szas == szas[np.argmin(np.abs(szas - sza))]
        e2 = vzas == vzas[np.argmin(np.abs(vzas - vza))]
        e3 = raas == raas[np.argmin(np.abs(raas - raa))]
        hit = np.where(e1 * e2 * e3)[0]
        if hit.size:
            return self.emulator_files[hit[0]]
        # no file matches all three independently-nearest angles (the reference
        # would raise IndexError here): nearest in joint angle space
        dist = (szas - sza) ** 2 + (vzas - vza) ** 2 + (raas - raa) ** 2
        return self.emulator_files[int(np.argmin(dist))]

    def _date_meta(self, timestep):
        """(angles dict, emulator set) of a date, parsed once."""
        if timestep not in self._meta_cache:
            folder = self.date_data[timestep]
            sza, saa, vza, vaa = parse_xml(os.path.join(folder, "metadata.xml"))
            metadata = dict(zip(["sza", "saa", "vza", "vaa"], [sza, saa, vza, vaa]))
            efile = self._find_emulator(sza, saa, vza, vaa)
            if efile not in self._emu_cache:  # the reference re-unpickled per band and iteration
                self._emu_cache[efile] = self._load_emulators(efile)
            self._meta_cache[timestep] = (metadata, self._emu_cache[efile])
        return self._meta_cache[timestep]

    def _load_emulators(self, efile):
        """Emulator set of a file.  Bound to a multi-rank engine, only rank 0
        reads and parses it; the others receive it by C4 (one tensor broadcast,
        ``Comm.broadcast_packed``).  Every rank asks for the same dates in the
        same order, so the collective is matched."""
        comm = getattr(self, "_comm", None)
        if comm is None or not comm.distributed:
            return load_emulator_set(efile)
        header, buf = pack_emulator_set(load_emulator_set(efile)) if comm.rank == 0 else (None, None)
        header, buf = comm.broadcast_packed(header, buf)
        self.c4_broadcasts = getattr(self, "c4_broadcasts", 0) + 1
        return unpack_emulator_set(header, buf)

    def get_band_data(self, timestep, band):
        folder = self.date_data[timestep]
        metadata, ems = self._date_meta(timestep)
        path = os.path.join(folder, f"B{self.band_map[band]}_sur.tif")
        if self.grid.geo:                  # warp onto the state grid (:166)
            rho = self.grid.read(path).astype(np.float64)
        else:
            rho = _crop(read_tiff(path)[0].astype(np.float64), self.roi)
        mask = rho > 0
        rho = np.where(mask, rho / 10000., 0.0)
        unc = _weights(rho * self.rel_unc, mask)
        key = f"S2A_MSI_{S2_EMULATOR_BANDS[band]:02d}"
        return S2MSIdata(rho, unc, mask, metadata, ems.get(key))

    # ---------------------------------------------------------- device path
    def bind_engine(self, engine):
        """Device ingest for ``engine``'s strip (called by LinearKalman)."""
        import torch

        from ..ops import kernels as K
        from .streaming import RasterIngest

        self._comm = getattr(engine, "comm", None)
        if not self.device_ingest:
            return
        self.partition = part = engine.partition
        self._device = engine.device
        self._K = K
        H, W = part.local_mask.shape
        self._warp_plan = None
        self._date_files = {}
        if self.grid.geo:
            if self.grid.shape != part.state_mask.shape:
                raise ValueError(f"state mask {self.grid.shape} differs from the engine's {part.state_mask.shape}")
            plan = self._plan_warp(self.dates[0])
            if plan is not None:
                self._warp_plan = plan
                elems = max((w[1] - w[0]) * (w[3] - w[2]) for w in plan["windows"].values())
                self._ingest = RasterIngest(len(self.band_map), (1, elems), torch.int16, self._device)
                return
        ulx, uly = (self.roi[0], self.roi[1]) if self.roi is not None else (0, 0)
        self._window = (uly + part.r0, uly + part.r0 + H, ulx, ulx + W)
        self._ingest = RasterIngest(len(self.band_map), (H, W), torch.int16, self._device)
        self._identity = part.N == H * W
        self._idx = None if self._identity else torch.from_numpy(part.local_idx).to(self._device)

    def _band_paths(self, timestep):
        folder = self.date_data[timestep]
        return [os.path.join(folder, f"B{b}_sur.tif") for b in self.band_map]

    def _plan_warp(self, timestep):
        """Per band grid: the strip's bounding source window and, for every
        active state pixel of the strip, its index into that window (-1 = not
        covered).  None when every band's grid is the state grid (the crop
        path is then exact)."""
        import torch

        part = self.partition
        warps = [self.grid.warp_for(p) for p in self._band_paths(timestep)]
        if all(w.identity for w in warps):
            return None
        windows, idx, band_key = {}, {}, []
        for w in warps:
            k = w.key()
            band_key.append(k)
            if k in windows:
                continue
            flat = w.index_of_mask(part.local_mask, row0=part.r0)
            win = w.window(flat)
            windows[k] = win
            idx[k] = torch.from_numpy(w.local(flat, win)).to(self._device)
        return {"windows": windows, "idx": idx, "band_key": band_key}

    def _files(self, timestep):
        hit = self._date_files.get(timestep)
        if hit is not None:
            return hit
        paths = self._band_paths(timestep)
        if self._warp_plan is None:
            files = [(p, 0, self._window) for p in paths]
        else:
            plan = self._warp_plan
            keys = [self.grid.warp_for(p).key() for p in paths]
            if keys != plan["band_key"]:
                raise ValueError(f"{self.date_data[timestep]}: band grids differ from the first date's; "
                                 "one reader covers one granule grid")
            files = [(p, 0, plan["windows"][k]) for p, k in zip(paths, keys)]
        if len(self._date_files) > 64:
            self._date_files.clear()
        self._date_files[timestep] = files
        return files

    def prefetch(self, timestep):
        if self._ingest is not None and timestep in self.date_data:
            self._ingest.prefetch(timestep, self._files(timestep))

    def __getattr__(self, name):
        # the engine probes hasattr(obs, "get_device_band_data"): only bound
        # readers expose the device protocol
        if name == "get_device_band_data" and self.__dict__.get("_ingest") is not None:
            return self._get_device_band_data
        raise AttributeError(name)

    def _get_device_band_data(self, timestep, band):
        from ..engine.bands import DeviceBand

        metadata, ems = self._date_meta(timestep)
        key = f"S2A_MSI_{S2_EMULATOR_BANDS[band]:02d}"
        planes = self._ingest.acquire(timestep, self._files(timestep))
        dn = planes[band].reshape(-1)
        if self._warp_plan is not None:    # warp + compaction: one gather (-1 -> DN 0)
            dn = self._K.gather(dn, self._warp_plan["idx"][self._warp_plan["band_key"][band]])
        elif not self._identity:
            dn = self._K.gather(dn, self._idx)
        return DeviceBand(self._K.OBS_DN16, dn=dn, scale=1e-4, rel_unc=self.rel_unc, unc_floor=0.0,
                          metadata=metadata, emulator=ems.get(key))


def write_s2_archive(root, dn_by_date: dict, emulators: dict, geotransform=None, projection=None,
                     angles=(31.0, 0.0, 8.0, 118.0), emulator_angles=((8.0, 31.0, 118.0),)):
    """Synthetic on-disk S2 archive in the reader's layout:
    ``root/data/YYYY/MM/DD/<granule>/{B02..B12}_sur.tif`` (uint16 DN x 1e4,
    tiled DEFLATE), ``aot.tif``, ``metadata.xml``; ``root/emus/*_{vza}_{sza}_{raa}.npz``.
    ``dn_by_date``: {date: uint16 array [10, H, W]}; ``emulators``: {key: emulator}
    with keys ``S2A_MSI_{band:02d}``.  Returns (data folder, emulator folder)."""
    data = os.path.join(root, "data")
    emus = os.path.join(root, "emus")
    os.makedirs(emus, exist_ok=True)
    for vza, sza, raa in emulator_angles:
        save_emulator_set(os.path.join(emus, f"prosail_{vza:g}_{sza:g}_{raa:g}.npz"), emulators)
    for date, dn in dn_by_date.items():
        g = os.path.join(data, f"{date.year:04d}", f"{date.month:02d}", f"{date.day:02d}", "S2A_GRANULE")
        os.makedirs(g, exist_ok=True)
        for i, b in enumerate(S2_BAND_MAP):
            write_tiff(os.path.join(g, f"B{b}_sur.tif"), np.asarray(dn[i], dtype=np.uint16), geotransform,
                       projection)
        write_tiff(os.path.join(g, "aot.tif"), np.zeros((8, 8), np.uint8))
        write_s2_metadata(os.path.join(g, "metadata.xml"), *angles)
    return data, emus


# ------------------------------------------------------------- Sentinel-1
class S1Observations:
    """Sentinel-1 sigma0 (``Sentinel1_Observations.py``).  With a georeferenced
    state mask (GeoTIFF path, or array plus ``mask_geotransform`` /
    ``mask_projection``) sigma0 and the incidence angle are warped onto the
    mask's grid, nearest neighbour, like the reference's ``reproject_image``
    calls (:178,194); uncovered pixels read -999 (no data)."""

    POLS = ("VV", "VH")

    def __init__(self, data_folder, state_mask, emulators=None, roi=None, rel_unc=0.05, mask_geotransform=None,
                 mask_projection=None):
        self.state_mask = state_mask
        self.grid = _StateGrid(state_mask, mask_geotransform, mask_projection)
        if self.grid.geo and roi is not None:
            raise ValueError("roi crops the acquisition grid; with a georeferenced state mask the mask defines it")
        self.roi = roi
        self.rel_unc = rel_unc
        self.dates, self.date_data = [], {}
        for d in sorted(glob.glob(os.path.join(data_folder, "S1_*"))):
            fields = os.path.basename(d).split("_")
            date = datetime.datetime.strptime(fields[5] if len(fields) > 5 else fields[-1], "%Y%m%dT%H%M%S")
            self.dates.append(date)
            self.date_data[date] = d
        self.emulators = emulators or {"VV": None, "VH": None}
        self.bands_per_observation = {d: 2 for d in self.dates}

    def define_output(self):
        if self.grid.geo:
            return self.grid.projection, list(self.grid.gt)
        from .tiff import tiff_info
        info = tiff_info(os.path.join(self.date_data[self.dates[0]], "theta.tif"))
        gt = list(info.get("geotransform", [0, 1, 0, 0, 0, -1]))
        if self.roi is not None:
            gt[0] += self.roi[0] * gt[1]
            gt[3] += self.roi[1] * gt[5]
        return info.get("projection", ""), gt

    def _read(self, path):
        if self.grid.geo:                  # warp onto the state grid (:178,194)
            return self.grid.read(path, nodata=WRONG_VALUE).astype(np.float64)
        return _crop(read_tiff(path)[0].astype(np.float64), self.roi)

    def get_band_data(self, timestep, band):
        pol = self.POLS[band]
        folder = self.date_data[timestep]
        s0 = self._read(os.path.join(folder, f"sigma0_{pol}.tif"))
        mask = s0 != WRONG_VALUE
        unc = _weights(np.where(mask, s0 * self.rel_unc, 0.0), mask)
        meta = {"incidence_angle": self._read(os.path.join(folder, "theta.tif"))}
        return SARdata(np.where(mask, s0, 0.0), unc, mask, meta, self.emulators.get(pol))


# ------------------------------------------------------------- MODIS BHR
class BHRObservations:
    """MCD43-like broadband BHR observations (VIS/NIR) from kernel-weight rasters."""

    def __init__(self, emulator, folder, start_time=None, end_time=None, period=16, ulx=0, uly=0, lrx=None,
                 lry=None):
        self.emulator = emulator if not isinstance(emulator, (str, os.PathLike)) else load_emulator_set(emulator)
        files = sorted(glob.glob(os.path.join(folder, "*_kernels_b0_k0.tif")))
        dates = [datetime.datetime.strptime(os.path.basename(f).split("_")[0], "A%Y%j") for f in files]
        if start_time is not None:
            dates = [d for d in dates if d >= start_time]
        if end_time is not None:
            dates = [d for d in dates if d <= end_time]
        self.folder = folder
        self.dates = dates[::period]
        self.bands_per_observation = {d: 2 for d in self.dates}
        self.apply_roi(ulx, uly, lrx, lry)

    def apply_roi(self, ulx, uly, lrx, lry):
        self.ulx, self.uly, self.lrx, self.lry = ulx, uly, lrx, lry
        self.roi = None if lrx is None else [ulx, uly, lrx, lry]

    def define_output(self):
        f = glob.glob(os.path.join(self.folder, self.dates[0].strftime("A%Y%j") + "_kernels_b0_k0.tif"))[0]
        info = read_tiff(f)[1]
        gt = list(info.get("geotransform", [0, 1, 0, 0, 0, -1]))
        gt[0] += self.ulx * gt[1]
        gt[3] += self.uly * gt[5]
        return info.get("projection", ""), gt

    def get_band_data(self, the_date, band_no):
        tag = the_date.strftime("A%Y%j")
        try:
            K = np.stack([read_tiff(os.path.join(self.folder, f"{tag}_kernels_b{band_no}_k{k}.tif"))[0]
                          for k in range(3)]).astype(np.float64)
        except FileNotFoundError:
            return None
        qa, _ = read_tiff(os.path.join(self.folder, f"{tag}_qa.tif"))
        K = np.stack([_crop(k, self.roi) for k in K])
        qa = _crop(qa, self.roi)
        mask = (qa <= 1) & np.all(np.isfinite(K), axis=0)
        bhr = np.where(mask, np.tensordot(TO_BHR, K, axes=1), 0.0)
        sig = np.where(qa == 1, np.maximum(2.5e-3, 0.07 * bhr), np.maximum(2.5e-3, 0.05 * bhr))
        em = self.emulator[band_no] if isinstance(self.emulator, (list, tuple)) else \
            (self.emulator.get(str(band_no)) if isinstance(self.emulator, dict) else self.emulator)
        return BHR_data(bhr, mask, _weights(sig, mask), None, em)


# ------------------------------------------------------------- Ross-Li
def ross_li_kernels(vza, sza, raa, br=1.0, hb=2.0):
    """RossThick and LiSparse-Reciprocal BRDF kernels (angles in degrees) — the
    MODIS kernel model the reference obtains from SIAC (observations.py:141-143)."""
    vz, sz, ra = (np.deg2rad(np.asarray(a, dtype=np.float64)) for a in (vza, sza, raa))
    cos_xi = np.cos(sz) * np.cos(vz) + np.sin(sz) * np.sin(vz) * np.cos(ra)
    xi = np.arccos(np.clip(cos_xi, -1, 1))
    k_vol = ((np.pi / 2 - xi) * cos_xi + np.sin(xi)) / (np.cos(sz) + np.cos(vz)) - np.pi / 4
    tvp = np.arctan(br * np.tan(vz))
    tip = np.arctan(br * np.tan(sz))
    cos_xip = np.cos(tip) * np.cos(tvp) + np.sin(tip) * np.sin(tvp) * np.cos(ra)
    D = np.sqrt(np.tan(tip) ** 2 + np.tan(tvp) ** 2 - 2 * np.tan(tip) * np.tan(tvp) * np.cos(ra))
    sec = 1 / np.cos(tip) + 1 / np.cos(tvp)
    cos_t = np.clip(hb * np.sqrt(D ** 2 + (np.tan(tip) * np.tan(tvp) * np.sin(ra)) ** 2) / sec, -1, 1)
    t = np.arccos(cos_t)
    O = (t - np.sin(t) * cos_t) * sec / np.pi
    k_geo = O - sec + 0.5 * (1 + cos_xip) / np.cos(tip) / np.cos(tvp)
    return np.ones_like(k_vol), k_vol, k_geo
