"""MODIS readers: MOD09 surface reflectance with Ross-Li kernels, and Synergy
kernel-weight stacks (``kafka/input_output/observations.py:89-211``).

The reference reads HDF4-EOS grids through GDAL and builds the BRDF kernels with
``SIAC.kernels.Kernels``.  Neither GDAL nor HDF4 nor SIAC exists in this stack:

* HDF access goes through a pluggable ``reader(filename, sds_name) -> ndarray``.
  The default reader takes a ``.npz`` archive (loaded with
  ``allow_pickle=False``) or a directory of ``<sds_name>.tif`` rasters holding
  the SDS arrays under their HDF names (``sur_refl_b01_1``, ``state_1km_1``,
  ``SolarZenith_1``, ...); a ``.hdf`` file without a reader raises.
* ``Kernels`` wraps ``sentinel.ross_li_kernels``, the MODIS kernel set the reference requests
  (``LiType="Sparse"``, ``RossType="Thick"``, ``RecipFlag=True``,
  ``MODISSPARSE=True``: h/b = 2, b/r = 1; Lucht, Schaaf & Strahler 2000,
  IEEE TGRS 38(2), eqs. 37-46).  Both kernels are zero at nadir/nadir, so the
  reference's ``normalise=1`` is the identity for this set.

``SynergyKernels.get_band_data`` computes the broadband BHR exactly like the
reference (``observations.py:186-211``) and, unlike it, returns the record
(the reference function falls off the end and returns ``None``).
"""
from __future__ import annotations

import datetime
import glob
import os

import numpy as np
import scipy.sparse as sp

from .observations import BHR_data
from .sentinel import ross_li_kernels

from .records import MOD09_data  # noqa: F401  (re-export)

# observations.py:100-103
MOD09_QA_OK = np.array([8, 72, 136, 200, 1032, 1288, 2056, 2120, 2184, 2248])
MOD09_BAND_SIGMA = [0.004, 0.015, 0.003, 0.004, 0.013, 0.010, 0.006]

# observations.py:191-196
TO_BHR = np.array([1.0, 0.189184, -1.377622])
TO_VIS = np.array([0.3265, 0., 0.4364, 0.2366, 0, 0, 0])
A_TO_VIS = -0.0019
TO_NIR = np.array([0., 0.5447, 0, 0, 0.1363, 0.0469, 0.2536])
A_TO_NIR = -0.0068


class Kernels:
    """Isotropic / RossThick / LiSparse-R kernel values (SIAC ``Kernels`` fields)."""

    def __init__(self, vza, sza, raa, hb: float = 2.0, br: float = 1.0):
        self.vza, self.sza, self.raa = (np.asarray(a, np.float64) for a in (vza, sza, raa))
        self.Isotropic, self.Ross, self.Li = ross_li_kernels(self.vza, self.sza, self.raa, br=br, hb=hb)

    def design_matrix(self):
        """(..., 3) [iso, vol, geo] — f = K @ [f_iso, f_vol, f_geo]."""
        return np.stack([self.Isotropic, self.Ross, self.Li], -1)


def default_hdf_reader(fname: str, sds: str) -> np.ndarray:
    """SDS arrays from a ``.npz`` archive or a directory of ``<sds>.tif``."""
    if os.path.isdir(fname):
        from .tiff import read_tiff
        return read_tiff(os.path.join(fname, sds + ".tif"))[0]
    if fname.endswith(".npz"):
        with np.load(fname, allow_pickle=False) as z:
            return np.asarray(z[sds])
    raise IOError(f"cannot read {sds} from {fname}: HDF4 needs a reader callable "
                  "(no GDAL/pyhdf in this stack); pass reader=")


def _zoom2(a):
    """2x nearest-neighbour zoom (scipy.ndimage.zoom(order=0) for factor 2)."""
    return np.repeat(np.repeat(np.asarray(a), 2, axis=0), 2, axis=1)


class MOD09_ObservationsKernels:
    """Generic M*D09GA reader (``observations.py:89-147``): reflectance /1e4
    (500 m), QA whitelist mask and angles /100 (1 km, zoomed 2x), Ross-Li
    kernels, a fixed per-band sigma.  Returns ``MOD09_data`` (``uncertainty``
    is sigma, as in the reference; ``weights()`` gives 1/sigma^2)."""

    def __init__(self, dates, filenames, reader=None):
        if not len(dates) == len(filenames):
            raise ValueError("{} dates, {} filenames".format(len(dates), len(filenames)))
        self.dates = list(dates)
        self.filenames = list(filenames)
        self.reader = reader or default_hdf_reader
        self.bands_per_observation = {d: 7 for d in self.dates}

    def get_band_data(self, the_date, band_no):
        try:
            iloc = self.dates.index(the_date)
        except ValueError:
            return None
        fname = self.filenames[iloc]
        rd = self.reader
        refl = rd(fname, "sur_refl_b0{}_1".format(band_no)) / 10000.
        qa = rd(fname, "state_1km_1")
        mask = np.isin(qa, MOD09_QA_OK).reshape(qa.shape)
        sza = rd(fname, "SolarZenith_1") / 100.
        saa = rd(fname, "SolarAzimuth_1") / 100.
        vza = rd(fname, "SensorZenith_1") / 100.
        vaa = rd(fname, "SensorAzimuth_1") / 100.
        raa = vaa - saa
        raa, vza, sza, mask = _zoom2(raa), _zoom2(vza), _zoom2(sza), _zoom2(mask)
        K = Kernels(vza, sza, raa)
        uncertainty = refl * 0 + MOD09_BAND_SIGMA[band_no - 1]
        return MOD09_data(refl, mask, uncertainty, K, sza, vza, raa)

    @staticmethod
    def weights(rec: MOD09_data):
        """Inverse-variance weights, 0 where masked."""
        return np.where(rec.mask, 1.0 / np.asarray(rec.uncertainty) ** 2, 0.0)


def _synergy_date(fname):
    return datetime.datetime.strptime(os.path.basename(fname).split(".")[1][1:], "%Y%j")


class SynergyKernels:
    """Linear kernel-weight stacks from the Synergy chain (``observations.py:150-211``).

    Files ``<dir>/*.<tile>*_b{0..6}_kernel_weights.tif`` hold (3, ny, nx)
    [iso, vol, geo] weights per MODIS band; ``..._kernel_unc.tif`` their sigmas
    (optional) and ``...mask.tif`` the valid mask (optional).  Band 0 of
    ``get_band_data`` is broadband VIS, band 1 NIR.

    The reference keeps dates with ``start_time >= date`` (``:163``), i.e. the
    dates *before* the start; the default here is the evident intent
    ``start_time <= date <= end_time``; ``reference_quirks=True`` restores it.
    """

    def __init__(self, directory, tile, start_time, end_time=None, emulator=None, reference_quirks: bool = False):
        fnames = sorted(glob.glob("%s/*.%s*_b0_kernel_weights.tif" % (directory, tile)))
        self.dates, self.kernels, self.uncertainties, self.masks = [], [], [], []
        for fname in fnames:
            date = _synergy_date(fname)
            keep = (start_time >= date) if reference_quirks else (start_time <= date)
            if keep and (end_time is None or date <= end_time):
                self.add_observations(date, fname, fname.replace("kernel_weights", "kernel_unc"),
                                      fname.replace("_b0_kernel_weights", "mask"))
        self.emulator = emulator

    @property
    def bands_per_observation(self):
        return {d: 2 for d in self.dates}

    def add_observations(self, the_date, the_kernels, the_uncs, the_mask):
        self.dates.append(the_date)
        self.kernels.append(the_kernels)
        self.uncertainties.append(the_uncs)
        self.masks.append(the_mask)

    def get_band_data(self, the_date, band_no):
        """Broadband BHR (VIS for 0, NIR for 1) with 1/sigma^2 weights."""
        from .tiff import read_tiff
        date_idx = self.dates.index(the_date)
        bhr, var = [], []
        for band in range(7):
            k = read_tiff(self.kernels[date_idx].replace("b0", "b%d" % band))[0].astype(np.float64)
            bhr.append(np.sum(k * TO_BHR[:, None, None], axis=0))
            ufile = self.uncertainties[date_idx].replace("b0", "b%d" % band)
            if os.path.exists(ufile):   # independent kernel errors
                u = read_tiff(ufile)[0].astype(np.float64)
                var.append(np.sum((u * TO_BHR[:, None, None]) ** 2, axis=0))
        bhr = np.array(bhr)
        coef, off = (TO_VIS, A_TO_VIS) if band_no == 0 else (TO_NIR, A_TO_NIR)
        bb = np.sum(bhr * coef[:, None, None], axis=0) + off
        if len(var) == 7:
            sigma2 = np.sum(np.array(var) * (coef ** 2)[:, None, None], axis=0)
        else:                           # the BHR uncertainty model of observations.py:300-302
            sigma2 = np.maximum(2.5e-3, 0.05 * np.abs(bb)) ** 2
        mask = np.isfinite(bb) & (sigma2 > 0)
        if os.path.exists(self.masks[date_idx]):
            mask &= read_tiff(self.masks[date_idx])[0].astype(bool)
        w = np.where(mask, 1.0 / np.where(sigma2 > 0, sigma2, 1.0), 0.0)
        unc = sp.dia_matrix((w.ravel(), 0), shape=(w.size, w.size)).tocsr()
        em = self.emulator[band_no] if isinstance(self.emulator, (list, tuple, dict)) else self.emulator
        return BHR_data(np.where(mask, bb, 0.0), mask, unc, {"band": ("VIS", "NIR")[band_no]}, em)
