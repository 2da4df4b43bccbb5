"""In-memory observation sources with the reference protocol.

* ``ArrayObservations`` — user-supplied rasters per (date, band): the
  generic way to feed real data (already on the state grid).
* ``BHRObservationsTest`` — single-pixel VIS/NIR albedo holder
  (``observations.py:313-335``), finished: ``get_band_data`` returns the BHR
  record with the 5 %/2.5e-3 uncertainty model.
* ``get_modis_dates`` — ``AYYYYDDD`` from MODIS file names (:75-83).
"""
from __future__ import annotations

import datetime
import os

import numpy as np
import scipy.sparse as sp

from .records import BHR_data, ObsData  # noqa: F401  (re-exports)


def get_modis_dates(fnames):
    dates = []
    for fname in fnames:
        txt = os.path.basename(fname).split(".")[1][1:]
        dates.append(datetime.datetime.strptime(txt, "%Y%j"))
    return dates


def bhr_uncertainty(bhr, qa_level=None, floor=2.5e-3):
    """sigma = max(floor, 5 % BHR) for QA 0, 7 % for QA 1 (observations.py:300-302)."""
    bhr = np.asarray(bhr, dtype=np.float64)
    rel = np.where(np.asarray(qa_level if qa_level is not None else 0) == 1, 0.07, 0.05)
    return np.maximum(floor, bhr * rel)


class ArrayObservations:
    """Observations from in-memory rasters.

    ``data[date] = [(y_raster, sigma_raster_or_weight, mask_raster), ...]`` per
    band; ``weights=True`` means the second item is already 1/sigma^2."""

    def __init__(self, data: dict, emulators=None, metadata=None, weights: bool = False):
        self.data = data
        self.dates = sorted(data.keys())
        self.bands_per_observation = {d: len(v) for d, v in data.items()}
        self.emulators = emulators
        self.metadata = metadata or {}
        self.weights = weights

    def get_band_data(self, the_date, band_no):
        y, s, m = self.data[the_date][band_no]
        y = np.asarray(y, dtype=np.float64)
        m = np.asarray(m).astype(bool)
        if self.weights:
            w = np.asarray(s, dtype=np.float64)
        else:
            s = np.asarray(s, dtype=np.float64)
            with np.errstate(divide="ignore"):
                w = np.where(m & (s > 0), 1.0 / np.where(s > 0, s, 1.0) ** 2, 0.0)
        w = np.where(m, w, 0.0)
        unc = sp.dia_matrix((w.ravel(), 0), shape=(w.size, w.size)).tocsr()
        em = self.emulators[band_no] if isinstance(self.emulators, (list, tuple)) else self.emulators
        return ObsData(np.where(m, y, 0.0), unc, m, self.metadata.get(band_no, {}), em)


class BHRObservationsTest:
    """One pixel, two broadband albedos per date (VIS, NIR)."""

    def __init__(self, dates, vis_albedo, nir_albedo, emulators=None):
        assert len(dates) == len(vis_albedo) == len(nir_albedo)
        self.dates = list(dates)
        self.values = {d: [float(v), float(n)] for d, v, n in zip(dates, vis_albedo, nir_albedo)}
        self.bands_per_observation = {d: 2 for d in self.dates}
        self.emulators = emulators

    def get_band_data(self, the_date, band_no):
        bhr = np.array([[self.values[the_date][band_no]]])
        mask = np.ones((1, 1), dtype=bool)
        R = 1. / bhr_uncertainty(bhr) ** 2
        em = self.emulators[band_no] if self.emulators is not None else None
        return BHR_data(bhr, mask, sp.csr_matrix(R.reshape(1, 1)), None, em)
