"""Priors: JRC-TIP (7 params) and SAIL/PROSAIL (10 params) Gaussian priors.

Constants from the reference: ``tip_prior`` (``kafka/inference/kf_tools.py:99-116``),
``JRCPrior._tip_prior`` (``kafka_test.py:102-119``, TLAI mean exp(-1)),
``SAILPrior`` (``kafka_test_S2.py:79-118``).  Every prior here implements the
reference protocol ``process_prior(date, inv_cov=True) -> (mean_vec,
sparse_inv_cov)`` and additionally exposes ``device_prior(date)`` — a per-pixel
constant ``(mean[n_p], cinv[n_p, n_p])`` (or per-pixel SoA arrays) that the
engine hands straight to the propagate/blend kernel without building an
(n_p·N)² matrix.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

from ..utils.blocks import blocks_to_sparse

TIP_PARAMETERS = ["w_vis", "x_vis", "a_vis", "w_nir", "x_nir", "a_nir", "TeLAI"]
SAIL_PARAMETERS = ["n", "cab", "car", "cbrown", "cw", "cm", "lai", "ala", "bsoil", "psoil"]


def tip_prior(tlai_mean: float = np.exp(-0.5 * 1.5)):
    """JRC-TIP prior (mean, covariance, inverse covariance) — kf_tools.py:99-116.

    TLAI = exp(-LAIe/2).  The covariance is assembled in float32 (as the
    reference does) and inverted in float64.
    """
    sigma = np.array([0.12, 0.7, 0.0959, 0.15, 1.5, 0.2, 0.5])
    x0 = np.array([0.17, 1.0, 0.1, 0.7, 2.0, 0.18, tlai_mean])
    little_p = np.diag(sigma ** 2).astype(np.float32)
    little_p[5, 2] = 0.8862 * 0.0959 * 0.2
    little_p[2, 5] = 0.8862 * 0.0959 * 0.2
    inv_p = np.linalg.inv(little_p)
    return x0, little_p, inv_p


def sail_prior():
    """SAIL (PROSAIL 10-parameter, transformed space) prior — kafka_test_S2.py:84-94."""
    mean = np.array([2.1, np.exp(-60. / 100.), np.exp(-7.0 / 100.), 0.1, np.exp(-50 * 0.0176),
                     np.exp(-100. * 0.002), np.exp(-4. / 2.), 70. / 90., 0.5, 0.9])
    sigma = np.array([0.01, 0.2, 0.01, 0.05, 0.01, 0.01, 0.50, 0.1, 0.1, 0.1])
    covar = np.diag(sigma ** 2).astype(np.float32)
    inv_covar = np.diag(1. / sigma ** 2).astype(np.float32)
    return mean, covar, inv_covar


@dataclass
class DevicePrior:
    """A prior the kernels consume directly: constant per pixel (mean[n], cinv[n,n])
    or spatially varying (mean_soa[n, N], cinv_packed[ntri, N])."""
    mean: np.ndarray | None = None
    cinv: np.ndarray | None = None
    mean_soa: object = None
    cinv_packed: object = None

    @property
    def constant(self) -> bool:
        return self.mean is not None


class GaussianPrior:
    """Per-pixel i.i.d. Gaussian prior with the reference ``process_prior`` API."""

    def __init__(self, parameter_list, state_mask, mean, covar):
        self.parameter_list = list(parameter_list)
        if isinstance(state_mask, (str, os.PathLike)):
            state_mask = _read_mask(state_mask)
        self.state_mask = np.asarray(state_mask).astype(bool)
        self.mean = np.asarray(mean, dtype=np.float64)
        self.covar = np.asarray(covar, dtype=np.float64)
        self.inv_covar = np.linalg.inv(self.covar)
        if len(self.mean) != len(self.parameter_list):
            raise ValueError("prior mean length differs from parameter list")

    def device_prior(self, date=None) -> DevicePrior:
        return DevicePrior(mean=self.mean.copy(), cinv=self.inv_covar.copy())

    def process_prior(self, time, inv_cov=True):
        n_pixels = int(self.state_mask.sum())
        x0 = np.tile(self.mean, n_pixels)
        mat = self.inv_covar if inv_cov else self.covar
        blocks = np.broadcast_to(mat.astype(np.float32), (n_pixels,) + mat.shape)
        return x0, blocks_to_sparse(np.ascontiguousarray(blocks), "csr")


class JRCPrior(GaussianPrior):
    """JRC-TIP prior object used by the BHR drivers (kafka_test.py:84-133)."""

    def __init__(self, parameter_list, state_mask, tlai_mean: float = np.exp(-0.5 * 2.0)):
        mean, covar, _ = tip_prior(tlai_mean)
        super().__init__(parameter_list, state_mask, mean, covar.astype(np.float64))
        self.inv_covar = np.linalg.inv(covar)  # float32 assembly, as the reference


class SAILPrior(GaussianPrior):
    """SAIL prior (kafka_test_S2.py:79-118); mean/covar are always defined here
    (the reference only set them when the mask was a filename)."""

    def __init__(self, parameter_list, state_mask):
        mean, covar, inv_covar = sail_prior()
        super().__init__(parameter_list, state_mask, mean, covar.astype(np.float64))
        self.inv_covar = inv_covar.astype(np.float64)


def _read_mask(fname):
    from ..input_output.tiff import read_tiff

    if not os.path.exists(fname):
        raise IOError("State mask is neither an array or a file that exists!")
    return read_tiff(fname)[0].astype(bool)
