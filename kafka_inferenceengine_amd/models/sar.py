"""Water Cloud Model SAR operator (kafka/observation_operators/sar_forward_model.py).

  tau       = exp(-2 B V / cos(theta))
  sigma_veg = A V^E cos(theta) (1 - tau)
  sigma_soil= 10^((C + D SM)/10)
  sigma0    = sigma_veg + tau sigma_soil           (linear units)

Parameters (``sar_forward_model.py:60-61``): VV = 0.0846, 0.0615, -14.8465,
15.907, 1; VH = 0.0795, 0.1464, -14.8332, 15.907, 0.  The device kernel is
``sar_eval`` in ``csrc/kf_core.h``; this NumPy version is the vectorised
reference (the original loops over pixels for the gradient, :82-98).
"""
from __future__ import annotations

import numpy as np

WCM_PARAMETERS = {"VV": (0.0846, 0.0615, -14.8465, 15.907, 1.0),
                  "VH": (0.0795, 0.1464, -14.8332, 15.907, 0.0)}
POLARISATIONS = ("VV", "VH")


def sar_observation_operator(x, theta, polarisation):
    """sigma0 and gradient wrt (V, SM) for rows of x = [[V, SM], ...]."""
    x = np.atleast_2d(np.asarray(x, dtype=np.float64))
    theta = np.deg2rad(np.asarray(theta, dtype=np.float64))
    mu = np.cos(theta)
    try:
        A, B, C, D, E = WCM_PARAMETERS[polarisation]
    except KeyError:
        raise ValueError("Only VV and VH polarisations available!")
    V, SM = x[:, 0], x[:, 1]
    if np.any(V <= 0.):
        raise ValueError("Negative LAI!")
    if np.any(SM <= 0.):
        raise ValueError("Negative SM!")
    tau = np.exp(-2. * B / mu * V)
    z = np.power(V, E)
    z1 = np.power(V, E - 1.)
    z = np.where(np.isnan(z), 1., z)
    z1 = np.where(np.isnan(z1), 1., z1)
    ssoil = 10. ** ((C + D * SM) / 10.)
    sigma0 = A * z * mu * (1. - tau) + tau * ssoil
    grad = np.zeros_like(x)
    grad[:, 0] = A * E * mu * z1 * (1. - tau) + 2. * A * B * z * tau - 2. * B * tau * ssoil / mu
    grad[:, 1] = D * np.log(10.) * tau * 10. ** ((C + D * SM) / 10. - 1.)
    if np.any(np.isnan(sigma0)):
        raise ValueError("Groan!")
    if np.any(np.isnan(grad)):
        raise ValueError("More Groan!")
    return sigma0, grad


class WaterCloudModel:
    """Device-capable WCM description.  ``state_map`` gives the state indices of
    (V, SM); the reference uses the first two state elements."""

    def __init__(self, polarisation: str = "VV", state_map=(0, 1), default_theta: float = 23.0,
                 coefficients=None):
        if polarisation not in WCM_PARAMETERS and coefficients is None:
            raise ValueError("Only VV and VH polarisations available!")
        self.polarisation = polarisation
        self.coefficients = tuple(coefficients) if coefficients is not None else WCM_PARAMETERS[polarisation]
        self.state_map = tuple(int(i) for i in state_map)
        self.default_theta = float(default_theta)

    def predict(self, X, theta=None):
        X = np.atleast_2d(X)
        th = self.default_theta if theta is None else theta
        th = np.broadcast_to(np.asarray(th, dtype=np.float64), (X.shape[0],))
        return sar_observation_operator(X[:, list(self.state_map)], th, self.polarisation)
