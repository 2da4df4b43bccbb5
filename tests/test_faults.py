"""Fault injection: corrupted observations and degenerate
blocks must be contained to their pixels and flagged."""
import datetime as dt

import numpy as np
import torch

import kafka_inferenceengine_amd as k
from kafka_inferenceengine_amd.engine.bands import DeviceBand
from kafka_inferenceengine_amd.ops import kernels as K


class NaNInjected:
    """Wraps a source and corrupts a tile of every band with NaN/inf."""

    def __init__(self, src, rows, cols):
        self.src = src
        self.dates = src.dates
        self.bands_per_observation = src.bands_per_observation
        self.partition = src.partition
        self.rows, self.cols = rows, cols

    def get_band_data(self, date, band):
        r = self.src.get_band_data(date, band)
        obs = r.observations.copy()
        obs[self.rows, self.cols] = np.nan
        unc = r.uncertainty.tolil()
        W = obs.shape[1]
        for rr in range(*self.rows.indices(obs.shape[0])):
            for cc in range(*self.cols.indices(W)):
                unc[rr * W + cc, rr * W + cc] = np.inf
        return r._replace(observations=obs, uncertainty=unc.tocsr())


def test_nan_tile_is_contained_and_flagged():
    mask = np.ones((16, 12), bool)
    src = k.SyntheticBHRObservations(mask, n_train=40, device="cpu", stream=False, n_pool=2, field_cell=4)
    bad = NaNInjected(src, slice(2, 5), slice(3, 7))
    grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(3)]
    res = []
    for obs in (src, bad):
        kf = k.LinearKalman(obs, None, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS,
                            device="cpu")
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
        st = kf.run(grid, kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask)), None, None)
        res.append((st.x.clone(), kf.last_status.clone()))
    (xa, sa), (xb, sb) = res
    assert torch.isfinite(xb).all()
    img = np.zeros(mask.shape, bool)
    img[2:5, 3:7] = True
    inside = torch.from_numpy(img.ravel())
    assert torch.all((sb[inside] & K.ST_NO_OBS) > 0)       # corrupted pixels saw no valid observation
    # pixels outside the tile: identical physics, only the global norm could differ
    assert torch.allclose(xa[:, ~inside], xb[:, ~inside], rtol=1e-5, atol=1e-6)


def test_nonspd_forecast_falls_back_per_pixel():
    n, N = 7, 64
    mu, _, Pi = k.tip_prior()
    x = torch.tensor(np.tile(mu[:, None], (1, N)), dtype=torch.float32)
    from kafka_inferenceengine_amd.utils.blocks import pack_matrix
    P = torch.tensor(np.tile(pack_matrix(Pi)[:, None], (1, N)), dtype=torch.float32)
    P[:, :5] = torch.tensor(pack_matrix(-np.eye(7)), dtype=torch.float32)[:, None]
    P[:, 5] = float("nan")
    y = torch.full((N,), 0.1)
    w = torch.zeros(N)   # no observations: A = P_f^-1 only
    spec = k.models.operators._linear_device_spec(n, None, None, 0)
    from kafka_inferenceengine_amd.engine.bands import RecordCache, build_table
    tab = build_table([spec], [DeviceBand(K.OBS_F32, y=y, w=w)], n, RecordCache(), "cpu")
    xo, ao = torch.zeros_like(x), torch.zeros_like(P)
    st = torch.zeros(N, dtype=torch.uint8)
    K.analysis(n, tab, x, x, P, xo, ao, None, st, K.partials_buffer(N, "cpu"))
    assert torch.all(st[:6] & K.ST_FALLBACK)
    assert torch.equal(xo[:, :6], x[:, :6])
    assert not torch.any(st[6:] & K.ST_FALLBACK)
    assert torch.isfinite(xo).all()
