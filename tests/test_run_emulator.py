"""run_emulator (reference utils.py:68-106): host NumPy path vs the resident
tensor path (torch.unique + K7 LUT assignment on the tensor's device)."""
import numpy as np
import pytest
import torch

from kafka_inferenceengine_amd.models.gp import GaussianProcessEmulator
from kafka_inferenceengine_amd.models.operators import locate_in_lut, run_emulator

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _gp(D=4, T=40, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.uniform(0, 1, (T, D))
    y = np.sin(X @ rng.normal(size=D))
    return GaussianProcessEmulator.fit(X, y, lengthscale=np.full(D, 0.5), noise=1e-3)


@pytest.mark.parametrize("device", DEVICES)
def test_run_emulator_unique_rows_device_equals_host(device):
    gp = _gp()
    rng = np.random.default_rng(1)
    base = rng.uniform(0, 1, (50, 4)).astype(np.float32)
    x = base[rng.integers(0, 50, 3000)]              # 3000 rows, 50 unique
    H, dH = run_emulator(gp, x.astype(np.float64))
    Ht, dHt = run_emulator(gp, torch.as_tensor(x, device=device))
    assert Ht.device.type == device and Ht.shape == (3000,) and dHt.shape == (3000, 4)
    np.testing.assert_allclose(Ht.cpu().numpy(), H, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(dHt.cpu().numpy(), dH, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("device", DEVICES)
def test_run_emulator_lut_branch_device_equals_host(device):
    gp = _gp()
    rng = np.random.default_rng(2)
    x = rng.normal(0.5, 0.1, (4000, 4)).astype(np.float32)
    H, dH = run_emulator(gp, x.astype(np.float64), lut_threshold=100, lut_size=300, seed=7)
    Ht, dHt = run_emulator(gp, torch.as_tensor(x, device=device), lut_threshold=100,
                           lut_size=300, seed=7)
    lut = np.random.default_rng(7).multivariate_normal(
        x.astype(np.float64).mean(0), np.cov(x.astype(np.float64), rowvar=False), 300)
    near = locate_in_lut(lut, x)
    # every pixel takes its nearest LUT row's emulator value; ties between
    # f32 (device) and f64 (host) distances are the only allowed difference
    same = np.isclose(Ht.cpu().numpy(), H, rtol=1e-4, atol=1e-5)
    assert same.mean() > 0.995
    pred = np.asarray(gp.predict(lut, do_unc=False)[0])
    np.testing.assert_allclose(H, pred[near], rtol=1e-12)
    assert dHt.shape == (4000, 4) and np.isfinite(dHt.cpu().numpy()).all()
