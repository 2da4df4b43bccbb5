"""Band-parallel (C5) guard: parallel/policy.py and the engine's refusal."""
import numpy as np
import pytest

import kafka_inferenceengine_amd as k
from kafka_inferenceengine_amd.parallel.policy import THRESHOLD, band_parallel_decision, band_parallel_ratio


def test_band_parallel_cost_model():
    # multisensor: 34 bands, T = 250, PROSAIL state, 2 band groups -> the all-reduce is ~3x the analysis
    r = band_parallel_ratio(10, 34, 250, 2)
    assert 2.0 < r < 4.0
    assert band_parallel_decision(10, 34, 250, 2, "cuda")[0] == 1
    # more GP work per pixel makes it pay
    assert band_parallel_ratio(10, 34, 4000, 2) < THRESHOLD
    assert band_parallel_decision(10, 34, 4000, 2, "cuda") == (2, None)
    # linear operators (no GP work): never
    assert band_parallel_decision(7, 7, 0, 2, "cuda")[0] == 1
    # forced, or the CPU logic harness: kept
    assert band_parallel_decision(10, 34, 250, 2, "cuda", force=True) == (2, None)
    assert band_parallel_decision(10, 34, 250, 2, "cpu") == (2, None)
    assert band_parallel_decision(10, 34, 250, 1, "cuda") == (1, None)
    # bigger groups move more bytes per rank for less work each
    assert band_parallel_ratio(10, 34, 250, 4) > band_parallel_ratio(10, 34, 250, 2)


def test_engine_refuses_band_parallel_on_gpu_cost(monkeypatch):
    """On a GPU device the engine refuses a band group whose all-reduce dwarfs
    the analysis (unless forced) at the first date, before any collective."""
    from kafka_inferenceengine_amd.parallel import Comm, StripPartition

    mask = np.ones((8, 8), bool)
    obs = k.SyntheticS2Observations(mask, n_bands=4, n_train=20, device="cpu", stream=False, n_pool=1)
    prior = k.SAILPrior(k.SAIL_PARAMETERS, mask)
    band = Comm(0, 2, "cpu")
    comm = Comm(0, 1, "cpu", band=band)
    kf = k.LinearKalman(obs, None, mask, k.create_prosail_observation_operator, k.SAIL_PARAMETERS,
                        state_propagation=None, prior=prior, device="cpu", comm=comm,
                        partition=StripPartition(mask, 0, 1), config=k.EngineConfig(gp_split="never"))
    import torch
    monkeypatch.setattr(kf, "device", torch.device("cuda", 0))   # the cost model of the GPU path
    monkeypatch.setattr(band, "max_float", lambda v: v)          # one-process stand-in for the group max
    specs = [kf._operator_spec(obs.get_device_band_data(obs.dates[0], b), b, obs.dates[0]) for b in range(2)]
    with pytest.raises(ValueError, match="band_parallel_force"):
        kf._band_parallel_check(specs, 4)
    kf.config.band_parallel_force = True
    kf._band_parallel_check(specs, 4)


def test_band_parallel_check_is_rank_uniform(monkeypatch):
    """10 bands dealt round-robin over B = 3 ranks give 4/3/3 bands.
    Near the threshold the old per-rank estimate (own bands x B) let rank 0
    proceed (12 bands) while the others refused (9): the survivors then waited
    in the band all-reduce.  The check now uses the date's band count and the
    group-wide largest emulator, so every rank decides alike."""
    from types import SimpleNamespace

    import torch

    from kafka_inferenceengine_amd.parallel import Comm, StripPartition

    n_train = 20000
    # the old estimate splits: 12 bands pass, 9 refuse
    assert band_parallel_decision(10, 12, n_train, 3, "cuda")[0] == 3
    assert band_parallel_decision(10, 9, n_train, 3, "cuda")[0] == 1
    mask = np.ones((4, 4), bool)
    obs = k.SyntheticS2Observations(mask, n_bands=4, n_train=20, device="cpu", stream=False, n_pool=1)
    prior = k.SAILPrior(k.SAIL_PARAMETERS, mask)
    decisions = []
    for rank, nb_mine in enumerate((4, 3, 3)):
        band = Comm(rank, 3, "cpu")
        # the group's max over the ranks' own largest emulators: the biggest sits on rank 2 only
        monkeypatch.setattr(band, "max_float", lambda v: max(v, float(n_train)))
        kf = k.LinearKalman(obs, None, mask, k.create_prosail_observation_operator, k.SAIL_PARAMETERS,
                            state_propagation=None, prior=prior, device="cpu", comm=Comm(0, 1, "cpu", band=band),
                            partition=StripPartition(mask, 0, 1))
        monkeypatch.setattr(kf, "device", torch.device("cuda", 0))
        own_T = n_train if rank == 2 else 100
        specs = [SimpleNamespace(emulator=SimpleNamespace(n_train=own_T)) for _ in range(nb_mine)]
        try:
            kf._band_parallel_check(specs, 10)
            decisions.append("run")
        except ValueError:
            decisions.append("refuse")
    assert decisions == ["refuse"] * 3
