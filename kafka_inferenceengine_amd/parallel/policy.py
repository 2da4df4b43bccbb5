"""When band-parallel (C5, SURVEY.md §2.8 "TP-like") pays on MI355X.

Band-parallel splits a date's bands over the B ranks of a strip: each rank
runs the GP operator for n_bands / B bands and the group all-reduces the
per-pixel packed normal equations [A | b] -- 4 (ntri + n) bytes per pixel
(260 B for the 10-parameter PROSAIL state) -- every Gauss-Newton iteration.
A ring all-reduce moves 2 (B - 1) / B of that per rank over xGMI.  The work it
removes per rank is (1 - 1/B) of the GP sums, n_bands * T training-point
evaluations per pixel at ~2e-13 s each on the matrix-core kernel (measured:
PROSAIL 10 bands x T = 250, 66 ms per 120.6 M-pixel launch; JRC-TIP 2 x 500,
4.9 us per point at 4096^2, BENCHMARKS.md).

The policy compares the all-reduce time with the analysis time that remains
per rank.  For the multisensor state (34 bands, T = 250, B = 2) the all-reduce
is ~3x the analysis: strips alone are faster.  It pays only from n_bands / B
* T >~ 50,000 point evaluations per pixel (e.g. 34 bands at T >~ 3000).
"""
from __future__ import annotations

from ..utils.blocks import ntri

# seconds per (training point, pixel, band) of the fused matrix-core analysis (MI355X)
T_POINT_S = 2e-13
# effective per-rank all-reduce bandwidth inside a band group (one xGMI link
# per neighbour; generous: ~2/3 of a link's 153 GB/s)
LINK_BYTES_PER_S = 100e9
# the all-reduce may cost at most this fraction of the per-rank analysis
THRESHOLD = 0.25


def band_parallel_ratio(n_params: int, n_bands: int, n_train: int, B: int, t_point: float = T_POINT_S,
                        link_bytes_per_s: float = LINK_BYTES_PER_S) -> float:
    """All-reduce time / per-rank analysis time of one GN iteration (per pixel,
    so the strip size cancels)."""
    if B <= 1:
        return 0.0
    allreduce = 2.0 * (B - 1) / B * 4.0 * (ntri(n_params) + n_params) / link_bytes_per_s
    analysis = max(n_bands / B, 1.0) * max(n_train, 1) * t_point
    return allreduce / analysis


def band_parallel_decision(n_params: int, n_bands: int, n_train: int, B: int, device_type: str = "cuda",
                           force: bool = False, threshold: float = THRESHOLD):
    """-> (band groups to use, reason or None).  ``force`` keeps B whatever it
    costs; on the CPU (the gloo logic harness) the MI355X cost model does not
    apply and B is kept."""
    if B <= 1:
        return 1, None
    if force or device_type != "cuda":
        return B, None
    r = band_parallel_ratio(n_params, n_bands, n_train, B)
    if r > threshold:
        return 1, (f"band_parallel={B}: the per-iteration all-reduce of the packed normal equations "
                   f"({4 * (ntri(n_params) + n_params)} B/px) would take {r:.2f}x the per-rank analysis "
                   f"({n_bands} bands, T={n_train}); running pure strips instead")
    return B, None
