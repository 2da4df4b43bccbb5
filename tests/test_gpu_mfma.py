"""GP emulator on the gfx950 matrix cores (csrc/kf_gp_mfma.h) against
independent float64 oracles: GaussianProcessEmulator.predict for the operator
value, and analysis_blocks (solvers.py) for the Gauss-Newton step.  The VALU
record loop (variant 4) runs next to it as a second device path."""
import numpy as np
import pytest
import torch

import kafka_inferenceengine_amd as k
from kafka_inferenceengine_amd.engine.bands import DeviceBand, RecordCache, build_table
from kafka_inferenceengine_amd.inference import analysis_blocks
from kafka_inferenceengine_amd.ops import kernels as K

import kernel_cases as C

pytestmark = pytest.mark.gpu


def gp_problem(ems, maps, n, N, seed, x_lo, x_hi):
    rng = np.random.default_rng(seed)
    x = x_lo + (x_hi - x_lo) * rng.random((N, n))
    xf = x + rng.normal(size=(N, n)) * 0.02 * (x_hi - x_lo)
    Pf = np.broadcast_to(np.diag(1.0 / (0.3 * (x_hi - x_lo)) ** 2), (N, n, n)) + 0.0
    specs = [k.gp_spec(em, mp) for em, mp in zip(ems, maps)]
    bands, obs = [], []
    for em, mp in zip(ems, maps):
        H, _ = em.predict(x[:, mp])
        y = (H + rng.normal(size=N) * 0.01).astype(np.float32)
        w = np.where(rng.random(N) > 0.2, 1e4, 0.0).astype(np.float32)
        bands.append((y.astype(np.float64), w.astype(np.float64)))
        obs.append((y, w))
    return dict(x=x, xf=xf, Pf=Pf, specs=specs, ems=ems, maps=maps, bands=bands, obs=obs, N=N, n=n)


def run(prob, device, variant=None):
    N, n = prob["N"], prob["n"]
    dbs = [DeviceBand(K.OBS_F32, y=torch.from_numpy(y).to(device), w=torch.from_numpy(w).to(device))
           for y, w in prob["obs"]]
    h0 = [torch.zeros(N, device=device) for _ in dbs]
    tab = build_table(prob["specs"], dbs, n, RecordCache(), device, h0)
    xo = torch.zeros((n, N), device=device)
    ao = torch.zeros((n * (n + 1) // 2, N), device=device)
    st = torch.zeros(N, dtype=torch.uint8, device=device)
    part = K.partials_buffer(N, device)
    K.analysis(n, tab, C.soa(prob["x"], device), C.soa(prob["xf"], device), C.packed(prob["Pf"], device), xo, ao,
               None, st, part, variant=variant)
    return tab, xo.cpu().numpy().T, ao.cpu().numpy(), st.cpu().numpy(), [t.cpu().numpy() for t in h0], \
        float(K.reduce_partials(part).cpu())


def oracle(prob):
    bands = []
    for em, mp, (y, w) in zip(prob["ems"], prob["maps"], prob["bands"]):
        H, dH = em.predict(prob["x"][:, mp])
        h = np.zeros((prob["N"], prob["n"]))
        h[:, mp] = dH
        bands.append((H, h, y, w))
    return analysis_blocks(prob["x"], prob["xf"], prob["Pf"], bands)


def tip_case(N=12000, seed=5, noise=1e-3):
    ems = k.make_tip_emulators(n_train=500, seed=seed, noise=noise)
    lo = np.array([0.05, 0.3, 0.05, 0.25, 0.6, 0.05, 0.1])
    hi = np.array([0.55, 3.0, 0.45, 0.9, 5.5, 0.7, 0.9])
    return gp_problem(ems, [k.TIP_BAND_MAPPER[0], k.TIP_BAND_MAPPER[1]], 7, N, seed, lo, hi)


def prosail_case(N=6000, seed=6, noise=1e-3):
    ems = k.make_prosail_emulators(n_bands=2, n_train=250, seed=seed, noise=noise)
    lo = np.min([em.inputs.min(0) for em in ems], 0)
    hi = np.max([em.inputs.max(0) for em in ems], 0)
    return gp_problem(ems, [np.arange(10), np.arange(10)], 10, N, seed, lo, hi)


@pytest.mark.parametrize("case", ["tip", "prosail"])
def test_gp_mfma_operator_value_vs_float64(cuda, case):
    prob = tip_case() if case == "tip" else prosail_case()
    tab, x, a, st, h0, _ = run(prob, cuda)
    assert tab.gpm_frags > 0, "matrix-core path not selected"
    _, _, _, _, h0v, _ = run(prob, cuda, variant=4)   # f32 VALU record loop
    for em, mp, (y, w), hd, hv in zip(prob["ems"], prob["maps"], prob["bands"], h0, h0v):
        H, _ = em.predict(prob["x"][:, mp])
        sel = w > 0
        err = np.abs(hd[sel] - H[sel]).max() / np.abs(H).max()
        err_valu = np.abs(hv[sel] - H[sel]).max() / np.abs(H).max()
        # emulators fitted with a realistic nugget (models/gp.py): |alpha| ~ |f|;
        # both device paths sit at the f32 exponent's limit (~3e-5 for TIP)
        assert err < 5e-5 and err < 1.5 * err_valu + 5e-6, (case, em.name, err, err_valu)
        assert np.all(hd[~sel] == 0)


@pytest.mark.parametrize("case", ["tip", "prosail"])
def test_gp_mfma_analysis_vs_oracle_and_valu(cuda, case):
    prob = tip_case() if case == "tip" else prosail_case()
    _, xm, am, sm, _, rm = run(prob, cuda)            # matrix cores
    _, xv, av, sv, _, rv = run(prob, cuda, variant=4)  # VALU record loop
    xr, Ar = oracle(prob)
    scale = np.abs(xr) + 0.05
    err_m = np.max(np.abs(xm - xr) / scale)
    err_v = np.max(np.abs(xv - xr) / scale)
    # SURVEY.md §7.3 asks 1e-4 relative on x against float64.  Both cases meet
    # it on the matrix cores since the tables alternate the two alpha-sign
    # groups (models/gp.py mfma_point_order: the f32 running sums stay near
    # the result).  Measured: TIP MFMA 5.4e-5 (1.47e-4 with the sign groups
    # one after the other), the f32 VALU record loop (grouped order) 1.73e-4;
    # PROSAIL 1.5e-5 -- the reference's own f32 cast of A, b
    # (solvers.py:127-128) is at the 1e-4 level
    tol = 1e-4
    print(f"x err mfma {err_m:.2e} valu {err_v:.2e}")
    from kafka_inferenceengine_amd.utils.blocks import unpack_blocks
    n = prob["n"]
    d = np.sqrt(np.einsum("nii->ni", Ar))
    norm = d[:, :, None] * d[:, None, :]              # |A_ij| <= sqrt(A_ii A_jj)
    rel_m = np.max(np.abs(unpack_blocks(am, n) - Ar) / norm)
    rel_v = np.max(np.abs(unpack_blocks(av, n) - Ar) / norm)
    print(f"A err mfma {rel_m:.2e} valu {rel_v:.2e}")
    assert err_m < tol and err_m <= err_v * 1.05 + 1e-6, (err_m, err_v)
    assert np.array_equal(sm, sv)
    assert rel_m < 1e-3 and rel_m < 1.5 * rel_v + 1e-5, (rel_m, rel_v)
    assert abs(rm - rv) / rv < 1e-2


@pytest.mark.parametrize("case", ["tip", "prosail"])
def test_interleaved_exponent_variant_bit_identical(cuda, case):
    """The default issues both column blocks' exponent MFMAs before the first
    block's exponentials (gpm_chunk IL); variant 16 keeps the round-3
    block-by-block order: the same operations per block, so the same bits."""
    prob = tip_case(N=5000) if case == "tip" else prosail_case(N=3000)
    _, x0, a0, s0, h0, r0 = run(prob, cuda)
    _, x1, a1, s1, h1, r1 = run(prob, cuda, variant=16)
    assert np.array_equal(x0, x1) and np.array_equal(a0, a1) and np.array_equal(s0, s1)
    assert all(np.array_equal(p, q) for p, q in zip(h0, h1)) and r0 == r1


# The cancelling regime: near-interpolating emulators (1e-5 nugget,
# |alpha| >> |f|) are the stress case of the f16 hi/lo split.  Round 2's bounds,
# measured on such emulators, still hold for the round-3 packed operand.
@pytest.mark.parametrize("case", ["tip", "prosail"])
def test_gp_mfma_cancelling_emulators(cuda, case):
    prob = tip_case(noise=1e-5) if case == "tip" else prosail_case(noise=1e-5)
    alpha_ratio = max(np.abs(em.alpha).max() / np.abs(em.predict(em.inputs)[0]).max() for em in prob["ems"])
    tab, xm, am, sm, h0, rm = run(prob, cuda)
    assert tab.gpm_frags > 0 or tab.gpm_global, "matrix-core path not selected"
    _, xv, av, sv, h0v, rv = run(prob, cuda, variant=4)
    for em, mp, (y, w), hd, hv in zip(prob["ems"], prob["maps"], prob["bands"], h0, h0v):
        H, _ = em.predict(prob["x"][:, mp])
        sel = w > 0
        err = np.abs(hd[sel] - H[sel]).max() / np.abs(H).max()
        err_valu = np.abs(hv[sel] - H[sel]).max() / np.abs(H).max()
        print(f"{case} {em.name}: |alpha|/|f| {alpha_ratio:.0f}, H0 err mfma {err:.2e} valu {err_valu:.2e}")
        assert err < max(2e-4, 2.0 * err_valu), (case, em.name, err, err_valu)
    xr, Ar = oracle(prob)
    scale = np.abs(xr) + 0.05
    err_m = np.max(np.abs(xm - xr) / scale)
    err_v = np.max(np.abs(xv - xr) / scale)
    from kafka_inferenceengine_amd.utils.blocks import unpack_blocks
    n = prob["n"]
    d = np.sqrt(np.einsum("nii->ni", Ar))
    norm = d[:, :, None] * d[:, None, :]
    rel_m = np.max(np.abs(unpack_blocks(am, n) - Ar) / norm)
    rel_v = np.max(np.abs(unpack_blocks(av, n) - Ar) / norm)
    print(f"{case} cancelling: x err mfma {err_m:.2e} valu {err_v:.2e}; A err mfma {rel_m:.2e} valu {rel_v:.2e}")
    assert err_m < 2e-3 and err_v < 4e-3 and err_m < 1.5 * err_v + 1e-4, (err_m, err_v)
    assert rel_m < 2e-2 and rel_m < 1.5 * rel_v + 1e-5, (rel_m, rel_v)


def test_gp_mfma_tail_and_cloud_waves(cuda):
    """N not a multiple of 64 (tail lanes) and a fully clouded wave (GP skipped)."""
    prob = tip_case(N=64 * 37 + 19, seed=8)
    for y, w in prob["obs"]:
        w[64 * 3:64 * 5] = 0.0
    prob["bands"] = [(y.astype(np.float64), w.astype(np.float64)) for y, w in prob["obs"]]
    _, xm, _, sm, h0, _ = run(prob, cuda)
    _, xv, _, sv, _, _ = run(prob, cuda, variant=4)
    assert np.array_equal(sm, sv)
    assert np.all(sm[64 * 3:64 * 5] & K.ST_NO_OBS)
    assert np.max(np.abs(xm - xv) / (np.abs(xv) + 0.05)) < 5e-4   # two f32 paths, each ~1.5e-4 off float64
    assert np.all(h0[0][64 * 3:64 * 5] == 0)


@pytest.mark.parametrize("cap", [0, 16])
def test_gp_mfma_realistic_tile_matches_valu(cuda, cap):
    """A 512^2 synthetic TIP tile with per-pixel states (one and many 64-pixel
    tiles per wave): every pixel of the matrix-core kernel agrees with the VALU
    loop to 5e-3.  Round 2's inline-asm hi/lo split once lost a wait state
    and corrupted a quarter of some waves; the split is compiler-visible now
    (tests/test_isa_lint.py checks the pads) and this stays as the runtime guard."""
    variant = 0
    from kafka_inferenceengine_amd.utils.blocks import pack_matrix
    mask = np.ones((512, 512), bool)
    obs = k.SyntheticBHRObservations(mask, n_train=500, device=cuda, stream=False, n_pool=1)
    bands = [(obs.band_specs[b], obs.get_device_band_data(obs.dates[0], b)) for b in range(2)]
    tab = build_table([s for s, _ in bands], [d for _, d in bands], 7, RecordCache(), cuda)
    N = obs.N
    mu, P, Pi = k.tip_prior()
    g = torch.Generator(device=cuda).manual_seed(0)
    sd = torch.tensor(np.sqrt(np.diag(P)) * 0.3, dtype=torch.float32, device=cuda)[:, None]
    xf = torch.tensor(mu, dtype=torch.float32, device=cuda)[:, None] + sd * torch.randn(7, N, device=cuda, generator=g)
    xf[6].clamp_(0.05, 0.95)
    Pf = torch.tensor(pack_matrix(Pi), dtype=torch.float32, device=cuda)[:, None].expand(28, N).contiguous()
    ext = K.ext()
    outs = {}
    try:
        ext.set_max_blocks(cap or ext.MAX_BLOCKS)
        for v in (4, variant):
            for _ in range(2):   # twice: the corruption was timing dependent
                xo = torch.zeros_like(xf)
                K.analysis(7, tab, xf, xf, Pf, xo, torch.zeros_like(Pf), None, None, None, variant=v)
                outs.setdefault(v, []).append(xo.cpu().numpy())
    finally:
        ext.set_max_blocks(ext.MAX_BLOCKS)
    ref = outs[4][0]
    for x in outs[variant]:
        d = np.abs(x - ref) / (np.abs(ref) + 0.05)
        assert d.max() < 5e-3, (variant, cap, float(d.max()), np.nonzero(d.max(0) > 5e-3)[0][:8])


def test_tip_layout_kernel_bit_identical_to_runtime_layout(cuda):
    """BAND_LAYOUT_TIP (band loop unrolled over the compile-time VIS / NIR maps,
    kf_gp_mfma.h) against the runtime-layout kernel (variant 10): the same
    operations per pixel, so x, A, status and the norm partials are identical."""
    prob = tip_case(N=64 * 53 + 7, seed=11)
    tab, xl, al, sl, hl, rl = run(prob, cuda)
    assert tab.layout == K.BAND_LAYOUT_TIP
    _, xr, ar, sr, hr, rr = run(prob, cuda, variant=10)
    assert np.array_equal(xl, xr) and np.array_equal(al, ar) and np.array_equal(sl, sr)
    for a, b in zip(hl, hr):
        assert np.array_equal(a, b)
    assert rl == rr
    # swapped band order is not the layout: the runtime kernel runs it
    swapped = dict(prob, specs=prob["specs"][::-1], obs=prob["obs"][::-1], ems=prob["ems"][::-1],
                   maps=prob["maps"][::-1], bands=prob["bands"][::-1])
    tab2, xs, *_ = run(swapped, cuda)
    assert tab2.layout == 0
    assert np.max(np.abs(xs - xl) / (np.abs(xl) + 0.05)) < 1e-5
