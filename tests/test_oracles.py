"""Every fast kernel instantiation against an INDEPENDENT float64 oracle
(``analysis_blocks`` / ``gain_blocks`` of inference/solvers.py, the NumPy GP
and water-cloud models, the reference-API propagators of kf_tools.py) — never
against the host runner built from the same kf_core.h source.

Each test runs twice: on the CPU (host runner; part of the default suite) and
on the MI355X (``gpu``): the gfx950 instantiations

* ``analysis_kernel<10,10>`` (fused PROSAIL, 10 GP bands of D = 10);
* the K2 split path: ``gp_operator`` chunks of ``band_chunk`` = 3 bands with the
  (A, b) accumulators chained through ``a_in`` / ``b_in`` (``solve=False``);
* the band-parallel partial sums (``solve=False``, forecast on slot 0 only,
  then one solve from the summed [A | b]);
* ``OP_SAR`` (water-cloud model, per-pixel incidence angle);
* the gain (covariance) form; the propagate modes 0-5 and the blend.

Tolerances: x relative to |x| + 0.05 (the analysis solve is f32) and A
entries scaled by sqrt(A_ii A_jj).  The PROSAIL and SAR problems meet 1e-4
in f32; the GP sums of the TIP emulators cancel (|alpha|
>> |f|) and are held to the measured f32 limit instead (test_gpu_mfma.py)."""
import numpy as np
import pytest
import torch

import kafka_inferenceengine_amd as k
from kafka_inferenceengine_amd.engine.bands import DeviceBand, RecordCache, build_table
from kafka_inferenceengine_amd.inference import analysis_blocks, gain_blocks
from kafka_inferenceengine_amd.models.operators import OP_PRECOMP, OperatorSpec, _sar_device_spec
from kafka_inferenceengine_amd.ops import kernels as K
from kafka_inferenceengine_amd.utils.blocks import ntri, pack_blocks, pack_matrix, unpack_blocks

import kernel_cases as C

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


@pytest.fixture(params=DEVICES)
def dev(request):
    if request.param == "cuda":
        if not torch.cuda.is_available():
            pytest.skip("no GPU")
        return torch.device("cuda", 0)
    return torch.device("cpu")


def x_err(x, xr):
    return float(np.max(np.abs(x - xr) / (np.abs(xr) + 0.05)))


def a_err(A_packed, Ar, n):
    d = np.sqrt(np.einsum("nii->ni", Ar))
    return float(np.max(np.abs(unpack_blocks(A_packed, n) - Ar) / (d[:, :, None] * d[:, None, :])))


# ------------------------------------------------------------------ problems
def prosail_problem(N=4096, n_bands=10, seed=21, n_train=250):
    """10-parameter PROSAIL state, ``n_bands`` GP bands over all 10 inputs."""
    rng = np.random.default_rng(seed)
    ems = k.make_prosail_emulators(n_bands=n_bands, n_train=n_train, seed=seed)
    mu, cov, Pi = k.sail_prior()
    lo = np.min([em.inputs.min(0) for em in ems], 0)
    hi = np.max([em.inputs.max(0) for em in ems], 0)
    x = lo + (hi - lo) * (0.2 + 0.6 * rng.random((N, 10)))
    xf = np.clip(mu[None] + 0.05 * (hi - lo) * rng.normal(size=(N, 10)), lo, hi)
    Pf = np.broadcast_to(Pi, (N, 10, 10)) + 0.0
    bands, obs = [], []
    for em in ems:
        H, _ = em.predict(x)
        y = (H + 0.01 * rng.normal(size=N)).astype(np.float32)
        w = np.where(rng.random(N) > 0.15, 1.0 / 0.02 ** 2, 0.0).astype(np.float32)
        bands.append((y.astype(np.float64), w.astype(np.float64)))
        obs.append((y, w))
    specs = [k.gp_spec(em, list(range(10))) for em in ems]
    return dict(x=x, xf=xf, Pf=Pf, ems=ems, specs=specs, bands=bands, obs=obs, N=N, n=10)


def oracle_bands(prob, x_lin):
    out = []
    for em, (y, w) in zip(prob["ems"], prob["bands"]):
        H, dH = em.predict(x_lin)
        out.append((H, dH, y, w))
    return out


def dbands(prob, device, idx=None):
    idx = range(len(prob["obs"])) if idx is None else idx
    return [DeviceBand(K.OBS_F32, y=torch.from_numpy(prob["obs"][i][0]).to(device),
                       w=torch.from_numpy(prob["obs"][i][1]).to(device)) for i in idx]


def run_fused(prob, device, specs=None, db=None, variant=None, expect_global=None):
    n, N = prob["n"], prob["N"]
    tab = build_table(specs or prob["specs"], db or dbands(prob, device), n, RecordCache(), device)
    if expect_global is not None:
        assert tab.gpm_global == expect_global and tab.gpm_frags == 0
    xo = torch.zeros((n, N), device=device)
    ao = torch.zeros((ntri(n), N), device=device)
    st = torch.zeros(N, dtype=torch.uint8, device=device)
    K.analysis(n, tab, C.soa(prob["x"], device), C.soa(prob["xf"], device), C.packed(prob["Pf"], device), xo, ao,
               None, st, None, variant=variant)
    return xo.cpu().numpy().T, ao.cpu().numpy(), st.cpu().numpy()


# ------------------------------------------------------------------ tests
@pytest.mark.parametrize("variant", [0, 4])
def test_prosail_fused_vs_oracle(dev, variant):
    """Ten PROSAIL GP bands (D = 10) fused in one pass: on the device variant 0
    is the matrix-core kernel with the tables read from global memory
    (analysis_mfma_g_kernel<10,10>: 10 bands x 8 chunks do not fit the LDS),
    variant 4 the VALU record loop (analysis_kernel<10,10>)."""
    prob = prosail_problem()
    x, a, st = run_fused(prob, dev, variant=variant, expect_global=True)
    xr, Ar = analysis_blocks(prob["x"], prob["xf"], prob["Pf"], oracle_bands(prob, prob["x"]))
    ex, ea = x_err(x, xr), a_err(a, Ar, 10)
    print(f"prosail fused on {dev}: x {ex:.2e} A {ea:.2e}")
    assert ex < 1e-4 and ea < 1e-4, (ex, ea)
    assert not np.any(st & K.ST_FALLBACK)


@pytest.mark.parametrize("variant", [0, 4])
def test_multisensor_34_band_fused_vs_oracle(dev, variant):
    """34 full-state GP bands (the S2 + OLCI-like multi-sensor date) in one
    fused pass: on the device the global-table matrix-core kernel, which the
    auto split policy now prefers to the split path for such dates."""
    prob = prosail_problem(N=2048, n_bands=34, seed=26)
    x, a, st = run_fused(prob, dev, variant=variant, expect_global=True)
    xr, Ar = analysis_blocks(prob["x"], prob["xf"], prob["Pf"], oracle_bands(prob, prob["x"]))
    ex, ea = x_err(x, xr), a_err(a, Ar, 10)
    print(f"34-band fused on {dev}: x {ex:.2e} A {ea:.2e}")
    # x: f32 normal equations of 34 well-observed bands (the host runner,
    # same f32 algebra without matrix cores, measures 4.3e-4 here)
    assert ex < 1e-3 and ea < 1e-4, (ex, ea)
    assert not np.any(st & K.ST_FALLBACK)


def test_split_path_chunked_accumulation_vs_oracle(dev):
    """K2 split: GP value + Jacobian of 3 bands per chunk into HBM (gp_operator),
    the analysis of each chunk from those precomputed rows, (A, b) chained
    through a_in / b_in with solve=False, the last chunk solves."""
    prob = prosail_problem(seed=22)
    n, N = prob["n"], prob["N"]
    nb, chunk = len(prob["specs"]), 3
    xs, xf, pf = C.soa(prob["x"], dev), C.soa(prob["xf"], dev), C.packed(prob["Pf"], dev)
    h0 = torch.zeros((chunk, N), device=dev)
    h = torch.zeros((chunk * n, N), device=dev)
    acc = [(torch.zeros((ntri(n), N), device=dev), torch.zeros((n, N), device=dev)) for _ in range(2)]
    xo = torch.zeros((n, N), device=dev)
    ao = torch.zeros((ntri(n), N), device=dev)
    st = torch.zeros(N, dtype=torch.uint8, device=dev)
    cache, prev = RecordCache(), None
    starts = list(range(0, nb, chunk))
    for ci, c0 in enumerate(starts):
        idx = list(range(c0, min(c0 + chunk, nb)))
        op_tab = build_table([prob["specs"][i] for i in idx], dbands(prob, dev, idx), n, cache, dev)
        K.gp_operator(n, op_tab, xs, h0[:len(idx)], h[:len(idx) * n], N=N, d=10)
        pre = [(h0[j], h[j * n:(j + 1) * n]) for j in range(len(idx))]
        an_tab = build_table([OperatorSpec(OP_PRECOMP, list(range(n)), [0.0] * n) for _ in idx],
                             dbands(prob, dev, idx), n, cache, dev, None, pre)
        a_in, b_in = prev if prev is not None else (None, None)
        if ci == len(starts) - 1:
            K.analysis(n, an_tab, xs, xf, pf, xo, ao, None, st, None, a_in=a_in, b_in=b_in)
        else:
            A_c, b_c = acc[ci % 2]
            K.analysis(n, an_tab, xs, xf, pf, None, A_c, b_c, st, None, solve=False, a_in=a_in, b_in=b_in)
            prev = (A_c, b_c)
    xr, Ar = analysis_blocks(prob["x"], prob["xf"], prob["Pf"], oracle_bands(prob, prob["x"]))
    ex, ea = x_err(xo.cpu().numpy().T, xr), a_err(ao.cpu().numpy(), Ar, n)
    print(f"split on {dev}: x {ex:.2e} A {ea:.2e}")
    assert ex < 1e-4 and ea < 1e-4, (ex, ea)


def test_band_parallel_partials_vs_oracle(dev):
    """C5 band-parallel: three band groups accumulate their partial [A | b]
    with solve=False (the forecast precision only on group 0, the others start
    from zero through a_in), the sum is solved by a band-less table."""
    prob = prosail_problem(seed=23)
    n, N = prob["n"], prob["N"]
    xs, xf, pf = C.soa(prob["x"], dev), C.soa(prob["xf"], dev), C.packed(prob["Pf"], dev)
    groups = [[0, 3, 6, 9], [1, 4, 7], [2, 5, 8]]
    cache = RecordCache()
    total = torch.zeros((ntri(n) + n, N), device=dev)
    st = torch.zeros(N, dtype=torch.uint8, device=dev)
    for g, idx in enumerate(groups):
        tab = build_table([prob["specs"][i] for i in idx], dbands(prob, dev, idx), n, cache, dev)
        buf = torch.zeros((ntri(n) + n, N), device=dev)
        A_p, b_p = buf[:ntri(n)], buf[ntri(n):]
        if g == 0:
            K.analysis(n, tab, xs, xf, pf, None, A_p, b_p, st, None, solve=False)
        else:
            K.analysis(n, tab, xs, xf, pf, None, A_p, b_p, st, None, solve=False, a_in=A_p, b_in=b_p)
        total += buf                       # the band-group all-reduce
    xo = torch.zeros((n, N), device=dev)
    ao = torch.zeros((ntri(n), N), device=dev)
    empty = build_table([], [], n, cache, dev)
    K.analysis(n, empty, xs, xf, pf, xo, ao, None, st, None, a_in=total[:ntri(n)], b_in=total[ntri(n):])
    xr, Ar = analysis_blocks(prob["x"], prob["xf"], prob["Pf"], oracle_bands(prob, prob["x"]))
    ex, ea = x_err(xo.cpu().numpy().T, xr), a_err(ao.cpu().numpy(), Ar, n)
    print(f"band-parallel on {dev}: x {ex:.2e} A {ea:.2e}")
    assert ex < 1e-4 and ea < 1e-4, (ex, ea)


def test_sar_analysis_vs_water_cloud_oracle(dev):
    """OP_SAR: VV + VH water-cloud bands with a per-pixel incidence angle."""
    rng = np.random.default_rng(24)
    N, n = 6000, 2
    x = np.stack([rng.uniform(0.3, 5.0, N), rng.uniform(0.08, 0.42, N)], 1)
    xf = np.stack([rng.uniform(0.5, 4.0, N), rng.uniform(0.1, 0.4, N)], 1)
    Pf = np.broadcast_to(np.diag([1.0, 100.0]), (N, 2, 2)) + 0.0
    th = rng.uniform(25, 45, N)
    th_t = torch.tensor(th, dtype=torch.float32, device=dev)
    specs, db, bands = [], [], []
    for b, pol in enumerate(("VV", "VH")):
        s0, _ = k.sar_observation_operator(x, th, pol)
        y = (s0 * (1 + 0.05 * rng.normal(size=N))).astype(np.float32)
        w = np.where(rng.random(N) > 0.1, 1.0 / (0.05 * np.abs(y) + 1e-3) ** 2, 0.0).astype(np.float32)
        specs.append(_sar_device_spec(n, None, None, b))
        db.append(DeviceBand(K.OBS_F32, y=torch.from_numpy(y).to(dev), w=torch.from_numpy(w).to(dev), aux=th_t))
        H, g = k.sar_observation_operator(x, th.astype(np.float32).astype(np.float64), pol)
        bands.append((H, g, y.astype(np.float64), w.astype(np.float64)))
    prob = dict(x=x, xf=xf, Pf=Pf, N=N, n=n)
    xo, ao, st = run_fused(prob, dev, specs, db)
    xr, Ar = analysis_blocks(x, xf, Pf, bands)
    ex, ea = x_err(xo, xr), a_err(ao, Ar, n)
    print(f"SAR on {dev}: x {ex:.2e} A {ea:.2e}")
    assert ex < 1e-4 and ea < 1e-4, (ex, ea)


@pytest.mark.parametrize("case", ["tip", "prosail"])
def test_gain_form_vs_gain_blocks(dev, case):
    """K1g sequential scalar updates vs the float64 covariance-form oracle."""
    if case == "tip":
        prob = C.tip_problem(N=4000, seed=25)
        tab = C.table(prob, dev)
        bands = C.oracle_bands(prob, prob["x"])
        tol_x = 1e-4
    else:
        prob = prosail_problem(N=3000, seed=25)
        tab = build_table(prob["specs"], dbands(prob, dev), 10, RecordCache(), dev)
        bands = oracle_bands(prob, prob["x"])
        tol_x = 1e-4
    n, N = prob["n"], prob["N"]
    Pcov = np.linalg.inv(prob["Pf"])
    xo = torch.zeros((n, N), device=dev)
    po = torch.zeros((ntri(n), N), device=dev)
    K.gain(n, tab, C.soa(prob["x"], dev), C.soa(prob["xf"], dev), C.packed(Pcov, dev), xo, po)
    xr, Pr = gain_blocks(prob["x"], prob["xf"], Pcov, bands)
    ex = x_err(xo.cpu().numpy().T, xr)
    d = np.sqrt(np.einsum("nii->ni", Pr))
    ep = float(np.max(np.abs(unpack_blocks(po.cpu().numpy(), n) - Pr) / (d[:, :, None] * d[:, None, :])))
    print(f"gain {case} on {dev}: x {ex:.2e} P {ep:.2e}")
    assert ex < tol_x and ep < 2e-4, (ex, ep)


def test_propagate_modes_vs_reference_api(dev):
    """Propagate kernel modes against the reference-API NumPy/SciPy propagators
    (kf_tools.py) and closed forms."""
    import scipy.sparse as sp
    from kafka_inferenceengine_amd.inference import kf_tools as T
    from kafka_inferenceengine_amd.utils.blocks import blocks_to_sparse, sparse_to_blocks

    rng = np.random.default_rng(26)
    n, N = 7, 2000
    A = C.spd_blocks(rng, N, n, 5.0)
    xa = rng.normal(size=(N, n))
    mu, _, Pi = k.tip_prior()
    q = rng.uniform(0.01, 0.2, n)
    m = rng.uniform(0.9, 1.1, n)
    Q, M = sp.diags(np.tile(q, N)), sp.diags(np.tile(m, N))

    def prop(mode, prop_mask=0, blend=False, quirk=False):
        spec = {"mode": mode, "m": m, "q": q, "prop_mask": prop_mask, "reset_mean": mu,
                "reset_cinv": pack_matrix(Pi), "blend": blend, "quirk_blend": quirk, "blend_mean": mu * 1.1,
                "blend_cinv": pack_matrix(Pi * 0.5)}
        xf = torch.zeros((n, N), device=dev)
        pf = torch.zeros((ntri(n), N), device=dev)
        K.propagate(n, spec, C.soa(xa, dev), C.packed(A, dev), xf, pf)
        return xf.cpu().numpy().T, unpack_blocks(pf.cpu().numpy(), n)

    def rel(a, b):
        return float(np.max(np.abs(a - b) / np.maximum(np.abs(b).max(axis=tuple(range(1, b.ndim)), keepdims=True),
                                                       1e-6)))

    xf, Pf = prop(T.PROP_INFO_EXACT)
    xr, _, Pr = T.propagate_information_filter_SLOW(xa.ravel(), None, blocks_to_sparse(A), M, Q, n_params=n)
    assert rel(xf, xr.reshape(N, n)) < 1e-5 and rel(Pf, sparse_to_blocks(Pr, n, check=False)) < 1e-4
    xf, Pf = prop(T.PROP_INFO_APPROX)
    _, _, Pr = T.propagate_information_filter_approx_SLOW(xa.ravel(), None, blocks_to_sparse(A), M, Q)
    assert rel(Pf, sparse_to_blocks(Pr, n, check=False)) < 1e-5
    xf, Pf = prop(T.PROP_PRIOR_PARTIAL, prop_mask=1 << 6)
    xr, _, Pr = T.propagate_information_filter_LAI(xa.ravel(), None, blocks_to_sparse(A), M, Q)
    assert rel(xf, xr.reshape(N, n)) < 1e-5 and rel(Pf, sparse_to_blocks(Pr, n, check=False)) < 1e-5
    xf, Pf = prop(T.PROP_STANDARD)
    assert rel(Pf, A + np.diag(q)[None]) < 1e-6
    xf, Pf = prop(T.PROP_PRIOR)
    assert rel(xf, np.broadcast_to(mu, (N, n))) < 1e-6 and rel(Pf, np.broadcast_to(Pi, (N, n, n))) < 1e-6
    for quirk in (False, True):
        xf, Pf = prop(T.PROP_IDENTITY, blend=True, quirk=quirk)
        xr, Cr = T.blend_prior(np.tile(mu * 1.1, N), blocks_to_sparse(np.broadcast_to(Pi * 0.5, (N, n, n)).copy()),
                               (xa * m).ravel(), blocks_to_sparse(A), quirk=quirk, n_params=n)
        assert rel(xf, xr.reshape(N, n)) < 1e-4 and rel(Pf, sparse_to_blocks(Cr, n, check=False)) < 1e-5


def test_gain_fused_forecast_and_output_vs_oracle(dev):
    """K1g with the LAI forecast fused (from the analysis COVARIANCE, first
    Gauss-Newton iteration: linearised at the forecast) and the output rasters
    written by the kernel, against NumPy: forecast precision = prior with the
    propagated diagonal 1/(1/(P_a^-1)_jj + q_j), gain_blocks, 1/sqrt(diag P^-1)."""
    prob = C.tip_problem(N=3000, seed=27)
    n, N = prob["n"], prob["N"]
    rng = np.random.default_rng(27)
    mu, _, Pi = k.tip_prior()
    Pa = np.linalg.inv(C.spd_blocks(rng, N, n, 20.0))          # analysis covariance
    xa = prob["x"]
    q = np.full(n, 0.0)
    q[6] = 0.04
    spec = {"mode": 1, "m": np.ones(n), "q": q, "prop_mask": 1 << 6, "reset_mean": mu,
            "reset_cinv": pack_matrix(Pi), "blend": False}
    # NumPy forecast
    Cf = np.broadcast_to(Pi, (N, n, n)).copy()
    Cf[:, 6, 6] = 1.0 / (1.0 / np.linalg.inv(Pa)[:, 6, 6] + q[6])
    Pf = np.linalg.inv(Cf)
    xf = np.broadcast_to(mu, (N, n)).copy()
    xf[:, 6] = xa[:, 6]
    bands = C.oracle_bands(prob, xf)
    xr, Pr = gain_blocks(xf, xf, Pf, bands)
    unc_r = 1.0 / np.sqrt(np.einsum("nii->ni", np.linalg.inv(Pr)))
    tab = C.table(prob, dev)
    xo = torch.zeros((n, N), device=dev)
    po = torch.zeros((ntri(n), N), device=dev)
    mean = torch.zeros((n, N), device=dev)
    unc = torch.zeros((n, N), device=dev)
    h = K.prop_args(n, spec, C.soa(xa, dev), C.packed(Pa, dev), fused=True)
    K.gain(n, tab, None, None, None, xo, po, prop=h, out=(mean, unc, None))
    ex = x_err(xo.cpu().numpy().T, xr)
    d = np.sqrt(np.einsum("nii->ni", Pr))
    ep = float(np.max(np.abs(unpack_blocks(po.cpu().numpy(), n) - Pr) / (d[:, :, None] * d[:, None, :])))
    eu = float(np.max(np.abs(unc.cpu().numpy().T - unc_r) / unc_r))
    print(f"gain fused on {dev}: x {ex:.2e} P {ep:.2e} unc {eu:.2e}")
    assert ex < 1e-4 and ep < 2e-4 and eu < 1e-4, (ex, ep, eu)
    assert torch.equal(mean, xo)


@pytest.mark.gpu
def test_global_table_prefetch_variant_bit_identical(cuda):
    """The global-table matrix-core kernel reads its tables through a raw buffer
    resource (rows past the table return zeros); the register double-buffered
    variant (7) loads the same fragments one chunk earlier: identical results."""
    prob = prosail_problem(N=3000, n_bands=10, seed=31)
    x0, a0, s0 = run_fused(prob, cuda, variant=0, expect_global=True)
    x7, a7, s7 = run_fused(prob, cuda, variant=7, expect_global=True)
    assert np.array_equal(x0, x7) and np.array_equal(a0, a7) and np.array_equal(s0, s7)


@pytest.mark.gpu
def test_shared_centre_operand_bit_identical(cuda):
    """PROSAIL emulators share one centre (models/gp.py set_center), so the
    global-table kernel builds the exponent operand once per iteration and each
    band patches its constant in (BAND_LAYOUT_SHARED_X); variant 14 builds it per
    band: identical results."""
    prob = prosail_problem(N=3000, n_bands=10, seed=33)
    db = dbands(prob, cuda)
    tab = build_table(prob["specs"], db, prob["n"], RecordCache(), cuda)
    assert tab.layout == K.BAND_LAYOUT_SHARED_X
    xs, as_, ss = run_fused(prob, cuda, variant=0, expect_global=True)
    xp, ap, sp = run_fused(prob, cuda, variant=14, expect_global=True)
    assert np.array_equal(xs, xp) and np.array_equal(as_, ap) and np.array_equal(ss, sp)
