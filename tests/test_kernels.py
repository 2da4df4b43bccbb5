"""Kernel numerics against the float64 oracle and plain-PyTorch references.

Every test runs on the CPU through the host runner (the same per-pixel source
as the gfx950 kernels); the ``gpu``-marked twins in test_gpu.py run the HIP
kernels and compare them to these references."""
import numpy as np
import pytest
import torch

import kafka_inferenceengine_amd as k
from kafka_inferenceengine_amd.inference import analysis_blocks, gain_blocks
from kafka_inferenceengine_amd.ops import kernels as K
from kafka_inferenceengine_amd.utils.blocks import pack_blocks, pack_matrix, unpack_blocks

import kernel_cases as C


def _run_analysis(prob, device):
    N, n = prob["N"], prob["n"]
    tab = C.table(prob, device)
    xo = torch.zeros((n, N), device=device)
    ao = torch.zeros((28, N), device=device)
    st = torch.zeros(N, dtype=torch.uint8, device=device)
    part = K.partials_buffer(N, device)
    K.analysis(n, tab, C.soa(prob["x"], device), C.soa(prob["xf"], device), C.packed(prob["Pf"], device), xo, ao,
               None, st, part)
    return xo.cpu().numpy().T, unpack_blocks(ao.cpu().numpy(), n), st.cpu().numpy(), K.reduce_partials(part).cpu()


@pytest.mark.parametrize("dn16", [False, True])
def test_analysis_vs_oracle(dn16):
    prob = C.tip_problem(dn16=dn16)
    xa, A, st, red = _run_analysis(prob, "cpu")
    xr, Ar = analysis_blocks(prob["x"], prob["xf"], prob["Pf"], C.oracle_bands(prob, prob["x"]))
    assert np.max(np.abs(xa - xr) / (np.abs(xr) + 0.05)) < 2e-3
    assert np.max(np.abs(A - Ar)) / np.abs(Ar).max() < 1e-5
    assert abs(red.item() - ((xr - prob["x"]) ** 2).sum()) / red.item() < 1e-3
    nobs = np.array([(w > 0) for _, w in prob["bands"]]).sum(0)
    assert np.all(((st & ~np.uint8(K.ST_OUT_OF_DOMAIN)) == K.ST_NO_OBS) == (nobs == 0))   # + the domain flag


def _expected_out_of_domain(prob, x):
    """Per band, as the reference emulators see it: the centred inputs outside
    the training box (OperatorSpec.domain_lo/hi), on any GP band."""
    out = np.zeros(len(x), bool)
    for sp in prob["specs"]:
        xi = x[:, list(sp.state_map)[:len(sp.domain_lo)]] - np.asarray(sp.center)[:len(sp.domain_lo)]
        out |= ((xi < np.asarray(sp.domain_lo)) | (xi > np.asarray(sp.domain_hi))).any(1)
    return out


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_domain_flag_marks_exactly_the_out_of_box_pixels(device):
    """ST_OUT_OF_DOMAIN: set on the pixels whose linearisation point lies
    outside some GP band's training box, observed or not, and on no other."""
    prob = C.tip_problem(N=2048, seed=4)
    x = prob["x"].copy()
    x[:100, 6] = -1.0           # TLAI below every band's box
    x[100:200, 0] = 5.0         # band 0's first input above its box
    x[200:260, 5] = -3.0        # band 1 only
    prob["x"] = x
    for bd in prob["raw"]:      # the flag does not depend on the band being observed
        for key in ("w", "dn"):
            if key in bd:
                bd[key][:50] = 0
    for y, w in prob["bands"]:
        w[:50] = 0.0
    _, _, st, _ = _run_analysis(prob, device)
    want = _expected_out_of_domain(prob, x.astype(np.float32).astype(np.float64))
    assert want[:260].all() and 0 < want.sum() < len(want)
    got = (st & K.ST_OUT_OF_DOMAIN) > 0
    assert np.array_equal(got, want)


def test_analysis_vs_torch_fp32_reference():
    """Plain PyTorch fp32 reference of the same op (batched normal equations)."""
    prob = C.tip_problem(seed=1)
    xa, A, _, _ = _run_analysis(prob, "cpu")
    bands = C.oracle_bands(prob, prob["x"])
    Pf = torch.tensor(prob["Pf"], dtype=torch.float32)
    x0 = torch.tensor(prob["x"], dtype=torch.float32)
    xf = torch.tensor(prob["xf"], dtype=torch.float32)
    At = Pf.clone()
    bt = (Pf @ xf[..., None])[..., 0]
    for H0, h, y, w in bands:
        h = torch.tensor(h, dtype=torch.float32)
        w = torch.tensor(w, dtype=torch.float32)
        yp = torch.tensor(y, dtype=torch.float32) + (h * x0).sum(1) - torch.tensor(H0, dtype=torch.float32)
        At += w[:, None, None] * h[:, :, None] * h[:, None, :]
        bt += (w * yp)[:, None] * h
    xt = torch.linalg.solve(At, bt).numpy()
    assert np.max(np.abs(xa - xt) / (np.abs(xt) + 0.05)) < 3e-3


def test_nonspd_fallback_keeps_forecast():
    prob = C.tip_problem(N=256, seed=2)
    prob["Pf"] = prob["Pf"].copy()
    prob["Pf"][:10] = -np.eye(7)[None]          # indefinite forecast precision
    for bd in prob["raw"]:
        bd["w"][:10] = 0.0
    for i, (y, w) in enumerate(prob["bands"]):
        w[:10] = 0.0
    xa, A, st, _ = _run_analysis(prob, "cpu")
    assert np.all(st[:10] & K.ST_FALLBACK)
    assert np.allclose(xa[:10], prob["xf"][:10].astype(np.float32))
    assert np.all(np.isfinite(xa))


def test_gain_kernel_vs_oracle():
    prob = C.tip_problem(seed=3)
    N, n = prob["N"], prob["n"]
    Pcov = np.linalg.inv(prob["Pf"])
    tab = C.table(prob, "cpu")
    xo = torch.zeros((n, N))
    po = torch.zeros((28, N))
    K.gain(n, tab, C.soa(prob["x"], "cpu"), C.soa(prob["xf"], "cpu"), C.packed(Pcov, "cpu"), xo, po)
    xr, Pr = gain_blocks(prob["x"], prob["xf"], Pcov, C.oracle_bands(prob, prob["x"]))
    xi, _ = analysis_blocks(prob["x"], prob["xf"], prob["Pf"], C.oracle_bands(prob, prob["x"]))
    assert np.allclose(xr, xi, atol=1e-6)  # oracle: gain form == information form
    assert np.max(np.abs(xo.numpy().T - xr) / (np.abs(xr) + 0.05)) < 2e-3
    assert np.max(np.abs(unpack_blocks(po.numpy(), n) - Pr)) / np.abs(Pr).max() < 1e-3


@pytest.mark.parametrize("n", [1, 2, 3, 4, 7, 10])
def test_invert(n):
    rng = np.random.default_rng(n)
    B = C.spd_blocks(rng, 500, n)
    out = torch.zeros((n * (n + 1) // 2, 500))
    K.invert(n, C.packed(B, "cpu"), out)
    ref = torch.linalg.inv(torch.tensor(B, dtype=torch.float32)).numpy()
    assert np.allclose(unpack_blocks(out.numpy(), n), ref, rtol=1e-4, atol=1e-6)


def _prop(mode, n=7, N=400, blend=False, quirk=False, seed=0, prop_mask=0):
    rng = np.random.default_rng(seed)
    A = C.spd_blocks(rng, N, n, 5.0)
    xa = rng.normal(size=(N, n))
    mu, cov, Pi = k.tip_prior()
    q = rng.uniform(0.01, 0.2, n)
    m = rng.uniform(0.9, 1.1, n)
    spec = {"mode": mode, "m": m, "q": q, "prop_mask": prop_mask, "reset_mean": mu, "reset_cinv": pack_matrix(Pi),
            "blend": blend, "quirk_blend": quirk, "blend_mean": mu * 1.1, "blend_cinv": pack_matrix(Pi * 0.5)}
    xf = torch.zeros((n, N))
    pf = torch.zeros((28, N))
    K.propagate(n, spec, C.soa(xa, "cpu"), C.packed(A, "cpu"), xf, pf)
    return xa, A, mu, Pi, q, m, xf.numpy().T, unpack_blocks(pf.numpy(), n)


def test_propagate_modes_vs_reference_api():
    import scipy.sparse as sp
    from kafka_inferenceengine_amd.inference import kf_tools as T
    from kafka_inferenceengine_amd.utils.blocks import blocks_to_sparse, interleaved_to_soa, sparse_to_blocks

    # exact information filter
    xa, A, mu, Pi, q, m, xf, Pf = _prop(T.PROP_INFO_EXACT)
    Q = sp.diags(np.tile(q, 400))
    M = sp.diags(np.tile(m, 400))
    xr, _, Pr = T.propagate_information_filter_SLOW(xa.ravel(), None, blocks_to_sparse(A), M, Q, n_params=7)
    assert np.allclose(xf, xr.reshape(400, 7), rtol=1e-5)
    assert np.allclose(Pf, sparse_to_blocks(Pr, 7, check=False), rtol=2e-3, atol=1e-3)
    # diagonal approximation
    xa, A, mu, Pi, q, m, xf, Pf = _prop(T.PROP_INFO_APPROX)
    _, _, Pr = T.propagate_information_filter_approx_SLOW(xa.ravel(), None, blocks_to_sparse(A), M, Q)
    assert np.allclose(Pf, sparse_to_blocks(Pr, 7, check=False), rtol=1e-5)
    # LAI (partial prior reset)
    xa, A, mu, Pi, q, m, xf, Pf = _prop(T.PROP_PRIOR_PARTIAL, prop_mask=1 << 6)
    xr, _, Pr = T.propagate_information_filter_LAI(xa.ravel(), None, blocks_to_sparse(A), M, Q)
    assert np.allclose(xf, xr.reshape(400, 7), rtol=1e-5)
    assert np.allclose(Pf, sparse_to_blocks(Pr, 7, check=False), rtol=1e-5, atol=1e-4)
    # standard (covariance form)
    xa, A, mu, Pi, q, m, xf, Pf = _prop(T.PROP_STANDARD)
    assert np.allclose(Pf, A + np.diag(q)[None], rtol=1e-6)
    # prior reset
    xa, A, mu, Pi, q, m, xf, Pf = _prop(T.PROP_PRIOR)
    assert np.allclose(xf, mu[None]) and np.allclose(Pf, Pi[None], rtol=1e-5)


@pytest.mark.parametrize("quirk", [False, True])
def test_blend_vs_reference_api(quirk):
    from kafka_inferenceengine_amd.inference import kf_tools as T
    from kafka_inferenceengine_amd.utils.blocks import blocks_to_sparse, sparse_to_blocks

    xa, A, mu, Pi, q, m, xf, Pf = _prop(T.PROP_IDENTITY, blend=True, quirk=quirk)
    N = xa.shape[0]
    xr, Cr = T.blend_prior(np.tile(mu * 1.1, N), blocks_to_sparse(np.broadcast_to(Pi * 0.5, (N, 7, 7)).copy()),
                           (xa * m).ravel(), blocks_to_sparse(A), quirk=quirk, n_params=7)
    assert np.allclose(xf, xr.reshape(N, 7), rtol=2e-3, atol=2e-4)
    assert np.allclose(Pf, sparse_to_blocks(Cr, 7, check=False), rtol=1e-5)


def test_operator_gp_sar_linear_vs_numpy():
    prob = C.tip_problem(N=800, seed=4)
    tab = C.table(prob, "cpu")
    xs = C.soa(prob["x"], "cpu")
    for b in range(2):
        h0 = torch.zeros(800)
        h = torch.zeros((7, 800))
        K.operator_eval(7, tab, b, xs, h0, h)
        H, dH = prob["ems"][b].predict(prob["x"][:, k.TIP_BAND_MAPPER[b]])
        full = np.zeros((800, 7))
        full[:, k.TIP_BAND_MAPPER[b]] = dH
        assert np.allclose(h0.numpy(), H, atol=5e-6)
        assert np.allclose(h.numpy().T, full, atol=5e-5)
    # SAR
    from kafka_inferenceengine_amd.engine.bands import RecordCache, operator_table
    from kafka_inferenceengine_amd.models.operators import _sar_device_spec
    rng = np.random.default_rng(5)
    x = np.stack([rng.uniform(0.2, 5, 600), rng.uniform(0.05, 0.45, 600)], 1)
    th = torch.tensor(rng.uniform(25, 45, 600), dtype=torch.float32)
    specs = [_sar_device_spec(2, None, None, b) for b in range(2)]
    tab = operator_table(specs, 2, RecordCache(), "cpu", aux=th)
    for b, pol in enumerate(("VV", "VH")):
        h0 = torch.zeros(600)
        h = torch.zeros((2, 600))
        K.operator_eval(2, tab, b, C.soa(x, "cpu"), h0, h)
        s0, g = k.sar_observation_operator(x, th.numpy().astype(np.float64), pol)
        assert np.allclose(h0.numpy(), s0, rtol=2e-5)
        assert np.allclose(h.numpy().T, g, rtol=2e-4, atol=1e-7)
    # linear
    lin = k.models.operators._linear_device_spec(4, k.LinearOperator(np.array([0.5, -1., 2., 0.]), 0.3), None, 0)
    tab = operator_table([lin], 4, RecordCache(), "cpu")
    x = rng.normal(size=(100, 4))
    h0 = torch.zeros(100)
    K.operator_eval(4, tab, 0, C.soa(x, "cpu"), h0)
    assert np.allclose(h0.numpy(), 0.3 + x @ np.array([0.5, -1., 2., 0.]), atol=1e-5)


def test_hessian_vs_numpy():
    hessian_vs_numpy("cpu")


def hessian_vs_numpy(device):
    prob = C.tip_problem(N=300, seed=6)
    tab = C.table(prob, device)
    a = torch.zeros((28, 300), device=device)
    K.hessian(7, tab, C.soa(prob["x"], device), a)
    ref = np.zeros((300, 7, 7))
    for b, (y, w) in enumerate(prob["bands"]):
        mp = k.TIP_BAND_MAPPER[b]
        f, _ = prob["ems"][b].predict(prob["x"][:, mp])
        Hs = prob["ems"][b].hessian(prob["x"][:, mp])
        ref[np.ix_(np.arange(300), mp, mp)] -= (w * (y - f))[:, None, None] * Hs
    got = unpack_blocks(a.cpu().numpy(), 7)
    assert np.max(np.abs(got - ref)) / (np.abs(ref).max() + 1e-9) < 2e-3


def test_gp_hessian_finite_difference():
    em = k.make_tip_emulators(n_train=40)[0]
    x = np.array([[0.3, 1.2, 0.4, 0.2]])
    Hs = em.hessian(x)[0]
    eps = 1e-5
    for j in range(4):
        e = np.zeros(4)
        e[j] = eps
        gp = em.predict(x + e)[1][0]
        gm = em.predict(x - e)[1][0]
        assert np.allclose((gp - gm) / (2 * eps), Hs[:, j], rtol=1e-4, atol=1e-6)


def test_unpack_and_gather_and_lut():
    unpack_gather_lut_vs_torch("cpu")


def unpack_gather_lut_vs_torch(device):
    rng = np.random.default_rng(7)
    N = 200
    x = rng.normal(size=(N, 7))
    A = C.spd_blocks(rng, N, 7)
    idx = torch.tensor(np.sort(rng.choice(400, N, replace=False)), dtype=torch.int64, device=device)
    mean = torch.zeros((7, 400), device=device)
    unc = torch.zeros((7, 400), device=device)
    K.unpack(7, C.soa(x, device), C.packed(A, device), mean, unc, idx=idx)
    ii = idx.cpu().numpy()
    assert np.allclose(mean.cpu().numpy()[:, ii], x.T.astype(np.float32))
    assert np.allclose(unc.cpu().numpy()[:, ii], 1 / np.sqrt(np.einsum("nii->ni", A)).T, rtol=1e-6)
    src = torch.arange(1000, dtype=torch.float32, device=device)
    g = K.gather(src, idx)
    assert torch.equal(g, src[idx])
    lut = torch.tensor(rng.normal(size=(50, 3)), dtype=torch.float32, device=device)
    pts = torch.tensor(rng.normal(size=(3, 300)), dtype=torch.float32, device=device)
    got = K.lut_nearest(lut, pts)
    ref = torch.cdist(pts.T.cpu(), lut.cpu()).argmin(1)
    assert torch.equal(got.long().cpu(), ref)


def test_jacobi_sweep_vs_numpy():
    jacobi_sweep_vs_numpy("cpu")


def jacobi_sweep_vs_numpy(device):
    from kafka_inferenceengine_amd.parallel import StripPartition
    rng = np.random.default_rng(8)
    mask = rng.random((12, 9)) > 0.2
    part = StripPartition(mask)
    N, n = part.N, 4
    A = C.spd_blocks(rng, N, n)
    b = rng.normal(size=(N, n))
    x = rng.normal(size=(N, n))
    nbr = torch.from_numpy(part.neighbour_table()).to(device)
    out = torch.zeros((n, N), device=device)
    gamma, regmask = 3.0, 0b0101
    K.jacobi(n, C.packed(A, device), C.soa(b, device), C.soa(x, device), nbr, C.soa(x, device), out, gamma, regmask,
             N)
    nb = nbr.cpu().numpy()
    ref = np.zeros((N, n))
    for p in range(N):
        Ap, bp = A[p].copy(), b[p].copy()
        qs = [q for q in nb[:, p] if q >= 0]
        for j in range(n):
            if (regmask >> j) & 1:
                Ap[j, j] += gamma * len(qs)
                bp[j] += gamma * sum(x[q, j] for q in qs)
        ref[p] = np.linalg.solve(Ap, bp)
    assert np.allclose(out.cpu().numpy().T, ref, rtol=1e-4, atol=1e-5)


def test_neighbour_table_matches_raster():
    from kafka_inferenceengine_amd.parallel import StripPartition
    rng = np.random.default_rng(9)
    mask = rng.random((10, 7)) > 0.3
    part = StripPartition(mask)
    nb = part.neighbour_table()
    lid = -np.ones(mask.shape, dtype=int)
    lid[mask] = np.arange(mask.sum())
    for p, flat in enumerate(part.local_idx):
        r, c = divmod(flat, 7)
        exp = [lid[r - 1, c] if r > 0 else -1, lid[r + 1, c] if r < 9 else -1,
               lid[r, c - 1] if c > 0 else -1, lid[r, c + 1] if c < 6 else -1]
        assert list(nb[:, p]) == exp


@pytest.mark.parametrize("mode,blend,quirk,pmask", C.FUSED_CASES)
def test_fused_propagation_equals_materialized(mode, blend, quirk, pmask):
    ref, fused = C.fused_vs_materialized("cpu", mode, blend, quirk, pmask)
    def rel(a, b):   # row-scaled: diag-approx forecasts are ill-conditioned per pixel
        return np.max(np.abs(a - b) / np.maximum(np.abs(b).max(1, keepdims=True), 1e-3))
    for (x1, a1, s1), (x2, a2, s2) in zip(ref, fused):
        assert np.array_equal(s1, s2)
        assert rel(x2, x1) < 1e-4 and rel(a2, a1) < 1e-4


@pytest.mark.parametrize("mode,blend", [(3, False), (4, False), (5, False), (1, True)])
def test_heavy_propagation_is_not_fused(mode, blend):
    with pytest.raises(ValueError, match="fused"):
        C.fused_vs_materialized("cpu", mode, blend, N=64)


def affine_vs_classic_jacobi(device, n=7, regmask=0b1000100, sweeps=4, seed=9):
    """The affine regulariser (prepare once, iterate the k regularised fields,
    finish) equals ``sweeps`` classic block-Jacobi sweeps, and writes A + g deg E_R."""
    from kafka_inferenceengine_amd.parallel import StripPartition
    rng = np.random.default_rng(seed)
    mask = rng.random((14, 11)) > 0.15
    part = StripPartition(mask)
    N = part.N
    A = C.spd_blocks(rng, N, n)
    b = rng.normal(size=(N, n))
    x0 = rng.normal(size=(N, n))
    nbr = torch.from_numpy(part.neighbour_table()).to(device)
    gamma = 2.5
    Ad, bd, xd = C.packed(A, device), C.soa(b, device), C.soa(x0, device)
    # classic: every sweep re-factors A + g deg E_R
    cur = xd.clone()
    for _ in range(sweeps):
        nxt = torch.zeros_like(cur)
        K.jacobi(n, Ad, bd, cur, nbr, xd, nxt, gamma, regmask, N)
        cur = nxt
    ref = cur.cpu().numpy()
    # affine
    rows = [j for j in range(n) if (regmask >> j) & 1]
    k = len(rows)
    u = torch.zeros((n, N), device=device)
    v = torch.zeros((k * n, N), device=device)
    A2 = Ad.clone()
    K.reg_prepare(n, A2, bd, nbr, u, v, gamma, regmask, N, a_out=A2)
    z = [xd[rows].clone().contiguous(), torch.zeros((k, N), device=device)]
    c = 0
    for _ in range(sweeps - 1):
        K.reg_sweep(n, u, v, z[c], nbr, z[1 - c], gamma, regmask, N)
        c = 1 - c
    out = torch.zeros((n, N), device=device)
    part_buf = K.partials_buffer(N, device)
    K.reg_finish(n, u, v, z[c], nbr, xd, out, gamma, regmask, N, partials=part_buf)
    got = out.cpu().numpy()
    assert np.allclose(got, ref, rtol=1e-4, atol=1e-5), float(np.abs(got - ref).max())
    norm = float(K.reduce_partials(part_buf).cpu()[0])
    assert np.isclose(norm, float(((got - x0.T) ** 2).sum()), rtol=1e-4)
    deg = (nbr >= 0).sum(0).cpu().numpy()
    Areg = unpack_blocks(A2.cpu().numpy(), n)
    for j in rows:
        assert np.allclose(Areg[:, j, j], A[:, j, j] + gamma * deg, rtol=1e-5)


@pytest.mark.parametrize("regmask", [0b1000000, 0b1000101])
def test_affine_jacobi_equals_classic(regmask):
    affine_vs_classic_jacobi("cpu", regmask=regmask)


def test_dense_geometry_equals_neighbour_table():
    """Index-derived neighbours (kf_core.h:StripGeo) reproduce the table for
    dense strips of a 3-rank partition (halo above, below, both)."""
    from kafka_inferenceengine_amd.parallel import StripPartition
    rng = np.random.default_rng(3)
    mask = np.ones((15, 7), bool)
    n, regmask, gamma = 4, 0b0110, 1.7
    for rank in range(3):
        part = StripPartition(mask, rank, 3)
        geo = part.dense_geometry()
        assert geo is not None
        N = part.N
        lay = part.halo_layout()
        cols = N + lay["n_up"] + lay["n_down"]
        u = torch.from_numpy(rng.normal(size=(n, N)).astype(np.float32))
        v = torch.from_numpy(rng.normal(size=(2 * n, N)).astype(np.float32))
        z = torch.from_numpy(rng.normal(size=(2, cols)).astype(np.float32))
        nbr = torch.from_numpy(part.neighbour_table())
        outs = []
        for g, t in ((geo, None), (None, nbr)):
            zo = torch.zeros((2, cols))
            K.reg_sweep(n, u, v, z, t, zo, gamma, regmask, N, geo=g)
            xo = torch.zeros((n, N))
            K.reg_finish(n, u, v, z, t, u, xo, gamma, regmask, N, geo=g)
            outs.append((zo, xo))
        assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    holes = mask.copy()
    holes[7, 3] = False
    assert StripPartition(holes, 1, 3).dense_geometry() is None


@pytest.mark.parametrize("case", [dict(), dict(omegas=(1.1, 1.2, 1.3), cheb=(True, True, False)),
                                  dict(h=7, w=5, omegas=(1.0,) * 8), dict(omegas=(1.0,), cheb=(False,))])
def test_reg_sweeps_tiled_equals_sequential(case):
    (zt, zpt), (zs, zps) = C.tiled_vs_sequential("cpu", **case)
    assert torch.equal(zt, zs) and torch.equal(zpt, zps)


DEEP_HALO_CASES = [dict(), dict(split=True), dict(r0=0, r1=90), dict(r0=120, r1=200, split=True),
                   dict(depth=6, omegas=(1.0,) * 6, cheb=(False,) * 6, split=True),
                   dict(device_sched=True, split=True), dict(device_sched=True, rho=0.3),
                   dict(device_sched=True, rho=0.0), dict(h_total=40, w=33, r0=9, r1=17, depth=8)]


@pytest.mark.parametrize("case", DEEP_HALO_CASES)
def test_reg_sweeps_tiled_deep_halo_equals_full_domain(case):
    """A strip's pass with the neighbours' rows in deep-halo planes equals the
    same rows of a pass over the whole raster: the ring's stale values never
    reach the strip (tile-DP C2 once per pass)."""
    (zs, zps), (zf, zpf) = C.deep_halo_vs_full("cpu", **case)
    assert torch.equal(zs, zf) and torch.equal(zps, zpf)


def test_reg_schedule_matches_host_formula():
    """The device-side Chebyshev schedule (kf_core.h:reg_cheb_schedule) gives
    the engine's host schedule: sweep count and weights."""
    kf = k.LinearKalman.__new__(k.LinearKalman)
    kf.config = k.EngineConfig(spatial_max_sweeps=40)
    for rho, tol in ((0.833, 1e-3), (0.2, 1e-1), (0.0, 1e-3), (0.99999, 1e-3), (1.2, 1e-3), (float("nan"), 1e-3)):
        rs = K.RegSchedule(100, 40, "cpu")
        rs.rho.fill_(rho)
        rs.schedule(tol)
        S = int(rs.info[1])
        r_h, S_h = kf._reg_sweeps_for(rho, tol)
        assert S == S_h and int(rs.sched[0]) == S - 1
        w = kf._cheb_weights(r_h, S - 1)
        assert [float(np.float32(o)) if c else 0.0 for o, c in w] == rs.omega[:S - 1].tolist()


def test_reg_boundary_tile_rows():
    assert K.reg_boundary_tile_rows(1373, 8, True, True) == (1, 21)
    assert K.reg_boundary_tile_rows(1373, 8, False, True) == (0, 21)
    assert K.reg_boundary_tile_rows(1373, 8, True, False) == (1, 22)
    assert K.reg_boundary_tile_rows(70, 8, True, True) == (1, 1)     # two tile rows, both boundary
    assert K.reg_boundary_tile_rows(6, 6, True, True) == (1, 1)


def test_reg_sweeps_tiled_rejects_bad_args():
    u = torch.zeros(7, 100)
    z = torch.zeros(1, 100)
    geo = {"w": 10, "h": 10, "halo": 0, "n_up": 0}
    with pytest.raises(ValueError):
        K.reg_sweeps_tiled(7, u, u, z, None, torch.zeros(1, 100), torch.zeros(1, 100), 1.0, 4, 100,
                           dict(geo, halo=1), [1.0], [False])
    with pytest.raises(ValueError):
        K.reg_sweeps_tiled(7, u, u, z, None, torch.zeros(1, 100), torch.zeros(1, 100), 1.0, 4, 100, geo,
                           [1.0] * 9, [False] * 9)
    with pytest.raises(ValueError):
        K.reg_sweeps_tiled(7, u, u, z, None, torch.zeros(1, 100), torch.zeros(1, 100), 1.0, 4, 100, geo,
                           [1.0], [True])
    with pytest.raises(ValueError):
        K.reg_sweeps_tiled(7, u, u, z, None, z, torch.zeros(1, 100), 1.0, 4, 100, geo, [1.0], [False])


def test_band_layout_detection():
    """BAND_LAYOUT_TIP (kf_core.h) is set only for two GP bands with the JRC-TIP
    VIS then NIR maps and matrix-core tables; any other set runs the
    runtime-layout kernel."""
    from kafka_inferenceengine_amd.engine.bands import DeviceBand, RecordCache, build_table

    ems = k.make_tip_emulators(n_train=64, seed=1)
    specs = [k.gp_spec(em, mp) for em, mp in zip(ems, [k.TIP_BAND_MAPPER[0], k.TIP_BAND_MAPPER[1]])]
    N = 100
    dbs = [DeviceBand(K.OBS_F32, y=torch.zeros(N), w=torch.ones(N)) for _ in specs]
    cache = RecordCache()
    assert build_table(specs, dbs, 7, cache, torch.device("cpu")).layout == K.BAND_LAYOUT_TIP
    assert build_table(specs[::-1], dbs, 7, cache, torch.device("cpu")).layout == 0
    assert build_table(specs[:1], dbs[:1], 7, cache, torch.device("cpu")).layout == 0
    assert build_table(specs + specs[:1], dbs + dbs[:1], 7, cache, torch.device("cpu")).layout == 0
