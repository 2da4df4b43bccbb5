"""Split-f16 matrix-core GP tables (models/gp.py:mfma_tables, the operand
layout of csrc/kf_gp_mfma.h) on the CPU: ``mfma_emulate`` reads the fragments
exactly as the kernel's lanes do (packed hi/lo sum rows, L'lo folded into the
sums operand, c_lo applied per pixel) and must reproduce the float64 GP value
and Jacobian (the emulator's own predict, /root/reference/kafka/inference/
utils.py:86-90 protocol)."""
import numpy as np
import pytest

from kafka_inferenceengine_amd.models import gp


def _case(kind):
    if kind == "tip":
        em = gp.make_tip_emulators(n_train=500, seed=3)[1]
    else:
        em = gp.make_prosail_emulators(n_bands=1, n_train=250, seed=4)[0]
    rng = np.random.default_rng(11)
    lo, hi = em.inputs.min(0), em.inputs.max(0)
    X = lo + (hi - lo) * rng.random((3000, em.n_inputs))
    return em, X


@pytest.mark.parametrize("kind", ["tip", "prosail"])
def test_emulated_tables_match_float64_gp(kind):
    em, X = _case(kind)
    D = em.n_inputs
    tab, nch, scale = gp.mfma_tables(em.records(), em.n_pos_pairs, em.lam)
    assert tab.shape == (nch, gp.gpm_frags_per_chunk(D), 8) and tab.dtype == np.float16
    assert 32 * nch >= em.n_train
    xi = X - em.center()[None, :]
    c = -0.5 * gp.LOG2E * (em.lam[None, :] * xi * xi).sum(1)
    S = gp.mfma_emulate(tab, nch, scale, D, xi, c)
    H = em.mean + S[:, 0]
    dH = -em.lam[None, :] * xi * S[:, :1] + np.log(2.0) * S[:, 1:]
    Hr, dHr = em.predict(X)
    eh = np.abs(H - Hr).max() / np.abs(Hr).max()
    ed = (np.abs(dH - dHr).max(0) / np.abs(dHr).max(0)).max()
    assert eh < 1e-5 and ed < 5e-5, (eh, ed)


def test_table_layout_packs_hi_lo_rows():
    """TIP (D = 4): one exponent K step (3D + 2 = 14 slots) and 2(D+1) = 10
    sums fragments per (K half, lane half); PROSAIL (D = 10): 32 slots = two K
    steps (was three with the lo constants in K slots)."""
    assert gp.gpm_k_steps(4) == 1 and gp.gpm_k_steps(10) == 2 and gp.gpm_k_steps(7) == 2
    assert gp.gpm_lo_row(4) == 8 and gp.gpm_lo_row(7) == 8 and gp.gpm_lo_row(10) == 16
    assert gp.gpm_frags_per_chunk(4) == 64 + 40 and gp.gpm_frags_per_chunk(10) == 128 + 88
    em, _ = _case("tip")
    tab, nch, _ = gp.mfma_tables(em.records(), em.n_pos_pairs, em.lam)
    t = tab.astype(np.float64)
    # exponent slots 3D = L'h, 3D + 1 = 1 (times c_hi), slots past 3D + 1 zero
    D = 4
    lanes = t[:, :64, :]                       # [chunk, lane, j]: K slot 8 (lane >> 5) + j
    slot = lambda k: lanes[:, 32 * (k // 8):32 * (k // 8) + 32, k % 8]
    assert np.all(slot(3 * D + 1)[:, :] == 1.0) or np.all(slot(3 * D + 1)[-1, -1] in (0.0, 1.0))
    assert np.all(slot(14) == 0) and np.all(slot(15) == 0)
    # sums: row 0 of the hi half is sgn * 2^L'lo (|.| within 1 %), lo rows are tiny
    base = 64
    hi0 = t[:, base + 0, :]
    lo0 = t[:, base + D + 1, :]
    nz = hi0 != 0
    assert np.all(np.abs(np.abs(hi0[nz]) - 1.0) < 1e-2)
    assert np.all(np.abs(lo0) <= 1e-3)


def _f32_accumulated(em, pts, sgn, X, step=16):
    """f and the Jacobian with exact point terms summed the matrix-core way: an
    f32 accumulator gets one exact 16-point partial at a time, in table order."""
    LOG2E = 1.0 / np.log(2.0)
    lam = em.lam
    xc = X - em.center()
    L, B = pts[:, 0], pts[:, 1:]
    E = L[None, :] - 0.5 * LOG2E * (lam * xc * xc).sum(1)[:, None] + xc @ B.T
    terms = np.exp2(E) * sgn[None, :]
    fields = np.concatenate([np.ones((len(sgn), 1)), B], 1)
    acc = np.zeros((len(X), fields.shape[1]), np.float32)
    for s in range(0, len(sgn), step):
        acc = (acc + (terms[:, s:s + step] @ fields[s:s + step]).astype(np.float32)).astype(np.float32)
    S = acc.astype(np.float64)
    return em.mean + S[:, 0], -lam * xc * S[:, [0]] + np.log(2.0) * S[:, 1:]


def test_table_point_order_cuts_f32_accumulation_error():
    """The tables alternate the signs of alpha (mfma_point_order): with the
    matrix cores' f32 accumulation of 16-point partials, f and its Jacobian
    are several times closer to float64 than in the records' sign-grouped
    order, for the cancelling sums of a realistic (1e-3 nugget) emulator."""
    em = gp.make_tip_emulators(n_train=500, seed=0)[0]
    rng = np.random.default_rng(1)
    lo, hi = em.inputs.min(0), em.inputs.max(0)
    X = lo + (hi - lo) * (0.1 + 0.8 * rng.random((2048, em.n_inputs)))
    H, G = em.predict(X)
    rec = em.records().astype(np.float64)
    pts = rec.transpose(0, 2, 1).reshape(-1, em.n_inputs + 1)
    sgn = np.where(np.arange(pts.shape[0]) < 2 * em.n_pos_pairs, 1.0, -1.0)
    keep = pts[:, 0] > -1e29
    grouped = _f32_accumulated(em, pts[keep], sgn[keep], X)
    ordered = _f32_accumulated(em, *gp.mfma_point_order(rec, em.n_pos_pairs), X)
    err = lambda r: (np.abs(r[0] - H).max() / np.abs(H).max(), np.abs(r[1] - G).max() / np.abs(G).max())  # noqa: E731
    (hg, gg), (ho, go) = err(grouped), err(ordered)
    assert ho < hg / 4 and go < gg / 3, (hg, gg, ho, go)
    assert ho < 4e-6 and go < 1e-5, (ho, go)


# --------------------------------------------------------------- line tables
def _tip_line_specs():
    import kafka_inferenceengine_amd as k

    ems = gp.make_tip_emulators(500, 0)
    return [k.gp_spec(ems[b], k.TIP_BAND_MAPPER[b]) for b in (0, 1)], np.asarray(k.tip_prior()[0], np.float32)


def _eval_f32(tab, t):
    """The kernels' arithmetic (line_pos / line_eval) in float32."""
    coef, t0, inv_h, n = tab
    t = np.asarray(t, np.float32)
    u = (t - np.float32(t0)) * np.float32(inv_h)
    uc = np.minimum(np.maximum(u, np.float32(0)), np.float32(n))
    kk = np.minimum(uc.astype(np.int64), n - 1)
    s = (uc - kk.astype(np.float32))[:, None, None]
    c = coef[kk]
    return ((c[..., 3] * s + c[..., 2]) * s + c[..., 1]) * s + c[..., 0]


def test_line_table_matches_float64_gp():
    """The JRC-TIP bands along the LAI propagator's forecast line: the float32
    evaluation of the cubic pieces equals the float64 GP value and gradient to
    a few 1e-8 of the GP's term scale over the whole table, on the emulator's
    parameters and on its float32 records alike."""
    specs, fixed = _tip_line_specs()
    tab = gp.line_table(specs, fixed, 6)
    assert tab is not None
    coef, t0, inv_h, n = tab
    assert coef.shape == (n, 2, 5, 4) and np.float32(t0) == t0 and np.log2(inv_h).is_integer()
    t = np.random.default_rng(0).uniform(t0, t0 + n / inv_h, 20000).astype(np.float32)
    p = _eval_f32(tab, t)
    for b, sp in enumerate(specs):
        F, _, scale = gp.line_functions(sp, fixed, 6, t.astype(np.float64))
        assert (np.abs(p[:, b] - F) / scale[:, None]).max() < 1e-7
        rec = gp.line_functions(type("S", (), dict(vars(sp), emulator=None))(), fixed, 6, t[:200].astype(np.float64))
        assert (np.abs(rec[0] - F[:200]) / scale[:200, None]).max() < 1e-6
    # every band input reading state 6 is covered (training box + margin)
    lo = min(sp.domain_lo[d] + sp.center[d] for sp in specs for d, s in enumerate(sp.state_map) if s == 6)
    assert t0 < lo


def test_line_table_derivatives_and_constant_point():
    """The tabulated t-derivatives are the GP's (finite differences), and with
    nothing propagated the table is one constant interval at the reset mean."""
    specs, fixed = _tip_line_specs()
    t = np.array([0.2, 0.45, 0.8])
    F, dF, _ = gp.line_functions(specs[1], fixed, 6, t)
    e = 1e-5
    Fp, _, _ = gp.line_functions(specs[1], fixed, 6, t + e)
    Fm, _, _ = gp.line_functions(specs[1], fixed, 6, t - e)
    assert np.allclose((Fp - Fm) / (2 * e), dF, rtol=1e-6, atol=1e-8)
    x = np.tile(fixed.astype(np.float64), (3, 1))
    x[:, 6] = t
    H, dH = specs[1].emulator.predict(x[:, specs[1].state_map])
    assert np.allclose(F[:, 0], H, rtol=0, atol=1e-12) and np.allclose(F[:, 1:], dH, rtol=0, atol=1e-12)
    coef, t0, inv_h, n = gp.line_table(specs, fixed, -1)
    assert n == 1 and t0 == 0.0 and not coef[..., 1:].any()
    H0, dH0 = specs[0].emulator.predict(fixed[specs[0].state_map].astype(np.float64)[None])
    assert np.isclose(coef[0, 0, 0, 0], H0[0], rtol=1e-7) and np.allclose(coef[0, 0, 1:, 0], dH0[0], rtol=1e-6)
