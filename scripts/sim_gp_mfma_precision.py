"""Host simulation of the split-f16 MFMA GP evaluation (csrc/kf_gp_mfma.h).

Emulates the exact rounding steps of the device path in NumPy — f16 hi/lo
operands, exact products, f32 accumulation, v_exp_f32, RTZ hi + RNE lo split
of m — and reports the error of (f, df/dx) against the float64 GP, next to
the error of the current f32 VALU algebra.  Used to choose the split (3 or 4
terms for the exponent) before writing the kernel.

    python scripts/sim_gp_mfma_precision.py
"""
import numpy as np

from kafka_inferenceengine_amd.models.gp import make_prosail_emulators, make_tip_emulators, LOG2E

f16 = np.float16


def rtz16(v):
    """f32 -> f16 round toward zero (v_cvt_pkrtz_f16_f32)."""
    h = v.astype(f16).astype(np.float32)
    over = np.abs(h) > np.abs(v)
    # step one ulp toward zero where RNE rounded away
    hb = h.astype(f16).view(np.uint16).astype(np.int32)
    hb = np.where(over, hb - 1, hb).astype(np.uint16)
    return hb.view(f16)


def split16(v):
    h = v.astype(np.float32).astype(f16)
    lo = (v.astype(np.float64) - h.astype(np.float64)).astype(np.float32).astype(f16)
    return h, lo


def simulate(em, X, terms=3, a_lo=True, c_split=False):
    t = em.inputs - em.center()[None, :]
    L = np.log2(em.signal) - 0.5 * LOG2E * (t * t * em.lam[None]).sum(1) + np.log2(np.abs(em.alpha))
    B = LOG2E * em.lam[None, :] * t
    sgn = np.sign(em.alpha)
    sigma = np.ceil(np.log2(em.signal * np.abs(em.alpha)).max()) - 14.0   # m <= s|alpha| <= 2^14 (f16 range)
    Ls = L - sigma
    xi = X - em.center()[None, :]
    c = (-0.5 * LOG2E * (em.lam[None] * xi * xi).sum(1)).astype(np.float32)
    Bh, Bl = split16(B)
    Lh, Ll = split16(Ls)
    xh, xl = split16(xi)
    f = lambda a: a.astype(np.float64)
    if c_split:   # c folded into the K slots as f16 hi + lo
        ch, cl = split16(c)
        c = (f(ch) + f(cl)).astype(np.float64)
    e = f(c)[:, None] + f(xh) @ f(Bh).T + f(xh) @ f(Bl).T + f(xl) @ f(Bh).T + f(Lh)[None] + f(Ll)[None]
    if terms == 4:
        e += f(xl) @ f(Bl).T
    e = e.astype(np.float32)
    m = np.exp2(e).astype(np.float32)
    mh = rtz16(m)
    ml = (f(m) - f(mh)).astype(np.float32).astype(f16)
    A = np.concatenate([sgn[:, None], sgn[:, None] * B], axis=1)     # [T, D+1]
    Ah, Al = split16(A)
    S = f(mh) @ f(Ah) + f(ml) @ f(Ah) + (f(mh) @ f(Al) if a_lo else 0.0)
    S *= 2.0 ** sigma
    H = em.mean + S[:, 0]
    dH = -em.lam[None] * xi * S[:, :1] + np.log(2.0) * S[:, 1:]
    return H, dH


def valu_f32(em, X):
    """The current f32 VALU algebra (gp_pairs), f32 everywhere."""
    rec = em.records().astype(np.float32)            # [T2, D+1, 2]
    T2, R, _ = rec.shape
    r = rec.transpose(0, 2, 1).reshape(-1, R)        # point-major
    npos = 2 * em.n_pos_pairs
    sg = np.where(np.arange(r.shape[0]) < npos, 1.0, -1.0).astype(np.float32)
    xi = (X - em.center()[None]).astype(np.float32)
    c = (-0.5 * LOG2E * (em.lam[None] * xi * xi).sum(1)).astype(np.float32)
    e = (c[:, None] + r[None, :, 0] + (xi[:, None, :] * r[None, :, 1:]).sum(-1)).astype(np.float32)
    m = np.exp2(e) * sg[None]
    S0 = m.sum(1, dtype=np.float32)
    Sd = (m[:, :, None] * r[None, :, 1:]).sum(1, dtype=np.float32)
    H = em.mean + S0
    dH = -em.lam[None] * xi * S0[:, None] + np.log(2.0) * Sd
    return H, dH


def report(name, em, X):
    H, dH = em.predict(X)
    scale_h = np.abs(H).max()
    scale_d = np.abs(dH).max(0)
    for label, fn in (("valu_f32", lambda: valu_f32(em, X)), ("mfma3", lambda: simulate(em, X, 3)),
                      ("mfma3_c", lambda: simulate(em, X, 3, c_split=True)),
                      ("mfma3_c_noAl", lambda: simulate(em, X, 3, a_lo=False, c_split=True))):
        h, d = fn()
        eh = np.abs(h - H).max() / scale_h
        ed = (np.abs(d - dH).max(0) / scale_d).max()
        print(f"{name:10s} {label:13s} max|dH0|/|H0|max={eh:.2e}  max|dJ|/|J|max={ed:.2e}")


def main():
    rng = np.random.default_rng(0)
    for i, em in enumerate(make_tip_emulators()):
        lo, hi = em.inputs.min(0), em.inputs.max(0)
        X = lo + (hi - lo) * rng.random((4000, em.n_inputs))
        report(f"tip{i}", em, X)
    for i, em in enumerate(make_prosail_emulators(n_bands=3, n_train=500)):
        lo, hi = em.inputs.min(0), em.inputs.max(0)
        X = lo + (hi - lo) * rng.random((2000, em.n_inputs))
        report(f"prosail{i}", em, X)


if __name__ == "__main__":
    main()
