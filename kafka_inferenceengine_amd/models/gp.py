"""Gaussian-process emulators (the "PROSAIL/SAIL/JRC-TIP" observation model).

The reference loads pickled ``gp_emulator.GaussianProcess`` objects and calls
``predict(X, do_unc=False) -> (H, dH)`` (``kafka/inference/utils.py:86-90``)
and optionally ``hessian(x)`` (``kf_tools.py:28``).  No pickles ship with the
reference and unpickling is not allowed here, so this module provides a
self-contained RBF/ARD GP with the same protocol, fitted on synthetic
radiative-transfer-like targets ("random-init emulators", BASELINE.json).

Kernel:  f(x) = mu + sum_i alpha_i * s * exp(-1/2 sum_d lambda_d (x_d - t_id)^2)

``records()`` emits the packed per-training-point rows the gfx950 kernel
streams through the scalar path (``csrc/kf_core.h`` ``gp_eval``).
"""
from __future__ import annotations

import numpy as np

LOG2E = 1.4426950408889634


class GaussianProcessEmulator:
    """RBF (ARD) GP emulator with analytic gradient and Hessian."""

    def __init__(self, inputs, alpha, lam, signal: float = 1.0, mean: float = 0.0, name: str = "gp"):
        self.inputs = np.asarray(inputs, dtype=np.float64)      # [T, D]
        self.alpha = np.asarray(alpha, dtype=np.float64)        # [T]
        self.lam = np.asarray(lam, dtype=np.float64)            # [D]  (1/lengthscale^2)
        self.signal = float(signal)
        self.mean = float(mean)
        self.name = name
        if self.inputs.ndim != 2 or self.inputs.shape[0] != self.alpha.shape[0]:
            raise ValueError("inputs must be [T, D] and alpha [T]")
        if self.lam.shape != (self.inputs.shape[1],):
            raise ValueError("lam must have one entry per input dimension")
        self._records = None
        self._center = None     # set_center: a shared reference point (else the training mean)

    # ------------------------------------------------------------------ shape
    @property
    def n_inputs(self) -> int:
        return self.inputs.shape[1]

    @property
    def n_train(self) -> int:
        return self.inputs.shape[0]

    # ------------------------------------------------------------- numerics
    def _kernel(self, X):
        X = np.atleast_2d(np.asarray(X, dtype=np.float64))
        diff = X[:, None, :] - self.inputs[None, :, :]                 # [n, T, D]
        k = self.signal * np.exp(-0.5 * np.einsum("ntd,d->nt", diff * diff, self.lam))
        return X, diff, k

    def predict(self, X, do_unc: bool = False, chunk: int = 65536):
        """(H, dH) like gp_emulator; with ``do_unc`` returns (H, var, dH)."""
        X = np.atleast_2d(np.asarray(X, dtype=np.float64))
        H = np.empty(X.shape[0])
        dH = np.empty_like(X)
        for s in range(0, X.shape[0], chunk):
            _, diff, k = self._kernel(X[s:s + chunk])
            ak = k * self.alpha[None, :]
            H[s:s + chunk] = self.mean + ak.sum(1)
            dH[s:s + chunk] = -self.lam[None, :] * np.einsum("nt,ntd->nd", ak, diff)
        if do_unc:
            return H, np.zeros_like(H), dH
        return H, dH

    def hessian(self, X):
        """d2f/dx2, [n, D, D]."""
        _, diff, k = self._kernel(X)
        ak = k * self.alpha[None, :]
        ld = diff * self.lam[None, None, :]
        H = np.einsum("nt,ntu,ntv->nuv", ak, ld, ld)
        H -= np.einsum("nt,u->nu", ak, self.lam)[:, :, None] * np.eye(self.n_inputs)[None]
        return H

    # ---------------------------------------------------------- kernel ABI
    def center(self) -> np.ndarray:
        """Reference point the kernel records are expressed around (inputs are
        centred on it): the training mean unless ``set_center`` chose one."""
        return self.inputs.mean(0) if self._center is None else self._center

    def set_center(self, c) -> "GaussianProcessEmulator":
        """Express the records around ``c`` instead of the training mean (the
        same predictions up to rounding).  Bands of one state that share a
        reference point share their centred GP inputs, and the matrix-core
        kernel then builds the exponent operand once for all of them
        (kf_gp_mfma.h, BAND_LAYOUT_SHARED_X)."""
        c = np.asarray(c, dtype=np.float64).reshape(-1)
        if c.shape != (self.n_inputs,):
            raise ValueError("center needs one value per input")
        self._center = c.copy()
        self._records = None
        self.__dict__.pop("_spec_cache", None)
        return self

    def records(self) -> np.ndarray:
        """float32 kernel records, training-point pairs field-major:
        [T2, D+1, 2] with fields L' = log2(s |alpha|) - 1/2 log2e sum lambda t^2
        and B = log2e lambda t (inputs centred).  Points with alpha > 0 come
        first (``n_pos_pairs`` pairs), then alpha < 0; each group is padded to
        an even count with an L' = -1e30 point (contributes 0); alpha = 0 points
        are dropped.  See ``csrc/kf_core.h`` (gp_pairs) for the algebra."""
        if self._records is None:
            c = self.center()
            t = self.inputs - c[None, :]
            L = np.log2(self.signal) - 0.5 * LOG2E * (t * t * self.lam[None, :]).sum(1)
            B = LOG2E * self.lam[None, :] * t
            groups = []
            for sel in (self.alpha > 0, self.alpha < 0):
                Lg = L[sel] + np.log2(np.abs(self.alpha[sel]))
                rec = np.concatenate([Lg[:, None], B[sel]], axis=1)          # [Tg, D+1]
                if rec.shape[0] % 2:
                    pad = np.zeros((1, rec.shape[1]))
                    pad[0, 0] = -1e30   # 2^(-1e30 + ...) = 0
                    rec = np.concatenate([rec, pad], axis=0)
                groups.append(rec.reshape(-1, 2, rec.shape[1]).transpose(0, 2, 1))   # [Tg/2, D+1, 2]
            self._n_pos_pairs = int(groups[0].shape[0])
            pairs = np.concatenate(groups, axis=0) if (groups[0].size + groups[1].size) else \
                np.zeros((0, self.n_inputs + 1, 2))
            self._records = np.ascontiguousarray(pairs.astype(np.float32))
        return self._records

    @property
    def n_pos_pairs(self) -> int:
        """Leading record pairs with alpha > 0 (``BandDesc.Tp``)."""
        self.records()
        return self._n_pos_pairs

    @property
    def n_records(self) -> int:
        """Padded number of training points the kernel iterates over."""
        return 2 * self.records().shape[0]

    # ------------------------------------------------------------ building
    @classmethod
    def fit(cls, X, y, lengthscale, signal=None, noise=1e-6, name="gp"):
        X = np.asarray(X, dtype=np.float64)
        y = np.asarray(y, dtype=np.float64)
        lam = 1.0 / np.asarray(lengthscale, dtype=np.float64) ** 2
        mu = float(y.mean())
        s = float(np.var(y)) if signal is None else float(signal)
        s = max(s, 1e-12)
        diff = X[:, None, :] - X[None, :, :]
        K = s * np.exp(-0.5 * np.einsum("ijd,d->ij", diff * diff, lam))
        K[np.diag_indices_from(K)] += noise * s + 1e-10
        alpha = np.linalg.solve(K, y - mu)
        return cls(X, alpha, lam, s, mu, name=name)

    @classmethod
    def synthetic(cls, target, lo, hi, n_train: int = 500, seed: int = 0, length_frac: float = 0.35,
                  noise: float = 1e-3, name: str = "gp"):
        """Fit an emulator to ``target`` on a Latin-hypercube design in [lo, hi].
        ``noise``: the nugget as a fraction of the signal variance.  1e-3 is a
        fitted emulator's typical noise level: alpha stays near |f| instead of
        the cancelling weights of a near-interpolating 1e-5 nugget."""
        rng = np.random.default_rng(seed)
        lo = np.asarray(lo, dtype=np.float64)
        hi = np.asarray(hi, dtype=np.float64)
        D = lo.size
        u = (np.argsort(rng.random((D, n_train)), axis=1).T + rng.random((n_train, D))) / n_train
        X = lo + u * (hi - lo)
        y = target(X)
        return cls.fit(X, y, length_frac * (hi - lo), noise=noise, name=name)


# --------------------------------------------------------------------------
# flat packing (C4 setup broadcast of emulator sets)

def pack_emulator_set(ems: dict):
    """{key: emulator} -> (header, float64 buffer): header = [(key, T, D, name)],
    buffer = per emulator [signal, mean, inputs (T x D), alpha (T), lam (D), center (D)]."""
    header, parts = [], []
    for key, em in ems.items():
        T, D = em.inputs.shape
        header.append((str(key), int(T), int(D), str(em.name)))
        parts += [np.array([em.signal, em.mean]), em.inputs.ravel(), em.alpha.ravel(), em.lam.ravel(),
                  np.asarray(em.center(), dtype=np.float64).ravel()]
    return header, (np.concatenate(parts) if parts else np.zeros(0))


def unpack_emulator_set(header, buf) -> dict:
    out, o = {}, 0
    for key, T, D, name in header:
        sig, mu = buf[o], buf[o + 1]
        o += 2
        inputs = buf[o:o + T * D].reshape(T, D)
        o += T * D
        alpha = buf[o:o + T]
        o += T
        lam = buf[o:o + D]
        o += D
        center = buf[o:o + D]
        o += D
        em = GaussianProcessEmulator(inputs.copy(), alpha.copy(), lam.copy(), float(sig), float(mu), name=name)
        out[key] = em.set_center(center) if not np.array_equal(center, em.center()) else em
    return out


# --------------------------------------------------------------------------
# split-f16 MFMA tables (csrc/kf_gp_mfma.h)

GPM_MAX_D = 10
GPM_M_LOG2 = 14          # m = 2^E is kept <= 2^14 (f16 max 65504)
_F16_SAFE = 6.0e4


def gpm_k_steps(d: int) -> int:
    """16-slot K steps of the exponent MFMA (3d + 2 slots used)."""
    return (3 * d + 2 + 15) // 16


def gpm_lo_row(d: int) -> int:
    """First row of the lo half of the packed sums operand (same lane as the hi row)."""
    return 8 if d + 1 <= 8 else 16


def gpm_sum_rows(d: int) -> int:
    return 2 * (d + 1)


def gpm_frags_per_chunk(d: int) -> int:
    return 64 * gpm_k_steps(d) + 4 * gpm_sum_rows(d)


def _split16(v):
    hi = np.asarray(v, dtype=np.float64).astype(np.float16)
    lo = (v - hi.astype(np.float64)).astype(np.float16)
    return hi, lo


def _sum_points():
    """[q, h, j] -> point of the chunk in K slot 8h + j of sums half q (the
    exponent MFMA's accumulator registers 8q..8q+7, csrc/kf_gp_mfma.h)."""
    q, h, j = np.meshgrid(np.arange(2), np.arange(2), np.arange(8), indexing="ij")
    return (j & 3) + 4 * h + 8 * (j >> 2) + 16 * q


def mfma_point_order(records, n_pos_pairs: int):
    """Training points ``(pts [T, D+1] = (L', B), sgn [T])`` in the order of the
    matrix-core tables (padding dropped).

    The sums cancel by ~300x between the alpha > 0 and alpha < 0 points, and
    the matrix cores add each 16-point partial into an f32 accumulator.  Summed
    one sign group after the other (the VALU records' order), the running sum
    first grows to ~300x the result and keeps that magnitude's rounding errors.
    The sums operand carries the sign, so the points may come in any order:
    the signs alternate (each group by L', log2 of its weight at the centre,
    largest first) and the running sum stays near the result -- 10x less error
    in f and 7x less in the Jacobian than grouped (tests/test_gp_tables.py
    models the accumulation; tests/test_mvp.py pins whole runs against float64)."""
    rec = np.asarray(records, dtype=np.float64)
    D = rec.shape[1] - 1
    pts = rec.transpose(0, 2, 1).reshape(-1, D + 1)          # point-major [T, D+1]: L', B
    sgn = np.where(np.arange(pts.shape[0]) < 2 * int(n_pos_pairs), 1.0, -1.0)
    keep = pts[:, 0] > -1e29                                  # drop the pair padding (m = 0)
    pts, sgn = pts[keep], sgn[keep]
    pos = np.flatnonzero(sgn > 0)
    neg = np.flatnonzero(sgn < 0)
    pos = pos[np.argsort(-pts[pos, 0], kind="stable")]
    neg = neg[np.argsort(-pts[neg, 0], kind="stable")]
    m2 = min(pos.size, neg.size)
    order = np.empty(pos.size + neg.size, dtype=np.int64)
    order[0:2 * m2:2], order[1:2 * m2:2] = pos[:m2], neg[:m2]
    order[2 * m2:] = np.concatenate([pos[m2:], neg[m2:]])
    return pts[order], sgn[order]


def mfma_tables(records, n_pos_pairs: int, lam):
    """Operand fragments of the matrix-core GP (``csrc/kf_gp_mfma.h``) from the
    packed VALU records (``GaussianProcessEmulator.records``), so any
    ``OperatorSpec`` with records gets them.

    Returns ``(table, n_chunks, scale)``: ``table`` is float16 ``[n_chunks,
    frags_per_chunk, 8]``; per 32-point chunk the exponent A fragments of all
    64 lanes for each 16-slot K step (rows = points, slots ``[Bh | Bl | Bh |
    L'h | 1]``), then for each K half q and lane half h the sums A fragments of
    the 2(D+1) used rows: hi of ``A' = A 2^L'l`` (rows ``sgn``, ``sgn B_d``) in
    rows 0..D, lo in rows LO..LO+D.  ``scale = 2^sigma`` undoes the shift that
    keeps every m below 2^14.  None when the values do not fit f16."""
    rec = np.asarray(records, dtype=np.float64)
    if rec.ndim != 3 or rec.shape[2] != 2:
        raise ValueError("records must be [T/2, D+1, 2]")
    D = rec.shape[1] - 1
    if not 1 <= D <= GPM_MAX_D:
        return None
    pts, sgn = mfma_point_order(rec, n_pos_pairs)
    L, B = pts[:, 0], pts[:, 1:]
    lam = np.asarray(lam, dtype=np.float64)[:D]
    # log2 m = L' + c + B.x <= L' + max_x (c + B.x) = L' + 1/2 sum_d B_d^2 / (log2e lambda_d)
    with np.errstate(divide="ignore", invalid="ignore"):
        q = np.where(lam[None, :] > 0, B * B / (LOG2E * lam[None, :]), 0.0)
    bound = L + 0.5 * q.sum(1)
    sigma = float(np.ceil(bound.max()) - GPM_M_LOG2) if bound.size else 0.0
    Ls = L - sigma
    if B.size and (np.abs(B).max() > _F16_SAFE or np.abs(Ls).max() > _F16_SAFE):
        return None
    T = pts.shape[0]
    nch = max(1, -(-T // 32))
    Tpad = 32 * nch
    NK = gpm_k_steps(D)
    Bh, Bl = _split16(B)
    Lh = Ls.astype(np.float16)
    Ll = Ls - Lh.astype(np.float64)                           # folded into the sums operand
    kexp = np.zeros((Tpad, 16 * NK), dtype=np.float16)        # exponent A rows (pad rows 0: m = 2^c, A = 0)
    kexp[:T, 0:D], kexp[:T, D:2 * D], kexp[:T, 2 * D:3 * D] = Bh, Bl, Bh
    kexp[:T, 3 * D] = Lh
    kexp[:T, 3 * D + 1] = 1.0
    A = np.zeros((D + 1, Tpad))
    A[0, :T] = sgn
    A[1:, :T] = (sgn[:, None] * B).T
    A[:, :T] *= np.exp2(Ll)[None, :]
    Ah, Al = _split16(A)
    NR = gpm_sum_rows(D)
    lane = np.arange(64)
    j = np.arange(8)
    sp = _sum_points()                                        # [q, h, j]
    out = np.zeros((nch, gpm_frags_per_chunk(D), 8), dtype=np.float16)
    for ch in range(nch):
        for kk in range(NK):
            out[ch, 64 * kk:64 * (kk + 1)] = kexp[ch * 32 + (lane & 31)[:, None],
                                                  16 * kk + 8 * (lane >> 5)[:, None] + j]
        base = 64 * NK
        for qq in range(2):
            for hh in range(2):
                pt = ch * 32 + sp[qq, hh]                     # [8]
                o = base + (2 * qq + hh) * NR
                out[ch, o:o + D + 1] = Ah[:, pt]
                out[ch, o + D + 1:o + NR] = Al[:, pt]
    return out, nch, float(2.0 ** sigma)


def mfma_emulate(table, n_chunks: int, scale: float, D: int, xi, c):
    """NumPy model of ``gp_mfma_sums`` read straight from the fragment table:
    ``S [n, D+1]`` (S0, S'_d, scaled) for centred inputs ``xi [n, D]`` and
    exponent constants ``c [n]``; f16 operand splits, exact products, float64
    sums (the device accumulates in f32 and rounds hi toward zero)."""
    xi = np.asarray(xi, dtype=np.float64)
    c = np.asarray(c, dtype=np.float64)
    NK, NR = gpm_k_steps(D), gpm_sum_rows(D)
    tab = np.asarray(table, dtype=np.float16).reshape(n_chunks, gpm_frags_per_chunk(D), 8).astype(np.float64)
    xh, xl = _split16(xi)
    ch_ = np.maximum(c, -6.0e4).astype(np.float16).astype(np.float64)
    cl_ = c - ch_
    xs = np.zeros((xi.shape[0], 16 * NK))
    xs[:, 0:D], xs[:, D:2 * D], xs[:, 2 * D:3 * D] = xh, xh, xl
    xs[:, 3 * D] = 1.0
    xs[:, 3 * D + 1] = ch_
    lane = np.arange(64)
    j = np.arange(8)
    sp = _sum_points()
    S = np.zeros((xi.shape[0], D + 1))
    for ch in range(n_chunks):
        kexp = np.zeros((32, 16 * NK))
        for kk in range(NK):
            kexp[(lane & 31)[:, None], 16 * kk + 8 * (lane >> 5)[:, None] + j] = tab[ch, 64 * kk:64 * (kk + 1)]
        e = (xs @ kexp.T).astype(np.float32)                   # [n, 32 points]
        A = np.zeros((2, D + 1, 32))
        base = 64 * NK
        for qq in range(2):
            for hh in range(2):
                o = base + (2 * qq + hh) * NR
                A[0][:, sp[qq, hh]] = tab[ch, o:o + D + 1]
                A[1][:, sp[qq, hh]] = tab[ch, o + D + 1:o + NR]
        m = np.exp2(e).astype(np.float32)
        mh = m.astype(np.float16).astype(np.float64)
        ml = (m - mh).astype(np.float16).astype(np.float64)
        S += (mh + ml) @ (A[0] + A[1]).T
    return S * (scale * np.exp2(cl_))[:, None]


# --------------------------------------------------------------------------
# line tables (csrc/kf_gp_mfma.h line_pos / line_eval)
#
# The first Gauss-Newton iteration of a date is linearised at the forecast
# (linear_kf.py:253-262: x_prev = x_forecast).  Under a partial prior reset
# (kf_tools.py:propagate_information_filter_LAI, the prior-only "propagator")
# every parameter but the propagated one is the prior mean at every pixel, so
# each band's H0 and dH/dx at the forecast are functions of one scalar t =
# x_f,j.  The table holds those D + 1 functions as cubic Hermite pieces built
# from float64 values and t-derivatives at the nodes; it is refined until the
# midpoint error is below LINE_RTOL of the GP's term scale (sum |alpha_i k_i|),
# i.e. well inside the float32 accumulation error of the GP sums it replaces.

LINE_RTOL = 2e-8
LINE_MIN_INTERVALS = 256
LINE_MAX_INTERVALS = 8192


def _gp_terms(spec, X):
    """Per training point weights m [n, P] and input-gradient factors a [n, P, D]
    of one GP band at inputs X [n, D] (f = offset + sum m, df/dx_d = sum m a_d):
    from the float64 emulator when it exposes its parameters, else from the
    band's float32 records (the values the VALU kernel reads)."""
    em = getattr(spec, "emulator", None)
    lam = np.asarray(spec.coef, dtype=np.float64)[:X.shape[1]]
    if em is not None and all(hasattr(em, k) for k in ("inputs", "alpha", "lam", "signal", "mean")):
        diff = X[:, None, :] - np.asarray(em.inputs, dtype=np.float64)[None]          # [n, P, D]
        lam = np.asarray(em.lam, dtype=np.float64)
        k = em.signal * np.exp(-0.5 * np.einsum("npd,d->np", diff * diff, lam))
        return float(em.mean), k * np.asarray(em.alpha, dtype=np.float64)[None], -lam[None, None, :] * diff, lam
    rec = np.asarray(spec.records, dtype=np.float64)
    D = rec.shape[1] - 1
    pts = rec.transpose(0, 2, 1).reshape(-1, D + 1)
    sgn = np.where(np.arange(pts.shape[0]) < 2 * int(spec.gp_pos_pairs), 1.0, -1.0)
    keep = pts[:, 0] > -1e29
    L, B, sgn = pts[keep, 0], pts[keep, 1:], sgn[keep]
    xi = X - np.asarray(spec.center, dtype=np.float64)[None, :D]
    c = -0.5 * LOG2E * (xi * xi * lam[None]).sum(1)
    m = sgn[None] * np.exp2(L[None] + xi @ B.T + c[:, None])
    a = np.log(2.0) * B[None] - lam[None, None, :] * xi[:, None, :]
    return float(spec.offset), m, a, lam


def line_functions(spec, fixed, j: int, t):
    """Value and input gradient of GP band ``spec`` along the forecast line and
    their t-derivatives: ``F, dF [len(t), D+1]`` (column 0 = H0, 1 + d = dH/dx_d).
    Inputs read the state through ``spec.state_map``; state j is t, every other
    state its ``fixed`` value (j < 0: no input varies)."""
    smap = [int(v) for v in spec.state_map]
    D = len(smap)
    t = np.asarray(t, dtype=np.float64)
    e = np.array([1.0 if (j >= 0 and s == j) else 0.0 for s in smap])
    X = np.empty((t.size, D))
    for d, s in enumerate(smap):
        X[:, d] = t if e[d] else float(fixed[s])
    off, m, a, lam = _gp_terms(spec, X)
    z = a @ e                                                  # [n, P]: d(log m)/dt
    S0 = m.sum(1)
    F = np.empty((t.size, D + 1))
    dF = np.empty_like(F)
    F[:, 0] = off + S0
    F[:, 1:] = np.einsum("np,npd->nd", m, a)
    dF[:, 0] = (m * z).sum(1)
    dF[:, 1:] = np.einsum("np,npd->nd", m * z, a) - (lam * e)[None, :] * S0[:, None]
    return F, dF, np.abs(m).sum(1)


def line_range(specs, j: int, margin: float = 0.5):
    """Table range of t = x_j: the training boxes of the inputs reading state j
    (OperatorSpec.domain_lo/hi, centred) widened by ``margin`` of their width
    per side; None when no band reads j or a box is unknown."""
    lo, hi = np.inf, -np.inf
    for sp in specs:
        for d, s in enumerate(sp.state_map):
            if int(s) != j:
                continue
            if sp.domain_lo is None or sp.domain_hi is None:
                return None
            a = float(sp.domain_lo[d]) + float(sp.center[d])
            b = float(sp.domain_hi[d]) + float(sp.center[d])
            lo, hi = min(lo, a), max(hi, b)
    if not np.isfinite(lo) or not hi > lo:
        return None
    w = hi - lo
    return lo - margin * w, hi + margin * w


def line_table(specs, fixed, j: int):
    """Cubic Hermite line tables of every band of ``specs`` (all GP with the same
    input count D) for the kernels' first iteration at a partial-reset forecast:
    ``(coef float32 [n, n_bands, D+1, 4], t0, inv_h, n)`` with coefficients of
    s = (t - t_k) * inv_h in [0, 1] (c0 + s c1 + s^2 c2 + s^3 c3), or None
    (no range, or the refinement limit reached).  ``fixed``: the forecast's
    state for the reset parameters (the kernel's float32 reset mean)."""
    if not specs:
        return None
    D = len(specs[0].state_map)
    if j < 0:
        # no propagated parameter: one constant point, one interval from t0 = 0
        cols = [line_functions(sp, fixed, -1, np.zeros(1))[0][0] for sp in specs]
        out = np.zeros((1, len(specs), D + 1, 4))
        out[0, :, :, 0] = np.stack(cols)
        return out.astype(np.float32), 0.0, 1.0, 1
    rng = line_range(specs, j)
    if rng is None:
        return None
    # t0 and the spacing (a power of two) exact in float32: the kernel's
    # u = (t - t0) * inv_h then only rounds t - t0
    t0 = float(np.float32(rng[0]))
    t1 = rng[1]
    h = 2.0 ** np.floor(np.log2((t1 - t0) / LINE_MIN_INTERVALS))
    while True:
        n = int(np.ceil((t1 - t0) / h))
        if n > LINE_MAX_INTERVALS:
            return None
        nodes = t0 + h * np.arange(n + 1)
        mids = nodes[:-1] + 0.5 * h
        coef = np.empty((n, len(specs), D + 1, 4))
        worst = 0.0
        for b, sp in enumerate(specs):
            F, dF, _ = line_functions(sp, fixed, j, nodes)
            y0, y1, d0, d1 = F[:-1], F[1:], h * dF[:-1], h * dF[1:]
            c = coef[:, b]
            c[..., 0], c[..., 1] = y0, d0
            c[..., 2] = 3.0 * (y1 - y0) - 2.0 * d0 - d1
            c[..., 3] = 2.0 * (y0 - y1) + d0 + d1
            Fm, _, scale = line_functions(sp, fixed, j, mids)
            pm = c[..., 0] + 0.5 * c[..., 1] + 0.25 * c[..., 2] + 0.125 * c[..., 3]
            worst = max(worst, float((np.abs(pm - Fm) / np.maximum(scale, 1e-300)[:, None]).max()))
        if worst <= LINE_RTOL:
            return coef.astype(np.float32), t0, float(1.0 / h), n
        h *= 0.5


# --------------------------------------------------------------------------
# synthetic targets ("random-init" physics stand-ins)

def tip_bhr_target(band: int):
    """Two-stream-like broadband albedo of (omega, asym, TLAI, soil) — the input
    order of the JRC-TIP band mapper ``[0,1,6,2]``/``[3,4,6,5]``
    (kafka/inference/utils.py:148-153)."""
    def f(X):
        w, d, t, s = X[:, 0], X[:, 1], np.clip(X[:, 2], 0.0, 1.0), X[:, 3]
        canopy = w * (1.0 - t) * (0.45 + 0.08 * np.tanh(d - 1.0)) / (1.0 - 0.3 * w * (1.0 - t))
        return canopy + s * t * t + (0.01 if band == 0 else 0.03)
    return f


def prosail_target(band: int, n_params: int = 10, hard: bool = False):
    """Smooth reflectance-like function of the 10 transformed PROSAIL parameters.
    ``hard``: a canopy/soil mixture with Beer-law gap fraction and leaf-optics
    saturation — curved enough that Gauss-Newton takes several iterations per
    date, as the reference's real PROSAIL emulators do (6)."""
    rng = np.random.default_rng(1000 + band)
    w = rng.normal(0, 0.08, n_params)
    b = rng.uniform(0.5, 2.0, n_params)
    if hard:
        from .priors import sail_prior
        wh = rng.normal(0, 1.2, n_params)
        ctr = sail_prior()[0][:n_params]

        def fh(X):
            lai_t = np.clip(X[:, 6], 0.0, 1.0)                      # exp(-LAI/2)
            gap = lai_t ** (1.5 + 0.25 * (band % 4))               # view/sun path gap fraction
            leaf = 0.05 + 0.45 / (1.0 + np.exp(-(X - ctr) @ wh))   # saturating leaf optics
            soil = 0.08 + 0.25 * np.clip(X[:, min(8, X.shape[1] - 1)], 0.0, 1.5) ** 2
            return leaf * (1.0 - gap) + soil * gap
        return fh

    def f(X):
        lai_t = np.clip(X[:, 6], 0.0, 1.0)  # exp(-LAI/2)
        soil = 0.1 + 0.1 * X[:, min(8, X.shape[1] - 1)]
        base = 0.05 + 0.02 * band + np.tanh(X @ (w * b)) * 0.05
        return base * (1.0 - lai_t) + soil * lai_t + 0.02 * np.sin(X[:, 1] * (1 + band % 3))
    return f


TIP_RANGES = {
    0: (np.array([0.0, 0.0, 0.0, 0.0]), np.array([0.6, 3.5, 1.0, 0.5])),
    1: (np.array([0.2, 0.0, 0.0, 0.0]), np.array([1.0, 6.5, 1.0, 0.8])),
}


def make_tip_emulators(n_train: int = 500, seed: int = 0, noise: float = 1e-3):
    """Two JRC-TIP band emulators (VIS, NIR), 4 inputs each.  ``noise``: the
    nugget (1e-5: near-interpolating weights that cancel, |alpha| >> |f|)."""
    ems = []
    for band in (0, 1):
        lo, hi = TIP_RANGES[band]
        ems.append(GaussianProcessEmulator.synthetic(tip_bhr_target(band), lo, hi, n_train, seed + band,
                                                     noise=noise, name=f"tip_{'vis' if band == 0 else 'nir'}"))
    return ems


def make_prosail_emulators(n_bands: int = 10, n_train: int = 250, seed: int = 0, n_params: int = 10,
                           hard: bool = False, noise: float = 1e-3):
    """Per-band PROSAIL-like emulators over the 10 transformed parameters
    (``hard``: the strongly non-linear targets of :func:`prosail_target`)."""
    from .priors import sail_prior

    mean, covar, _ = sail_prior()
    sig = np.sqrt(np.diag(covar))
    lo = mean - 3 * np.maximum(sig, 0.05)
    hi = mean + 3 * np.maximum(sig, 0.05)
    # every band's records around the SAIL prior mean (the centre of the design
    # box): the bands share their centred inputs (BAND_LAYOUT_SHARED_X)
    return [GaussianProcessEmulator.synthetic(prosail_target(b, n_params, hard), lo[:n_params], hi[:n_params],
                                              n_train, seed + b, noise=noise,
                                              name=f"prosail_b{b}{'h' if hard else ''}")
            .set_center(mean[:n_params]) for b in range(n_bands)]
