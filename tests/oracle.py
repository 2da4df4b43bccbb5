"""Float64 NumPy oracle of the reference run loop (kafka/linear_kf.py:171-307).

Independent of the kernels: it drives the reference-API functions of this
package (sparse matrices, operator factories, ``variational_kalman_multiband``,
``propagate_and_blend_prior``) exactly the way ``LinearKalman.run`` of the
reference does, so engine results can be checked against it.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

from kafka_inferenceengine_amd.inference import (iterate_time_grid, propagate_and_blend_prior,
                                                 variational_kalman_multiband)


def oracle_run(obs, state_mask, factory, n_params, time_grid, x0, Pinv0, propagator=None, prior=None, Q=None,
               tol=1e-3, min_iterations=2, max_iterations=25, on_step=None):
    """``on_step(timestep, x_a, P_a^-1)``: called after every time-grid step
    (the state the engine's output writer sees, linear_kf.py:211-212)."""
    state_mask = np.asarray(state_mask).astype(bool)
    N = int(state_mask.sum())
    M = sp.eye(n_params * N, format="csr")
    Qm = sp.diags(np.zeros(n_params * N) if Q is None else np.asarray(Q, dtype=np.float64)).tocsr()
    x_f, Pi_f = np.asarray(x0, dtype=np.float64), Pinv0
    x_a, Pi_a = None, None
    iters = []
    for timestep, locate, is_first in iterate_time_grid(time_grid, obs.dates):
        if not is_first:
            x_f, _, Pi_f = propagate_and_blend_prior(x_a, None, Pi_a, M, Qm, prior=prior,
                                                     state_propagator=propagator, date=timestep)
        if len(locate) == 0:
            x_a, Pi_a = x_f, Pi_f
            if on_step is not None:
                on_step(timestep, x_a, Pi_a)
            continue
        for date in locate:
            data = [obs.get_band_data(date, b) for b in range(obs.bands_per_observation[date])]
            x_prev = x_f * 1.0
            n_iter = 1
            while True:
                H = [factory(n_params, d.emulator, d.metadata, d.mask, state_mask, x_prev, b)
                     for b, d in enumerate(data)]
                xa, _, A, _, _ = variational_kalman_multiband([d.observations for d in data], [d.mask for d in data],
                                                              state_mask, [d.uncertainty for d in data], H, n_params,
                                                              x_prev, x_f, None, Pi_f, None)
                norm = np.linalg.norm(xa - x_prev) / float(len(xa))
                x_prev = xa
                if norm < tol and n_iter >= min_iterations:
                    break
                if n_iter > max_iterations:
                    break
                n_iter += 1
            iters.append(n_iter)
            x_f, Pi_f = xa, A
        x_a, Pi_a = x_f, Pi_f
        if on_step is not None:
            on_step(timestep, x_a, Pi_a)
    return x_a, Pi_a, iters


def gp_predict64(em, X, chunk=16384):
    """float64 RBF GP value and gradient through GEMMs (an implementation
    independent of the emulator's ``predict``): with centred inputs, d2 =
    |x|^2_lam + |t|^2_lam - 2 x lam t^T, k = s exp(-d2 / 2), f = mean + k alpha,
    df/dx_d = -lam_d (x_d (k alpha) - k (alpha t_d))."""
    X = np.atleast_2d(np.asarray(X, dtype=np.float64))
    T = np.asarray(em.inputs, dtype=np.float64)
    c = T.mean(0)
    Tc = T - c
    lam = np.asarray(em.lam, dtype=np.float64)
    alpha = np.asarray(em.alpha, dtype=np.float64)
    tt = np.einsum("td,td,d->t", Tc, Tc, lam)
    B = np.concatenate([alpha[:, None], alpha[:, None] * Tc], axis=1)       # [T, 1 + D]
    H = np.empty(X.shape[0])
    dH = np.empty_like(X)
    for s in range(0, X.shape[0], chunk):
        Xc = X[s:s + chunk] - c
        xx = np.einsum("nd,nd,d->n", Xc, Xc, lam)
        d2 = xx[:, None] + tt[None, :] - 2.0 * (Xc * lam[None, :]) @ Tc.T
        k = em.signal * np.exp(-0.5 * np.maximum(d2, 0.0))
        S = k @ B
        H[s:s + chunk] = em.mean + S[:, 0]
        dH[s:s + chunk] = -lam[None, :] * (Xc * S[:, :1] - S[:, 1:])
    return H, dH


def oracle_run_blocks(obs, state_mask, maps, time_grid, prior_mean, prior_cinv, propagated=(6,), q=None,
                      tol=1e-3, min_iterations=2, max_iterations=25, on_step=None, x0=None, A0=None):
    """The same run loop with every matrix held as its per-pixel n x n blocks,
    all in float64 (no float32 cast of the normal equations): the GP value and
    gradient from :func:`gp_predict64` on each band's input subset ``maps[b]``,
    ``analysis_blocks`` for the analysis and the partial prior-reset
    propagation of ``propagate_information_filter_LAI`` (kf_tools.py:292-314:
    every parameter back to the prior except ``propagated``, whose precision
    is inflated by q).  Fast enough for 256^2 tiles; checked against
    :func:`oracle_run` on small tiles (tests/test_mvp.py).

    Returns (x [N, n], A [N, n, n], iters); ``on_step(timestep, x, A)``."""
    from kafka_inferenceengine_amd.inference import analysis_blocks

    sm = np.asarray(state_mask).astype(bool)
    N = int(sm.sum())
    mu = np.asarray(prior_mean, dtype=np.float64)
    ci = np.asarray(prior_cinv, dtype=np.float64)
    n = mu.size
    q = np.zeros(n) if q is None else np.asarray(q, dtype=np.float64)
    # initial state: the given per-pixel constants (x0 [n], A0 [n, n]), else the prior
    x_f = np.broadcast_to(mu if x0 is None else np.asarray(x0, np.float64), (N, n)).copy()
    A_f = np.broadcast_to(ci if A0 is None else np.asarray(A0, np.float64), (N, n, n)).copy()
    x_a, A_a = None, None
    iters = []
    for timestep, locate, is_first in iterate_time_grid(time_grid, obs.dates):
        if not is_first:
            x_f = np.broadcast_to(mu, (N, n)).copy()
            A_f = np.broadcast_to(ci, (N, n, n)).copy()
            for kk in propagated:
                x_f[:, kk] = x_a[:, kk]
                A_f[:, kk, kk] = 1.0 / (1.0 / A_a[:, kk, kk] + q[kk])
        if len(locate) == 0:
            x_a, A_a = x_f, A_f
            if on_step is not None:
                on_step(timestep, x_a, A_a)
            continue
        for date in locate:
            data = [obs.get_band_data(date, b) for b in range(obs.bands_per_observation[date])]
            raw = []
            for d in data:
                m = np.asarray(d.mask)[sm]
                w = np.asarray(d.uncertainty.diagonal())[sm.ravel()] if sp.issparse(d.uncertainty) else \
                    np.asarray(d.uncertainty)[sm]
                w = np.where(m & np.isfinite(w), w, 0.0)
                raw.append((np.where(m, np.asarray(d.observations)[sm], 0.0), w, d.emulator))
            x_prev = x_f.copy()
            n_iter = 1
            while True:
                bands = []
                for b, (y, w, em) in enumerate(raw):
                    H0, dH = gp_predict64(em, x_prev[:, maps[b]])
                    h = np.zeros((N, n))
                    h[:, maps[b]] = dH
                    bands.append((H0, h, y, w))
                xa, A = analysis_blocks(x_prev, x_f, A_f, bands)
                norm = np.linalg.norm((xa - x_prev).ravel()) / float(N * n)
                x_prev = xa
                if norm < tol and n_iter >= min_iterations:
                    break
                if n_iter > max_iterations:
                    break
                n_iter += 1
            iters.append(n_iter)
            x_f, A_f = xa, A
        x_a, A_a = x_f, A_f
        if on_step is not None:
            on_step(timestep, x_a, A_a)
    return x_a, A_a, iters


def gp_predict64_torch(em, X, chunk=65536, f32=()):
    """gp_predict64 in float64 torch on X's device (the 1024^2 slice: ~10^9
    kernel evaluations per band and iteration, minutes in NumPy).  ``f32``:
    parts evaluated in float32 instead, to locate a float32 pipeline's loss
    ("exponent": the squared distances; "sums": the kernel-weighted sums)."""
    import torch

    dev = X.device
    T = torch.as_tensor(np.asarray(em.inputs, dtype=np.float64), device=dev)
    c = T.mean(0)
    Tc = T - c
    lam = torch.as_tensor(np.asarray(em.lam, dtype=np.float64), device=dev)
    alpha = torch.as_tensor(np.asarray(em.alpha, dtype=np.float64), device=dev)
    tt = (Tc * Tc * lam).sum(1)
    B = torch.cat([alpha[:, None], alpha[:, None] * Tc], 1)
    H = torch.empty(X.shape[0], dtype=torch.float64, device=dev)
    dH = torch.empty_like(X)
    for s in range(0, X.shape[0], chunk):
        Xc = X[s:s + chunk] - c
        xx = (Xc * Xc * lam).sum(1)
        if "exponent" in f32:
            Xf, Tf, lf = Xc.float(), Tc.float(), lam.float()
            d2 = ((Xf * Xf * lf).sum(1)[:, None] + (Tf * Tf * lf).sum(1)[None, :] - 2.0 * (Xf * lf) @ Tf.T).double()
        else:
            d2 = xx[:, None] + tt[None, :] - 2.0 * (Xc * lam) @ Tc.T
        k = em.signal * torch.exp(-0.5 * torch.clamp(d2, min=0.0))
        S = (k.float() @ B.float()).double() if "sums" in f32 else k @ B
        H[s:s + chunk] = em.mean + S[:, 0]
        dH[s:s + chunk] = -lam * (Xc * S[:, :1] - S[:, 1:])
    return H, dH


def oracle_run_blocks_torch(obs, state_mask, maps, time_grid, prior_mean, prior_cinv, propagated=(6,), q=None,
                            tol=1e-3, min_iterations=2, max_iterations=25, x0=None, A0=None, device="cuda",
                            cast_f32=False, gp_f32=()):
    """:func:`oracle_run_blocks` in float64 torch on ``device`` (same loop, same
    per-pixel normal equations, solved by batched float64 Cholesky): the
    oracle of the 1024^2 slice.  Returns (x [N, n], A [N, n, n], iters) on the
    host.

    ``cast_f32``: the reference's one precision loss -- its solver casts the
    normal equations to float32 and solves in single precision
    (solvers.py:127-134); everything else stays float64.  ``gp_f32``: GP parts
    in float32 (:func:`gp_predict64_torch`)."""
    import torch

    dev = torch.device(device)
    sm = np.asarray(state_mask).astype(bool)
    N = int(sm.sum())
    f64 = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=dev)  # noqa: E731
    mu, ci = f64(prior_mean), f64(prior_cinv)
    n = mu.numel()
    qv = torch.zeros(n, dtype=torch.float64, device=dev) if q is None else f64(q)
    x_f = (mu if x0 is None else f64(x0)).expand(N, n).clone()
    A_f = (ci if A0 is None else f64(A0)).expand(N, n, n).clone()
    x_a = A_a = None
    iters = []
    for timestep, locate, is_first in iterate_time_grid(time_grid, obs.dates):
        if not is_first:
            x_f = mu.expand(N, n).clone()
            A_f = ci.expand(N, n, n).clone()
            for kk in propagated:
                x_f[:, kk] = x_a[:, kk]
                A_f[:, kk, kk] = 1.0 / (1.0 / A_a[:, kk, kk] + qv[kk])
        if len(locate) == 0:
            x_a, A_a = x_f, A_f
            continue
        for date in locate:
            raw = []
            for b in range(obs.bands_per_observation[date]):
                d = obs.get_band_data(date, b)
                m = np.asarray(d.mask)[sm]
                w = np.asarray(d.uncertainty.diagonal())[sm.ravel()] if sp.issparse(d.uncertainty) else \
                    np.asarray(d.uncertainty)[sm]
                w = np.where(m & np.isfinite(w) & (w > 0), w, 0.0)
                raw.append((f64(np.where(m, np.asarray(d.observations)[sm], 0.0)), f64(w), d.emulator))
            x_prev = x_f.clone()
            n_iter = 1
            while True:
                A = A_f.clone()
                rhs = torch.einsum("nij,nj->ni", A_f, x_f)
                for b, (y, w, em) in enumerate(raw):
                    H0, dH = gp_predict64_torch(em, x_prev[:, list(maps[b])].contiguous(), f32=gp_f32)
                    h = torch.zeros((N, n), dtype=torch.float64, device=dev)
                    h[:, list(maps[b])] = dH
                    yp = y + (h * x_prev).sum(1) - H0
                    A += w[:, None, None] * h[:, :, None] * h[:, None, :]
                    rhs += (w * yp)[:, None] * h
                if cast_f32:
                    A32, r32 = A.float(), rhs.float()
                    xa = torch.cholesky_solve(r32[..., None], torch.linalg.cholesky(A32))[..., 0].double()
                    A = A32.double()
                else:
                    xa = torch.cholesky_solve(rhs[..., None], torch.linalg.cholesky(A))[..., 0]
                norm = float(torch.linalg.norm((xa - x_prev).reshape(-1))) / float(N * n)
                x_prev = xa
                if norm < tol and n_iter >= min_iterations:
                    break
                if n_iter > max_iterations:
                    break
                n_iter += 1
            iters.append(n_iter)
            x_f, A_f = xa, A
        x_a, A_a = x_f, A_f
    return x_a.cpu().numpy(), A_a.cpu().numpy(), iters
