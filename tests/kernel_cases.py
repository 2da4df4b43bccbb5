"""Random problem instances shared by the host-runner and GPU kernel tests."""
from __future__ import annotations

import numpy as np
import torch

import kafka_inferenceengine_amd as k
from kafka_inferenceengine_amd.engine.bands import DeviceBand, RecordCache, build_table, operator_table
from kafka_inferenceengine_amd.ops import kernels as K
from kafka_inferenceengine_amd.utils.blocks import pack_blocks


def spd_blocks(rng, N, n, scale=10.0):
    A = rng.normal(size=(N, n, n))
    return np.einsum("nij,nkj->nik", A, A) + scale * np.eye(n)[None]


def tip_problem(N=3000, seed=0, n_train=64, dn16=False, mask_frac=0.2):
    """7-param TIP state, 2 GP bands; returns numpy inputs + descriptors factory."""
    rng = np.random.default_rng(seed)
    ems = k.make_tip_emulators(n_train=n_train, seed=seed)
    mu, P, Pi = k.tip_prior()
    x = mu[None, :] + rng.normal(size=(N, 7)) * np.sqrt(np.diag(P)) * 0.3
    x[:, 6] = np.clip(x[:, 6], 0.05, 0.95)
    xf = mu[None, :] + rng.normal(size=(N, 7)) * 0.01
    Pf = np.broadcast_to(Pi, (N, 7, 7)) + 0.0
    specs = [k.gp_spec(ems[b], k.TIP_BAND_MAPPER[b]) for b in range(2)]
    bands_np = []
    raw = []
    for b in range(2):
        H, _ = ems[b].predict(x[:, k.TIP_BAND_MAPPER[b]])
        y = np.clip(H + rng.normal(size=N) * 0.01, 0.01, 1.0)
        valid = rng.random(N) > mask_frac
        if dn16:
            dn = np.where(valid, np.clip(np.round(y / 1e-4), 1, 65535), 0).astype(np.int32)
            yy = dn * 1e-4
            sig = np.maximum(0.05 * yy, 2.5e-3)
            w = np.where(dn > 0, 1 / sig ** 2, 0.0)
            raw.append(dict(dn=np.where(dn > 32767, dn - 65536, dn).astype(np.int16)))
            yv = np.where(dn > 0, yy, 0.0)
        else:
            w = np.where(valid, 1 / 0.01 ** 2, 0.0)
            raw.append(dict(y=y.astype(np.float32), w=w.astype(np.float32)))
            yv = y
        bands_np.append((yv, w))
    return dict(x=x, xf=xf, Pf=Pf, specs=specs, ems=ems, bands=bands_np, raw=raw, dn16=dn16, N=N, n=7)


def device_bands(prob, device):
    obs = []
    for r in prob["raw"]:
        if prob["dn16"]:
            obs.append(DeviceBand(K.OBS_DN16, dn=torch.from_numpy(r["dn"]).to(device), scale=1e-4, rel_unc=0.05,
                                  unc_floor=2.5e-3))
        else:
            obs.append(DeviceBand(K.OBS_F32, y=torch.from_numpy(r["y"]).to(device),
                                  w=torch.from_numpy(r["w"]).to(device)))
    return obs


def table(prob, device, h0_outs=None):
    return build_table(prob["specs"], device_bands(prob, device), prob["n"], RecordCache(), device, h0_outs)


def soa(a, device):
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a).T, dtype=np.float32)).to(device)


def packed(blocks, device):
    return torch.from_numpy(np.ascontiguousarray(pack_blocks(blocks), dtype=np.float32)).to(device)


def oracle_bands(prob, x_lin):
    out = []
    for b, (y, w) in enumerate(prob["bands"]):
        mp = k.TIP_BAND_MAPPER[b]
        H, dH = prob["ems"][b].predict(x_lin[:, mp])
        h = np.zeros((prob["N"], prob["n"]))
        h[:, mp] = dH
        out.append((H, h, y, w))
    return out


def fused_vs_materialized(device, mode, blend=False, quirk=False, prop_mask=0, N=2000, seed=3):
    """Analysis with the propagation fused into the kernel vs propagate pass +
    analysis; both linearise at the forecast (first Gauss-Newton iteration) and
    then at a perturbed point.  Returns the two (x, A, status) results."""
    from kafka_inferenceengine_amd.utils.blocks import pack_matrix
    prob = tip_problem(N=N, seed=seed)
    rng = np.random.default_rng(seed)
    n = prob["n"]
    mu, _, Pi = k.tip_prior()
    A = spd_blocks(rng, N, n, 5.0) * 0.2 + prob["Pf"]
    spec = {"mode": mode, "m": np.ones(n), "q": rng.uniform(0.01, 0.1, n), "prop_mask": prop_mask,
            "reset_mean": mu, "reset_cinv": pack_matrix(Pi), "blend": blend, "quirk_blend": quirk,
            "blend_mean": mu * 1.05, "blend_cinv": pack_matrix(Pi * 0.5)}
    xa, pa = soa(prob["x"], device), packed(A, device)
    tab = table(prob, device)
    nt = n * (n + 1) // 2
    res = []
    for fused in (False, True):
        out = []
        x_lin = None
        for it in range(2):
            xo = torch.zeros((n, N), device=device)
            ao = torch.zeros((nt, N), device=device)
            st = torch.zeros(N, dtype=torch.uint8, device=device)
            if fused:
                h = K.prop_args(n, spec, xa, pa, fused=True)
                K.analysis(n, tab, x_lin, None, None, xo, ao, None, st, None, prop=h)
            else:
                xf = torch.zeros((n, N), device=device)
                pf = torch.zeros((nt, N), device=device)
                K.propagate(n, spec, xa, pa, xf, pf)
                K.analysis(n, tab, xf if x_lin is None else x_lin, xf, pf, xo, ao, None, st, None)
            out.append((xo.cpu().numpy(), ao.cpu().numpy(), st.cpu().numpy()))
            x_lin = soa(prob["x"] * 0.5 + 0.5 * xo.cpu().numpy().T, device)
        res.append(out)
    return res


FUSED_CASES = [(1, False, False, 1 << 6), (1, False, False, 0b1010011), (0, False, False, 0),
               (2, False, False, 0)]


def tiled_vs_sequential(device, h=150, w=300, omegas=(1.0, 1.3, 1.2, 1.25, 1.22), cheb=None, n=7, j0=2, seed=5):
    """K9 temporal blocking (reg_sweeps_tiled) against one reg_sweep launch per
    sweep on a dense strip without halo rows.  Returns ((z, zp) tiled, (z, zp)
    sequential) as CPU tensors."""
    rng = np.random.default_rng(seed)
    N = h * w
    ld = N + 64
    geo = {"w": w, "h": h, "halo": 0, "n_up": 0}
    cheb = [s > 0 for s in range(len(omegas))] if cheb is None else list(cheb)
    u = torch.tensor(rng.normal(size=(n, ld)), dtype=torch.float32, device=device)
    v = torch.tensor(rng.uniform(0.0, 0.2, size=(n, ld)), dtype=torch.float32, device=device)
    z0 = torch.tensor(rng.normal(size=(1, ld)), dtype=torch.float32, device=device)
    zm1 = torch.tensor(rng.normal(size=(1, ld)), dtype=torch.float32, device=device)
    gamma, mask = 0.9, 1 << j0
    zo, zpo = (torch.zeros(1, ld, device=device) for _ in range(2))
    K.reg_sweeps_tiled(n, u, v, z0, zm1, zo, zpo, gamma, mask, N, geo, list(omegas), cheb)
    cur, prev = z0.clone(), zm1.clone()
    for om, c in zip(omegas, cheb):
        nxt = torch.zeros(1, ld, device=device)
        K.reg_sweep(n, u, v, cur, None, nxt, gamma, mask, N, geo=geo, z_prev=prev if c else None, omega=om)
        prev, cur = cur, nxt
    return (zo[:, :N].cpu(), zpo[:, :N].cpu()), (cur[:, :N].cpu(), prev[:, :N].cpu())


def deep_halo_vs_full(device, h_total=200, w=150, r0=70, r1=150, depth=8, omegas=(1.0, 1.3, 1.2, 1.25, 1.22, 1.21),
                      cheb=None, device_sched=False, split=False, n=7, j0=6, seed=11, rho=None):
    """K9 deep halo: a tiled pass over strip rows [r0, r1) of a dense raster,
    with `depth` rows of u, v, z, zp of each neighbour in halo planes (as the
    engine receives them), against the same pass over the whole raster (no
    halo).  ``device_sched``: the weights come from a RegSchedule (``rho``) and
    the pass from its table; ``split``: boundary tile rows, then the interior
    (the C2 overlap order).  Returns ((z, zp) strip, (z, zp) full rows r0..r1)."""
    rng = np.random.default_rng(seed)
    Nf = h_total * w
    ld = Nf + 32
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=device)  # noqa: E731
    u = t(rng.normal(size=(n, ld)))
    v = t(rng.uniform(0.0, 0.2, size=(n, ld)))
    z0 = t(rng.normal(size=(1, ld)))
    zm1 = t(rng.normal(size=(1, ld)))
    gamma, mask = 0.9, 1 << j0
    kw_host = {}
    if device_sched:
        rs = K.RegSchedule(Nf, 32, device)
        rs.rho.fill_(0.8 if rho is None else rho)
        rs.schedule(1e-3)
        kw = dict(sched=(rs.sched, rs.omega), s_base=1, nsweep=len(omegas))
        kw_host = kw
    else:
        cheb = [s > 0 for s in range(len(omegas))] if cheb is None else list(cheb)
        kw = dict(omegas=list(omegas), chebyshev=cheb)
        kw_host = kw
    geo_full = {"w": w, "h": h_total, "halo": 0, "n_up": 0}
    zo, zpo = (torch.zeros(1, ld, device=device) for _ in range(2))
    K.reg_sweeps_tiled(n, u, v, z0, zm1, zo, zpo, gamma, mask, Nf, geo_full, **kw_host)
    # the strip's own arrays and its neighbours' rows
    h = r1 - r0
    N = h * w
    lds = N + 16

    def rows_of(a, ra, rb):
        return a[..., ra * w:rb * w]
    us = torch.zeros(n, lds, device=device)
    vs = torch.zeros(n, lds, device=device)
    us[:, :N] = rows_of(u, r0, r1)
    vs[:, :N] = rows_of(v, r0, r1)
    zs = torch.zeros(1, lds, device=device)
    zps = torch.zeros(1, lds, device=device)
    zs[:, :N] = rows_of(z0, r0, r1)
    zps[:, :N] = rows_of(zm1, r0, r1)
    hu = depth if r0 > 0 else 0
    hd = depth if r1 < h_total else 0
    up = dn = None
    if hu:
        up = torch.stack([rows_of(f[j], r0 - hu, r0) for f, j in ((u, j0), (v, j0), (z0, 0), (zm1, 0))]).contiguous()
    if hd:
        dn = torch.stack([rows_of(f[j], r1, r1 + hd) for f, j in ((u, j0), (v, j0), (z0, 0), (zm1, 0))]).contiguous()
    geo = {"w": w, "h": h, "halo": (1 if hu else 0) | (2 if hd else 0), "n_up": w if hu else 0}
    so, spo = (torch.zeros(1, lds, device=device) for _ in range(2))
    halo = (hu, hd, up, dn)
    if split:
        T = K.reg_tile_rows(h)
        a, b = K.reg_boundary_tile_rows(h, depth, hu > 0, hd > 0)
        for tr in ((0, a), (b, T), (a, b)):
            K.reg_sweeps_tiled(n, us, vs, zs, zps, so, spo, gamma, mask, N, geo, halo=halo, tile_rows=tr, **kw)
    else:
        K.reg_sweeps_tiled(n, us, vs, zs, zps, so, spo, gamma, mask, N, geo, halo=halo, **kw)
    return ((so[:, :N].cpu(), spo[:, :N].cpu()), (rows_of(zo, r0, r1).cpu(), rows_of(zpo, r0, r1).cpu()))


def dense_finish(device, h_total=30, w=44, ranks=3, rank=1, n=7, j0=6, out=True, seed=9):
    """reg_finish on a dense strip of a ``ranks``-strip partition (halo rows
    above/below) with the output dump; returns (x_out, mean, unc) on the CPU.
    On the device with w % 4 == 0 this takes the 16-byte path (FINISH4)."""
    from kafka_inferenceengine_amd.parallel import StripPartition
    rng = np.random.default_rng(seed)
    part = StripPartition(np.ones((h_total, w), bool), rank, ranks)
    geo = part.dense_geometry()
    N = part.N
    lay = part.halo_layout()
    cols = N + lay["n_up"] + lay["n_down"]
    ld = N + 12
    mk = lambda r, c, lo=-1.0, hi=1.0: torch.tensor(rng.uniform(lo, hi, size=(r, c)), dtype=torch.float32,
                                                   device=device)
    u, v, xr = mk(n, ld), mk(n, ld, 0.0, 0.2), mk(n, ld)
    z = mk(1, cols)
    a_prec = mk(n * (n + 1) // 2, ld, 0.5, 4.0)
    xo = torch.zeros(n, ld, device=device)
    part_buf = torch.zeros(4096, dtype=torch.float64, device=device)
    mean = torch.zeros(n, N, device=device)
    unc = torch.zeros(n, N, device=device)
    # out="mean": the mean only (the analysis wrote the uncertainty raster)
    K.reg_finish(n, u, v, z, None, xr, xo, 0.8, 1 << j0, N, partials=part_buf, geo=geo,
                 out=(mean, None if out == "mean" else unc, None) if out else None,
                 a_prec=a_prec if out is True else None)
    return xo[:, :N].cpu(), mean.cpu(), unc.cpu(), float(part_buf.sum())
