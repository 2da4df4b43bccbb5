// kf_host.cpp — CPU runner for the per-pixel kernels of kf_core.h.
// Compiled by g++ (-fopenmp); the math is byte-for-byte the source the
// gfx950 kernels run, so CPU CI exercises the kernel code paths.
#include <omp.h>
#include <math.h>
#include <string.h>
#include "kf_launch.h"
#include "kf_deflate.h"
#include <algorithm>
#include <vector>

namespace kf {

static constexpr int HBLOCK = 256;

#define KF_HOST_NP_SWITCH(np, FN, ...)   \
  switch (np) {                          \
    case 1: return FN<1>(__VA_ARGS__);   \
    case 2: return FN<2>(__VA_ARGS__);   \
    case 3: return FN<3>(__VA_ARGS__);   \
    case 4: return FN<4>(__VA_ARGS__);   \
    case 7: return FN<7>(__VA_ARGS__);   \
    case 10: return FN<10>(__VA_ARGS__); \
    default: return -1;                  \
  }

bool host_supported(int np) { return np == 1 || np == 2 || np == 3 || np == 4 || np == 7 || np == 10; }

// Block b handles pixels p = b*256 + t + k*grid*256 (same as the device).
template <typename F>
static void grid_stride(int64_t N, int grid, double* partials, F&& f) {
  const int64_t stride = (int64_t)grid * HBLOCK;
#pragma omp parallel for schedule(dynamic, 4)
  for (int b = 0; b < grid; ++b) {
    double acc = 0.0;
    for (int t = 0; t < HBLOCK; ++t)
      for (int64_t p = (int64_t)b * HBLOCK + t; p < N; p += stride) acc += (double)f(p);
    if (partials) partials[b] = acc;
  }
}

template <int NP>
static int h_analysis(const AnalysisArgs& a, int grid) {
  const int64_t stride = (int64_t)grid * HBLOCK;
  const int64_t nv = visit_count(a);
#pragma omp parallel for schedule(dynamic, 4)
  for (int b = 0; b < grid; ++b) {
    double acc = 0.0, acc1 = 0.0;
    for (int t = 0; t < HBLOCK; ++t)
      for (int64_t q = (int64_t)b * HBLOCK + t; q < nv; q += stride) {
        float dn1;
        const int64_t p = visit_px(a.order, q);
        const float dn = pixel_analysis<NP>(a, p, dn1);
        if (a.dn_out) a.dn_out[p] = dn;
        acc += (double)dn;
        acc1 += (double)dn1;
      }
    if (a.partials) a.partials[b] = acc;
    if (a.partials_first) a.partials_first[b] = acc1;
  }
  return 0;
}
template <int NP>
static int h_gain(const GainArgs& a, int grid) {
  const int64_t stride = (int64_t)grid * HBLOCK;
  const int64_t nv = visit_count(a);
#pragma omp parallel for schedule(dynamic, 4)
  for (int b = 0; b < grid; ++b) {
    double acc = 0.0, acc1 = 0.0;
    for (int t = 0; t < HBLOCK; ++t)
      for (int64_t q = (int64_t)b * HBLOCK + t; q < nv; q += stride) {
        float dn1;
        acc += (double)pixel_gain<NP>(a, visit_px(a.order, q), dn1);
        acc1 += (double)dn1;
      }
    if (a.partials) a.partials[b] = acc;
    if (a.partials_first) a.partials_first[b] = acc1;
  }
  return 0;
}
template <int NP>
static int h_jacobi(const JacobiArgs& a, int grid) {
  grid_stride(a.pn > 0 ? a.pn : a.N, grid, a.partials, [&](int64_t i) { return pixel_jacobi<NP>(a, a.p0 + i); });
  return 0;
}
template <int NP>
static int h_propagate(const PropArgs& a) {
#pragma omp parallel for schedule(static)
  for (int64_t p = 0; p < a.N; ++p) pixel_propagate<NP>(a, p);
  return 0;
}
template <int NP>
static int h_invert(const float* src, float* dst, int64_t N, int64_t ld, uint8_t* st) {
#pragma omp parallel for schedule(static)
  for (int64_t p = 0; p < N; ++p) {
    const bool ok = pixel_invert<NP>(src, dst, ld, p);
    if (st && !ok) st[p] |= ST_NONSPD;
  }
  return 0;
}
template <int NP>
static int h_operator(const BandDesc* b, int band, const float* x, int64_t N, int64_t ld, float* h0, float* h,
                      int64_t h_ld, uint8_t* okp) {
  const BandDesc& bd = b[band];
#pragma omp parallel for schedule(static)
  for (int64_t p = 0; p < N; ++p) {
    float xv[NP], hv[NP], H0;
    for (int j = 0; j < NP; ++j) xv[j] = x[j * ld + p];
    const bool ok = eval_operator<NP>(bd, p, ld, xv, H0, hv);
    h0[p] = H0;
    if (h)
      for (int j = 0; j < NP; ++j) h[j * h_ld + p] = hv[j];
    if (okp) okp[p] = ok ? 1 : 0;
  }
  return 0;
}
template <int NP>
static int h_gp_operator(const BandDesc* bands, int nb, const float* x, int64_t N, int64_t ld, float* h0, float* h,
                         int64_t ldh) {
#pragma omp parallel for schedule(static)
  for (int64_t p = 0; p < N; ++p) {
    float xv[NP];
    for (int j = 0; j < NP; ++j) xv[j] = x[j * ld + p];
    for (int b = 0; b < nb; ++b) {
      const BandDesc& bd = bands[b];
      float y, w, H0 = 0.f, hv[NP];
      for (int j = 0; j < NP; ++j) hv[j] = 0.f;
      decode_obs(bd, p, y, w);
      if (w > 0.f) eval_operator<NP>(bd, p, ld, xv, H0, hv);
      h0[b * ldh + p] = H0;
      for (int j = 0; j < NP; ++j) h[((int64_t)b * NP + j) * ldh + p] = hv[j];
    }
  }
  return 0;
}

template <int NP>
static int h_hessian(const BandDesc* bands, int nb, const float* x, float* a, int64_t N, int64_t ld) {
  constexpr int NT = ntri(NP);
#pragma omp parallel for schedule(static)
  for (int64_t p = 0; p < N; ++p) {
    float xv[NP], acc[NT];
    for (int j = 0; j < NP; ++j) xv[j] = x[j * ld + p];
    for (int t = 0; t < NT; ++t) acc[t] = 0.f;
    for (int bi = 0; bi < nb; ++bi) {
      const BandDesc& bd = bands[bi];
      if (bd.op != OP_GP) continue;
      float y, w;
      decode_obs(bd, p, y, w);
      if (!(w > 0.f)) continue;
      float f, Hs[NT];
      if (!gp_hessian_dispatch<NP>(bd, xv, f, Hs)) continue;
      const float s = w * (y - f);
      for (int t = 0; t < NT; ++t) acc[t] = fmaf(s, Hs[t], acc[t]);
    }
    for (int t = 0; t < NT; ++t) a[t * ld + p] -= acc[t];
  }
  return 0;
}
template <int NP>
static int h_unpack(const float* x, const float* a, int64_t N, int64_t ld, const int64_t* idx, float* mean,
                    float* unc, int64_t plane) {
#pragma omp parallel for schedule(static)
  for (int64_t p = 0; p < N; ++p) {
    const int64_t r = idx ? idx[p] : p;
    for (int j = 0; j < NP; ++j) {
      if (mean) mean[j * plane + r] = x[j * ld + p];
      if (unc) unc[j * plane + r] = kf_rsqrt(a[tri(NP, j, j) * ld + p]);
    }
  }
  return 0;
}

// GeoTIFF tiles on the host: the same row encoder as dfl_tile_kernel, rows in
// order into one byte stream per tile (bit-identical streams)
int host_deflate_tiles(const DflArgs& a) {
  const int per = a.tiles_x * a.tiles_y, n = a.nplanes * per;
  if (n <= 0) return -1;
#pragma omp parallel for schedule(dynamic, 1)
  for (int tile = 0; tile < n; ++tile) {
    const int plane = tile / per, tt = tile - plane * per;
    const int ty = tt / a.tiles_x, tx = tt - ty * a.tiles_x;
    const int x0 = tx * DFL_TILE;
    const int ncol = a.W - x0 < DFL_TILE ? a.W - x0 : DFL_TILE;
    uint8_t* o = a.out + (int64_t)tile * DFL_BOUND;
    int64_t nb = 0;
    uint64_t acc = 0;
    int nacc = 0;
    auto sink = [&](uint32_t bits, int len) {
      acc |= (uint64_t)bits << nacc;
      nacc += len;
      while (nacc >= 8) {
        o[nb++] = (uint8_t)(acc & 0xFFu);
        acc >>= 8;
        nacc -= 8;
      }
    };
    sink(0x78u, 8);
    sink(0x01u, 8);
    sink(1u, 1);                 // BFINAL
    sink(1u, 2);                 // BTYPE 01: fixed Huffman
    uint64_t t1 = 0, t2 = 0;
    for (int r = 0; r < DFL_TILE; ++r) {
      const int64_t y = (int64_t)ty * DFL_TILE + r;
      const bool rin = y < a.H;
      const float* rowp = a.src + (int64_t)plane * a.plane_ld + (rin ? y : 0) * a.W + x0;
      auto row = [&](int c) -> uint32_t {
        if (!(rin && c < ncol)) return 0u;
        uint32_t u;
        memcpy(&u, rowp + c, 4);
        return u;
      };
      uint64_t s1, s2;
      dfl_encode_row(row, DFL_RAW - (int64_t)r * DFL_ROW, sink, s1, s2);
      t1 += s1;
      t2 += s2;
    }
    sink(0u, 7);                 // end of block
    if (nacc) sink(0u, 8 - nacc);
    const uint32_t adler = dfl_adler(t1, t2, DFL_RAW);
    for (int k = 3; k >= 0; --k) sink((adler >> (8 * k)) & 0xFFu, 8);
    a.sizes[tile] = (uint32_t)nb;
  }
  return 0;
}

int host_analysis(int np, const AnalysisArgs& a, int grid) { KF_HOST_NP_SWITCH(np, h_analysis, a, grid); }
int host_gain(int np, const GainArgs& a, int grid) { KF_HOST_NP_SWITCH(np, h_gain, a, grid); }
int host_jacobi(int np, const JacobiArgs& a, int grid) { KF_HOST_NP_SWITCH(np, h_jacobi, a, grid); }
int host_propagate(int np, const PropArgs& a) { KF_HOST_NP_SWITCH(np, h_propagate, a); }
int host_invert(int np, const float* src, float* dst, int64_t N, int64_t ld, uint8_t* st) {
  KF_HOST_NP_SWITCH(np, h_invert, src, dst, N, ld, st);
}
int host_operator(int np, const BandDesc* b, int band, const float* x, int64_t N, int64_t ld, float* h0, float* h,
                  int64_t h_ld, uint8_t* ok) {
  KF_HOST_NP_SWITCH(np, h_operator, b, band, x, N, ld, h0, h, h_ld, ok);
}
int host_gp_operator(int np, const BandDesc* b, int nb, const float* x, int64_t N, int64_t ld, float* h0, float* h,
                     int64_t ldh) {
  KF_HOST_NP_SWITCH(np, h_gp_operator, b, nb, x, N, ld, h0, h, ldh);
}
int host_hessian(int np, const BandDesc* b, int nb, const float* x, float* a, int64_t N, int64_t ld) {
  KF_HOST_NP_SWITCH(np, h_hessian, b, nb, x, a, N, ld);
}
int host_unpack(int np, const float* x, const float* a, int64_t N, int64_t ld, const int64_t* idx, float* mean,
                float* unc, int64_t plane) {
  KF_HOST_NP_SWITCH(np, h_unpack, x, a, N, ld, idx, mean, unc, plane);
}
int host_obs_order(const BandDesc* bands, const int32_t* grp, int nb, int G, int64_t N, int32_t* order, bool local) {
  if (G < 1 || G > 3) return -1;
  std::vector<uint8_t> cls((size_t)N);
#pragma omp parallel for schedule(static)
  for (int64_t p = 0; p < N; ++p) cls[p] = (uint8_t)obs_class(bands, grp, nb, G, p);
  // local: each KF_ORD_CHUNK-pixel chunk partitioned in place
  const int64_t span = local ? (int64_t)KF_ORD_CHUNK : N;
  for (int64_t c0 = 0; c0 < N; c0 += span) {
    const int64_t c1 = std::min(N, c0 + span);
    int64_t k = c0;
    for (int c = 0; c < (1 << G); ++c)
      for (int64_t p = c0; p < c1; ++p)
        if (cls[p] == c) order[k++] = (int32_t)p;
  }
  return 0;
}
// Per-chunk Gauss-Newton convergence: each pixel's |dx|^2 in integer quanta
// of its chunk (chunk_quant) summed exactly, as on the device (any order
// gives the same total).
int host_chunk_partials(const ChunkPartialArgs& a) {
#pragma omp parallel for schedule(dynamic, 1)
  for (int c = 0; c < a.n_local; ++c) {
    const int g = a.lc_gid[c];
    if (!a.active[g]) continue;
    const double qi = a.qinv[g];
    int64_t tot = 0;
    for (int sg = a.lc_ptr[c]; sg < a.lc_ptr[c + 1]; ++sg) {
      const int st = a.seg_start[sg], len = a.seg_len[sg];
      for (int i = 0; i < len; ++i) tot += chunk_quant(a.dn[st + i], qi, a.clamp);
    }
    a.part[g] = tot;
  }
  return 0;
}

int host_chunk_decide(const ChunkDecideArgs& a) {
  double mx = 0.0;
  int n_act = 0, px = 0, n_new = 0;
  for (int g = 0; g < a.nc; ++g) {
    const bool was = a.active[g] != 0;
    bool stop = false;
    if (was) {
      int64_t tot = 0;
      for (int r = 0; r < a.world; ++r) tot += a.part_all[(int64_t)r * a.nc + g];
      const double norm = sqrt((double)tot * a.unit);
      mx = std::max(mx, norm);
      stop = chunk_stops(norm, a.n_iter, a.min_iter, a.max_iter, a.tol);
    }
    a.newly[g] = stop ? 1 : 0;
    if (stop) {
      a.active[g] = 0;
      a.iters[g] = a.n_iter;
      ++n_new;
    } else if (was) {
      ++n_act;
      px += a.local_count[g];
    }
  }
  a.info[0] = (double)n_act;
  a.info[1] = mx;
  a.info[2] = (double)px;
  a.info[3] = (double)n_new;
  if (a.px_out) *a.px_out = px;
  return 0;
}

int64_t host_chunk_compact(const ChunkCompactArgs& a) {
  int64_t k = 0;
  const int64_t n_in = visit_bounded(a.n_in, a.n_in, a.n_in_dev);
  for (int64_t q = 0; q < n_in; ++q) {
    const int p = a.order_in ? a.order_in[q] : (int)q;
    const int g = a.chunk_of[p];
    if (a.active[g]) {
      a.order_out[k++] = p;
    } else if (a.newly[g] && a.x_dst) {
      for (int j = 0; j < a.np; ++j) a.x_dst[(int64_t)j * a.ld + p] = a.x_src[(int64_t)j * a.ld + p];
    }
  }
  return k;
}

int host_lut_nearest(const float* lut, int M, int D, const float* x, int64_t N, int64_t ld, int32_t* out) {
#pragma omp parallel for schedule(static)
  for (int64_t p = 0; p < N; ++p) {
    float best = 3.4e38f;
    int bi = 0;
    for (int m = 0; m < M; ++m) {
      float s = 0.f;
      for (int d = 0; d < D; ++d) {
        const float t = lut[m * D + d] - x[d * ld + p];
        s = fmaf(t, t, s);
      }
      if (s < best) { best = s; bi = m; }
    }
    out[p] = bi;
  }
  return 0;
}

// RegTileArgs on the host: the same sweeps over the whole domain (strip plus
// deep halo rows), one at a time (scratch planes), then the strip rows of the
// launch's tile rows are written -- a host run equals the device's tiled pass.
int host_reg_tiled(const RegTileArgs& a) {
  const int64_t w = a.w;
  if (a.nsweep < 1 || a.nsweep > REG_TILE_MAX_SWEEPS || a.w <= 0 || a.h <= 0) return 1;
  if (a.hu < 0 || a.hd < 0 || (a.hu && a.hu < a.nsweep) || (a.hd && a.hd < a.nsweep)) return 1;
  if ((a.hu && !a.halo_up) || (a.hd && !a.halo_dn) || (a.sched && !a.omega_tab)) return 1;
  const int K = reg_tile_nsweep(a);
  bool cheb0 = false;
  if (K > 0) reg_tile_omega(a, 0, cheb0);
  const int H = a.hu + a.h + a.hd;          // domain rows, row 0 = strip row -hu
  const int64_t n = (int64_t)H * w;
  std::vector<float> cur(n), prev(n, 0.f), nxt(n), u(n), v(n);
  const float* ug = a.u + a.j0 * a.ld;
  const float* vg = a.v + a.j0 * a.ld;
  for (int R = 0; R < H; ++R) {
    const int gr = R - a.hu;
    const float *su = ug, *sv = vg, *sz = a.z, *szp = a.zp;
    int64_t off = (int64_t)gr * w;
    if (gr < 0) {
      off = (int64_t)(gr + a.hu) * w;
      su = a.halo_up, sv = a.halo_up + a.halo_plane, sz = a.halo_up + 2 * a.halo_plane;
      szp = a.halo_up + 3 * a.halo_plane;
    } else if (gr >= a.h) {
      off = (int64_t)(gr - a.h) * w;
      su = a.halo_dn, sv = a.halo_dn + a.halo_plane, sz = a.halo_dn + 2 * a.halo_plane;
      szp = a.halo_dn + 3 * a.halo_plane;
    }
    for (int64_t c = 0; c < w; ++c) {
      const int64_t q = (int64_t)R * w + c;
      cur[q] = sz[off + c];
      u[q] = su[off + c];
      v[q] = sv[off + c];
      if ((cheb0 || K == 0) && szp) prev[q] = szp[off + c];
    }
  }
  for (int s = 0; s < K; ++s) {
#pragma omp parallel for schedule(static)
    for (int64_t q = 0; q < n; ++q) {
      const int64_t r = q / w, c = q - r * w;
      const float sn = reg_tile_nsum(cur.data(), q, w, r > 0, r + 1 < H, c > 0, c + 1 < w);
      nxt[q] = reg_tile_step(a, s, sn, u[q], v[q], prev[q]);
    }
    std::swap(prev, cur);
    std::swap(cur, nxt);
  }
  const int tiles_y = (a.h + 63) / 64;
  const int ty0 = a.ty1 == 0 ? 0 : a.ty0, ty1 = a.ty1 == 0 ? tiles_y : a.ty1;
  if (ty0 < 0 || ty1 > tiles_y || ty0 > ty1) return 1;
  const int64_t r_lo = (int64_t)ty0 * 64, r_hi = std::min<int64_t>((int64_t)ty1 * 64, a.h);
  for (int64_t r = r_lo; r < r_hi; ++r) {
    const int64_t src = (r + a.hu) * w;
    std::copy(cur.begin() + src, cur.begin() + src + w, a.z_out + r * w);
    std::copy(prev.begin() + src, prev.begin() + src + w, a.zp_out + r * w);
  }
  return 0;
}

int host_reg_rho(const float* vrow, const StripGeo& g, int64_t N, const RegScheduleArgs& a) {
  if (N <= 0 || g.w <= 0) return 1;
  float m = 0.f;
  for (int64_t p = 0; p < N; ++p) m = std::max(m, reg_rho_term(vrow, g, p));
  a.rho[0] = (double)(m * a.gamma);
  return 0;
}

int host_reg_schedule(const RegScheduleArgs& a) {
  if (a.max_sweeps < 1 || !a.sched || !a.omega_tab || !a.info || !a.rho) return 1;
  double used;
  const int S = reg_cheb_schedule(a.rho[0], a.tol, a.max_sweeps, a.omega_tab, &used);
  a.sched[0] = S - 1;
  a.info[0] = used;
  a.info[1] = (double)S;
  return 0;
}

}  // namespace kf
