// kf_reg_tiled.hip — K9 temporal blocking on gfx950: up to 8 sweeps of the
// regularised field per launch (RegTileArgs, kf_core.h), plus the device-side
// Chebyshev schedule (rho bound -> sweep count and weights, no host read-back
// ahead of the sweeps).
//
// One sweep streams ~20 B/px (u, v, the iterate, the previous iterate, the
// result) for ~10 flops, so the per-sweep kernel runs at the HBM floor of a
// single sweep.  Here a 1024-thread workgroup stages a 64 x 128 tile plus a
// ring nsweep pixels wide in LDS (46 KB at 8 sweeps), keeps u, v and the
// previous iterate of its pixels in registers, and runs every sweep out of
// LDS: 4 neighbour reads + 1 write per pixel and sweep, two barriers.  HBM
// sees one read of the region and one write of the interior's last two
// iterates per launch.  Workgroups are dealt to the 8 XCDs in contiguous runs
// of tiles so a tile's ring is mostly in its own XCD's L2.
//
// Tile-DP strips (C2): the ring of a strip's first / last tile row reaches
// into the neighbours' rows, read from a deep halo (hu / hd rows of u, v, z,
// zp) that the engine exchanges once per pass, not once per sweep.  A launch
// covers a range of tile rows, so the boundary rows can run first, their
// exchange go on the wire, and the interior run under it
// (engine/linear_kf.py:_reg_tiled_sweeps).
#include "kf_device.h"

namespace kf {

constexpr int RT_TH = 64, RT_TW = 128, RT_NT = 1024;
constexpr int RT_MAXR = (RT_TH + 2 * REG_TILE_MAX_SWEEPS) * (RT_TW + 2 * REG_TILE_MAX_SWEEPS);
constexpr int RT_PER = (RT_MAXR + RT_NT - 1) / RT_NT;

// per-pixel flags: in domain, then which neighbours are read (in the domain and in the region)
constexpr uint32_t RT_IN = 1, RT_UP = 2, RT_DN = 4, RT_LF = 8, RT_RT = 16, RT_OUT = 32;

__global__ __launch_bounds__(RT_NT) void reg_tiled_kernel(RegTileArgs a, int tiles_x, int ntiles, int per_xcd) {
  __shared__ float zs[RT_MAXR];
  const int b = blockIdx.x;
  const int tile = (b & 7) * per_xcd + (b >> 3);
  if (tile >= ntiles) return;   // whole workgroup, before any barrier
  const int tyl = tile / tiles_x, tx = tile - tyl * tiles_x;
  const int ty = a.ty0 + tyl;
  const int K = reg_tile_nsweep(a);   // uniform (scalar load of the schedule); 0: copy the inputs
  const int RW = RT_TW + 2 * K, RH = RT_TH + 2 * K, R = RW * RH;
  const int r0 = ty * RT_TH - K, c0 = tx * RT_TW - K;
  const int64_t w = a.w;
  const int lo = -a.hu, hi = a.h + a.hd;   // rows of the domain (strip + halo)
  const float* ug = a.u + a.j0 * a.ld;
  const float* vg = a.v + a.j0 * a.ld;
  bool cheb0 = false;
  if (K > 0) reg_tile_omega(a, 0, cheb0);
  const bool use_zp = cheb0 || K == 0;

  float u[RT_PER], v[RT_PER], zc[RT_PER], zp[RT_PER];
  uint32_t fl[RT_PER];
#pragma unroll
  for (int j = 0; j < RT_PER; ++j) {
    const int i = threadIdx.x + j * RT_NT;
    const int rr = i / RW, cc = i - rr * RW;
    const int gr = r0 + rr, gc = c0 + cc;
    const bool in = i < R && gr >= lo && gr < hi && gc >= 0 && gc < a.w;
    uint32_t f = 0;
    if (in) {
      f = RT_IN;
      if (gr > lo && rr > 0) f |= RT_UP;
      if (gr + 1 < hi && rr + 1 < RH) f |= RT_DN;
      if (gc > 0 && cc > 0) f |= RT_LF;
      if (gc + 1 < a.w && cc + 1 < RW) f |= RT_RT;
      if (rr >= K && rr < K + RT_TH && cc >= K && cc < K + RT_TW && gr >= 0 && gr < a.h) f |= RT_OUT;
    }
    fl[j] = f;
    // source of the pixel: the strip, or a halo plane (u, v, z, zp at 0..3 planes)
    const float *su = ug, *sv = vg, *sz = a.z, *szp = a.zp;
    int64_t p = 0;
    if (in) {
      if (gr < 0) {
        p = (int64_t)(gr + a.hu) * w + gc;
        su = a.halo_up;
        sv = a.halo_up + a.halo_plane;
        sz = a.halo_up + 2 * a.halo_plane;
        szp = a.halo_up + 3 * a.halo_plane;
      } else if (gr >= a.h) {
        p = (int64_t)(gr - a.h) * w + gc;
        su = a.halo_dn;
        sv = a.halo_dn + a.halo_plane;
        sz = a.halo_dn + 2 * a.halo_plane;
        szp = a.halo_dn + 3 * a.halo_plane;
      } else {
        p = (int64_t)gr * w + gc;
      }
    }
    zc[j] = in ? sz[p] : 0.f;
    zp[j] = in && use_zp && szp ? szp[p] : 0.f;
    u[j] = in ? su[p] : 0.f;
    v[j] = in ? sv[p] : 0.f;
    if (i < R) zs[i] = zc[j];
  }
  __syncthreads();
  for (int s = 0; s < K; ++s) {
    float zn[RT_PER];
#pragma unroll
    for (int j = 0; j < RT_PER; ++j) {
      const int i = threadIdx.x + j * RT_NT;
      const uint32_t f = fl[j];
      float sn = 0.f;
      if (f & RT_UP) sn += zs[i - RW];
      if (f & RT_DN) sn += zs[i + RW];
      if (f & RT_LF) sn += zs[i - 1];
      if (f & RT_RT) sn += zs[i + 1];
      zn[j] = reg_tile_step(a, s, sn, u[j], v[j], zp[j]);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RT_PER; ++j) {
      const int i = threadIdx.x + j * RT_NT;
      if (fl[j] & RT_IN) {
        zp[j] = zc[j];
        zc[j] = zn[j];
        zs[i] = zn[j];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < RT_PER; ++j) {
    if (!(fl[j] & RT_OUT)) continue;
    const int i = threadIdx.x + j * RT_NT;
    const int rr = i / RW, cc = i - rr * RW;
    const int64_t p = (int64_t)(r0 + rr) * w + (c0 + cc);
    a.z_out[p] = zc[j];
    a.zp_out[p] = zp[j];
  }
}

hipError_t dev_reg_tiled(const RegTileArgs& a, hipStream_t s) {
  if (a.nsweep < 1 || a.nsweep > REG_TILE_MAX_SWEEPS || a.w <= 0 || a.h <= 0) return hipErrorInvalidValue;
  if (a.hu < 0 || a.hd < 0 || a.hu > REG_TILE_MAX_SWEEPS || a.hd > REG_TILE_MAX_SWEEPS) return hipErrorInvalidValue;
  if ((a.hu && (!a.halo_up || a.halo_plane < (int64_t)a.hu * a.w)) ||
      (a.hd && (!a.halo_dn || a.halo_plane < (int64_t)a.hd * a.w)))
    return hipErrorInvalidValue;
  // a halo shallower than the sweeps would let stale ring values reach the strip
  if ((a.hu && a.hu < a.nsweep) || (a.hd && a.hd < a.nsweep)) return hipErrorInvalidValue;
  if (a.sched && !a.omega_tab) return hipErrorInvalidValue;
  const int tiles_x = (a.w + RT_TW - 1) / RT_TW, tiles_y = (a.h + RT_TH - 1) / RT_TH;
  RegTileArgs b = a;
  if (b.ty1 == 0) {
    b.ty0 = 0;
    b.ty1 = tiles_y;
  }
  if (b.ty0 < 0 || b.ty1 > tiles_y || b.ty0 > b.ty1) return hipErrorInvalidValue;
  const int64_t nt = (int64_t)tiles_x * (b.ty1 - b.ty0);
  if (nt == 0) return hipSuccess;
  if (nt > (1 << 28)) return hipErrorInvalidValue;
  const int per = (int)((nt + 7) / 8);
  hipLaunchKernelGGL(reg_tiled_kernel, dim3(8 * per), dim3(RT_NT), 0, s, b, tiles_x, (int)nt, per);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Schedule of the coupled solve on the device: the per-block maxima of
// v_RR * deg (one regularised field, dense strip), their max (times gamma)
// into rho, then -- after the engine's all-rank max of rho -- the sweep count
// and the Chebyshev weights (reg_cheb_schedule).  The tiled passes read them,
// so the host queues the first pass without waiting for rho.
constexpr int RHO_BS = 256;

__global__ __launch_bounds__(RHO_BS) void reg_rho_kernel(const float* vrow, StripGeo g, int64_t N, float* pmax) {
  __shared__ float red[RHO_BS / 64];
  float m = 0.f;
  for (int64_t p = (int64_t)blockIdx.x * RHO_BS + threadIdx.x; p < N; p += (int64_t)gridDim.x * RHO_BS)
    m = fmaxf(m, reg_rho_term(vrow, g, p));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = red[0];
#pragma unroll
    for (int k = 1; k < RHO_BS / 64; ++k) t = fmaxf(t, red[k]);
    pmax[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(64) void reg_rho_reduce_kernel(RegScheduleArgs a) {
  float m = 0.f;
  for (int i = threadIdx.x; i < a.npart; i += 64) m = fmaxf(m, a.pmax[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (threadIdx.x == 0) a.rho[0] = (double)(m * a.gamma);
}

__global__ __launch_bounds__(64) void reg_schedule_kernel(RegScheduleArgs a) {
  if (threadIdx.x != 0) return;
  double used;
  const int S = reg_cheb_schedule(a.rho[0], a.tol, a.max_sweeps, a.omega_tab, &used);
  a.sched[0] = S - 1;
  a.info[0] = used;
  a.info[1] = (double)S;
}

int reg_rho_blocks(int64_t N) {
  const int64_t b = (N + RHO_BS - 1) / RHO_BS;
  return (int)(b < 1024 ? (b < 1 ? 1 : b) : 1024);
}

hipError_t dev_reg_rho(const float* vrow, const StripGeo& g, int64_t N, const RegScheduleArgs& a, hipStream_t s) {
  if (N <= 0 || g.w <= 0 || a.npart != reg_rho_blocks(N)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(reg_rho_kernel, dim3(a.npart), dim3(RHO_BS), 0, s, vrow, g, N, const_cast<float*>(a.pmax));
  hipLaunchKernelGGL(reg_rho_reduce_kernel, dim3(1), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t dev_reg_schedule(const RegScheduleArgs& a, hipStream_t s) {
  if (a.max_sweeps < 1 || !a.sched || !a.omega_tab || !a.info || !a.rho) return hipErrorInvalidValue;
  hipLaunchKernelGGL(reg_schedule_kernel, dim3(1), dim3(64), 0, s, a);
  return hipGetLastError();
}

}  // namespace kf
