// kf_reg_tiled.hip — K9 temporal blocking on gfx950: up to 8 sweeps of the
// regularised field per launch (RegTileArgs, kf_core.h).
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
  const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
  const int K = a.nsweep;
  const int RW = RT_TW + 2 * K, RH = RT_TH + 2 * K, R = RW * RH;
  const int r0 = ty * RT_TH - K, c0 = tx * RT_TW - K;
  const int64_t w = a.w;
  const float* ug = a.u + a.j0 * a.ld;
  const float* vg = a.v + a.j0 * a.ld;
  const bool use_zp = a.prev_mask & 1u;

  float u[RT_PER], v[RT_PER], zc[RT_PER], zp[RT_PER];
  uint32_t fl[RT_PER];
#pragma unroll
  for (int j = 0; j < RT_PER; ++j) {
    const int i = threadIdx.x + j * RT_NT;
    const int rr = i / RW, cc = i - rr * RW;
    const int gr = r0 + rr, gc = c0 + cc;
    const bool in = i < R && gr >= 0 && gr < a.h && gc >= 0 && gc < a.w;
    uint32_t f = 0;
    if (in) {
      f = RT_IN;
      if (gr > 0 && rr > 0) f |= RT_UP;
      if (gr + 1 < a.h && rr + 1 < RH) f |= RT_DN;
      if (gc > 0 && cc > 0) f |= RT_LF;
      if (gc + 1 < a.w && cc + 1 < RW) f |= RT_RT;
      if (rr >= K && rr < K + RT_TH && cc >= K && cc < K + RT_TW) f |= RT_OUT;
    }
    fl[j] = f;
    const int64_t p = in ? (int64_t)gr * w + gc : 0;
    zc[j] = in ? a.z[p] : 0.f;
    zp[j] = in && use_zp ? a.zp[p] : 0.f;
    u[j] = in ? ug[p] : 0.f;
    v[j] = in ? vg[p] : 0.f;
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
  const int tiles_x = (a.w + RT_TW - 1) / RT_TW, tiles_y = (a.h + RT_TH - 1) / RT_TH;
  const int64_t nt = (int64_t)tiles_x * tiles_y;
  if (nt > (1 << 28)) return hipErrorInvalidValue;
  const int per = (int)((nt + 7) / 8);
  hipLaunchKernelGGL(reg_tiled_kernel, dim3(8 * per), dim3(RT_NT), 0, s, a, tiles_x, (int)nt, per);
  return hipGetLastError();
}

}  // namespace kf
