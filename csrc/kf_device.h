// kf_device.h — gfx950 (MI355X) kernel templates for the KaFKA engine, shared by
// the translation units kf_kernels.hip, kf_analysis7.hip and kf_analysis10.hip
// (split so the heavy analysis instantiations compile in parallel, _build.py).
//
// Design: every matrix the reference builds is block
// diagonal with n_p x n_p per-pixel blocks, so the whole Gauss-Newton
// analysis (operator + Jacobian, normal equations, Cholesky, convergence
// partial) is one pixel per lane, SoA layout ([param][pixel], coalesced
// 256-B wave loads), grid-stride over pixels, 256-thread workgroups
// (4 wave64 per workgroup).  GP training records are wave-uniform and are
// read through the scalar path (s_load) so they cost no VGPRs/LDS traffic.
// Deterministic reductions: per-block f64 partials, summed in fixed order
// by reduce_partials_kernel.
#pragma once
#include <hip/hip_runtime.h>
#include "kf_core.h"
#include "kf_launch.h"
#include "kf_gp_mfma.h"

namespace kf {

constexpr int BLOCK = 256;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <int BS = BLOCK>
__device__ __forceinline__ void block_partial(double v, double* partials) {
  __shared__ double red[BS / 64];
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < BS / 64; ++i) s += red[i];
    partials[blockIdx.x] = s;
  }
}

// Both norm partials of a fused two-iteration launch in one reduction pass.
template <int BS = BLOCK>
__device__ __forceinline__ void block_partials2(double v, double v1, double* partials, double* partials1) {
  __shared__ double red[2][BS / 64];
  v = wave_sum(v);
  v1 = wave_sum(v1);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wid] = v;
    red[1][wid] = v1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0, s1 = 0.0;
#pragma unroll
    for (int i = 0; i < BS / 64; ++i) {
      s += red[0][i];
      s1 += red[1][i];
    }
    if (partials) partials[blockIdx.x] = s;
    if (partials1) partials1[blockIdx.x] = s1;
  }
}

template <int BS = BLOCK>
__device__ __forceinline__ void analysis_partials(const AnalysisArgs& a, double acc, double acc1) {
  if (a.partials_first) block_partials2<BS>(acc, acc1, a.partials, a.partials_first);
  else if (a.partials) block_partial<BS>(acc, a.partials);
}

template <int NP, int FD = 0, int FOBS = 0, int UNR = 4, bool FOLD = false>
__global__ __launch_bounds__(BLOCK) void analysis_kernel(AnalysisArgs a) {
  double acc = 0.0, acc1 = 0.0;
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  const int64_t nv = visit_count(a);
  for (int64_t q = (int64_t)blockIdx.x * BLOCK + threadIdx.x; q < nv; q += stride) {
    float dn1;
    const int64_t p = visit_px(a.order, q);
    const float dn = pixel_analysis<NP, FD, FOBS, UNR, FOLD>(a, p, dn1);
    if (a.dn_out) a.dn_out[p] = dn;
    acc += (double)dn;
    acc1 += (double)dn1;
  }
  analysis_partials(a, acc, acc1);
}

// K1 with the GP on the matrix cores (kf_gp_mfma.h).  Every band's split-f16
// table is staged in LDS once per workgroup (a.gpm_frags x 16 B of dynamic
// LDS), then each wave walks 64-pixel tiles grid-stride.  BS = 512 with
// MINW = 4 waves per SIMD (<= 128 VGPRs, 2 workgroups per CU for two bands'
// tables) lets the HBM phases (state loads, result stores) of some waves run
// under the record loops of others; BS = 256 gives 3 waves per SIMD.
template <int NP, int D, int FOBS, int BS = BLOCK, int MINW = 1, int LAYOUT = BAND_LAYOUT_RUNTIME, bool IL = false,
          int SPEC = SPEC_ANY>
__global__ __launch_bounds__(BS, MINW) void analysis_mfma_kernel(AnalysisArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  extern __shared__ kf_h8 gpm_lds[];
  KF_PHASE_KERNEL_BEGIN
  {
    int off = 0;
    for (int bi = 0; bi < a.n_bands; ++bi) {
      const KF_CONST_AS BandDesc* bd = cptr(a.bands) + bi;
      const int n = bd->gpm_nchunk * gpm_frags_per_chunk(D);
      const kf_h8* src = (const kf_h8*)bd->gpm;
      for (int i = threadIdx.x; i < n; i += BS) gpm_lds[off + i] = src[i];
      off += n;
    }
    if (threadIdx.x == 0) gpm_lds[a.gpm_frags - 1] = kf_h8{};   // shared zero fragment
  }
  __syncthreads();
  KF_PHASE(KF_PH_PROLOGUE)
  double acc = 0.0, acc1 = 0.0;
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * BS;
  const int64_t nv = visit_count(a);
  if constexpr (SPEC == SPEC_PROP_PF) {
    // small emulators (short GP loops): the next pixel group's index and its
    // single propagated parameter's x_a / P_a,jj are loaded before this group's
    // analysis, so the forecast starts from registers instead of a dependent
    // order -> state load chain (pixel indices < 2^31: one VGPR carried)
    const KF_CONST_AS PropArgs* pa = cptr(a.prop);
    const int pj = prop_single(pa->prop_mask);
    int64_t base = (int64_t)blockIdx.x * BS + (threadIdx.x - lane);
    uint32_t p32 = base < nv ? (uint32_t)visit_px(a.order, base + lane < nv ? base + lane : nv - 1) : 0u;
    float px = 0.f, pp = 0.f;
    if (pj >= 0 && base < nv) {
      px = KF_PX(pa->x_a, pj * pa->ld, (int64_t)p32);
      pp = KF_PX(pa->p_a, tri(NP, pj, pj) * pa->ld, (int64_t)p32);
    }
    for (; base < nv; base += stride) {
      const int64_t q = base + lane;
      const bool act = q < nv;
      const int64_t p = (int64_t)p32;
      const int64_t bn = base + stride;
      uint32_t pn = 0u;
      float pxn = 0.f, ppn = 0.f;
      if (bn < nv) {
        pn = (uint32_t)visit_px(a.order, bn + lane < nv ? bn + lane : nv - 1);
        if (pj >= 0) {
          pxn = KF_PX(pa->x_a, pj * pa->ld, (int64_t)pn);
          ppn = KF_PX(pa->p_a, tri(NP, pj, pj) * pa->ld, (int64_t)pn);
        }
      }
      float dn1;
      const float dn = pixel_analysis_mfma<NP, D, FOBS, false, false, LAYOUT, IL, SPEC>(
          a, p, act, gpm_lds, dn1 KF_PHASE_ARG, pj, px, pp);
      {
        float* dno = opaque((const KF_CONST_AS AnalysisArgs*)__builtin_amdgcn_kernarg_segment_ptr())->dn_out;
        if (act && dno) KF_PX(dno, 0, p) = dn;
      }
      acc += act ? (double)dn : 0.0;
      acc1 += act ? (double)dn1 : 0.0;
      p32 = pn;
      px = pxn;
      pp = ppn;
    }
  } else {
    for (int64_t base = (int64_t)blockIdx.x * BS + (threadIdx.x - lane); base < nv; base += stride) {
      const int64_t q = base + lane;
      const bool act = q < nv;
      const int64_t p = visit_px(a.order, act ? q : nv - 1);
      float dn1;
      const float dn = pixel_analysis_mfma<NP, D, FOBS, false, false, LAYOUT, IL, SPEC>(a, p, act, gpm_lds,
                                                                                       dn1 KF_PHASE_ARG);
      {
        // re-read through the opaque kernarg pointer: not pinned in SGPRs across the GP loop
        float* dno = opaque((const KF_CONST_AS AnalysisArgs*)__builtin_amdgcn_kernarg_segment_ptr())->dn_out;
        if (act && dno) KF_PX(dno, 0, p) = dn;
      }
      acc += act ? (double)dn : 0.0;
      acc1 += act ? (double)dn1 : 0.0;
    }
  }
  analysis_partials<BS>(a, acc, acc1);
  KF_PHASE_KERNEL_END
#endif
}

// K1 on the matrix cores with every band's table read from global memory
// (gp_mfma_sums_g): many-band GP states (PROSAIL: ten bands, 358-716 KiB of
// tables) whose tables exceed the LDS.  No LDS, so the waves per SIMD follow
// the VGPR count alone.
template <int NP, int D, int FOBS, bool PF = false, bool IL = false, int SPEC = SPEC_ANY>
__global__ __launch_bounds__(BLOCK, 2) void analysis_mfma_g_kernel(AnalysisArgs a) {
  static_assert(BLOCK / 64 == GPM_G_WAVES, "per-wave LDS transpose buffers of gp_mfma_sums_g_xb");
#if defined(__HIP_DEVICE_COMPILE__)
  KF_PHASE_KERNEL_BEGIN
  double acc = 0.0, acc1 = 0.0;
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  const int64_t nv = visit_count(a);
  for (int64_t base = (int64_t)blockIdx.x * BLOCK + (threadIdx.x - lane); base < nv; base += stride) {
    const int64_t q = base + lane;
    const bool act = q < nv;
    const int64_t p = visit_px(a.order, act ? q : nv - 1);
    float dn1;
    const float dn = pixel_analysis_mfma<NP, D, FOBS, true, PF, BAND_LAYOUT_RUNTIME, IL, SPEC>(
        a, p, act, nullptr, dn1 KF_PHASE_ARG);
    {
      // re-read through the opaque kernarg pointer: not pinned in SGPRs across the GP loop
      float* dno = opaque((const KF_CONST_AS AnalysisArgs*)__builtin_amdgcn_kernarg_segment_ptr())->dn_out;
      if (act && dno) KF_PX(dno, 0, p) = dn;
    }
    acc += act ? (double)dn : 0.0;
    acc1 += act ? (double)dn1 : 0.0;
  }
  analysis_partials(a, acc, acc1);
  KF_PHASE_KERNEL_END
#endif
}

// dynamic LDS above the 64 KiB default (tables of several bands, up to the
// 160 KiB of a gfx950 CU)
template <typename K>
static void gpm_lds_attr(K kernel, size_t bytes) {
  if (bytes > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)bytes);
}

// K1g with the GP on the matrix cores (JRC-TIP: tables staged in LDS once per
// workgroup, as analysis_mfma_kernel).  3 workgroups per CU (168 VGPRs, 80 B
// of scratch per lane) run 6 % faster than 2 (201 VGPRs, 64 B): tip7 gain
// 24.05 vs 25.52 ms/step (profiles/r6_v25_gain_three_waves_ab.jsonl).
template <int NP, int D, int FOBS>
__global__ __launch_bounds__(BLOCK, 3) void gain_mfma_kernel(GainArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  extern __shared__ kf_h8 gpm_lds[];
  {
    int off = 0;
    for (int bi = 0; bi < a.n_bands; ++bi) {
      const KF_CONST_AS BandDesc* bd = cptr(a.bands) + bi;
      const int n = bd->gpm_nchunk * gpm_frags_per_chunk(D);
      const kf_h8* src = (const kf_h8*)bd->gpm;
      for (int i = threadIdx.x; i < n; i += BLOCK) gpm_lds[off + i] = src[i];
      off += n;
    }
    if (threadIdx.x == 0) gpm_lds[a.gpm_frags - 1] = kf_h8{};   // shared zero fragment
  }
  __syncthreads();
  double acc = 0.0, acc1 = 0.0;
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  const int64_t nv = visit_count(a);
  for (int64_t base = (int64_t)blockIdx.x * BLOCK + (threadIdx.x - lane); base < nv; base += stride) {
    const int64_t q = base + lane;
    const bool act = q < nv;
    const int64_t p = visit_px(a.order, act ? q : nv - 1);
    float dn1;
    const float dn = pixel_gain_mfma<NP, D, FOBS>(a, p, act, gpm_lds, dn1);
    acc += act ? (double)dn : 0.0;
    acc1 += act ? (double)dn1 : 0.0;
  }
  if (a.partials_first) block_partials2<BLOCK>(acc, acc1, a.partials, a.partials_first);
  else if (a.partials) block_partial(acc, a.partials);
#endif
}

template <int NP, int FD = 0, int FOBS = 0>
__global__ __launch_bounds__(BLOCK) void gain_kernel(GainArgs a) {
  double acc = 0.0, acc1 = 0.0;
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  const int64_t nv = visit_count(a);
  for (int64_t q = (int64_t)blockIdx.x * BLOCK + threadIdx.x; q < nv; q += stride) {
    float dn1;
    acc += (double)pixel_gain<NP, FD, FOBS>(a, visit_px(a.order, q), dn1);
    acc1 += (double)dn1;
  }
  if (a.partials_first) block_partials2<BLOCK>(acc, acc1, a.partials, a.partials_first);
  else if (a.partials) block_partial(acc, a.partials);
}

// K1g launch: the all-GP fast instantiations (as l_analysis) or the generic kernel.
template <int NP>
static void l_gain(const GainArgs& a, int grid, hipStream_t s) {
#define KF_GAIN_FAST(D_)                                                                                 \
  if (a.fast_d == D_) {                                                                                 \
    if (a.fast_obs == OBS_DN16) {                                                                       \
      hipLaunchKernelGGL((gain_kernel<NP, D_, OBS_DN16>), dim3(grid), dim3(BLOCK), 0, s, a);            \
      return;                                                                                           \
    }                                                                                                   \
    if (a.fast_obs == OBS_F32) {                                                                        \
      hipLaunchKernelGGL((gain_kernel<NP, D_, OBS_F32>), dim3(grid), dim3(BLOCK), 0, s, a);             \
      return;                                                                                           \
    }                                                                                                   \
  }
  if constexpr (NP == 7) {
    if (a.fast_d == 4 && a.gpm_frags > 0 && a.n_bands <= GPM_MAX_BANDS &&
        (a.fast_obs == OBS_DN16 || a.fast_obs == OBS_F32)) {
      const size_t lds = (size_t)a.gpm_frags * sizeof(kf_h8);
      if (a.fast_obs == OBS_DN16) {
        gpm_lds_attr(gain_mfma_kernel<NP, 4, OBS_DN16>, lds);
        hipLaunchKernelGGL((gain_mfma_kernel<NP, 4, OBS_DN16>), dim3(grid), dim3(BLOCK), lds, s, a);
      } else {
        gpm_lds_attr(gain_mfma_kernel<NP, 4, OBS_F32>, lds);
        hipLaunchKernelGGL((gain_mfma_kernel<NP, 4, OBS_F32>), dim3(grid), dim3(BLOCK), lds, s, a);
      }
      return;
    }
    KF_GAIN_FAST(4)
  } else if constexpr (NP == 10) {
    KF_GAIN_FAST(10)
  }
#undef KF_GAIN_FAST
  hipLaunchKernelGGL(gain_kernel<NP>, dim3(grid), dim3(BLOCK), 0, s, a);
}

// MODE < 0: runtime a.mode (prepare / classic: Cholesky-sized registers);
// the streaming sweep and finish passes get instantiations of their own so
// that their occupancy is not set by the prepare path's register count.
template <int NP, int MODE = -1>
__global__ __launch_bounds__(BLOCK) void jacobi_kernel(JacobiArgs a) {
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  const int64_t n = a.pn > 0 ? a.pn : a.N;
  if constexpr (MODE == JACOBI_SWEEP1D || MODE == JACOBI_FINISH1D) {
    // whole rows [p0 / w, (p0 + n) / w) of a dense strip (checked by the launcher)
    const uint32_t w = (uint32_t)a.geo.w;
    const uint32_t r0 = (uint32_t)(a.p0 / w), nr = (uint32_t)(n / w);
    const int j0 = __builtin_ctz(a.reg_mask);
    for (uint32_t rr = blockIdx.x; rr < nr; rr += gridDim.x) {
      const uint32_t r = r0 + rr;
      // the finish carries NP values per pixel: 2 pixels per thread keep it at
      // 4 waves per SIMD (<= 128 VGPRs; 4 pixels: 147, 3 waves)
      constexpr int UU = MODE == JACOBI_SWEEP1D ? JACOBI_U : 2;
      for (uint32_t c0 = threadIdx.x; c0 < w; c0 += UU * BLOCK) {
        if constexpr (MODE == JACOBI_SWEEP1D) reg_sweep1d<NP, UU, BLOCK>(a, r, c0, j0);
        else acc += (double)reg_finish1d<NP, UU, BLOCK>(a, r, c0);
      }
    }
  } else if constexpr (MODE == JACOBI_FINISH4) {
    // 4-pixel groups of whole rows (w % 4 == 0 and 16-byte alignment: launcher)
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n / 4; i += stride)
      acc += (double)reg_finish4<NP>(a, a.p0 + 4 * i);
  } else if constexpr (MODE == JACOBI_SWEEP1 || MODE == JACOBI_FINISH1) {
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += JACOBI_U * stride) {
      if constexpr (MODE == JACOBI_SWEEP1) reg_sweep1<NP, JACOBI_U>(a, i, stride, n);
      else acc += (double)reg_finish1<NP, JACOBI_U>(a, i, stride, n);
    }
  } else {
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) {
      if constexpr (MODE == JACOBI_SWEEP) acc += (double)pixel_reg_sweep<NP>(a, a.p0 + i);
      else if constexpr (MODE == JACOBI_FINISH) acc += (double)pixel_reg_finish<NP>(a, a.p0 + i);
      else acc += (double)pixel_jacobi<NP>(a, a.p0 + i);
    }
  }
  if (a.partials) block_partial(acc, a.partials);
}

template <int NP>
__global__ __launch_bounds__(BLOCK) void propagate_kernel(PropArgs a) {
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  for (int64_t p = (int64_t)blockIdx.x * BLOCK + threadIdx.x; p < a.N; p += stride)
    pixel_propagate<NP>(a, p);
}

template <int NP>
__global__ __launch_bounds__(BLOCK) void invert_kernel(const float* src, float* dst, int64_t N, int64_t ld,
                                                      uint8_t* status) {
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  for (int64_t p = (int64_t)blockIdx.x * BLOCK + threadIdx.x; p < N; p += stride) {
    const bool ok = pixel_invert<NP>(src, dst, ld, p);
    if (status && !ok) status[p] |= ST_NONSPD;
  }
}

// Standalone operator evaluation (H0 and Jacobian rows) for one band.
template <int NP>
__global__ __launch_bounds__(BLOCK) void operator_kernel(const BandDesc* bands, int band, const float* x,
                                                        int64_t N, int64_t ld, float* h0, float* h,
                                                        int64_t h_ld, uint8_t* ok_out) {
  const BandDesc bd = cptr(bands)[band];
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  for (int64_t p = (int64_t)blockIdx.x * BLOCK + threadIdx.x; p < N; p += stride) {
    float xv[NP], hv[NP], H0;
#pragma unroll
    for (int j = 0; j < NP; ++j) xv[j] = x[j * ld + p];
    const bool ok = eval_operator<NP>(bd, p, ld, xv, H0, hv);
    h0[p] = H0;
    if (h) {
#pragma unroll
      for (int j = 0; j < NP; ++j) h[j * h_ld + p] = hv[j];
    }
    if (ok_out) ok_out[p] = ok ? 1 : 0;
  }
}

// K2 split path: GP emulator value + Jacobian for a chunk of bands into HBM
// (h0[b][p], h[b*NP+j][p]).  Without the analysis' packed A/b in registers it
// runs at high occupancy; used for large input counts (PROSAIL D=10) and many
// bands (multi-sensor), followed by the OP_PRECOMP analysis kernel.  Pixels
// whose observation is masked skip the GP (wave-level skip under clouds).
template <int NP, int D, int UNR>
__global__ __launch_bounds__(BLOCK) void gp_operator_kernel(const BandDesc* bands, int nb, const float* x,
                                                           int64_t N, int64_t ld, float* h0, float* h,
                                                           int64_t ldh) {
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  for (int64_t p = (int64_t)blockIdx.x * BLOCK + threadIdx.x; p < N; p += stride) {
    float xv[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) xv[j] = x[j * ld + p];
    for (int b = 0; b < nb; ++b) {
      const BandDesc bd = cptr(bands)[b];
      float y, w, H0 = 0.f, hv[NP];
#pragma unroll
      for (int j = 0; j < NP; ++j) hv[j] = 0.f;
      decode_obs(bd, p, y, w);
      // RELOAD: the descriptor's epilogue fields are re-read after the record
      // stream (61 instead of 91 VGPRs, 26 instead of 233 SGPR spills at D=10)
      if (w > 0.f) gp_eval<NP, D, UNR, false, true>(bd, xv, H0, hv, bands + b);
      h0[b * ldh + p] = H0;
#pragma unroll
      for (int j = 0; j < NP; ++j) h[((int64_t)b * NP + j) * ldh + p] = hv[j];
    }
  }
}

// K6 Hessian correction: A -= w (y - H0(x)) d2f/dx2 for every GP band.
template <int NP>
__global__ __launch_bounds__(BLOCK) void hessian_kernel(const BandDesc* bands, int n_bands, const float* x,
                                                       float* a, int64_t N, int64_t ld) {
  constexpr int NT = ntri(NP);
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  for (int64_t p = (int64_t)blockIdx.x * BLOCK + threadIdx.x; p < N; p += stride) {
    float xv[NP], acc[NT];
#pragma unroll
    for (int j = 0; j < NP; ++j) xv[j] = x[j * ld + p];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = 0.f;
    for (int bi = 0; bi < n_bands; ++bi) {
      const BandDesc bd = cptr(bands)[bi];
      if (bd.op != OP_GP) continue;
      float y, w;
      decode_obs(bd, p, y, w);
      if (!(w > 0.f)) continue;
      float f, Hs[NT];
      if (!gp_hessian_dispatch<NP>(bd, xv, f, Hs)) continue;
      const float s = w * (y - f);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = fmaf(s, Hs[t], acc[t]);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) a[t * ld + p] -= acc[t];
  }
}

// Output unpack (observations.py:374-376, 392-393): mean and 1/sqrt(diag(P^-1))
// scattered onto the raster; idx==nullptr means the identity map.
template <int NP>
__global__ __launch_bounds__(BLOCK) void unpack_kernel(const float* x, const float* a, int64_t N, int64_t ld,
                                                      const int64_t* idx, float* mean, float* unc,
                                                      int64_t plane) {
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  for (int64_t p = (int64_t)blockIdx.x * BLOCK + threadIdx.x; p < N; p += stride) {
    const int64_t r = idx ? idx[p] : p;
    KF_DCHECK(r >= 0 && r < plane);
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      if (mean) mean[j * plane + r] = x[j * ld + p];
      if (unc) unc[j * plane + r] = kf_rsqrt(a[tri(NP, j, j) * ld + p]);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(BLOCK) void gather_kernel(const T* src, const int64_t* idx, T* dst, int64_t n,
                                                      int rows, int64_t src_ld, int64_t dst_ld) {
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  for (int64_t p = (int64_t)blockIdx.x * BLOCK + threadIdx.x; p < n; p += stride) {
    const int64_t s = idx[p];  // s < 0: no source pixel (a warp's uncovered target) -> 0 = no data
    KF_DCHECK(s < src_ld);
    for (int r = 0; r < rows; ++r) dst[r * dst_ld + p] = s >= 0 ? src[r * src_ld + s] : T(0);
  }
}

// ---------------------------------------------------------------------------
// launchers
inline int grid_for(int64_t N, int max_blocks) {
  int64_t g = (N + BLOCK - 1) / BLOCK;
  if (g > max_blocks) g = max_blocks;
  if (g < 1) g = 1;
  return (int)g;
}

#define KF_NP_SWITCH(np, FN, ...)                 \
  switch (np) {                                   \
    case 1: FN<1>(__VA_ARGS__); break;            \
    case 2: FN<2>(__VA_ARGS__); break;            \
    case 3: FN<3>(__VA_ARGS__); break;            \
    case 4: FN<4>(__VA_ARGS__); break;            \
    case 7: FN<7>(__VA_ARGS__); break;            \
    case 10: FN<10>(__VA_ARGS__); break;          \
    default: return hipErrorInvalidValue;         \
  }

// Interleaved exponent MFMAs (gpm_chunk IL: both column blocks' exponent
// MFMAs before the first block's exponentials) by default where the second
// live block costs no waves per SIMD and no scratch (ISA lint,
// tests/test_isa_lint.py): the JRC-TIP layout kernel (156 -> 168 VGPRs, 3
// waves either way) and 10-parameter states (2 waves either way); +0.5% tip7,
// +1.0% prosail10 interleaved on one box (profiles/r4_v2_ab_fixed_tip7T.jsonl).
// Elsewhere (7-parameter runtime layout: 8-24 B scratch; 3-4 parameters: 4 ->
// 3 waves) the block-by-block order stays.
template <int NP, int LAYOUT>
constexpr bool gpm_il_default() {
  return (NP == 7 && LAYOUT == BAND_LAYOUT_TIP) || NP >= 10;
}

// Launch of a matrix-core analysis kernel on the static grid-stride mapping
// (partials per workgroup; the hardware dispatcher hands a finished
// workgroup's slot to the next one, which balances the cloud-skip load).
// Round 5's persistent tile queue with per-XCD counters measured within
// 0.5 % of it at 10980^2, 3882^2 and for PROSAIL and was removed in round 6.
// *n_part: the partial entries written.
template <typename KernT>
static void launch_tiles(KernT kernel, int bs, size_t lds, const AnalysisArgs& a, int grid, hipStream_t s,
                         int* n_part) {
  *n_part = grid;
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(bs), lds, s, a);
}

template <int NP, int FD>
static bool l_analysis_fast(const AnalysisArgs& a, int grid, hipStream_t s, int* n_part) {
  *n_part = grid;
  // GP on the matrix cores when the host attached split-f16 tables to every band
  // (AV_VALU_ORACLE: the f32 VALU record loop, the tests' second device path)
  if constexpr (FD > 0 && FD <= GPM_MAX_D) {
    if (a.gpm_frags > 0 && a.variant != AV_VALU_ORACLE && a.n_bands <= GPM_MAX_BANDS) {
      const size_t lds = (size_t)a.gpm_frags * sizeof(kf_h8);
#define KF_MFMA_GO1(OBS_, BS_, MINW_, LAY_, IL_, SPEC_)                                                        \
  {                                                                                                           \
    gpm_lds_attr(analysis_mfma_kernel<NP, FD, OBS_, BS_, MINW_, LAY_, IL_, SPEC_>, lds);                      \
    launch_tiles(analysis_mfma_kernel<NP, FD, OBS_, BS_, MINW_, LAY_, IL_, SPEC_>, BS_, lds, a, grid, s, n_part); \
  }
      // Both column blocks' exponent MFMAs issued before the first block's
      // exponentials (gpm_chunk IL) where that costs no occupancy
      // (gpm_il_default); AV_BLOCK_ORDER: the other order
#define KF_MFMA_GO(OBS_, BS_, MINW_, LAY_)                                   \
  {                                                                         \
    if (gpm_il_default<NP, LAY_>() != (a.variant == AV_BLOCK_ORDER))        \
      KF_MFMA_GO1(OBS_, BS_, MINW_, LAY_, true, SPEC_ANY)                   \
    else KF_MFMA_GO1(OBS_, BS_, MINW_, LAY_, false, SPEC_ANY)               \
  }
      // JRC-TIP layout with the forecast fused (every date after the first):
      // the launch's paths fixed at compile time (SPEC_PROP / SPEC_PROP_REG,
      // kf_core.h); AV_GENERIC_SPEC: the generic kernel
#define KF_MFMA_GO_SPEC(OBS_, BS_, MINW_, LAY_)                                                      \
  {                                                                                                 \
    constexpr bool IL_ = gpm_il_default<NP, LAY_>();                                                \
    if (!a.prop || a.variant == AV_BLOCK_ORDER || a.variant == AV_GENERIC_SPEC)                     \
      KF_MFMA_GO(OBS_, BS_, MINW_, LAY_)                                                            \
    else if (a.reg_v) KF_MFMA_GO1(OBS_, BS_, MINW_, LAY_, IL_, SPEC_PROP_REG)                      \
    else if (small) KF_MFMA_GO1(OBS_, BS_, MINW_, LAY_, IL_, SPEC_PROP_PF)                          \
    else KF_MFMA_GO1(OBS_, BS_, MINW_, LAY_, IL_, SPEC_PROP)                                        \
  }
      // Launch bound of 3 workgroups per CU (MINW = 3, as the LDS tables
      // allow) up to 7 parameters: the compiler holds the kernel to <= 168
      // VGPRs itself (A/B neutral against landing there unconstrained,
      // profiles/r3_v13_*); 10 parameters would spill, so no bound there.
      constexpr int MW = NP <= 7 ? 3 : 1;
      // JRC-TIP band layout (AnalysisArgs.band_layout, checked on the host):
      // band loop unrolled over the two compile-time maps (AV_RUNTIME_LAYOUT:
      // the runtime-layout kernel, its oracle)
      bool tip = false;
      // small emulators (<= 4 chunks of 32 training points per band): the GP
      // loop is too short to hide the next group's forecast loads, so the
      // SPEC_PROP_PF kernel loads them ahead (T = 32: -2.2 %; at T = 500 the
      // extra registers cost +0.5 %, profiles/r5_forecast_prefetch_ab.jsonl)
      const bool small = a.gpm_frags <= 4 * a.n_bands * gpm_frags_per_chunk(FD) + 1;
      (void)small;
      if constexpr (NP == 7 && FD == 4)
        tip = a.band_layout == BAND_LAYOUT_TIP && a.n_bands == 2 && a.variant != AV_RUNTIME_LAYOUT;
      if (a.fast_obs == OBS_DN16) {
        if constexpr (NP == 7 && FD == 4) {
          if (tip) {
            KF_MFMA_GO_SPEC(OBS_DN16, BLOCK, 3, BAND_LAYOUT_TIP)
            return true;
          }
        }
        KF_MFMA_GO(OBS_DN16, BLOCK, MW, BAND_LAYOUT_RUNTIME)
      } else if (a.fast_obs == OBS_F32) {
        if constexpr (NP == 7 && FD == 4) {
          if (tip) {
            KF_MFMA_GO(OBS_F32, BLOCK, 3, BAND_LAYOUT_TIP)
            return true;
          }
        }
        KF_MFMA_GO(OBS_F32, BLOCK, MW, BAND_LAYOUT_RUNTIME)
      } else {
        return false;
      }
#undef KF_MFMA_GO_SPEC
#undef KF_MFMA_GO
#undef KF_MFMA_GO1
      return true;
    }
    if constexpr (FD == NP && NP >= 7) {
      if (a.gpm_global && a.variant != AV_VALU_ORACLE) {
        // AV_GT_PREFETCH: register double buffer (next chunk's fragments
        // loaded under the current one): 191.7 vs 191.6 ms/step without, so
        // the default leaves the latency to the other wave
        constexpr bool IL = gpm_il_default<NP, BAND_LAYOUT_RUNTIME>();
        if (a.fast_obs == OBS_DN16 && a.variant == AV_GT_PREFETCH)
          launch_tiles(analysis_mfma_g_kernel<NP, FD, OBS_DN16, true>, BLOCK, 0, a, grid, s, n_part);
        else if (a.fast_obs == OBS_DN16 && a.prop && !a.reg_v && a.variant == AV_DEFAULT && IL)
          // fused forecast, no regulariser: the launch's paths fixed at compile time (SPEC_PROP)
          launch_tiles(analysis_mfma_g_kernel<NP, FD, OBS_DN16, false, true, SPEC_PROP>, BLOCK, 0, a, grid, s, n_part);
        else if (a.fast_obs == OBS_DN16 && (a.variant == AV_BLOCK_ORDER) != IL)
          launch_tiles(analysis_mfma_g_kernel<NP, FD, OBS_DN16, false, true>, BLOCK, 0, a, grid, s, n_part);
        else if (a.fast_obs == OBS_DN16)
          launch_tiles(analysis_mfma_g_kernel<NP, FD, OBS_DN16>, BLOCK, 0, a, grid, s, n_part);
        else if (a.fast_obs == OBS_F32)
          launch_tiles(analysis_mfma_g_kernel<NP, FD, OBS_F32, false, IL>, BLOCK, 0, a, grid, s, n_part);
        else
          return false;
        return true;
      }
    }
  }
  if (a.fast_obs == OBS_DN16) {
    hipLaunchKernelGGL((analysis_kernel<NP, FD, OBS_DN16>), dim3(grid), dim3(BLOCK), 0, s, a);
  } else if (a.fast_obs == OBS_F32) {
    hipLaunchKernelGGL((analysis_kernel<NP, FD, OBS_F32>), dim3(grid), dim3(BLOCK), 0, s, a);
  } else if constexpr (FD <= 0) {
    // bf16 (y, w) observations: precomputed / linear operators only
    if (a.fast_obs == OBS_BF16)
      hipLaunchKernelGGL((analysis_kernel<NP, FD, OBS_BF16>), dim3(grid), dim3(BLOCK), 0, s, a);
    else if (a.fast_obs == OBS_BF16Y)
      hipLaunchKernelGGL((analysis_kernel<NP, FD, OBS_BF16Y>), dim3(grid), dim3(BLOCK), 0, s, a);
    else
      return false;
  } else {
    return false;
  }
  return true;
}

// Fast-path instantiations: JRC-TIP (7 params, 4-input band GPs), PROSAIL
// (10 params, full-state GPs) and full-state GPs for small states.
template <int NP>
static void l_analysis(const AnalysisArgs& a, int grid, hipStream_t s, int* n_part) {
  bool done = false;
  *n_part = grid;
  if (a.fast_d > 0) {
    if constexpr (NP == 7) {
      if (a.fast_d == 4) done = l_analysis_fast<7, 4>(a, grid, s, n_part);
      else if (a.fast_d == 7) done = l_analysis_fast<7, 7>(a, grid, s, n_part);
    } else if constexpr (NP == 10) {
      if (a.fast_d == 10) done = l_analysis_fast<10, 10>(a, grid, s, n_part);
    } else if constexpr (NP <= 4) {
      if (a.fast_d == NP) done = l_analysis_fast<NP, NP>(a, grid, s, n_part);
    }
  }
  else if (a.fast_d == FD_PRECOMP) {
    done = l_analysis_fast<NP, FD_PRECOMP>(a, grid, s, n_part);
  } else if (a.fast_d == FD_LINEAR) {
    done = l_analysis_fast<NP, FD_LINEAR>(a, grid, s, n_part);
  }
  if (!done) {
    *n_part = grid;
    hipLaunchKernelGGL(analysis_kernel<NP>, dim3(grid), dim3(BLOCK), 0, s, a);
  }
}
}  // namespace kf
