// kf_gp_mfma.h — GP emulator operator + Jacobian on the gfx950 matrix cores.
//
// The GP sums of kf_core.h (gp_eval) for a wave's 64 pixels are two GEMMs
// over the T training points (replaces utils.py:181-219 + gp.predict):
//   E[i][p]  = L'_i + c_p + sum_d B_id x_pd                    (exponent, K = D)
//   m[i][p]  = 2^E[i][p]                                        (v_exp_f32)
//   S[f][p]  = sum_i A[f][i] m[i][p],  A = [sgn_i; sgn_i B_i]   (K = T)
// Both run on v_mfma_f32_32x32x16_f16 with split-f16 operands (v = hi + lo,
// hi = f16(v), lo = f16(v - hi); products hi.hi + hi.lo + lo.hi accumulated in
// f32): 22 significant bits per operand, as accurate as the f32 VALU loop it
// replaces (scripts/sim_gp_mfma_precision.py).  The exponent comes out of the
// accumulator in f32; only v_exp and the hi/lo split of m stay on the VALU.
//
// Layout (lane l, h = l >> 5, col = l & 31; fragment element j = K index 8h + j
// of a 16-wide K step; C row of accumulator register r = (r&3) + 8(r>>2) + 4h):
//   exponent  A rows = 32 training points, B cols = 32 pixels, K slots
//             [Bh(D) | Bl(D) | Bh(D) | L'h | L'l | 1 | 1 | 0..] x
//             [xh(D) | xh(D) | xl(D) | 1   | 1   | ch | cl | 0..]   (ceil((3D+4)/16) K steps)
//             -> lane l holds E of pixel col at points (r&3) + 8(r>>2) + 4h, r = 0..15
//   sums      A rows = fields (S0, S'_1..S'_D; rows > D unused), B cols = 32 pixels,
//             two K = 16 halves q: K slot 8h + j <-> point (j&3) + 4h + 8(j>>2) + 16q,
//             i.e. exactly accumulator registers 8q .. 8q+7 of the exponent MFMA.
// Host tables (models/gp.py: mfma_tables), per 32-point chunk: the exponent A
// fragments of every lane, then for q = 0, 1 the hi and lo sums A fragments of
// the lanes with row <= D.  A band's table is staged in LDS once per
// workgroup.  m is kept <= 2^14 (f16 range) by a per-band power-of-two shift
// folded into L' and undone on S (BandDesc.gpm_scale).
#pragma once
#include <hip/hip_runtime.h>
#include "kf_core.h"

namespace kf {

typedef _Float16 kf_h8 __attribute__((ext_vector_type(8)));
typedef float kf_f16v __attribute__((ext_vector_type(16)));
typedef uint32_t kf_u4 __attribute__((ext_vector_type(4)));
typedef __fp16 kf_hp2 __attribute__((ext_vector_type(2)));

// exponent K steps of 16 slots (3D + 4 used)
KF_HD constexpr int gpm_k_steps(int D) { return (3 * D + 4 + 15) / 16; }
// sums fragments per (q, hi/lo): lanes with row <= D in both K halves
KF_HD constexpr int gpm_sum_lanes(int D) { return 2 * (D + 1); }
// 16-byte fragments per 32-point chunk
KF_HD constexpr int gpm_frags_per_chunk(int D) { return 64 * gpm_k_steps(D) + 4 * gpm_sum_lanes(D); }
constexpr int GPM_MAX_D = 10;
// bands whose sums are held across the record loops (larger tables fall back to VALU)
constexpr int GPM_MAX_BANDS = 4;

#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ uint32_t gpm_pack(_Float16 a, _Float16 b) {
  return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
}

// K slot k of the exponent B operand
template <int D>
__device__ __forceinline__ _Float16 gpm_xslot(int k, const _Float16 (&xh)[D], const _Float16 (&xl)[D],
                                              _Float16 ch, _Float16 cl) {
  if (k < D) return xh[k];
  if (k < 2 * D) return xh[k - D];
  if (k < 3 * D) return xl[k - 2 * D];
  if (k < 3 * D + 2) return (_Float16)1.f;
  if (k == 3 * D + 2) return ch;
  if (k == 3 * D + 3) return cl;
  return (_Float16)0.f;
}

template <int D>
__device__ __forceinline__ kf_u4 gpm_xfrag(int k0, const _Float16 (&xh)[D], const _Float16 (&xl)[D], _Float16 ch,
                                           _Float16 cl) {
  kf_u4 v;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    v[q] = gpm_pack(gpm_xslot<D>(k0 + 2 * q, xh, xl, ch, cl), gpm_xslot<D>(k0 + 2 * q + 1, xh, xl, ch, cl));
  return v;
}

// x of lane l ^ 32 (v_permlane32_swap: a VALU op, no LDS round trip; the
// compiler pads its VALU-write hazard itself).  Call it unconditionally from
// every lane and select afterwards: under a divergent branch the swap would
// read inactive partner lanes (fetch-inactive is also set for safety).
__device__ __forceinline__ float gpm_partner32(float x) {
  const unsigned u = __builtin_bit_cast(unsigned, x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, true, false);
  return __builtin_bit_cast(float, (threadIdx.x & 32) ? r[0] : r[1]);
}

__device__ __forceinline__ void gpm_split16(float v, _Float16& h, _Float16& l) {
  h = (_Float16)v;
  l = (_Float16)(v - (float)h);
}

// Exponent B operands (all K steps) of column block `blk` (pixels 32 blk ..
// 32 blk + 31 of the wave).
template <int D>
__device__ __forceinline__ void gpm_operand(const float (&xi)[D], float c, int blk,
                                            kf_h8 (&xb)[gpm_k_steps(D)]) {
  // column col of block blk is pixel 32 blk + col: this lane's own pixel when
  // its half h equals blk, else the pixel of lane l ^ 32
  const bool h1 = (threadIdx.x & 32) != 0;
  const bool own = (h1 ? 1 : 0) == blk;
  _Float16 xh[D], xl[D], ch, cl;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const float pv = gpm_partner32(xi[d]);
    const float v = own ? xi[d] : pv;
    // clamp: f16 range (a state that far out has k = 0 anyway through c)
    gpm_split16(fminf(fmaxf(v, -6.0e4f), 6.0e4f), xh[d], xl[d]);
  }
  const float pc = gpm_partner32(c);
  gpm_split16(fmaxf(own ? c : pc, -6.0e4f), ch, cl);
#pragma unroll
  for (int kk = 0; kk < gpm_k_steps(D); ++kk) {
    const kf_u4 f0 = gpm_xfrag<D>(16 * kk, xh, xl, ch, cl), f1 = gpm_xfrag<D>(16 * kk + 8, xh, xl, ch, cl);
    xb[kk] = __builtin_bit_cast(kf_h8, h1 ? f1 : f0);
  }
}

// Both column blocks' exponent B operands at once (BPP = 2): the lane splits
// and packs its OWN pixel's values into both K halves (F0: slots 16kk..+7,
// F1: 16kk+8..+15) and sends the half its partner l ^ 32 needs, so each value
// is split once and one dword per fragment register crosses the wave halves,
// instead of every raw input being swapped and split again per block.
//   block 0 (pixels 0..31):  lanes h = 0 own F0, lanes h = 1 the partner's F1
//   block 1 (pixels 32..63): lanes h = 0 the partner's F0, lanes h = 1 own F1
template <int D>
__device__ __forceinline__ void gpm_operands(const float (&xi)[D], float c, kf_h8 (&xb)[2][gpm_k_steps(D)]) {
  const bool h1 = (threadIdx.x & 32) != 0;
  _Float16 xh[D], xl[D], ch, cl;
#pragma unroll
  for (int d = 0; d < D; ++d) gpm_split16(fminf(fmaxf(xi[d], -6.0e4f), 6.0e4f), xh[d], xl[d]);
  gpm_split16(fmaxf(c, -6.0e4f), ch, cl);
#pragma unroll
  for (int kk = 0; kk < gpm_k_steps(D); ++kk) {
    const kf_u4 f0 = gpm_xfrag<D>(16 * kk, xh, xl, ch, cl), f1 = gpm_xfrag<D>(16 * kk + 8, xh, xl, ch, cl);
    kf_u4 b0, b1;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // h = 0 sends F1 (its partner's half), h = 1 sends F0
      const uint32_t send = h1 ? f0[q] : f1[q];
      const uint32_t recv = __builtin_bit_cast(uint32_t, gpm_partner32(__builtin_bit_cast(float, send)));
      b0[q] = h1 ? recv : f0[q];
      b1[q] = h1 ? f1[q] : recv;
    }
    xb[0][kk] = __builtin_bit_cast(kf_h8, b0);
    xb[1][kk] = __builtin_bit_cast(kf_h8, b1);
  }
}

// The lane's own pixel (32 h + col) is column col of block h.  Field f of
// that column sits in register (f&3) + 4(f>>3) of lane 32 ((f>>2)&1) + col,
// the lane itself or its partner l ^ 32, so each lane sends the OTHER block's
// value (the one its partner's pixel needs): one exchange per field.
template <int D>
__device__ __forceinline__ void gpm_extract2(const kf_f16v (&acc)[2], float (&S)[D + 1]) {
  const bool h1 = (threadIdx.x & 32) != 0;
#pragma unroll
  for (int f = 0; f <= D; ++f) {
    const int r = (f & 3) + 4 * (f >> 3);
    const float own = h1 ? acc[1][r] : acc[0][r];
    const float send = h1 ? acc[0][r] : acc[1][r];
    const float recv = gpm_partner32(send);
    S[f] = (((f >> 2) & 1) == (h1 ? 1 : 0)) ? own : recv;
  }
}

// m = 2^e for 8 accumulator registers, split into f16 hi (round toward zero)
// and lo = f16(m - hi).
__device__ __forceinline__ void gpm_exp_split(const kf_f16v& e, int r0, kf_h8& mh, kf_h8& ml) {
  kf_u4 hv, lv;
  // two pairs at a time: both low halves, then both high halves (no
  // back-to-back partial writes of one register, which cost an s_nop)
#pragma unroll
  for (int q = 0; q < 4; q += 2) {
    float m[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) m[j] = kexp2(e[r0 + 2 * q + j]);
    hv[q] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(m[0], m[1]));
    hv[q + 1] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(m[2], m[3]));
    // lo = f16(m - hi) with mixed-precision FMAs (-hi * 1 + m): v_fma_mix reads
    // hi as f16 straight from the packed register
    asm volatile("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lv[q]) : "v"(hv[q]), "v"(m[0]));
    asm volatile("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lv[q + 1]) : "v"(hv[q + 1]), "v"(m[2]));
    asm volatile("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
                 : "+v"(lv[q]) : "v"(hv[q]), "v"(m[1]));
    if (q == 0) {
      asm volatile("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
                   : "+v"(lv[q + 1]) : "v"(hv[q + 1]), "v"(m[3]));
    } else {
      // last writer of the MFMA B operand ml: VALU write -> MFMA SrcB read needs
      // 2 wait states, and hipcc pads only one after an asm statement
      asm volatile("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\ts_nop 1"
                   : "+v"(lv[q + 1]) : "v"(hv[q + 1]), "v"(m[3]));
    }
  }
  mh = __builtin_bit_cast(kf_h8, hv);
  ml = __builtin_bit_cast(kf_h8, lv);
}

// Wave-cooperative GP sums for the 64 pixels of the wave (lane = pixel).
// tab: the band's fragments (LDS), nchunk 32-point chunks.  Returns the lane's
// S[0] = sum sgn m, S[1 + d] = sum sgn m B_d, unscaled.  Every lane of the wave
// must call it (MFMA); lanes without an observation pass any finite x.
// BPP = column blocks (of 32 pixels) per pass sharing each chunk's A fragments.
template <int D, int BPP = 2>
__device__ __forceinline__ void gp_mfma_sums(const kf_h8* __restrict__ tab, const kf_h8* __restrict__ zf, int nchunk,
                                             const float (&xi)[D], float c, float (&S)[D + 1]) {
  static_assert(D >= 1 && D <= GPM_MAX_D, "GP input count for the matrix-core path");
  static_assert(BPP == 1 || BPP == 2, "column blocks per pass");
  constexpr int NK = gpm_k_steps(D), NLS = gpm_sum_lanes(D), FPC = gpm_frags_per_chunk(D);
  const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31;
  // sums fragments of this lane; rows > D read the shared zero fragment zf
  // (stride 0): no exec-mask branch, and zero rows keep the matrix cores'
  // switching energy (and so the DVFS clock penalty) down
  const bool ls = col <= D;
  const kf_h8* sp = ls ? tab + 64 * NK + h * (D + 1) + col : zf;
  const int sstep = ls ? FPC : 0, soff = ls ? NLS : 0;
  const kf_f16v zero = {};
#pragma unroll
  for (int f = 0; f <= D; ++f) S[f] = 0.f;
  for (int pass = 0; pass < 2 / BPP; ++pass) {
    kf_h8 xb[BPP][NK];
    kf_f16v acc[BPP];
    if constexpr (BPP == 2) {
      gpm_operands<D>(xi, c, xb);
    } else {
#pragma unroll
      for (int i = 0; i < BPP; ++i) gpm_operand<D>(xi, c, pass * BPP + i, xb[i]);
    }
#pragma unroll
    for (int i = 0; i < BPP; ++i) acc[i] = zero;
    // (a software-pipelined order -- next chunk's exponent MFMAs between the two
    // K halves -- removes the s_nop padding but measured 4-7 % slower: more
    // VGPRs, fewer waves; the other waves already fill the MFMA latency)
    for (int ch = 0; ch < nchunk; ++ch) {
      const kf_h8* t = tab + ch * FPC;
      kf_h8 ea[NK], sa[2][2];
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) ea[kk] = t[64 * kk + lane];
      const kf_h8* st = sp + ch * sstep;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        sa[q][0] = st[(2 * q) * soff];
        sa[q][1] = st[(2 * q + 1) * soff];
      }
#pragma unroll
      for (int i = 0; i < BPP; ++i) {
        kf_f16v e = __builtin_amdgcn_mfma_f32_32x32x16_f16(ea[0], xb[i][0], zero, 0, 0, 0);
#pragma unroll
        for (int kk = 1; kk < NK; ++kk) e = __builtin_amdgcn_mfma_f32_32x32x16_f16(ea[kk], xb[i][kk], e, 0, 0, 0);
        kf_h8 mh[2], ml[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          gpm_exp_split(e, 8 * q, mh[q], ml[q]);
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(sa[q][0], mh[q], acc[i], 0, 0, 0);
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(sa[q][0], ml[q], acc[i], 0, 0, 0);
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(sa[q][1], mh[q], acc[i], 0, 0, 0);
        }
      }
    }
    // field f of pixel 32 blk + col sits in register (f&3) + 4(f>>3) of lane
    // 32 ((f>>2)&1) + col: the lane itself or its partner l ^ 32
    if constexpr (BPP == 2) {
      gpm_extract2<D>(acc, S);
    } else {
#pragma unroll
      for (int i = 0; i < BPP; ++i) {
        const int blk = pass * BPP + i;
#pragma unroll
        for (int f = 0; f <= D; ++f) {
          const float mine = acc[i][(f & 3) + 4 * (f >> 3)];
          const float theirs = gpm_partner32(mine);
          const float v = (((f >> 2) & 1) == h) ? mine : theirs;
          S[f] = h == blk ? v : S[f];
        }
      }
    }
  }
}

// The same sums with the band's table read from global memory (L2-resident:
// used when the tables of all bands do not fit the 160 KiB of LDS, e.g. ten
// PROSAIL bands).  The next chunk's fragments are loaded while the current one
// runs (register double buffer), so the L2 latency sits under the exp/MFMA
// work of the chunk.  tab + nchunk * FPC holds a zero fragment (models/gp.py).
typedef const __attribute__((address_space(1))) kf_h8* kf_gtab;

template <int D, int BPP = 2, bool PF = true>
__device__ __forceinline__ void gp_mfma_sums_g(const void* tab_, int nchunk, const float (&xi)[D], float c,
                                               float (&S)[D + 1]) {
  static_assert(D >= 1 && D <= GPM_MAX_D, "GP input count for the matrix-core path");
  static_assert(BPP == 2, "global-table path: both column blocks per pass");
  constexpr int NK = gpm_k_steps(D), NLS = gpm_sum_lanes(D), FPC = gpm_frags_per_chunk(D);
  const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31;
  const kf_gtab tab = (kf_gtab)tab_;
  const bool ls = col <= D;
  const kf_gtab sp = ls ? tab + 64 * NK + h * (D + 1) + col : tab + (int64_t)nchunk * FPC;
  const int sstep = ls ? FPC : 0, soff = ls ? NLS : 0;
  const kf_f16v zero = {};
#pragma unroll
  for (int f = 0; f <= D; ++f) S[f] = 0.f;
  kf_h8 xb[2][NK];
  kf_f16v acc[2];
  gpm_operands<D>(xi, c, xb);
#pragma unroll
  for (int i = 0; i < 2; ++i) acc[i] = zero;
  kf_h8 ea[NK], sa[2][2];
  if constexpr (PF) {
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) ea[kk] = tab[64 * kk + lane];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      sa[q][0] = sp[(2 * q) * soff];
      sa[q][1] = sp[(2 * q + 1) * soff];
    }
  }
  for (int ch = 0; ch < nchunk; ++ch) {
    // prefetch chunk ch + 1 (the last chunk re-reads itself); PF = false: load
    // chunk ch here (no register double buffer, the waves hide the latency)
    const int nx = PF ? (ch + 1 < nchunk ? ch + 1 : ch) : ch;
    const kf_gtab t = tab + (int64_t)nx * FPC;
    const kf_gtab st = sp + (int64_t)nx * sstep;
    kf_h8 ean[NK], san[2][2];
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) ean[kk] = t[64 * kk + lane];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      san[q][0] = st[(2 * q) * soff];
      san[q][1] = st[(2 * q + 1) * soff];
    }
    if constexpr (!PF) {
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) ea[kk] = ean[kk];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        sa[q][0] = san[q][0];
        sa[q][1] = san[q][1];
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      kf_f16v e = __builtin_amdgcn_mfma_f32_32x32x16_f16(ea[0], xb[i][0], zero, 0, 0, 0);
#pragma unroll
      for (int kk = 1; kk < NK; ++kk) e = __builtin_amdgcn_mfma_f32_32x32x16_f16(ea[kk], xb[i][kk], e, 0, 0, 0);
      kf_h8 mh[2], ml[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        gpm_exp_split(e, 8 * q, mh[q], ml[q]);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(sa[q][0], mh[q], acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(sa[q][0], ml[q], acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(sa[q][1], mh[q], acc[i], 0, 0, 0);
      }
    }
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) ea[kk] = ean[kk];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      sa[q][0] = san[q][0];
      sa[q][1] = san[q][1];
    }
  }
  gpm_extract2<D>(acc, S);
}

#endif

}  // namespace kf

namespace kf {
#if defined(__HIP_DEVICE_COMPILE__)
// K1 on the matrix cores: pixel_analysis (kf_core.h) with lane = pixel and the
// GP sums of every band evaluated wave-cooperatively by gp_mfma_sums.  All 64
// lanes run the band loop (act = false for the tail lanes past N: clamped
// reads, no stores); the GP is skipped only when no lane of the wave has an
// observation of the band (wave-level cloud skip).
// (A two-phase variant -- every band's GP sums first, the forecast precision
// and normal equations afterwards, 8 fewer VGPRs -- gave intermittently wrong
// pixels on some waves under full occupancy on MI355X while this order never
// did (scripts/debug_mfma_tiles.py, r2 bisect); tests/test_gpu_mfma.py
// ::test_gp_mfma_realistic_tile_matches_valu guards it.)
// Centred GP inputs and the exponent constant sum_d lambda_d xi_d^2 of a band.
// A full-state GP (map[d] == d, wave-uniform flag) reads x0 directly; other
// maps select through gather_state (NP - 1 v_cndmask per input).
template <int NP, int D>
__device__ __forceinline__ void gpm_inputs(const KF_CONST_AS BandDesc* bdp, const float (&x0)[NP], float (&xi)[D],
                                           float& c) {
  if (bdp->map_identity) {
#pragma unroll
    for (int d = 0; d < D; ++d) xi[d] = x0[d < NP ? d : NP - 1] - bdp->center[d];
  } else {
#pragma unroll
    for (int d = 0; d < D; ++d) xi[d] = gather_state<NP>(x0, bdp->map[d]) - bdp->center[d];
  }
#pragma unroll
  for (int d = 0; d < D; ++d) c = fmaf(bdp->coef[d] * xi[d], xi[d], c);
}

// gp_epilogue with the same identity-map shortcut (h[d] = g_d, no scatter).
template <int NP, int D>
__device__ __forceinline__ void gpm_epilogue(const KF_CONST_AS BandDesc* q, const float (&xi)[D], float S0,
                                             const float (&S)[D], float& H0, float (&h)[NP]) {
  if (q->map_identity) {
    H0 = q->offset + S0;
#pragma unroll
    for (int j = 0; j < NP; ++j) h[j] = 0.f;
#pragma unroll
    for (int d = 0; d < D && d < NP; ++d) h[d] = fmaf(-q->coef[d] * xi[d], S0, LN2 * S[d]);
  } else {
    gp_epilogue<NP, D>(q->offset, q->coef, q->map, xi, S0, S, H0, h);
  }
}

template <int NP, int D, int FOBS, int BPP = 2, int NBM = 2, bool GT = false, bool PF = true>
__device__ __forceinline__ float pixel_analysis_mfma(const AnalysisArgs& a, int64_t p, bool act,
                                                     const kf_h8* lds) {
  constexpr int NT = ntri(NP);
  const int64_t ld = a.ld;
  float x0[NP], A[NT], b[NP];
  uint8_t st = 0;
  if (a.x_prev) {
#pragma unroll
    for (int j = 0; j < NP; ++j) x0[j] = a.x_prev[j * ld + p];
  }
  if (a.prop) {
    float xf[NP];
    forecast_partial<NP>(opaque(cptr(a.prop)), p, xf, A);
    symv<NP>(A, xf, b);
    if (!a.x_prev) {
#pragma unroll
      for (int j = 0; j < NP; ++j) x0[j] = xf[j];
    }
  } else if (a.a_in) {
#pragma unroll
    for (int t = 0; t < NT; ++t) A[t] = a.a_in[t * ld + p];
#pragma unroll
    for (int j = 0; j < NP; ++j) b[j] = a.b_in[j * ld + p];
  } else {
    float xf[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) xf[j] = a.x_f[j * ld + p];
#pragma unroll
    for (int t = 0; t < NT; ++t) A[t] = a.pf_inv[t * ld + p];
    symv<NP>(A, xf, b);
  }
  int nobs = 0;
  int off = 0;
  for (int bi = 0; bi < a.n_bands; ++bi) {
    const KF_CONST_AS BandDesc* bdp = cptr(a.bands) + bi;
    float y, w;
    decode_obs<FOBS>(*bdp, p, y, w);
    const bool use = act && (w > 0.f);
    float H0 = 0.f, h[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) h[j] = 0.f;
    bool ok = false;
    const int nch = bdp->gpm_nchunk;
    const bool any = __any(use);
    if (any) {
      float xi[D], c = 0.f;
      gpm_inputs<NP, D>(bdp, x0, xi, c);
      c *= -0.5f * LOG2E;
      float S[D + 1];
      if constexpr (GT) gp_mfma_sums_g<D, BPP, PF>(bdp->gpm, nch, xi, c, S);
      else gp_mfma_sums<D, BPP>(lds + off, lds + a.gpm_frags - 1, nch, xi, c, S);
      const KF_CONST_AS BandDesc* q = opaque(bdp);   // epilogue fields: not live across the chunk loop
      const float sc = q->gpm_scale;
      float Sd[D];
#pragma unroll
      for (int d = 0; d < D; ++d) Sd[d] = S[1 + d] * sc;
      gpm_epilogue<NP, D>(q, xi, S[0] * sc, Sd, H0, h);
      ok = finitef(H0);
#pragma unroll
      for (int j = 0; j < NP; ++j) ok = ok && finitef(h[j]);
    }
    off += nch * gpm_frags_per_chunk(D);
    float* h0o = opaque(bdp)->h0_out;
    if (act && h0o) h0o[p] = use ? H0 : 0.f;
    if (use && !ok) st |= ST_BAD_OP;
    if (use && ok) {
      ++nobs;
      float yp = y - H0;
#pragma unroll
      for (int j = 0; j < NP; ++j) yp = fmaf(h[j], x0[j], yp);
      const float wy = w * yp;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const float wh = w * h[i];
        b[i] = fmaf(h[i], wy, b[i]);
#pragma unroll
        for (int j = i; j < NP; ++j) A[tri(NP, i, j)] = fmaf(wh, h[j], A[tri(NP, i, j)]);
      }
    }
  }
  if (nobs == 0) st |= ST_NO_OBS;
  if (!act) return 0.f;
  const KF_CONST_AS AnalysisArgs* ka =
      opaque((const KF_CONST_AS AnalysisArgs*)__builtin_amdgcn_kernarg_segment_ptr());
  return analysis_epilogue<NP>(ka, p, A, b, x0, st);
}

// K1g (gain / covariance form) with the GP on the matrix cores: pixel_gain
// (kf_core.h) with lane = pixel, the band's GP sums wave-cooperative as in
// pixel_analysis_mfma, then the same scalar-band update and tail.
template <int NP, int D, int FOBS>
__device__ __forceinline__ float pixel_gain_mfma(const GainArgs& a, int64_t p, bool act, const kf_h8* lds) {
  constexpr int NT = ntri(NP);
  const int64_t ld = a.ld;
  float x0[NP], x[NP], P[NT];
  uint8_t st = 0;
  if (a.prop) {
    st |= forecast_partial_cov<NP>(opaque(cptr(a.prop)), p, x, P);
  } else {
#pragma unroll
    for (int j = 0; j < NP; ++j) x[j] = a.x_f[j * ld + p];
#pragma unroll
    for (int t = 0; t < NT; ++t) P[t] = a.p_f[t * ld + p];
  }
  if (a.x_prev) {
#pragma unroll
    for (int j = 0; j < NP; ++j) x0[j] = a.x_prev[j * ld + p];
  } else {
#pragma unroll
    for (int j = 0; j < NP; ++j) x0[j] = x[j];
  }
  int nobs = 0;
  int off = 0;
  for (int bi = 0; bi < a.n_bands; ++bi) {
    const KF_CONST_AS BandDesc* bdp = cptr(a.bands) + bi;
    float y, w;
    decode_obs<FOBS>(*bdp, p, y, w);
    const bool use = act && (w > 0.f);
    float H0 = 0.f, h[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) h[j] = 0.f;
    bool ok = false;
    const int nch = bdp->gpm_nchunk;
    if (__any(use)) {
      float xi[D], c = 0.f;
      gpm_inputs<NP, D>(bdp, x0, xi, c);
      c *= -0.5f * LOG2E;
      float S[D + 1];
      gp_mfma_sums<D, 2>(lds + off, lds + a.gpm_frags - 1, nch, xi, c, S);
      const KF_CONST_AS BandDesc* q = opaque(bdp);
      const float sc = q->gpm_scale;
      float Sd[D];
#pragma unroll
      for (int d = 0; d < D; ++d) Sd[d] = S[1 + d] * sc;
      gpm_epilogue<NP, D>(q, xi, S[0] * sc, Sd, H0, h);
      ok = finitef(H0);
#pragma unroll
      for (int j = 0; j < NP; ++j) ok = ok && finitef(h[j]);
    }
    off += nch * gpm_frags_per_chunk(D);
    float* h0o = opaque(bdp)->h0_out;
    if (act && h0o) h0o[p] = use ? H0 : 0.f;
    if (use && !ok) st |= ST_BAD_OP;
    if (use && ok) {
      ++nobs;
      gain_band_update<NP>(P, x, x0, h, H0, y, w, a.joseph != 0);
    }
  }
  if (!act) return 0.f;
  return gain_finish<NP>(a, p, x, P, x0, st, nobs);
}
#endif
}  // namespace kf
