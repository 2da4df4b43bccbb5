// kf_gp_mfma.h — GP emulator operator + Jacobian on the gfx950 matrix cores.
//
// The GP sums of kf_core.h (gp_eval) for a wave's 64 pixels are two GEMMs
// over the T training points (replaces utils.py:181-219 + gp.predict):
//   E[i][p]  = L'_i + c_p + sum_d B_id x_pd                    (exponent, K = D)
//   m[i][p]  = 2^E[i][p]                                        (v_exp_f32)
//   S[f][p]  = sum_i A[f][i] m[i][p],  A = [sgn_i; sgn_i B_i]   (K = T)
// Both run on v_mfma_f32_32x32x16_f16 with split-f16 operands (v = hi + lo,
// hi = f16(v), lo = f16(v - hi)): 22 significant bits per operand, as
// accurate as the f32 VALU loop it replaces (scripts/sim_gp_mfma_precision.py).
//
// Exponent (A rows = 32 training points, B cols = 32 pixels), K slots
//   [Bh(D) | Bl(D) | Bh(D) | L'h | 1 ] x [xh(D) | xh(D) | xl(D) | 1 | ch]
// (3D + 2 slots: one K step of 16 for D <= 4, two for D <= 10).  The low
// parts of the two constants are not K slots: L'l_i is folded into the sums
// operand on the host (A'_i = A_i 2^L'l_i, exact) and cl_p = c_p - ch_p is
// applied once per pixel afterwards (S *= 2^cl), so E carries only hi parts.
//
// Sums (A rows = fields, B cols = 32 pixels, K = 32 points in two halves q):
// ONE A operand holds both split halves of A' -- hi in rows 0..D, lo in rows
// LO..LO+D (LO = 8 for D <= 7, 16 for D <= 15) -- so per K half two MFMAs,
// [A'h; A'l] x mh and [A'h; A'l] x ml, give all four hi/lo products
// (2 + 2 NK MFMAs per 32 x 32 block instead of 3 + NK with separate hi/lo
// operands: TIP 7 -> 5, PROSAIL 9 -> 6).  Row LO + f sits in the same lane as
// row f, accumulator register + LO/2, so S_f = acc[r_f] + acc[r_f + LO/2]
// needs no lane movement.  K slot 8h + j of half q <-> point (j&3) + 4h +
// 8(j>>2) + 16q, i.e. exactly accumulator registers 8q .. 8q+7 of the
// exponent MFMA (no shuffles between the two GEMMs).
//
// The hi/lo split of m is plain C++ (hipcc selects v_cvt_pkrtz_f16_f32 +
// v_fma_mixlo/mixhi_f16 and inserts the VALU -> MFMA SrcB wait states
// itself; the analysis TUs are built with -fno-slp-vectorize, _build.py, so
// the f32 subtraction is not packed into v_pk_fma_f32 first).
//
// Host tables (models/gp.py: mfma_tables), per 32-point chunk: the exponent A
// fragments of every lane (NK x 64), then for q = 0, 1 and h = 0, 1 the sums
// A fragments of the 2(D+1) lanes whose row is used.  m is kept <= 2^14 (f16
// range) by a per-band power-of-two shift folded into L' and undone on S
// (BandDesc.gpm_scale).
#pragma once
#include <hip/hip_runtime.h>
#include <type_traits>
#include "kf_core.h"

namespace kf {

typedef _Float16 kf_h8 __attribute__((ext_vector_type(8)));
typedef float kf_f16v __attribute__((ext_vector_type(16)));
typedef uint32_t kf_u4 __attribute__((ext_vector_type(4)));
typedef __fp16 kf_hp2 __attribute__((ext_vector_type(2)));

// exponent K steps of 16 slots (3D + 2 used)
KF_HD constexpr int gpm_k_steps(int D) { return (3 * D + 2 + 15) / 16; }
// first row of the lo half of the sums operand
KF_HD constexpr int gpm_lo_row(int D) { return D + 1 <= 8 ? 8 : 16; }
// sums fragments per (q, h): the lanes whose row is used (hi and lo rows)
KF_HD constexpr int gpm_sum_rows(int D) { return 2 * (D + 1); }
// 16-byte fragments per 32-point chunk
KF_HD constexpr int gpm_frags_per_chunk(int D) { return 64 * gpm_k_steps(D) + 4 * gpm_sum_rows(D); }
constexpr int GPM_MAX_D = 10;
// bands whose sums are held across the record loops (larger tables fall back to VALU)
constexpr int GPM_MAX_BANDS = 4;
// waves per workgroup of the global-table kernels (analysis_mfma_g_kernel,
// BLOCK = 256): the sizes of their per-wave LDS transpose buffers
constexpr int GPM_G_WAVES = 4;

#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ uint32_t gpm_pack(_Float16 a, _Float16 b) {
  return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
}

// K slot k of the exponent B operand
template <int D>
__device__ __forceinline__ _Float16 gpm_xslot(int k, const _Float16 (&xh)[D], const _Float16 (&xl)[D],
                                              _Float16 ch) {
  if (k < D) return xh[k];
  if (k < 2 * D) return xh[k - D];
  if (k < 3 * D) return xl[k - 2 * D];
  if (k == 3 * D) return (_Float16)1.f;
  if (k == 3 * D + 1) return ch;
  return (_Float16)0.f;
}

template <int D>
__device__ __forceinline__ kf_u4 gpm_xfrag(int k0, const _Float16 (&xh)[D], const _Float16 (&xl)[D], _Float16 ch) {
  kf_u4 v;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    v[q] = gpm_pack(gpm_xslot<D>(k0 + 2 * q, xh, xl, ch), gpm_xslot<D>(k0 + 2 * q + 1, xh, xl, ch));
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

// Both 32-pixel column blocks' exponent B operands: the lane splits and packs
// its OWN pixel's values into both K halves (F0: slots 16kk..+7, F1:
// 16kk+8..+15) and sends the half its partner l ^ 32 needs, so each value is
// split once and one dword per fragment register crosses the wave halves.
//   block 0 (pixels 0..31):  lanes h = 0 own F0, lanes h = 1 the partner's F1
//   block 1 (pixels 32..63): lanes h = 0 the partner's F0, lanes h = 1 own F1
// cl: the lane's own c - f16(c), applied to its sums afterwards.
template <int D>
__device__ __forceinline__ void gpm_operands(const float (&xi)[D], float c, kf_h8 (&xb)[2][gpm_k_steps(D)],
                                             float& cl) {
  const bool h1 = (threadIdx.x & 32) != 0;
  _Float16 xh[D], xl[D];
#pragma unroll
  for (int d = 0; d < D; ++d) gpm_split16(fminf(fmaxf(xi[d], -6.0e4f), 6.0e4f), xh[d], xl[d]);
  // clamp: f16 range (a state that far out has m = 0 anyway, through cl)
  const _Float16 ch = (_Float16)fmaxf(c, -6.0e4f);
  cl = c - (float)ch;
#pragma unroll
  for (int kk = 0; kk < gpm_k_steps(D); ++kk) {
    const kf_u4 f0 = gpm_xfrag<D>(16 * kk, xh, xl, ch), f1 = gpm_xfrag<D>(16 * kk + 8, xh, xl, ch);
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
// value (the one its partner's pixel needs): one exchange per field.  The lo
// row LO + f of the same field is register + LO/2 of the same lane.
template <int D>
__device__ __forceinline__ void gpm_extract2(const kf_f16v (&acc)[2], float (&S)[D + 1]) {
  constexpr int LR = gpm_lo_row(D) / 2;
  const bool h1 = (threadIdx.x & 32) != 0;
#pragma unroll
  for (int f = 0; f <= D; ++f) {
    const int r = (f & 3) + 4 * (f >> 3);
    const float a0 = acc[0][r] + acc[0][r + LR], a1 = acc[1][r] + acc[1][r + LR];
    const float own = h1 ? a1 : a0;
    const float send = h1 ? a0 : a1;
    const float recv = gpm_partner32(send);
    S[f] = (((f >> 2) & 1) == (h1 ? 1 : 0)) ? own : recv;
  }
}

// gpm_extract2 through LDS, for the global-table kernels (whose LDS is
// otherwise unused): each lane adds its own hi and lo rows (the same adds) and
// stores its fields of both column blocks, [block][column][field], then reads
// its own pixel's D + 1 fields back -- 2 G ds_write_b128 + ceil((D+1)/4)
// ds_read_b128 per band instead of ~6 VALU per field (own/partner selects and
// the wave-half swap).  Bit-identical to gpm_extract2.  LDS of one wave: the
// ds ops of a wave execute in order, so the wave barriers (no instruction:
// they only stop the compiler moving the accesses across) suffice.
template <int D>
__device__ __forceinline__ void gpm_extract_lds(const kf_f16v (&acc)[2], float (&S)[D + 1], float* wbuf) {
  constexpr int LR = gpm_lo_row(D) / 2;
  constexpr int G = (D + 1 + 7) / 8;   // 8-row groups holding fields 0..D
  const int lane = threadIdx.x & 63, n = lane & 31, q = lane >> 5;
  typedef float f4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      // fields 8g + 4q + i of column n sit in register 4g + i (hi row) and
      // 4g + i + LR (lo row) of this lane
      f4 v;
      v.x = acc[blk][4 * g + 0] + acc[blk][4 * g + 0 + LR];
      v.y = acc[blk][4 * g + 1] + acc[blk][4 * g + 1 + LR];
      v.z = acc[blk][4 * g + 2] + acc[blk][4 * g + 2 + LR];
      v.w = acc[blk][4 * g + 3] + acc[blk][4 * g + 3 + LR];
      *(f4*)(wbuf + (blk * 32 + n) * 16 + 8 * g + 4 * q) = v;
    }
  }
  __builtin_amdgcn_wave_barrier();
  const f4* src = (const f4*)(wbuf + (q * 32 + n) * 16);   // own pixel 32 q + n: column n of block q
#pragma unroll
  for (int f4i = 0; f4i < (D + 4) / 4; ++f4i) {
    const f4 v = src[f4i];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (4 * f4i + i <= D) S[4 * f4i + i] = v[i];
  }
  __builtin_amdgcn_wave_barrier();
}

// m = 2^e for 8 accumulator registers, split into f16 hi (round toward zero)
// and lo = f16(m - hi).  lo is fma(hi, -1, m) with the -1 in an SGPR the
// optimiser cannot see through, so it stays an FMA with an f16-extended
// operand and a rounded f16 result: v_fma_mixlo/mixhi_f16, one instruction
// per element (a visible -1 folds to an f32 subtraction plus conversions).
__device__ __forceinline__ void gpm_exp_split(const kf_f16v& e, int r0, float neg1, kf_h8& mh, kf_h8& ml) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float m0 = kexp2(e[r0 + 2 * q]), m1 = kexp2(e[r0 + 2 * q + 1]);
    const kf_hp2 hp = __builtin_amdgcn_cvt_pkrtz(m0, m1);
    const _Float16 h0 = (_Float16)hp[0], h1 = (_Float16)hp[1];
    mh[2 * q] = h0;
    mh[2 * q + 1] = h1;
    ml[2 * q] = (_Float16)__builtin_fmaf((float)h0, neg1, m0);
    ml[2 * q + 1] = (_Float16)__builtin_fmaf((float)h1, neg1, m1);
  }
}

__device__ __forceinline__ float gpm_neg1() {
  float v = -1.0f;
  asm volatile("" : "+s"(v));   // opaque SGPR -1 (see gpm_exp_split)
  return v;
}

// The sums operand lane: compact row index of lane column `col`, or -1 (the
// lane reads the shared zero fragment).
template <int D>
__device__ __forceinline__ int gpm_sum_row(int col) {
  constexpr int LO = gpm_lo_row(D);
  return col <= D ? col : ((col >= LO && col <= LO + D) ? D + 1 + (col - LO) : -1);
}

// One 32-point chunk for both column blocks: exponent, split, packed sums.
// FIRST: the first chunk starts the sums from a zero accumulator operand (an
// inline constant of the MFMA) instead of 32 zeroed registers.
// IL: both column blocks' exponent MFMAs are issued first, so the second
// block's exponent runs on the matrix cores under the first block's
// exponentials and split (one more 16-register accumulator live).
template <int D, bool FIRST = false, bool IL = false>
__device__ __forceinline__ void gpm_chunk(const kf_h8 (&ea)[gpm_k_steps(D)], const kf_h8 (&sa)[2],
                                          const kf_h8 (&xb)[2][gpm_k_steps(D)], float neg1, kf_f16v (&acc)[2]) {
  constexpr int NK = gpm_k_steps(D);
  const kf_f16v zero = {};
  if constexpr (IL) {
    kf_f16v e[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      e[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ea[0], xb[i][0], zero, 0, 0, 0);
#pragma unroll
      for (int kk = 1; kk < NK; ++kk) e[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ea[kk], xb[i][kk], e[i], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        kf_h8 mh, ml;
        gpm_exp_split(e[i], 8 * q, neg1, mh, ml);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(sa[q], mh, (FIRST && q == 0) ? zero : acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(sa[q], ml, acc[i], 0, 0, 0);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    kf_f16v e = __builtin_amdgcn_mfma_f32_32x32x16_f16(ea[0], xb[i][0], zero, 0, 0, 0);
#pragma unroll
    for (int kk = 1; kk < NK; ++kk) e = __builtin_amdgcn_mfma_f32_32x32x16_f16(ea[kk], xb[i][kk], e, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      kf_h8 mh, ml;
      gpm_exp_split(e, 8 * q, neg1, mh, ml);
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(sa[q], mh, (FIRST && q == 0) ? zero : acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(sa[q], ml, acc[i], 0, 0, 0);
    }
  }
}

// Wave-cooperative GP sums for the 64 pixels of the wave (lane = pixel).
// tab: the band's fragments (LDS), nchunk 32-point chunks, zf: a zero
// fragment.  Returns the lane's S[0] = sum sgn m, S[1 + d] = sum sgn m B_d,
// unscaled (gpm_scale not applied; 2^cl is).  Every lane of the wave must call
// it (MFMA); lanes without an observation pass any finite x.
template <int D, bool IL = false>
__device__ __forceinline__ void gp_mfma_sums(const kf_h8* __restrict__ tab, const kf_h8* __restrict__ zf, int nchunk,
                                             const float (&xi)[D], float c, float (&S)[D + 1]) {
  static_assert(D >= 1 && D <= GPM_MAX_D, "GP input count for the matrix-core path");
  constexpr int NK = gpm_k_steps(D), NR = gpm_sum_rows(D), FPC = gpm_frags_per_chunk(D);
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int cr = gpm_sum_row<D>(lane & 31);
  // rows not used read the shared zero fragment zf (stride 0): no exec-mask
  // branch, and zero rows keep the matrix cores' switching energy (and so the
  // DVFS clock penalty) down
  const bool ls = cr >= 0;
  const kf_h8* sp = ls ? tab + 64 * NK + h * NR + cr : zf;
  const int sstep = ls ? FPC : 0, soff = ls ? 2 * NR : 0;
  const float neg1 = gpm_neg1();
  kf_h8 xb[2][NK];
  float cl;
  gpm_operands<D>(xi, c, xb, cl);
  kf_f16v acc[2];
  auto load = [&](int ch, kf_h8 (&ea)[NK], kf_h8 (&sa)[2]) {
    const kf_h8* t = tab + ch * FPC;
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) ea[kk] = t[64 * kk + lane];
    const kf_h8* st = sp + ch * sstep;
    sa[0] = st[0];
    sa[1] = st[soff];
  };
  // every table has >= 1 chunk (models/gp.py mfma_tables); the first one is
  // peeled so the sums start from the MFMA's zero operand
  KF_DCHECK(nchunk >= 1);
  {
    kf_h8 ea[NK], sa[2];
    load(0, ea, sa);
    gpm_chunk<D, true, IL>(ea, sa, xb, neg1, acc);
  }
  for (int ch = 1; ch < nchunk; ++ch) {
    kf_h8 ea[NK], sa[2];
    load(ch, ea, sa);
    gpm_chunk<D, false, IL>(ea, sa, xb, neg1, acc);
  }
  gpm_extract2<D>(acc, S);
  const float s = kexp2(cl);
#pragma unroll
  for (int f = 0; f <= D; ++f) S[f] *= s;
}

// The same sums with the band's table read from global memory (L2-resident:
// used when the tables of all bands do not fit the 160 KiB of LDS, e.g. ten
// PROSAIL bands).  PF: the next chunk's fragments are loaded while the current
// one runs (register double buffer).

template <int D, bool PF = false, bool IL = false>
__device__ __forceinline__ void gp_mfma_sums_g_xb(const void* tab_, int nchunk, const kf_h8 (&xb)[2][gpm_k_steps(D)],
                                                  float cl, float (&S)[D + 1]) {
  static_assert(D >= 1 && D <= GPM_MAX_D, "GP input count for the matrix-core path");
  constexpr int NK = gpm_k_steps(D), NR = gpm_sum_rows(D), FPC = gpm_frags_per_chunk(D);
  const int lane = threadIdx.x & 63, h = lane >> 5;
  // The table through a raw buffer resource: per-lane byte offsets fixed for
  // the whole loop (VGPR), the chunk offset in the scalar soffset, so a chunk
  // costs no VALU address arithmetic (64-bit pointer adds per load before).
  // Lanes whose sums row is unused read past num_records: the hardware
  // returns zeros, the shared zero fragment of the LDS path.
  const int chunk_bytes = FPC * 16;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(tab_), (short)0, nchunk * chunk_bytes, 0x00020000);
  const int cr = gpm_sum_row<D>(lane & 31);
  const bool ls = cr >= 0;
  constexpr int OOB = 0x40000000;
  const int soff0 = ls ? (64 * NK + h * NR + cr) * 16 : OOB;
  const int soff1 = ls ? soff0 + 2 * NR * 16 : OOB;
  const float neg1 = gpm_neg1();
  kf_f16v acc[2];
  kf_h8 ea[NK], sa[2];
  auto ld = [&](int voff, int ch) {
    return __builtin_bit_cast(kf_h8, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, ch * chunk_bytes, 0));
  };
  if constexpr (PF) {
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) ea[kk] = ld((64 * kk + lane) * 16, 0);
    sa[0] = ld(soff0, 0);
    sa[1] = ld(soff1, 0);
  }
  // one chunk: PF prefetches chunk ch + 1 (the last chunk re-reads itself);
  // otherwise chunk ch is loaded here and the latency left to the other waves.
  // The first chunk is peeled (sums from the MFMA's zero operand, >= 1 chunk).
  auto step = [&](int ch, auto first) {
    const int nx = PF ? (ch + 1 < nchunk ? ch + 1 : ch) : ch;
    kf_h8 ean[NK], san[2];
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) ean[kk] = ld((64 * kk + lane) * 16, nx);
    san[0] = ld(soff0, nx);
    san[1] = ld(soff1, nx);
    if constexpr (!PF) {
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) ea[kk] = ean[kk];
      sa[0] = san[0];
      sa[1] = san[1];
    }
    gpm_chunk<D, decltype(first)::value, IL>(ea, sa, xb, neg1, acc);
    if constexpr (PF) {
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) ea[kk] = ean[kk];
      sa[0] = san[0];
      sa[1] = san[1];
    }
  };
  KF_DCHECK(nchunk >= 1);
  step(0, std::true_type{});
  for (int ch = 1; ch < nchunk; ++ch) step(ch, std::false_type{});
  __shared__ float gpm_xbuf[GPM_G_WAVES * 2 * 32 * 16];
  KF_DCHECK((int)(threadIdx.x >> 6) < GPM_G_WAVES);
  gpm_extract_lds<D>(acc, S, gpm_xbuf + (threadIdx.x >> 6) * (2 * 32 * 16));
  const float s = kexp2(cl);
#pragma unroll
  for (int f = 0; f <= D; ++f) S[f] *= s;
}

template <int D, bool PF = false, bool IL = false>
__device__ __forceinline__ void gp_mfma_sums_g(const void* tab_, int nchunk, const float (&xi)[D], float c,
                                               float (&S)[D + 1]) {
  kf_h8 xb[2][gpm_k_steps(D)];
  float cl;
  gpm_operands<D>(xi, c, xb, cl);
  gp_mfma_sums_g_xb<D, PF, IL>(tab_, nchunk, xb, cl, S);
}

// BAND_LAYOUT_SHARED_X: every band is a full-state GP around the same centre,
// so the exponent operand (split, packed and half-swapped centred inputs,
// gpm_operands) is built once per Gauss-Newton iteration and each band only
// patches the K slot 3D + 1 that carries its own constant c.  D even: slots 3D
// ("1") and 3D + 1 (c) share one packed dword.  Which lanes hold the dword of
// their own pixel and which their partner's follows gpm_operands.
template <int D>
__device__ __forceinline__ void gpm_patch_c(kf_h8 (&xb)[2][gpm_k_steps(D)], float c, float& cl) {
  static_assert(D % 2 == 0, "slots 3D and 3D + 1 share a dword for even D");
  constexpr int K = 3 * D + 1, KK = K / 16, W = K % 16, F = W / 8, Q = (W % 8) / 2;
  const _Float16 ch = (_Float16)fmaxf(c, -6.0e4f);
  cl = c - (float)ch;
  const uint32_t own = gpm_pack((_Float16)1.f, ch);
  const uint32_t par = __builtin_bit_cast(uint32_t, gpm_partner32(__builtin_bit_cast(float, own)));
  const bool h1 = (threadIdx.x & 32) != 0;
  // F1 slot: lanes h = 1 hold their own dword in block 1 and the partner's in
  // block 0; F0 slot: lanes h = 0 their own in block 0, the partner's in block 1
  const bool mine = F == 1 ? h1 : !h1;
  kf_u4 b0 = __builtin_bit_cast(kf_u4, xb[0][KK]), b1 = __builtin_bit_cast(kf_u4, xb[1][KK]);
  if (F == 1) {
    b1[Q] = mine ? own : b1[Q];
    b0[Q] = mine ? par : b0[Q];
  } else {
    b0[Q] = mine ? own : b0[Q];
    b1[Q] = mine ? par : b1[Q];
  }
  xb[0][KK] = __builtin_bit_cast(kf_h8, b0);
  xb[1][KK] = __builtin_bit_cast(kf_h8, b1);
}

// Line tables (AnalysisArgs.line_* / GainArgs.line_*): the first Gauss-Newton
// iteration at a partial-reset forecast sees every parameter but the
// propagated one at the reset mean, so each band's GP value and gradient are
// cubic pieces in that one parameter (models/gp.py:line_table).  line_pos finds
// the lane's interval (in: x_f,j inside the table; outside, or not finite, the
// wave takes the GP sums) and line_eval one band's D + 1 polynomials.
struct LinePos {
  const float* row;   // the interval's coefficients, band 0
  float s;            // (t - t_k) / h in [0, 1]
  bool in;
};

template <int NP, typename LA>
__device__ __forceinline__ LinePos line_pos(const KF_CONST_AS LA* la, const float (&x0)[NP], int row_floats) {
  const int n = la->line_n;
  const float t = la->line_j >= 0 ? gather_state_u<NP>(x0, la->line_j) : la->line_t0;
  const float u = (t - la->line_t0) * la->line_inv_h;
  LinePos r;
  r.in = u >= 0.f && u <= (float)n;
  // clamped (NaN -> 0) so every lane's loads stay inside the table
  const float uc = fminf(fmaxf(u, 0.f), (float)n);
  const int k = min((int)uc, n - 1);
  r.s = uc - (float)k;
  r.row = la->line_tab + (int64_t)k * row_floats;
  return r;
}

template <int D>
__device__ __forceinline__ void line_eval(const float* row, float s, float& H0, float (&g)[D]) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const f4* r = (const f4*)row;
  f4 c = r[0];
  H0 = fmaf(fmaf(fmaf(c.w, s, c.z), s, c.y), s, c.x);
#pragma unroll
  for (int d = 0; d < D; ++d) {
    c = r[1 + d];
    g[d] = fmaf(fmaf(fmaf(c.w, s, c.z), s, c.y), s, c.x);
  }
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
// (Round 2 abandoned a two-phase variant -- every band's GP sums first, the
// normal equations afterwards -- that gave intermittently wrong pixels under
// full occupancy.  That build split m with inline-asm v_fma_mix and a
// hand-placed s_nop before the MFMA SrcB read, a hazard the compiler's
// recognizer cannot see; the split is now plain C++ (gpm_exp_split), so every
// VALU -> MFMA wait state is the compiler's, and tests/test_isa_lint.py checks
// the built code object for them.)
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
    for (int d = 0; d < D; ++d) xi[d] = gather_state_u<NP>(x0, bdp->map[d]) - bdp->center[d];
  }
#pragma unroll
  for (int d = 0; d < D; ++d) c = fmaf(bdp->coef[d] * xi[d], xi[d], c);
}

// Compile-time maps (BandDesc.map_kind, JRC-TIP): the gather of gpm_inputs and
// the normal-equation update of the dense path restricted to the touched
// entries, in the same operand order (bit-identical: the dense update adds
// exact zeros elsewhere).
struct GpmMap {
  int m[4];
  int inv[16];   // input index of state j, -1 if none
};
__device__ constexpr GpmMap gpm_const_map(int kind) {
  GpmMap r{{0, 1, 6, 2}, {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1}};
  if (kind == GPM_MAP_TIP_NIR) {
    r.m[0] = 3; r.m[1] = 4; r.m[2] = 6; r.m[3] = 5;
  }
  for (int d = 0; d < 4; ++d) r.inv[r.m[d]] = d;
  return r;
}

template <int NP, int D, int K>
__device__ __forceinline__ void gpm_inputs_const(const KF_CONST_AS BandDesc* bdp, const float (&x0)[NP],
                                                 float (&xi)[D], float& c) {
  constexpr GpmMap M = gpm_const_map(K);
#pragma unroll
  for (int d = 0; d < D; ++d) xi[d] = x0[M.m[d]] - bdp->center[d];
#pragma unroll
  for (int d = 0; d < D; ++d) c = fmaf(bdp->coef[d] * xi[d], xi[d], c);
}

template <int NP, int D, int K>
__device__ __forceinline__ void gpm_update_const(float (&A)[ntri(NP)], float (&b)[NP], const float (&g)[D],
                                                 float w, float wy) {
  constexpr GpmMap M = gpm_const_map(K);
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    if (M.inv[i] < 0) continue;
    const float hi = g[M.inv[i]];
    const float wh = w * hi;
    b[i] = fmaf(hi, wy, b[i]);
#pragma unroll
    for (int j = i; j < NP; ++j)
      if (M.inv[j] >= 0) A[tri(NP, i, j)] = fmaf(wh, g[M.inv[j]], A[tri(NP, i, j)]);
  }
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

template <int NP, int D, int FOBS, bool GT = false, bool PF = false, int LAYOUT = BAND_LAYOUT_RUNTIME,
          bool IL = false, int SPEC = SPEC_ANY>
__device__ __forceinline__ float pixel_analysis_mfma(const AnalysisArgs& a, int64_t p, bool act,
                                                     const kf_h8* lds, float& dn_first KF_PHASE_PARAM,
                                                     int pre_j = -1, float pre_x = 0.f, float pre_p = 0.f) {
  constexpr int NT = ntri(NP);
  // LAYOUT == BAND_LAYOUT_TIP: two bands with the JRC-TIP VIS / NIR maps, the
  // band loop unrolled with both maps compile-time (no runtime map branches
  // and no register copies at their joins)
  static_assert(LAYOUT == BAND_LAYOUT_RUNTIME || (NP == 7 && D == 4 && !GT), "JRC-TIP layout: 7 params, 4 inputs");
  const int64_t ld = a.ld;
  float x0[NP], A[NT], b[NP];
  if (a.x_prev) {
#pragma unroll
    for (int j = 0; j < NP; ++j) x0[j] = KF_PX(a.x_prev, j * ld, p);
  }
  dn_first = 0.f;
  KF_PHASE_COUNT(KF_PH_GROUPS)
  // wave-uniform loop over the fused Gauss-Newton iterations (AnalysisArgs.gn_fused)
  for (int it = 0;; ++it) {
  p = opaque_lane(p);
  uint8_t st = 0;
  // correction form throughout (kf_core.h analysis_epilogue, DELTA)
  if (SPEC != SPEC_ANY || a.prop) {
    float xf[NP];
    // SPEC_PROP_PF: the single propagated parameter's x_a / P_a,jj of the first
    // iteration were loaded ahead by the kernel's loop (pre_j >= 0)
    if (SPEC == SPEC_PROP_PF && pre_j >= 0 && it == 0)
      forecast_partial_pre<NP>(opaque(cptr(a.prop)), p, pre_j, pre_x, pre_p, xf, A);
    else
      forecast_partial<NP>(opaque(cptr(a.prop)), p, xf, A);
    if (!a.x_prev && it == 0) {
      // linearised at the forecast: the prior part P_f^-1 (x_f - x0) is 0
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        x0[j] = xf[j];
        b[j] = 0.f;
      }
    } else {
      prior_rhs<NP, true>(A, xf, x0, b);
    }
  } else if (a.a_in) {
#pragma unroll
    for (int t = 0; t < NT; ++t) A[t] = KF_PX(a.a_in, t * ld, p);
#pragma unroll
    for (int j = 0; j < NP; ++j) b[j] = KF_PX(a.b_in, j * ld, p);
    float t[NP];
    symv<NP>(A, x0, t);
#pragma unroll
    for (int j = 0; j < NP; ++j) b[j] -= t[j];
  } else {
    float xf[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) xf[j] = KF_PX(a.x_f, j * ld, p);
#pragma unroll
    for (int t = 0; t < NT; ++t) A[t] = KF_PX(a.pf_inv, t * ld, p);
    prior_rhs<NP, true>(A, xf, x0, b);
  }
  int nobs = 0;
  int off = 0;
  // BAND_LAYOUT_SHARED_X (global tables, full-state GPs around one centre):
  // the exponent operand of the centred inputs once per iteration, each band
  // patches its constant in (gpm_patch_c).  AV_PER_BAND_OPERAND: per band (oracle).
  constexpr bool SXC = GT && D == NP && D % 2 == 0;
  bool sx = false;
  kf_h8 sxb[2][gpm_k_steps(D)];
  // the centred inputs too: every band of the layout has the same centre and
  // the identity map, so gpm_inputs would recompute exactly these values
  float sxi[SXC ? D : 1];
  if constexpr (SXC) {
    sx = a.band_layout == BAND_LAYOUT_SHARED_X && a.variant != AV_PER_BAND_OPERAND && a.n_bands > 0;
    if (sx) {
      const KF_CONST_AS BandDesc* b0 = cptr(a.bands);
      float c0;
#pragma unroll
      for (int d = 0; d < D; ++d) sxi[d] = x0[d] - b0->center[d];
      gpm_operands<D>(sxi, 0.f, sxb, c0);
    }
  }
  // the first iteration at the fused forecast: line tables when the host set
  // them (the kernels specialised for the fused forecast only: SPEC_ANY is the
  // first date's launch, without one, and the generic oracle, variant 18)
  const bool line = SPEC != SPEC_ANY && it == 0 && !a.x_prev &&
                    opaque((const KF_CONST_AS AnalysisArgs*)__builtin_amdgcn_kernarg_segment_ptr())->line_tab;
  // one band: GP sums on the matrix cores, value and Jacobian, normal equations.
  // MKC: the band's map kind when known at compile time (LAYOUT), else -1
  auto band = [&](int bi, auto mkc) {
    constexpr int MKC = decltype(mkc)::value;
    const KF_CONST_AS BandDesc* bdp = cptr(a.bands) + bi;
    float y, w;
    decode_obs<FOBS>(*bdp, p, y, w);
    const bool use = act && (w > 0.f);
    float H0 = 0.f, g[D];
#pragma unroll
    for (int d = 0; d < D; ++d) g[d] = 0.f;
    bool ok = false;
    const int nch = bdp->gpm_nchunk;
    // wave-uniform: a compiled-in JRC-TIP map, or the runtime / identity map
    constexpr bool TIPK = NP == 7 && D == 4;
    const int mk = MKC >= 0 ? MKC : (TIPK ? bdp->map_kind : GPM_MAP_RUNTIME);
    const bool any = __any(use);
    bool tabled = false;
    if (any && line) {
      // wave-uniform: every observed lane's x_f,j inside the table
      const KF_CONST_AS AnalysisArgs* la =
          opaque((const KF_CONST_AS AnalysisArgs*)__builtin_amdgcn_kernarg_segment_ptr());
      const LinePos lp = line_pos<NP>(la, x0, a.n_bands * (D + 1) * 4);
      if (__all(lp.in || !use)) {
        line_eval<D>(lp.row + bi * (D + 1) * 4, lp.s, H0, g);
        tabled = true;
        ok = finitef(H0);
#pragma unroll
        for (int d = 0; d < D; ++d) ok = ok && finitef(g[d]);
      }
    }
    if (any && !tabled) {
      float xi[D], c = 0.f;
      if (TIPK && mk == GPM_MAP_TIP_VIS) {
        gpm_inputs_const<NP, D, GPM_MAP_TIP_VIS>(bdp, x0, xi, c);
      } else if (TIPK && mk == GPM_MAP_TIP_NIR) {
        gpm_inputs_const<NP, D, GPM_MAP_TIP_NIR>(bdp, x0, xi, c);
      } else if (SXC && sx) {
#pragma unroll
        for (int d = 0; d < D; ++d) xi[d] = sxi[SXC ? d : 0];
#pragma unroll
        for (int d = 0; d < D; ++d) c = fmaf(bdp->coef[d] * xi[d], xi[d], c);
      } else {
        gpm_inputs<NP, D>(bdp, x0, xi, c);
      }
      c *= -0.5f * LOG2E;
      float S[D + 1];
      KF_PHASE(KF_PH_BAND_IN)
      if constexpr (SXC) {
        if (sx) {
          kf_h8 xb[2][gpm_k_steps(D)];
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int kk = 0; kk < gpm_k_steps(D); ++kk) xb[i][kk] = sxb[i][kk];
          float cl;
          gpm_patch_c<D>(xb, c, cl);
          gp_mfma_sums_g_xb<D, PF, IL>(bdp->gpm, nch, xb, cl, S);
        } else {
          gp_mfma_sums_g<D, PF, IL>(bdp->gpm, nch, xi, c, S);
        }
      } else if constexpr (GT) {
        gp_mfma_sums_g<D, PF, IL>(bdp->gpm, nch, xi, c, S);
      } else {
        gp_mfma_sums<D, IL>(lds + off, lds + a.gpm_frags - 1, nch, xi, c, S);
      }
      KF_PHASE(KF_PH_GP)
      const KF_CONST_AS BandDesc* q = opaque(bdp);   // epilogue fields: not live across the chunk loop
      const float sc = q->gpm_scale;
      const float S0 = S[0] * sc;
      // f = offset + S0, df/dx_d = -lambda_d x_d S0 + ln2 S'_d (gp_epilogue)
      H0 = q->offset + S0;
#pragma unroll
      for (int d = 0; d < D; ++d) g[d] = fmaf(-q->coef[d] * xi[d], S0, LN2 * (S[1 + d] * sc));
      ok = finitef(H0);
#pragma unroll
      for (int d = 0; d < D; ++d) ok = ok && finitef(g[d]);
    }
    off += nch * gpm_frags_per_chunk(D);
    float* h0o = opaque(bdp)->h0_out;
    if (act && h0o) KF_PX(h0o, 0, p) = use ? H0 : 0.f;
    if (use && !ok) st |= ST_BAD_OP;
    if (use && ok) {
      ++nobs;
      const float wy = w * (y - H0);   // correction form: the residual at x0
      if (TIPK && mk == GPM_MAP_TIP_VIS) {
        gpm_update_const<NP, D, GPM_MAP_TIP_VIS>(A, b, g, w, wy);
      } else if (TIPK && mk == GPM_MAP_TIP_NIR) {
        gpm_update_const<NP, D, GPM_MAP_TIP_NIR>(A, b, g, w, wy);
      } else {
        // scatter to the state (identity map: h[d] = g_d)
        float h[NP];
        const KF_CONST_AS BandDesc* q = opaque(bdp);
#pragma unroll
        for (int j = 0; j < NP; ++j) h[j] = 0.f;
        if (q->map_identity) {
#pragma unroll
          for (int d = 0; d < D && d < NP; ++d) h[d] = g[d];
        } else {
#pragma unroll
          for (int d = 0; d < D; ++d) {
#pragma unroll
            for (int j = 0; j < NP; ++j) h[j] += (q->map[d] == j) ? g[d] : 0.f;
          }
        }
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          const float wh = w * h[i];
          b[i] = fmaf(h[i], wy, b[i]);
#pragma unroll
          for (int j = i; j < NP; ++j) A[tri(NP, i, j)] = fmaf(wh, h[j], A[tri(NP, i, j)]);
        }
      }
    }
    KF_PHASE(KF_PH_BAND_OUT)
  };
  KF_PHASE(KF_PH_FORECAST)
  if constexpr (LAYOUT == BAND_LAYOUT_TIP) {
    band(0, std::integral_constant<int, GPM_MAP_TIP_VIS>{});
    band(1, std::integral_constant<int, GPM_MAP_TIP_NIR>{});
  } else {
    for (int bi = 0; bi < a.n_bands; ++bi) band(bi, std::integral_constant<int, -1>{});
  }
  if (nobs == 0) st |= ST_NO_OBS;
  const KF_CONST_AS AnalysisArgs* ka =
      opaque((const KF_CONST_AS AnalysisArgs*)__builtin_amdgcn_kernarg_segment_ptr());
  // the linearisation point outside the GP bands' domain box (state space, one
  // test for every band: AnalysisArgs.dom_*)
  if (state_out_of_domain<NP>(ka, x0)) st |= ST_OUT_OF_DOMAIN;
  // one epilogue call site for the fused intermediate and the final iteration
  // (bit-identical intermediate x, kf_core.h); tail lanes (act = false) solve
  // too but store nothing: their x0 only feeds the next iteration's MFMA
  // operands and must stay finite
  const bool last = it + 1 >= ka->gn_fused;
  const float dn = analysis_epilogue<NP, true, SPEC>(ka, p, A, b, x0, st, last && act, last);
  KF_PHASE(KF_PH_SOLVE)
  if (last) return act ? dn : 0.f;
  dn_first = dn;
#pragma unroll
  for (int j = 0; j < NP; ++j) x0[j] = b[j];
  }
}

// K1g (gain / covariance form) with the GP on the matrix cores: gain_pixel
// (kf_core.h) with lane = pixel, each band's GP sums wave-cooperative as in
// pixel_analysis_mfma (every lane of the wave takes part, act = false lanes
// included), then the same scalar-band update and tail.
template <int NP, int D, int FOBS>
__device__ __forceinline__ float pixel_gain_mfma(const GainArgs& a, int64_t p, bool act, const kf_h8* lds,
                                                 float& dn1) {
  return gain_pixel<NP>(a, p, act, dn1, [&](int bi, int it, const float (&x0)[NP], float& y, float& w, float& H0,
                                            float (&h)[NP], bool& ok) -> bool {
    int off = 0;
    for (int bj = 0; bj < bi; ++bj) off += cptr(a.bands)[bj].gpm_nchunk * gpm_frags_per_chunk(D);
    const KF_CONST_AS BandDesc* bdp = cptr(a.bands) + bi;
    decode_obs<FOBS>(*bdp, p, y, w);
    const bool use = act && (w > 0.f);
    H0 = 0.f;
#pragma unroll
    for (int j = 0; j < NP; ++j) h[j] = 0.f;
    ok = false;
    const int nch = bdp->gpm_nchunk;
    bool tabled = false;
    const KF_CONST_AS GainArgs* la = opaque((const KF_CONST_AS GainArgs*)__builtin_amdgcn_kernarg_segment_ptr());
    if (it == 0 && !a.x_prev && la->line_tab && __any(use)) {
      // the first iteration at the fused forecast: line tables (pixel_analysis_mfma)
      const LinePos lp = line_pos<NP>(la, x0, a.n_bands * (D + 1) * 4);
      if (__all(lp.in || !use)) {
        float g[D];
        line_eval<D>(lp.row + bi * (D + 1) * 4, lp.s, H0, g);
        const KF_CONST_AS BandDesc* q = opaque(bdp);
        if (q->map_identity) {
#pragma unroll
          for (int d = 0; d < D && d < NP; ++d) h[d] = g[d];
        } else {
#pragma unroll
          for (int d = 0; d < D; ++d) {
#pragma unroll
            for (int j = 0; j < NP; ++j) h[j] += (q->map[d] == j) ? g[d] : 0.f;
          }
        }
        tabled = true;
        ok = finitef(H0);
#pragma unroll
        for (int j = 0; j < NP; ++j) ok = ok && finitef(h[j]);
      }
    }
    if (!tabled && __any(use)) {
      float xi[D], c = 0.f;
      gpm_inputs<NP, D>(bdp, x0, xi, c);
      c *= -0.5f * LOG2E;
      float S[D + 1];
      gp_mfma_sums<D>(lds + off, lds + a.gpm_frags - 1, nch, xi, c, S);
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
    float* h0o = opaque(bdp)->h0_out;
    if (act && h0o) KF_PX(h0o, 0, p) = use ? H0 : 0.f;
    return use;
  });
}
#endif
}  // namespace kf
