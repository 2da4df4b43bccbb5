// Issue-overlap probe for the GP inner loop on gfx950 (VERDICT r3 #4a): do the
// instruction streams of different waves on one SIMD overlap, or do their
// issue costs add?  Streams: v_exp_f32 (transcendental), v_fma_mixlo_f16,
// v_cvt_pkrtz_f16_f32, v_fma_f32, v_mfma_f32_32x32x16_f16 (4 independent
// accumulators) and the GP loop's own per-value mix.
//
// One workgroup per CU (a large dynamic LDS request holds it there), 4 * wps
// waves: waves w, w + 4, w + 8 share SIMD w.  Each wave runs ONE stream,
// chosen by its slot on the SIMD (slot = wave / 4), for a fixed instruction
// count.  For streams A, B on two slots:
//   t_AA, t_BB: both waves run A (B);  t_AB: one wave A, one wave B.
//   additive issue (one shared issue port):   t_AB = (t_AA + t_BB) / 2
//   fully overlapped (separate pipes):        t_AB = max(t_AA, t_BB) / 2
// overlap = ((t_AA + t_BB) / 2 - t_AB) / (min(t_AA, t_BB) / 2): 0 = the costs
// add, 1 = the cheaper stream is completely hidden.  Kernel time by hipEvent
// (median of interleaved repeats), so clock changes hit every mode alike.
// Build: hipcc --offload-arch=gfx950 -O3 -o issue_overlap_probe issue_overlap_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

enum { S_EXP = 0, S_MIX = 1, S_CVT = 2, S_FMA = 3, S_MFMA = 4, S_GPMIX = 5, S_IDLE = 6 };
static const char* NAMES[] = {"exp", "fma_mixlo", "cvt_pkrtz", "fma_f32", "mfma32x32x16", "gp_mix", "idle"};

#define EXP(r) asm volatile("v_exp_f32 %0, %1" : "+v"(r) : "v"(src));
#define FMA(r) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(r) : "v"(src), "v"(src2));
#define CVT(r) asm volatile("v_cvt_pkrtz_f16_f32 %0, %1, %2" : "+v"(r) : "v"(src), "v"(src2));
#define MIX(r) asm volatile("v_fma_mixlo_f16 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "+v"(r) : "v"(src), "s"(neg1), "v"(src2));

template <int S>
__device__ __forceinline__ void stream_body(float src, float src2, float neg1, float (&r)[8], h8 a, h8 b,
                                            f16v (&acc)[4]) {
  if constexpr (S == S_EXP) { EXP(r[0]) EXP(r[1]) EXP(r[2]) EXP(r[3]) EXP(r[4]) EXP(r[5]) EXP(r[6]) EXP(r[7]) }
  if constexpr (S == S_MIX) { MIX(r[0]) MIX(r[1]) MIX(r[2]) MIX(r[3]) MIX(r[4]) MIX(r[5]) MIX(r[6]) MIX(r[7]) }
  if constexpr (S == S_CVT) { CVT(r[0]) CVT(r[1]) CVT(r[2]) CVT(r[3]) CVT(r[4]) CVT(r[5]) CVT(r[6]) CVT(r[7]) }
  if constexpr (S == S_FMA) { FMA(r[0]) FMA(r[1]) FMA(r[2]) FMA(r[3]) FMA(r[4]) FMA(r[5]) FMA(r[6]) FMA(r[7]) }
  if constexpr (S == S_MFMA) {
    // 4 MFMAs per body (4 independent accumulators)
    acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[1], 0, 0, 0);
    acc[2] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[2], 0, 0, 0);
    acc[3] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[3], 0, 0, 0);
  }
  if constexpr (S == S_GPMIX) { EXP(r[0]) EXP(r[1]) CVT(r[2]) MIX(r[3]) MIX(r[4]) EXP(r[5]) EXP(r[6]) CVT(r[7]) }
}

// the whole loop of one stream: the wave branches once, outside the loop
template <int S>
__device__ __forceinline__ void run_stream(int iters, float src, float src2, float neg1, float (&r)[8], h8 a, h8 b,
                                        f16v (&acc)[4]) {
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) stream_body<S>(src, src2, neg1, r, a, b, acc);
  }
}

__global__ void probe(float* out, int iters, float seed, int4 slot_stream) {
  float src = seed + threadIdx.x, src2 = seed * 0.5f;
  float neg1 = -1.0f;
  asm volatile("" : "+s"(neg1));
  float r[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  h8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (_Float16)(src * 1e-3f + i);
    b[i] = (_Float16)(src2 * 1e-3f - i);
  }
  f16v acc[4];
  for (int j = 0; j < 4; ++j)
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
  const int slot = (threadIdx.x >> 6) >> 2;
  const int s = __builtin_amdgcn_readfirstlane(slot == 0 ? slot_stream.x : slot == 1 ? slot_stream.y : slot_stream.z);
  __syncthreads();
  switch (s) {
    case S_EXP: run_stream<S_EXP>(iters, src, src2, neg1, r, a, b, acc); break;
    case S_MIX: run_stream<S_MIX>(iters, src, src2, neg1, r, a, b, acc); break;
    case S_CVT: run_stream<S_CVT>(iters, src, src2, neg1, r, a, b, acc); break;
    case S_FMA: run_stream<S_FMA>(iters, src, src2, neg1, r, a, b, acc); break;
    case S_MFMA: run_stream<S_MFMA>(iters, src, src2, neg1, r, a, b, acc); break;
    case S_GPMIX: run_stream<S_GPMIX>(iters, src, src2, neg1, r, a, b, acc); break;
    default: break;
  }
  float t = 0.f;
  for (int i = 0; i < 8; ++i) t += r[i];
  for (int j = 0; j < 4; ++j) t += acc[j][threadIdx.x & 15];
  if (t == 12345.678f) out[blockIdx.x] = t;   // keep the streams alive
}

static float time_mode(int wps, int4 ss, float* d, int ncu, int iters) {
  const int threads = 256 * wps;
  const size_t lds = 96 * 1024;   // one workgroup per CU
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(probe, dim3(ncu), dim3(threads), lds, 0, d, iters, 1.0f, ss);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return ms;
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  float* d;
  hipMalloc(&d, (size_t)ncu * sizeof(float));
  hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  const int iters = 4000, reps = 7;
  // (A, B) pairs on 2 waves / SIMD; the GP loop question is exp vs mix / mfma
  const int pairs[][2] = {{S_EXP, S_FMA}, {S_EXP, S_MIX}, {S_EXP, S_CVT}, {S_MIX, S_CVT},
                          {S_EXP, S_MFMA}, {S_MIX, S_MFMA}, {S_GPMIX, S_MFMA}, {S_FMA, S_MFMA}};
  hipLaunchKernelGGL(probe, dim3(ncu), dim3(512), 96 * 1024, 0, d, 64, 1.0f, make_int4(0, 0, 0, 0));   // warm-up
  hipDeviceSynchronize();
  for (auto& p : pairs) {
    const int A = p[0], B = p[1];
    std::vector<float> taa, tbb, tab, ta1, tb1;
    for (int rep = 0; rep < reps; ++rep) {
      taa.push_back(time_mode(2, make_int4(A, A, S_IDLE, 0), d, ncu, iters));
      tbb.push_back(time_mode(2, make_int4(B, B, S_IDLE, 0), d, ncu, iters));
      tab.push_back(time_mode(2, make_int4(A, B, S_IDLE, 0), d, ncu, iters));
      ta1.push_back(time_mode(2, make_int4(A, S_IDLE, S_IDLE, 0), d, ncu, iters));
      tb1.push_back(time_mode(2, make_int4(B, S_IDLE, S_IDLE, 0), d, ncu, iters));
    }
    auto med = [](std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    const float aa = med(taa), bb = med(tbb), ab = med(tab), a1 = med(ta1), b1 = med(tb1);
    const float add = 0.5f * (aa + bb), ovl = 0.5f * std::max(aa, bb);
    const float overlap = (add - ab) / (0.5f * std::min(aa, bb));
    printf("{\"A\": \"%s\", \"B\": \"%s\", \"waves_per_simd\": 2, \"t_AA_ms\": %.4f, \"t_BB_ms\": %.4f, "
           "\"t_AB_ms\": %.4f, \"t_A_alone_ms\": %.4f, \"t_B_alone_ms\": %.4f, \"additive_ms\": %.4f, "
           "\"overlapped_ms\": %.4f, \"overlap\": %.3f}\n",
           NAMES[A], NAMES[B], aa, bb, ab, a1, b1, add, ovl, overlap);
    fflush(stdout);
  }
  // 3 waves / SIMD: the GP loop runs 3 waves per SIMD (exp + mix + cvt + mfma
  // spread over them): gp_mix x3 vs gp_mix, gp_mix, mfma
  {
    std::vector<float> t3, t2m;
    for (int rep = 0; rep < reps; ++rep) {
      t3.push_back(time_mode(3, make_int4(S_GPMIX, S_GPMIX, S_GPMIX, 0), d, ncu, iters));
      t2m.push_back(time_mode(3, make_int4(S_GPMIX, S_GPMIX, S_MFMA, 0), d, ncu, iters));
    }
    std::sort(t3.begin(), t3.end());
    std::sort(t2m.begin(), t2m.end());
    printf("{\"waves_per_simd\": 3, \"gp_mix_x3_ms\": %.4f, \"gp_mix_x2_plus_mfma_ms\": %.4f}\n", t3[reps / 2],
           t2m[reps / 2]);
  }
  hipFree(d);
  return 0;
}
