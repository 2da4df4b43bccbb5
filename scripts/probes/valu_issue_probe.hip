// VALU issue-cost probe for the GP inner loop's instruction mix on gfx950:
// v_exp_f32, v_cvt_pkrtz_f16_f32, v_fma_mixlo_f16, v_fma_f32, v_pk_add_f32,
// alone and mixed, at 1 / 2 / 3 waves per SIMD (one workgroup per CU, held
// there by a large dynamic LDS request; waves w and w + 4 share a SIMD).
// Also: does one wave's v_exp overlap another wave's plain VALU on the same
// SIMD (a separate transcendental pipe) or do their issue costs add?
// Prints one line per (mode, waves/SIMD): shader cycles per instruction per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_issue_probe valu_issue_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));

#define EXP(r) asm volatile("v_exp_f32 %0, %1" : "+v"(r) : "v"(src));
#define FMA(r) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(r) : "v"(src), "v"(src2));
#define CVT(r) asm volatile("v_cvt_pkrtz_f16_f32 %0, %1, %2" : "+v"(r) : "v"(src), "v"(src2));
#define MIX(r) asm volatile("v_fma_mixlo_f16 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "+v"(r) : "v"(src), "s"(neg1), "v"(src2));
#define PKA(r) asm volatile("v_pk_add_f32 %0, %1, %2" : "+v"(r) : "v"(p0), "v"(p1));

template <int MODE>
__global__ void probe(long long* out, int iters, float seed) {
  float src = seed + threadIdx.x, src2 = seed * 0.5f;
  float neg1 = -1.0f;
  asm volatile("" : "+s"(neg1));
  f2 p0 = {src, src2}, p1 = {src2, src};
  float r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0, r5 = 0, r6 = 0, r7 = 0;
  f2 q0 = p0, q1 = p1, q2 = p0, q3 = p1;
  const int wave = threadIdx.x >> 6;
  __syncthreads();
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if constexpr (MODE == 0) { EXP(r0) EXP(r1) EXP(r2) EXP(r3) EXP(r4) EXP(r5) EXP(r6) EXP(r7) }
      if constexpr (MODE == 1) { MIX(r0) MIX(r1) MIX(r2) MIX(r3) MIX(r4) MIX(r5) MIX(r6) MIX(r7) }
      if constexpr (MODE == 2) { CVT(r0) CVT(r1) CVT(r2) CVT(r3) CVT(r4) CVT(r5) CVT(r6) CVT(r7) }
      if constexpr (MODE == 3) { FMA(r0) FMA(r1) FMA(r2) FMA(r3) FMA(r4) FMA(r5) FMA(r6) FMA(r7) }
      if constexpr (MODE == 4) { PKA(q0) PKA(q1) PKA(q2) PKA(q3) PKA(q0) PKA(q1) PKA(q2) PKA(q3) }
      // exp and fma interleaved in one wave (do their costs add?)
      if constexpr (MODE == 5) { EXP(r0) FMA(r1) EXP(r2) FMA(r3) EXP(r4) FMA(r5) EXP(r6) FMA(r7) }
      // waves 0-3 exp, waves 4-7 (their SIMD partners) fma: separate pipes?
      if constexpr (MODE == 6) {
        if (wave < 4) { EXP(r0) EXP(r1) EXP(r2) EXP(r3) EXP(r4) EXP(r5) EXP(r6) EXP(r7) }
        else { FMA(r0) FMA(r1) FMA(r2) FMA(r3) FMA(r4) FMA(r5) FMA(r6) FMA(r7) }
      }
      // the GP loop's per-value mix: 2 exp, 1 cvt, 2 mix per 2 values
      if constexpr (MODE == 7) { EXP(r0) EXP(r1) CVT(r2) MIX(r3) MIX(r4) EXP(r5) EXP(r6) CVT(r7) }
    }
  }
  const long long t1 = clock64();
  asm volatile("" ::"v"(r0), "v"(r1), "v"(r2), "v"(r3), "v"(r4), "v"(r5), "v"(r6), "v"(r7));
  if constexpr (MODE == 4) asm volatile("" ::"v"(q0), "v"(q1), "v"(q2), "v"(q3));
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x >> 6) + wave] = t1 - t0;
}

template <int MODE>
static void run(const char* name, int wps, long long* d, int ncu) {
  const int threads = 256 * wps, iters = 4000;
  const size_t lds = 96 * 1024;   // one workgroup per CU
  hipFuncSetAttribute((const void*)probe<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  probe<MODE><<<ncu, threads, lds>>>(d, 16, 1.0f);
  hipEventRecord(a);
  probe<MODE><<<ncu, threads, lds>>>(d, iters, 1.0f);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const int nw = ncu * threads / 64;
  std::vector<long long> h(nw);
  hipMemcpy(h.data(), d, nw * sizeof(long long), hipMemcpyDeviceToHost);
  double mean = 0;
  for (auto v : h) mean += (double)v;
  mean /= nw;
  const double insts = (double)iters * 32;
  // waves on one SIMD run concurrently: SIMD cycles per instruction
  const double cpi = mean / (insts * wps);
  const double mhz = mean / (ms * 1e3);
  printf("{\"mode\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_inst_per_simd\": %.2f, "
         "\"wave_cycles\": %.0f, \"kernel_ms\": %.3f, \"clock_mhz_est\": %.0f}\n",
         name, wps, cpi, mean, ms, mhz);
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  long long* d;
  hipMalloc(&d, (size_t)ncu * 16 * sizeof(long long));
  for (int w = 1; w <= 3; ++w) {
    run<0>("exp", w, d, ncu);
    run<1>("fma_mixlo", w, d, ncu);
    run<2>("cvt_pkrtz", w, d, ncu);
    run<3>("fma_f32", w, d, ncu);
    run<4>("pk_add_f32", w, d, ncu);
    run<5>("exp+fma same wave", w, d, ncu);
    if (w >= 2) run<6>("exp waves0-3 | fma waves4-7", w, d, ncu);
    run<7>("gp mix 4exp 2cvt 2mix", w, d, ncu);
  }
  hipFree(d);
  return 0;
}
