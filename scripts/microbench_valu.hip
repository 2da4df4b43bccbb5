// microbench_valu.hip — issue cost of the GP loop's VALU instructions on gfx950.
// Each kernel runs ITER iterations of 8 independent dependency chains of one
// instruction type in every lane of 256 CUs x WAVES waves; cycles per
// instruction per SIMD = elapsed * clock / (instructions per SIMD).
//   hipcc --offload-arch=gfx950 -O3 scripts/microbench_valu.hip -o /tmp/mb && /tmp/mb
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 4096;

__global__ void k_fma(float* out, float a, float b) {
  float x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_fmaf(x[i], a, b);
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_pkfma(float* out, float a, float b) {
  f2 x[8];
  const f2 av = {a, a + 1.f}, bv = {b, b - 1.f};
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = f2{(float)threadIdx.x + i, (float)i};
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_elementwise_fma(x[i], av, bv);
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_exp(float* out, float a) {
  float x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = (threadIdx.x & 7) * 0.01f + i * 0.001f;
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_amdgcn_exp2f(x[i]) * a;   // exp + mul
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul(float* out, float a) {
  float x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = (threadIdx.x & 7) * 0.01f + i * 0.001f;
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = x[i] * a;
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  int dev = 0;
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, dev);
  const int cus = prop.multiProcessorCount;
  const double clk_ghz = prop.clockRate / 1e6;   // kHz -> GHz (peak)
  float* out;
  hipMalloc(&out, (size_t)cus * 64 * 1024 * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int waves = 4; waves <= 32; waves *= 2) {       // waves per CU (x4 SIMDs)
    const int blocks = cus * waves / 4;
    const int threads = 256;
    const double inst_per_simd = (double)ITER * 8 * (waves / 4);   // per SIMD (one wave64 instruction each)
    struct K { const char* name; int kind; double extra; };
    const K ks[] = {{"v_fma_f32", 0, 0}, {"v_pk_fma_f32", 1, 0}, {"v_exp_f32+v_mul_f32", 2, 0}, {"v_mul_f32", 3, 0}};
    for (const K& k : ks) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (k.kind == 0) hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(threads), 0, 0, out, 0.999f, 0.001f);
        if (k.kind == 1) hipLaunchKernelGGL(k_pkfma, dim3(blocks), dim3(threads), 0, 0, out, 0.999f, 0.001f);
        if (k.kind == 2) hipLaunchKernelGGL(k_exp, dim3(blocks), dim3(threads), 0, 0, out, 0.5f);
        if (k.kind == 3) hipLaunchKernelGGL(k_mul, dim3(blocks), dim3(threads), 0, 0, out, 0.999f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep == 1)
          std::printf("{\"waves_per_cu\": %d, \"op\": \"%s\", \"ms\": %.4f, \"cycles_per_inst_per_simd_at_%.2fGHz\": %.3f}\n",
                      waves, k.name, ms, clk_ghz, ms * 1e-3 * clk_ghz * 1e9 / inst_per_simd);
      }
    }
  }
  hipFree(out);
  return 0;
}
