// proto_gp_mfma.hip — prototype: GP emulator sums with the exponent GEMM on
// the f32 matrix cores (v_mfma_f32_16x16x4_f32) vs the current VALU loop.
//
// Per pixel p (one per lane) and training point i:
//   E_ip = L_i + c_p + sum_d B_id x_pd,  k_ip = 2^E_ip,
//   S0_p = sum_i alpha_i k_ip,  S_dp = sum_i (alpha t_d)_i k_ip.
// VALU kernel: records in SGPRs, 2 points per v_pk_fma_f32 (production path).
// MFMA kernel: a wave = 64 pixels = 4 column blocks of 16; per tile of 16
// points the exponents come from 2 k-steps x 4 blocks of 16x16x4 MFMAs
// (A = point features [L, 1, B_1..B_D, 0, 0], B = pixel features
// [1, c, x_1..x_D, 0, 0]); lane l then holds k for points 4(l>>4)+r, r<4, of
// pixels 16 cb + (l&15) and accumulates the sums on the VALU; a butterfly over
// the 4 lane groups gives every lane its own pixel's sums at the end.
//   hipcc --offload-arch=gfx950 -O3 scripts/proto_gp_mfma.hip -o /tmp/proto && /tmp/proto
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int D = 4;
constexpr int NF = 8;          // exponent features, padded to 2 k-steps of 4
constexpr int NV = D + 1;      // sums per pixel
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

// ---------------------------------------------------------------- VALU path
__global__ __launch_bounds__(256) void gp_valu(const float* __restrict__ rec_g, int T, const float* __restrict__ x,
                                               int N, float* __restrict__ out) {
  const __attribute__((address_space(4))) f2* r2 = (const __attribute__((address_space(4))) f2*)rec_g;
  constexpr int R = 2 * D + 2;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < N; p += gridDim.x * 256) {
    float xi[D], c = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) { xi[d] = x[d * N + p]; c = fmaf(xi[d], xi[d], c); }
    c *= -0.5f;
    f2 xv[D], S0 = {0.f, 0.f}, S[D];
#pragma unroll
    for (int d = 0; d < D; ++d) { xv[d] = f2{xi[d], xi[d]}; S[d] = f2{0.f, 0.f}; }
    const f2 cv = {c, c};
#pragma unroll 4
    for (int i = 0; i < T / 2; ++i) {
      const __attribute__((address_space(4))) f2* ri = r2 + (size_t)i * R;
      f2 e = ri[0] + cv;
#pragma unroll
      for (int d = 0; d < D; ++d) e = __builtin_elementwise_fma(ri[1 + d], xv[d], e);
      f2 k;
      k.x = __builtin_amdgcn_exp2f(e.x);
      k.y = __builtin_amdgcn_exp2f(e.y);
      S0 = __builtin_elementwise_fma(ri[1 + D], k, S0);
#pragma unroll
      for (int d = 0; d < D; ++d) S[d] = __builtin_elementwise_fma(ri[2 + D + d], k, S[d]);
    }
    out[0 * N + p] = S0.x + S0.y;
#pragma unroll
    for (int d = 0; d < D; ++d) out[(1 + d) * N + p] = S[d].x + S[d].y;
  }
}

// ---------------------------------------------------------------- MFMA path
// aop [T/16][2][64]: lane l of k-step s = feature 4s + (l>>4) of point 16t + (l&15)
// vop [T/16][NV][16]: value m of point 16t + j
__global__ __launch_bounds__(256) void gp_mfma(const float* __restrict__ aop, const float* __restrict__ vop, int T,
                                               const float* __restrict__ x, int N, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, col = lane & 15;
  const int nwaves = gridDim.x * 4;
  for (int w0 = blockIdx.x * 4 + (threadIdx.x >> 6); w0 * 64 < N; w0 += nwaves) {
    const int p = w0 * 64 + lane;
    const bool live = p < N;
    // own pixel features [1, c, x_1..x_D, 0, 0]
    float pf[NF];
    float c = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) { pf[2 + d] = live ? x[d * N + p] : 0.f; c = fmaf(pf[2 + d], pf[2 + d], c); }
    pf[0] = 1.f;
    pf[1] = -0.5f * c;
#pragma unroll
    for (int f = 2 + D; f < NF; ++f) pf[f] = 0.f;
    // B operands: lane l, block cb, k-step s -> feature 4s + g of pixel 16 cb + col
    float bop[4][2];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int src = cb * 16 + col;
        float v = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float t = __shfl(pf[4 * s + j], src, 64);
          v = (g == j) ? t : v;
        }
        bop[cb][s] = v;
      }
    float acc[4][NV];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int m = 0; m < NV; ++m) acc[cb][m] = 0.f;
    const int ntile = T / 16;
    // software pipeline: operands of tile t+1 are loaded while tile t computes;
    // all 8 MFMAs of a tile are issued before their results are consumed
    float a0 = aop[0 * 64 + lane], a1 = aop[1 * 64 + lane];
    f4 v[NV];
#pragma unroll
    for (int m = 0; m < NV; ++m) v[m] = *(const f4*)(vop + m * 16 + 4 * g);
    for (int t = 0; t < ntile; ++t) {
      f4 e[4];
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        e[cb] = f4{0.f, 0.f, 0.f, 0.f};
        e[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, bop[cb][0], e[cb], 0, 0, 0);
      }
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) e[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, bop[cb][1], e[cb], 0, 0, 0);
      f4 vn[NV];
      float a0n = 0.f, a1n = 0.f;
      if (t + 1 < ntile) {
        a0n = aop[((t + 1) * 2 + 0) * 64 + lane];
        a1n = aop[((t + 1) * 2 + 1) * 64 + lane];
#pragma unroll
        for (int m = 0; m < NV; ++m) vn[m] = *(const f4*)(vop + ((t + 1) * NV + m) * 16 + 4 * g);
      }
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float k = __builtin_amdgcn_exp2f(e[cb][r]);
#pragma unroll
          for (int m = 0; m < NV; ++m) acc[cb][m] = fmaf(v[m][r], k, acc[cb][m]);
        }
      }
      a0 = a0n;
      a1 = a1n;
#pragma unroll
      for (int m = 0; m < NV; ++m) v[m] = vn[m];
    }
    // butterfly over the 4 lane groups, then lane l keeps block cb = g (its own pixel)
    float res[NV];
#pragma unroll
    for (int m = 0; m < NV; ++m) {
      float mine = 0.f;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        float s = acc[cb][m];
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        mine = (g == cb) ? s : mine;
      }
      res[m] = mine;
    }
    if (live)
#pragma unroll
      for (int m = 0; m < NV; ++m) out[m * N + p] = res[m];
  }
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? std::atoi(argv[1]) : (1 << 24);
  const int T = 512;
  std::srand(7);
  auto U = [](float a, float b) { return a + (b - a) * (std::rand() / (float)RAND_MAX); };
  // training points and weights (centred inputs, lambda folded into B)
  std::vector<float> L(T), B(T * D), al(T), at(T * D);
  for (int i = 0; i < T; ++i) {
    float tt = 0.f;
    for (int d = 0; d < D; ++d) {
      const float t = U(-1.f, 1.f);
      B[i * D + d] = t;
      at[i * D + d] = 0.f;
      tt += t * t;
    }
    L[i] = -0.5f * tt;
    al[i] = U(-0.05f, 0.05f);
    for (int d = 0; d < D; ++d) at[i * D + d] = al[i] * B[i * D + d];
  }
  // VALU records: pairs [T/2][2D+2][2]: L, B[D], alpha, alpha t[D]
  const int R = 2 * D + 2;
  std::vector<float> rec((size_t)T * R);
  for (int i = 0; i < T; ++i) {
    auto put = [&](int f, float v) { rec[((size_t)(i >> 1) * R + f) * 2 + (i & 1)] = v; };
    put(0, L[i]);
    for (int d = 0; d < D; ++d) put(1 + d, B[i * D + d]);
    put(1 + D, al[i]);
    for (int d = 0; d < D; ++d) put(2 + D + d, at[i * D + d]);
  }
  // MFMA operands
  std::vector<float> aop((size_t)T / 16 * 2 * 64), vop((size_t)T / 16 * NV * 16);
  for (int t = 0; t < T / 16; ++t) {
    for (int s = 0; s < 2; ++s)
      for (int l = 0; l < 64; ++l) {
        const int f = 4 * s + (l >> 4), i = 16 * t + (l & 15);
        float v = 0.f;
        if (f == 0) v = L[i];
        else if (f == 1) v = 1.f;
        else if (f < 2 + D) v = B[i * D + f - 2];
        aop[(t * 2 + s) * 64 + l] = v;
      }
    for (int j = 0; j < 16; ++j) {
      const int i = 16 * t + j;
      vop[(t * NV + 0) * 16 + j] = al[i];
      for (int d = 0; d < D; ++d) vop[(t * NV + 1 + d) * 16 + j] = at[i * D + d];
    }
  }
  std::vector<float> x((size_t)D * N);
  for (auto& v : x) v = U(-1.f, 1.f);

  float *d_rec, *d_aop, *d_vop, *d_x, *d_o1, *d_o2;
  CHECK(hipMalloc(&d_rec, rec.size() * 4));
  CHECK(hipMalloc(&d_aop, aop.size() * 4));
  CHECK(hipMalloc(&d_vop, vop.size() * 4));
  CHECK(hipMalloc(&d_x, x.size() * 4));
  CHECK(hipMalloc(&d_o1, (size_t)NV * N * 4));
  CHECK(hipMalloc(&d_o2, (size_t)NV * N * 4));
  CHECK(hipMemcpy(d_rec, rec.data(), rec.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_aop, aop.data(), aop.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_vop, vop.data(), vop.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_x, x.data(), x.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int grid = 4096;
  float best[2] = {1e9f, 1e9f};
  for (int rep = 0; rep < 6; ++rep) {
    for (int k = 0; k < 2; ++k) {
      CHECK(hipEventRecord(e0));
      if (k == 0) hipLaunchKernelGGL(gp_valu, dim3(grid), dim3(256), 0, 0, d_rec, T, d_x, N, d_o1);
      else hipLaunchKernelGGL(gp_mfma, dim3(grid), dim3(256), 0, 0, d_aop, d_vop, T, d_x, N, d_o2);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (rep > 0 && ms < best[k]) best[k] = ms;
    }
  }
  std::vector<float> o1((size_t)NV * N), o2((size_t)NV * N);
  CHECK(hipMemcpy(o1.data(), d_o1, o1.size() * 4, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(o2.data(), d_o2, o2.size() * 4, hipMemcpyDeviceToHost));
  double maxrel = 0.0;
  for (int m = 0; m < NV; ++m) {
    double scale = 0.0;
    for (int p = 0; p < N; ++p) scale = std::fmax(scale, std::fabs(o1[(size_t)m * N + p]));
    for (int p = 0; p < N; ++p)
      maxrel = std::fmax(maxrel, std::fabs(o1[(size_t)m * N + p] - o2[(size_t)m * N + p]) / (scale + 1e-30));
  }
  // host f64 check of a few pixels
  double maxref = 0.0;
  for (int p = 0; p < N; p += N / 97 + 1) {
    double c = 0.0;
    for (int d = 0; d < D; ++d) c += (double)x[(size_t)d * N + p] * x[(size_t)d * N + p];
    double s[NV] = {0};
    for (int i = 0; i < T; ++i) {
      double e = L[i] - 0.5 * c;
      for (int d = 0; d < D; ++d) e += (double)B[i * D + d] * x[(size_t)d * N + p];
      const double kk = std::exp2(e);
      s[0] += al[i] * kk;
      for (int d = 0; d < D; ++d) s[1 + d] += at[i * D + d] * kk;
    }
    for (int m = 0; m < NV; ++m) maxref = std::fmax(maxref, std::fabs(s[m] - o2[(size_t)m * N + p]) / (std::fabs(s[m]) + 1e-3));
  }
  const double pts = (double)N * T;
  std::printf("{\"N\": %d, \"T\": %d, \"D\": %d, \"valu_ms\": %.3f, \"mfma_ms\": %.3f, \"valu_gpts\": %.1f, "
              "\"mfma_gpts\": %.1f, \"max_rel_diff\": %.3g, \"max_rel_vs_f64\": %.3g}\n",
              N, T, D, best[0], best[1], pts / best[0] * 1e-6, pts / best[1] * 1e-6, maxrel, maxref);
  return 0;
}
