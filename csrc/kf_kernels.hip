// kf_kernels.hip — gfx950 (MI355X) launchers for the KaFKA engine kernels
// (templates in kf_device.h; the NP = 7 / 10 analysis instantiations live in
// kf_analysis7.hip / kf_analysis10.hip).
#include "kf_device.h"

namespace kf {

constexpr int RED_BLOCK = 1024;
__global__ __launch_bounds__(RED_BLOCK) void reduce_partials_kernel(const double* partials, int n, double* out) {
  // one workgroup, fixed order (bit-reproducible): thread-strided sums, a fixed
  // shuffle tree per wave, then the 16 wave sums in wave order
  __shared__ double red[RED_BLOCK / 64];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += RED_BLOCK) s += partials[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < RED_BLOCK / 64; ++w) t += red[w];
    out[0] = t;
  }
}

// K7: nearest LUT entry (utils.py:225-234); LUT staged in LDS.
__global__ __launch_bounds__(BLOCK) void lut_nearest_kernel(const float* lut, int M, int D, const float* x,
                                                           int64_t N, int64_t ld, int32_t* out) {
  extern __shared__ __attribute__((aligned(16))) float slut[];
  for (int i = threadIdx.x; i < M * D; i += BLOCK) slut[i] = lut[i];
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  for (int64_t p = (int64_t)blockIdx.x * BLOCK + threadIdx.x; p < N; p += stride) {
    float xv[MAX_D];
    for (int d = 0; d < D; ++d) xv[d] = x[d * ld + p];
    float best = 3.4e38f;
    int bi = 0;
    for (int m = 0; m < M; ++m) {
      float s = 0.f;
      for (int d = 0; d < D; ++d) { const float t = slut[m * D + d] - xv[d]; s = fmaf(t, t, s); }
      if (s < best) { best = s; bi = m; }
    }
    out[p] = bi;
  }
}

template <int NP>
static void l_jacobi(const JacobiArgs& a, int grid, hipStream_t s) {
  const bool one = a.k == 1 && a.reg_mask != 0 && (a.reg_mask & (a.reg_mask - 1)) == 0;
  // dense strip, whole rows: the row-loop kernels (no per-pixel index division)
  const int64_t n = a.pn > 0 ? a.pn : a.N;
  const bool rows = one && a.geo.w > 0 && a.p0 % a.geo.w == 0 && n % a.geo.w == 0 && n > 0;
  const auto al16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  const bool four = rows && a.mode == JACOBI_FINISH && a.geo.w % 4 == 0 && a.ld % 4 == 0 && a.ld_ext % 4 == 0 &&
                    a.p0 % 4 == 0 && a.N % 4 == 0 && al16(a.u) && al16(a.v) && al16(a.x_ext) && al16(a.x_ref) &&
                    al16(a.x_out) &&
                    (!a.out_mean || (!a.out_idx && a.out_plane % 4 == 0 && al16(a.out_mean) && al16(a.out_unc) &&
                                     al16(a.a_in)));
  if (four) {
    hipLaunchKernelGGL((jacobi_kernel<NP, JACOBI_FINISH4>), dim3(grid), dim3(BLOCK), 0, s, a);
    return;
  }
  if (rows && (a.mode == JACOBI_SWEEP || a.mode == JACOBI_FINISH)) {
    const int64_t nr = n / a.geo.w;
    const int g = (int)(nr < grid ? nr : grid);   // partials hold >= grid entries
    // the norm sums all `grid` partials: blocks g.. do not exist here, so their
    // entries are cleared (nothing written earlier into the buffer leaks in)
    if (a.mode == JACOBI_FINISH && a.partials && g < grid)
      (void)hipMemsetAsync(a.partials + g, 0, sizeof(double) * (size_t)(grid - g), s);
    if (a.mode == JACOBI_SWEEP)
      hipLaunchKernelGGL((jacobi_kernel<NP, JACOBI_SWEEP1D>), dim3(g), dim3(BLOCK), 0, s, a);
    else
      hipLaunchKernelGGL((jacobi_kernel<NP, JACOBI_FINISH1D>), dim3(g), dim3(BLOCK), 0, s, a);
    return;
  }
  if (a.mode == JACOBI_SWEEP && one)
    hipLaunchKernelGGL((jacobi_kernel<NP, JACOBI_SWEEP1>), dim3(grid), dim3(BLOCK), 0, s, a);
  else if (a.mode == JACOBI_FINISH && one)
    hipLaunchKernelGGL((jacobi_kernel<NP, JACOBI_FINISH1>), dim3(grid), dim3(BLOCK), 0, s, a);
  else if (a.mode == JACOBI_SWEEP)
    hipLaunchKernelGGL((jacobi_kernel<NP, JACOBI_SWEEP>), dim3(grid), dim3(BLOCK), 0, s, a);
  else if (a.mode == JACOBI_FINISH)
    hipLaunchKernelGGL((jacobi_kernel<NP, JACOBI_FINISH>), dim3(grid), dim3(BLOCK), 0, s, a);
  else
    hipLaunchKernelGGL(jacobi_kernel<NP>, dim3(grid), dim3(BLOCK), 0, s, a);
}
template <int NP>
static void l_propagate(const PropArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL(propagate_kernel<NP>, dim3(grid), dim3(BLOCK), 0, s, a);
}
template <int NP>
static void l_invert(const float* src, float* dst, int64_t N, int64_t ld, uint8_t* st, int grid, hipStream_t s) {
  hipLaunchKernelGGL(invert_kernel<NP>, dim3(grid), dim3(BLOCK), 0, s, src, dst, N, ld, st);
}
template <int NP>
static void l_operator(const BandDesc* b, int band, const float* x, int64_t N, int64_t ld, float* h0, float* h,
                       int64_t h_ld, uint8_t* ok, int grid, hipStream_t s) {
  hipLaunchKernelGGL(operator_kernel<NP>, dim3(grid), dim3(BLOCK), 0, s, b, band, x, N, ld, h0, h, h_ld, ok);
}
template <int NP>
static void l_hessian(const BandDesc* b, int nb, const float* x, float* a, int64_t N, int64_t ld, int grid,
                      hipStream_t s) {
  hipLaunchKernelGGL(hessian_kernel<NP>, dim3(grid), dim3(BLOCK), 0, s, b, nb, x, a, N, ld);
}
template <int NP>
static void l_unpack(const float* x, const float* a, int64_t N, int64_t ld, const int64_t* idx, float* mean,
                     float* unc, int64_t plane, int grid, hipStream_t s) {
  hipLaunchKernelGGL(unpack_kernel<NP>, dim3(grid), dim3(BLOCK), 0, s, x, a, N, ld, idx, mean, unc, plane);
}

// Grid cap for the per-pixel kernels (one f64 partial per workgroup).  The
// default keeps grid-stride loops; raising it to >= N/256 gives one pixel per
// thread so workgroups start and finish at different times and their memory
// phases overlap other workgroups' compute.
static int g_max_blocks = KF_MAX_BLOCKS;
void set_max_blocks(int n) { g_max_blocks = n > 0 ? n : KF_MAX_BLOCKS; }
static int g_gp_unroll = 4;
void set_gp_unroll(int n) { g_gp_unroll = n; }
int get_max_blocks() { return g_max_blocks; }
int dev_grid(int64_t N) { return grid_for(N, g_max_blocks); }

// ---------------------------------------------------------------------------
// obs_order: a stable partition of 0..N-1 by observation class (obs_class:
// pixels observed in every band group first, unobserved last), so each class
// fills whole waves and a wave skips the GP of the groups it has no data for
// (AnalysisArgs.order).  Chunks of ORD_CHUNK pixels: class counts per chunk,
// a scan per class (one workgroup), a scatter with a workgroup-wide ballot
// prefix per class and 256-pixel tile.
constexpr int ORD_CHUNK = 4096;
constexpr int ORD_MAX_CLASSES = 8;   // <= 3 band groups

__global__ __launch_bounds__(BLOCK) void obs_count_kernel(const BandDesc* bands, const int32_t* grp, int nb, int G,
                                                          int64_t N, int32_t* counts) {
  __shared__ int red[ORD_MAX_CLASSES];
  const int K = 1 << G;
  if (threadIdx.x < ORD_MAX_CLASSES) red[threadIdx.x] = 0;
  __syncthreads();
  const int64_t c0 = (int64_t)blockIdx.x * ORD_CHUNK;
  int n[ORD_MAX_CLASSES] = {};
  for (int64_t p = c0 + threadIdx.x; p < N && p < c0 + ORD_CHUNK; p += BLOCK) ++n[obs_class(bands, grp, nb, G, p)];
  for (int c = 0; c < K; ++c) {
    int v = n[c];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(&red[c], v);   // LDS atomics
  }
  __syncthreads();
  if (threadIdx.x < K) counts[(int64_t)blockIdx.x * K + threadIdx.x] = red[threadIdx.x];
}

// counts [nc][K] -> exclusive slot offsets in place (class c's pixels start
// after every pixel of the classes before it); counts[nc * K] = N
__global__ __launch_bounds__(1024) void obs_scan_kernel(int32_t* counts, int nc, int K) {
  __shared__ int part[1024];
  __shared__ int cbase;
  const int per = (nc + 1023) / 1024;
  const int i0 = threadIdx.x * per, i1 = min(nc, i0 + per);
  if (threadIdx.x == 0) cbase = 0;
  __syncthreads();
  for (int c = 0; c < K; ++c) {
    int s = 0;
    for (int i = i0; i < i1; ++i) s += counts[(int64_t)i * K + c];
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
      int run = cbase;
      for (int i = 0; i < 1024; ++i) {
        const int v = part[i];
        part[i] = run;
        run += v;
      }
      cbase = run;
    }
    __syncthreads();
    int run = part[threadIdx.x];
    for (int i = i0; i < i1; ++i) {
      const int v = counts[(int64_t)i * K + c];
      counts[(int64_t)i * K + c] = run;
      run += v;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) counts[(int64_t)nc * K] = cbase;
}

__global__ __launch_bounds__(BLOCK) void obs_scatter_kernel(const BandDesc* bands, const int32_t* grp, int nb, int G,
                                                            int64_t N, const int32_t* offs, int32_t* order) {
  __shared__ int wave_n[BLOCK / 64][ORD_MAX_CLASSES];
  __shared__ int base[ORD_MAX_CLASSES];
  const int K = 1 << G;
  const int64_t c0 = (int64_t)blockIdx.x * ORD_CHUNK;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x < K) base[threadIdx.x] = offs[(int64_t)blockIdx.x * K + threadIdx.x];
  __syncthreads();
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int64_t t0 = c0; t0 < N && t0 < c0 + ORD_CHUNK; t0 += BLOCK) {
    const int64_t p = t0 + threadIdx.x;
    const bool in = p < N && p < c0 + ORD_CHUNK;
    const int cls = in ? obs_class(bands, grp, nb, G, p) : -1;
    int rank = 0;
    for (int c = 0; c < K; ++c) {
      const uint64_t m = __ballot(cls == c);
      if (lane == 0) wave_n[wv][c] = __popcll(m);
      if (cls == c) rank = __popcll(m & below);
    }
    __syncthreads();
    if (in) {
      int slot = base[cls] + rank;
      for (int i = 0; i < wv; ++i) slot += wave_n[i][cls];
      order[slot] = (int32_t)p;
    }
    __syncthreads();
    if (threadIdx.x < K)
      for (int i = 0; i < BLOCK / 64; ++i) base[threadIdx.x] += wave_n[i][threadIdx.x];
    __syncthreads();
  }
}

int obs_order_chunks(int64_t N) { return (int)((N + ORD_CHUNK - 1) / ORD_CHUNK); }

hipError_t dev_obs_order(const BandDesc* bands, const int32_t* grp, int nb, int G, int64_t N, int32_t* counts,
                         int32_t* order, hipStream_t s) {
  if (G < 1 || G > 3) return hipErrorInvalidValue;
  const int nc = obs_order_chunks(N);
  if (N <= 0) return hipSuccess;
  hipLaunchKernelGGL(obs_count_kernel, dim3(nc), dim3(BLOCK), 0, s, bands, grp, nb, G, N, counts);
  hipLaunchKernelGGL(obs_scan_kernel, dim3(1), dim3(1024), 0, s, counts, nc, 1 << G);
  hipLaunchKernelGGL(obs_scatter_kernel, dim3(nc), dim3(BLOCK), 0, s, bands, grp, nb, G, N, counts, order);
  return hipGetLastError();
}

bool gp_operator_supported(int np, int d) {
  return (np == 10 && (d == 10 || d == 4)) || (np == 7 && (d == 7 || d == 4)) || (np == d && np >= 2 && np <= 4);
}

hipError_t dev_analysis(int np, const AnalysisArgs& a, int grid, hipStream_t s) {
  switch (np) {
    case 7: return dev_analysis_np7(a, grid, s);     // kf_analysis7.hip
    case 10: return dev_analysis_np10(a, grid, s);   // kf_analysis10.hip
    case 1: l_analysis<1>(a, grid, s); break;
    case 2: l_analysis<2>(a, grid, s); break;
    case 3: l_analysis<3>(a, grid, s); break;
    case 4: l_analysis<4>(a, grid, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
hipError_t dev_gain(int np, const GainArgs& a, int grid, hipStream_t s) {
  KF_NP_SWITCH(np, l_gain, a, grid, s);
  return hipGetLastError();
}
hipError_t dev_jacobi(int np, const JacobiArgs& a, int grid, hipStream_t s) {
  KF_NP_SWITCH(np, l_jacobi, a, grid, s);
  return hipGetLastError();
}
hipError_t dev_propagate(int np, const PropArgs& a, hipStream_t s) {
  KF_NP_SWITCH(np, l_propagate, a, grid_for(a.N, KF_MAX_BLOCKS), s);
  return hipGetLastError();
}
hipError_t dev_invert(int np, const float* src, float* dst, int64_t N, int64_t ld, uint8_t* st, hipStream_t s) {
  KF_NP_SWITCH(np, l_invert, src, dst, N, ld, st, grid_for(N, KF_MAX_BLOCKS), s);
  return hipGetLastError();
}
hipError_t dev_operator(int np, const BandDesc* b, int band, const float* x, int64_t N, int64_t ld, float* h0,
                        float* h, int64_t h_ld, uint8_t* ok, hipStream_t s) {
  KF_NP_SWITCH(np, l_operator, b, band, x, N, ld, h0, h, h_ld, ok, grid_for(N, KF_MAX_BLOCKS), s);
  return hipGetLastError();
}
hipError_t dev_gp_operator(int np, int d, const BandDesc* b, int nb, const float* x, int64_t N, int64_t ld,
                           float* h0, float* h, int64_t ldh, hipStream_t s) {
  const int g = grid_for(N, KF_MAX_BLOCKS);
  // record-stream unroll: 4 pairs by default, 2 selectable (set_gp_unroll) for A/B
#define KF_GPOP(NP_, D_)                                                                                     \
  if (np == NP_ && d == D_) {                                                                               \
    if (g_gp_unroll == 2)                                                                                   \
      hipLaunchKernelGGL((gp_operator_kernel<NP_, D_, 2>), dim3(g), dim3(BLOCK), 0, s, b, nb, x, N, ld, h0, \
                         h, ldh);                                                                           \
    else                                                                                                    \
      hipLaunchKernelGGL((gp_operator_kernel<NP_, D_, 4>), dim3(g), dim3(BLOCK), 0, s, b, nb, x, N, ld, h0, \
                         h, ldh);                                                                           \
    return hipGetLastError();                                                                               \
  }
  KF_GPOP(10, 10) KF_GPOP(10, 4) KF_GPOP(7, 7) KF_GPOP(7, 4) KF_GPOP(4, 4) KF_GPOP(3, 3) KF_GPOP(2, 2)
#undef KF_GPOP
  return hipErrorInvalidValue;
}

hipError_t dev_hessian(int np, const BandDesc* b, int nb, const float* x, float* a, int64_t N, int64_t ld,
                       hipStream_t s) {
  KF_NP_SWITCH(np, l_hessian, b, nb, x, a, N, ld, grid_for(N, KF_MAX_BLOCKS), s);
  return hipGetLastError();
}
hipError_t dev_unpack(int np, const float* x, const float* a, int64_t N, int64_t ld, const int64_t* idx,
                      float* mean, float* unc, int64_t plane, hipStream_t s) {
  KF_NP_SWITCH(np, l_unpack, x, a, N, ld, idx, mean, unc, plane, grid_for(N, KF_MAX_BLOCKS), s);
  return hipGetLastError();
}
hipError_t dev_reduce(const double* partials, int n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(1), dim3(RED_BLOCK), 0, s, partials, n, out);
  return hipGetLastError();
}
hipError_t dev_gather(int elem_bytes, const void* src, const int64_t* idx, void* dst, int64_t n, int rows,
                      int64_t src_ld, int64_t dst_ld, hipStream_t s) {
  const int g = grid_for(n, KF_MAX_BLOCKS);
  switch (elem_bytes) {
    case 1: hipLaunchKernelGGL(gather_kernel<uint8_t>, dim3(g), dim3(BLOCK), 0, s, (const uint8_t*)src, idx,
                               (uint8_t*)dst, n, rows, src_ld, dst_ld); break;
    case 2: hipLaunchKernelGGL(gather_kernel<uint16_t>, dim3(g), dim3(BLOCK), 0, s, (const uint16_t*)src, idx,
                               (uint16_t*)dst, n, rows, src_ld, dst_ld); break;
    case 4: hipLaunchKernelGGL(gather_kernel<float>, dim3(g), dim3(BLOCK), 0, s, (const float*)src, idx,
                               (float*)dst, n, rows, src_ld, dst_ld); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
hipError_t dev_lut_nearest(const float* lut, int M, int D, const float* x, int64_t N, int64_t ld, int32_t* out,
                           hipStream_t s) {
  const size_t lds = (size_t)M * D * sizeof(float);
  if (lds > 160 * 1024 || D > MAX_D) return hipErrorInvalidValue;
  hipLaunchKernelGGL(lut_nearest_kernel, dim3(grid_for(N, KF_MAX_BLOCKS)), dim3(BLOCK), lds, s, lut, M, D, x, N,
                     ld, out);
  return hipGetLastError();
}

}  // namespace kf
