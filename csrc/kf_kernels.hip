// kf_kernels.hip — gfx950 (MI355X) launchers for the KaFKA engine kernels
// (templates in kf_device.h; the NP = 7 / 10 analysis instantiations live in
// kf_analysis7.hip / kf_analysis10.hip).
#include "kf_device.h"
#include <map>
#include <mutex>
#include <tuple>

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
// (AnalysisArgs.order).  Chunks of ORD_CHUNK pixels, ORD_PT consecutive pixels
// per thread (two 16-byte loads per DN16 band): class counts per chunk, a scan
// per class (one workgroup), a scatter that ranks the chunk's pixels in LDS and
// writes each class's run coalesced.  Three passes of ~4 B/px read + 4 B/px
// written; per-pixel decode (one pixel per thread) cost 1.0 ms per 10980^2 date
// (r4_v27), these ~0.3 ms.
constexpr int ORD_PT = 16;
constexpr int ORD_CHUNK = BLOCK * ORD_PT;
static_assert(ORD_CHUNK == KF_ORD_CHUNK, "host chunk-local partition (kf_host.cpp)");
constexpr int ORD_MAX_CLASSES = 8;   // <= 3 band groups

// bit i: pixel p0 + i (< N) has an observation in band bd (p0: this lane's
// first pixel, lane * ORD_PT past the wave's).  DN16 whose weight is positive
// exactly when dn > 0 (decode_obs: an uncertainty floor > 0, or a relative
// uncertainty that cannot underflow; no overflow of sig^2) on aligned full
// tiles: two vector loads.  Anything else: decode_obs with consecutive lanes on
// consecutive pixels (coalesced), a ballot per 64 pixels, each lane picking its
// 16 bits out of the wave's 16 ballots.
__device__ __forceinline__ uint32_t obs_bits(const BandDesc& bd, int64_t p0, int64_t N) {
  static_assert(ORD_PT == 16, "two 16-byte loads of uint16 DNs");
  const float ru = bd.rel_unc * bd.scale;
  const bool fast = bd.obs == OBS_DN16 && !(bd.unc_floor >= 1e18f) && fabsf(ru) < 1e13f &&
                    (bd.unc_floor > 0.f || (bd.rel_unc > 0.f && bd.scale > 0.f && ru > 1e-30f));
  const bool vec = fast && p0 + ORD_PT <= N && (((uintptr_t)(bd.dn + p0)) & 15) == 0;
  if (__all(vec)) {
    const uint4* v = reinterpret_cast<const uint4*>(bd.dn + p0);
    const uint4 lo = v[0], hi = v[1];
    const uint32_t u[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      m |= ((u[i] & 0xffffu) ? 1u : 0u) << (2 * i) | ((u[i] >> 16) ? 1u : 0u) << (2 * i + 1);
    return m;
  }
  const int lane = threadIdx.x & 63;
  const int64_t w0 = p0 - (int64_t)lane * ORD_PT;   // the wave's first pixel
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < ORD_PT; ++i) {
    const int64_t q = w0 + (int64_t)i * 64 + lane;
    float y = 0.f, w = 0.f;
    if (q < N) decode_obs<0>(bd, q, y, w);
    const uint64_t bal = __ballot(w > 0.f);
    // lane L owns pixels 16 L .. 16 L + 15 of the wave: ballot L / 4, bits 16 (L % 4) ..
    if ((lane >> 2) == i) m = (uint32_t)(bal >> (16 * (lane & 3))) & 0xffffu;
  }
  return m;
}

// classes of the ORD_PT pixels from p0 as 4-bit fields (obs_class numbering:
// (2^G - 1) - observed-group mask; fields of pixels >= N are not used)
template <int G>
__device__ __forceinline__ uint64_t obs_classes(const BandDesc* bands, const int32_t* grp, int nb, int64_t p0,
                                                int64_t N) {
  uint32_t g0 = 0u, g1 = 0u, g2 = 0u;
  for (int b = 0; b < nb; ++b) {
    const int g = (G > 1 && grp) ? grp[b] : 0;
    const uint32_t have = g == 0 ? g0 : (g == 1 ? g1 : g2);
    if (__all(have == 0xffffu)) continue;   // every pixel of the wave already observed in g (wave-uniform:
                                             // obs_bits' fallback is wave-cooperative)
    const uint32_t bits = obs_bits(bands[b], p0, N);
    if (g == 0) g0 |= bits;
    else if (g == 1) g1 |= bits;
    else g2 |= bits;
  }
  constexpr uint32_t K1 = (1u << G) - 1u;
  uint64_t cls = 0;
#pragma unroll
  for (int i = 0; i < ORD_PT; ++i) {
    const uint32_t key = ((g0 >> i) & 1u) | (((g1 >> i) & 1u) << 1) | (((g2 >> i) & 1u) << 2);
    cls |= (uint64_t)(K1 - key) << (4 * i);
  }
  return cls;
}

__device__ __forceinline__ int ord_valid(int64_t p0, int64_t N) {
  return p0 >= N ? 0 : (N - p0 < ORD_PT ? (int)(N - p0) : ORD_PT);
}

// pixels of class c among the first nv fields of cls
__device__ __forceinline__ int ord_count(uint64_t cls, int nv, int c) {
  int n = 0;
#pragma unroll
  for (int i = 0; i < ORD_PT; ++i) n += (i < nv && (int)((cls >> (4 * i)) & 15u) == c) ? 1 : 0;
  return n;
}

template <int G>
__global__ __launch_bounds__(BLOCK) void obs_count_kernel(const BandDesc* bands, const int32_t* grp, int nb,
                                                          int64_t N, int32_t* counts) {
  constexpr int K = 1 << G;
  __shared__ int red[BLOCK / 64][K];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t p0 = (int64_t)blockIdx.x * ORD_CHUNK + (int64_t)threadIdx.x * ORD_PT;
  const int nv = ord_valid(p0, N);
  const uint64_t cls = obs_classes<G>(bands, grp, nb, p0, N);   // every lane: wave-cooperative
#pragma unroll
  for (int c = 0; c < K; ++c) {
    int v = ord_count(cls, nv, c);
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) red[wv][c] = v;
  }
  __syncthreads();
  if (threadIdx.x < K) {
    int s = 0;
    for (int i = 0; i < BLOCK / 64; ++i) s += red[i][threadIdx.x];
    counts[(int64_t)blockIdx.x * K + threadIdx.x] = s;
  }
}

// counts [nc][K] -> each class's exclusive prefix over the chunks, in place;
// counts[nc * K + c] = class c's total (the scatter adds the totals of the
// classes before c).  Tiles of 1024 x ORD_SCAN_PT chunks: a load round trip per
// tile, a shuffle scan per wave, LDS wave totals, a carry per class.
constexpr int ORD_SCAN_PT = 8;

template <int K>
__global__ __launch_bounds__(1024) void obs_scan_kernel(int32_t* counts, int nc) {
  __shared__ int wtot[16][K];
  __shared__ int tot[K];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int carry[K];
#pragma unroll
  for (int c = 0; c < K; ++c) carry[c] = 0;
  for (int t0 = 0; t0 < nc; t0 += 1024 * ORD_SCAN_PT) {
    const int i0 = t0 + threadIdx.x * ORD_SCAN_PT;
    int v[ORD_SCAN_PT][K];
#pragma unroll
    for (int i = 0; i < ORD_SCAN_PT; ++i)
#pragma unroll
      for (int c = 0; c < K; ++c) v[i][c] = i0 + i < nc ? counts[(int64_t)(i0 + i) * K + c] : 0;
    int sum[K], incl[K];
#pragma unroll
    for (int c = 0; c < K; ++c) {
      int t = 0;
#pragma unroll
      for (int i = 0; i < ORD_SCAN_PT; ++i) t += v[i][c];
      sum[c] = t;
      for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(t, o);
        if (lane >= o) t += u;
      }
      incl[c] = t;
      if (lane == 63) wtot[wv][c] = t;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < K; ++c) {
      int add = 0;
      for (int w = 0; w < wv; ++w) add += wtot[w][c];
      if (threadIdx.x == 1023) tot[c] = add + incl[c];
      int run = carry[c] + add + incl[c] - sum[c];
#pragma unroll
      for (int i = 0; i < ORD_SCAN_PT; ++i) {
        if (i0 + i < nc) counts[(int64_t)(i0 + i) * K + c] = run;
        run += v[i][c];
      }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < K; ++c) carry[c] += tot[c];
    __syncthreads();
  }
  if (threadIdx.x < K) counts[(int64_t)nc * K + threadIdx.x] = carry[threadIdx.x];
}

template <int G>
__global__ __launch_bounds__(BLOCK) void obs_scatter_kernel(const BandDesc* bands, const int32_t* grp, int nb,
                                                            int64_t N, const int32_t* offs, int32_t* order) {
  constexpr int K = 1 << G;
  __shared__ int32_t buf[ORD_CHUNK];
  __shared__ int wtot[BLOCK / 64][K];
  __shared__ int start[K + 1];
  __shared__ int gbase[K];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t p0 = (int64_t)blockIdx.x * ORD_CHUNK + (int64_t)threadIdx.x * ORD_PT;
  const int nv = ord_valid(p0, N);
  const uint64_t cls = obs_classes<G>(bands, grp, nb, p0, N);   // every lane: wave-cooperative
  if (threadIdx.x < K && offs) {
    // the chunk's place in its class, after every pixel of the classes before it
    int g = offs[(int64_t)blockIdx.x * K + threadIdx.x];
    const int32_t* totals = offs + (int64_t)gridDim.x * K;
    for (int c = 0; c < (int)threadIdx.x; ++c) g += totals[c];
    gbase[threadIdx.x] = g;
  }
  // per class: this thread's exclusive rank within its wave, the wave totals
  int excl[K];
#pragma unroll
  for (int c = 0; c < K; ++c) {
    const int n = ord_count(cls, nv, c);
    int v = n;
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(v, o);
      if (lane >= o) v += t;
    }
    excl[c] = v - n;
    if (lane == 63) wtot[wv][c] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int c = 0; c < K; ++c) {
      start[c] = run;
      for (int i = 0; i < BLOCK / 64; ++i) run += wtot[i][c];
    }
    start[K] = run;
  }
  __syncthreads();
  // chunk-local partition (offs null): the classes in place, chunk-aligned
  // (read after the barrier below)
  if (threadIdx.x < K && !offs) gbase[threadIdx.x] = (int)(blockIdx.x * ORD_CHUNK) + start[threadIdx.x];
  // chunk-local slots in LDS (stable: thread order, then pixel order)
#pragma unroll
  for (int c = 0; c < K; ++c) {
    int slot = start[c] + excl[c];
    for (int i = 0; i < wv; ++i) slot += wtot[i][c];
#pragma unroll
    for (int i = 0; i < ORD_PT; ++i)
      if (i < nv && (int)((cls >> (4 * i)) & 15u) == c) buf[slot++] = (int32_t)(p0 + i);
  }
  __syncthreads();
  // each class's run of the chunk to its global range, coalesced
  const int n_all = start[K];
  for (int j = threadIdx.x; j < n_all; j += BLOCK) {
    int c = 0;
#pragma unroll
    for (int k = 1; k < K; ++k) c += j >= start[k] ? 1 : 0;
    order[gbase[c] + (j - start[c])] = buf[j];
  }
}

int obs_order_chunks(int64_t N) { return (int)((N + ORD_CHUNK - 1) / ORD_CHUNK); }

hipError_t dev_obs_order(const BandDesc* bands, const int32_t* grp, int nb, int G, int64_t N, int32_t* counts,
                         int32_t* order, bool local, hipStream_t s) {
  if (G < 1 || G > 3) return hipErrorInvalidValue;
  const int nc = obs_order_chunks(N);
  if (N <= 0) return hipSuccess;
#define KF_ORD_GO(G_)                                                                                   \
  if (local) {                                                                                          \
    hipLaunchKernelGGL(obs_scatter_kernel<G_>, dim3(nc), dim3(BLOCK), 0, s, bands, grp, nb, N,          \
                       (const int32_t*)nullptr, order);                                                 \
  } else {                                                                                              \
    hipLaunchKernelGGL(obs_count_kernel<G_>, dim3(nc), dim3(BLOCK), 0, s, bands, grp, nb, N, counts);   \
    hipLaunchKernelGGL(obs_scan_kernel<1 << G_>, dim3(1), dim3(1024), 0, s, counts, nc);                \
    hipLaunchKernelGGL(obs_scatter_kernel<G_>, dim3(nc), dim3(BLOCK), 0, s, bands, grp, nb, N, counts,  \
                       order);                                                                          \
  }
  if (G == 1) KF_ORD_GO(1)
  else if (G == 2) KF_ORD_GO(2)
  else KF_ORD_GO(3)
#undef KF_ORD_GO
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Per-chunk Gauss-Newton convergence (kf_core.h ChunkPartialArgs ...).

// Stage 1, one workgroup per (local chunk, group of CHUNK_GROUP_RUNS runs):
// thread t sums column offsets t, t + 256, .. of the group's runs in row
// order, then a fixed shuffle tree per wave and the wave sums in wave order.
// Stage 2, one thread per local chunk: the group totals in group order.  The
// host runner repeats exactly this order (kf_host.cpp), so a chunk's sum does
// not depend on the device or on the order the analysis visited its pixels in.
// (One workgroup per whole chunk was latency-bound: 256 dependent run loads
// per thread, one workgroup per CU on a 3882^2 share, 131 us per call.)
__global__ __launch_bounds__(BLOCK) void chunk_group_kernel(ChunkPartialArgs a) {
  const int c = blockIdx.x / a.groups, q = blockIdx.x - c * a.groups;
  const int g = a.lc_gid[c];
  if (!a.active[g]) return;   // frozen: its sum is no longer read (workgroup-uniform)
  const int s0 = a.lc_ptr[c] + q * CHUNK_GROUP_RUNS, s1 = a.lc_ptr[c + 1];
  if (s0 >= s1) return;       // past this chunk's runs (workgroup-uniform)
  const int n = s1 - s0 < CHUNK_GROUP_RUNS ? s1 - s0 : CHUNK_GROUP_RUNS;
  __shared__ int sst[CHUNK_GROUP_RUNS], slen[CHUNK_GROUP_RUNS];
  const int t = threadIdx.x;
  if (t < n) {
    sst[t] = a.seg_start[s0 + t];
    slen[t] = a.seg_len[s0 + t];
  }
  __syncthreads();
  bool short_runs = true;     // every run within one element per thread (chunk width <= 256)
  for (int k = 0; k < n; ++k) short_runs = short_runs && slen[k] <= BLOCK;
  const double qi = a.qinv[g];
  const int64_t cl = a.clamp;
  // integer quanta (chunk_quant): exact sums, any order
  int64_t acc = 0;
  if (short_runs) {
    // all the group's loads in flight before the adds
    float v[CHUNK_GROUP_RUNS];
#pragma unroll
    for (int k = 0; k < CHUNK_GROUP_RUNS; ++k) v[k] = (k < n && t < slen[k]) ? a.dn[sst[k] + t] : 0.f;
#pragma unroll
    for (int k = 0; k < CHUNK_GROUP_RUNS; ++k)
      if (k < n && t < slen[k]) acc += chunk_quant(v[k], qi, cl);
  } else {
    for (int k = 0; k < n; ++k)
      for (int i = t; i < slen[k]; i += BLOCK) acc += chunk_quant(a.dn[sst[k] + i], qi, cl);
  }
  __shared__ unsigned long long tot;
  if (t == 0) tot = 0ull;
  __syncthreads();
  if (acc) atomicAdd(&tot, (unsigned long long)acc);   // LDS integer adds: exact in any order
  __syncthreads();
  if (t == 0) a.gpart[(int64_t)c * a.groups + q] = (int64_t)tot;
}

__global__ __launch_bounds__(BLOCK) void chunk_total_kernel(ChunkPartialArgs a) {
  const int c = blockIdx.x * BLOCK + threadIdx.x;
  if (c >= a.n_local) return;
  const int g = a.lc_gid[c];
  if (!a.active[g]) return;
  const int ng = (a.lc_ptr[c + 1] - a.lc_ptr[c] + CHUNK_GROUP_RUNS - 1) / CHUNK_GROUP_RUNS;
  int64_t tot = 0;
  for (int q = 0; q < ng; ++q) tot += a.gpart[(int64_t)c * a.groups + q];
  a.part[g] = tot;
}

constexpr int DEC_BLOCK = 1024;
__global__ __launch_bounds__(DEC_BLOCK) void chunk_decide_kernel(ChunkDecideArgs a) {
  __shared__ double smax[DEC_BLOCK / 64];
  __shared__ int sact[DEC_BLOCK / 64], spx[DEC_BLOCK / 64], snew[DEC_BLOCK / 64];
  double mx = 0.0;
  int n_act = 0, px = 0, n_new = 0;
  for (int g = threadIdx.x; g < a.nc; g += DEC_BLOCK) {
    const bool was = a.active[g] != 0;
    bool stop = false;
    if (was) {
      int64_t tot = 0;
      for (int r = 0; r < a.world; ++r) tot += a.part_all[(int64_t)r * a.nc + g];   // exact
      const double norm = sqrt((double)tot * a.unit);
      mx = norm > mx ? norm : mx;
      stop = chunk_stops(norm, a.n_iter, a.min_iter, a.max_iter, a.tol);
    }
    a.newly[g] = stop ? 1 : 0;
    if (stop) {
      a.active[g] = 0;
      a.iters[g] = a.n_iter;
      ++n_new;
    } else if (was) {
      ++n_act;
      px += a.local_count[g];
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const double om = __shfl_xor(mx, off, 64);
    mx = om > mx ? om : mx;
    n_act += __shfl_xor(n_act, off, 64);
    px += __shfl_xor(px, off, 64);
    n_new += __shfl_xor(n_new, off, 64);
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    smax[wv] = mx;
    sact[wv] = n_act;
    spx[wv] = px;
    snew[wv] = n_new;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double m = 0.0;
    int na = 0, np_ = 0, nn = 0;
    for (int w = 0; w < DEC_BLOCK / 64; ++w) {
      m = smax[w] > m ? smax[w] : m;
      na += sact[w];
      np_ += spx[w];
      nn += snew[w];
    }
    a.info[0] = (double)na;
    a.info[1] = m;
    a.info[2] = (double)np_;
    a.info[3] = (double)nn;
    if (a.px_out) *a.px_out = np_;
  }
}

// Stable compaction of the visiting order to the active chunks' pixels, the
// x of pixels whose chunk stopped at this iteration copied into the next
// launch's output buffer on the way (16 consecutive slots per thread): counts
// per 4096-slot block, a scan (obs_scan_kernel), a scatter.
constexpr int CMP_PT = 16;
static_assert(BLOCK * CMP_PT == KF_CMP_CHUNK, "compaction block");

__device__ __forceinline__ int cmp_slot_px(const ChunkCompactArgs& a, int64_t q) {
  return a.order_in ? a.order_in[q] : (int)q;
}

__global__ __launch_bounds__(BLOCK) void chunk_count_kernel(ChunkCompactArgs a) {
  __shared__ int red[BLOCK / 64];
  const int64_t q0 = (int64_t)blockIdx.x * KF_CMP_CHUNK + (int64_t)threadIdx.x * CMP_PT;
  const int64_t n_in = visit_bounded(a.n_in, a.n_in, a.n_in_dev);
  int n = 0;
  for (int i = 0; i < CMP_PT; ++i) {
    const int64_t q = q0 + i;
    if (q >= n_in) break;
    const int p = cmp_slot_px(a, q);
    const int g = a.chunk_of[p];
    if (a.active[g]) {
      ++n;
    } else if (a.newly[g] && a.x_dst) {
      for (int j = 0; j < a.np; ++j) a.x_dst[(int64_t)j * a.ld + p] = a.x_src[(int64_t)j * a.ld + p];
    }
  }
  for (int off = 32; off > 0; off >>= 1) n += __shfl_xor(n, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < BLOCK / 64; ++w) t += red[w];
    a.counts[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(BLOCK) void chunk_scatter_kernel(ChunkCompactArgs a) {
  __shared__ int wtot[BLOCK / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t q0 = (int64_t)blockIdx.x * KF_CMP_CHUNK + (int64_t)threadIdx.x * CMP_PT;
  const int64_t n_in = visit_bounded(a.n_in, a.n_in, a.n_in_dev);
  uint32_t keep = 0;
  int px[CMP_PT];
  for (int i = 0; i < CMP_PT; ++i) {
    const int64_t q = q0 + i;
    px[i] = 0;
    if (q < n_in) {
      px[i] = cmp_slot_px(a, q);
      if (a.active[a.chunk_of[px[i]]]) keep |= 1u << i;
    }
  }
  const int n = __popc(keep);
  int v = n;
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  if (lane == 63) wtot[wv] = v;
  __syncthreads();
  int base = a.counts[blockIdx.x] + v - n;
  for (int w = 0; w < wv; ++w) base += wtot[w];
  for (int i = 0; i < CMP_PT; ++i)
    if ((keep >> i) & 1u) a.order_out[base++] = px[i];
}

int chunk_compact_blocks(int64_t n) { return (int)((n + KF_CMP_CHUNK - 1) / KF_CMP_CHUNK); }

hipError_t dev_chunk_partials(const ChunkPartialArgs& a, hipStream_t s) {
  if (a.n_local <= 0) return hipSuccess;
  if (a.groups <= 0 || a.gpart == nullptr || (int64_t)a.n_local * a.groups > INT32_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(chunk_group_kernel, dim3(a.n_local * a.groups), dim3(BLOCK), 0, s, a);
  hipLaunchKernelGGL(chunk_total_kernel, dim3((a.n_local + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, a);
  return hipGetLastError();
}

hipError_t dev_chunk_decide(const ChunkDecideArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(chunk_decide_kernel, dim3(1), dim3(DEC_BLOCK), 0, s, a);
  return hipGetLastError();
}

hipError_t dev_chunk_compact(const ChunkCompactArgs& a, hipStream_t s) {
  const int nb = chunk_compact_blocks(a.n_in);
  if (nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(chunk_count_kernel, dim3(nb), dim3(BLOCK), 0, s, a);
  hipLaunchKernelGGL(obs_scan_kernel<1>, dim3(1), dim3(1024), 0, s, a.counts, nb);
  hipLaunchKernelGGL(chunk_scatter_kernel, dim3(nb), dim3(BLOCK), 0, s, a);
  return hipGetLastError();
}

bool gp_operator_supported(int np, int d) {
  return (np == 10 && (d == 10 || d == 4)) || (np == 7 && (d == 7 || d == 4)) || (np == d && np >= 2 && np <= 4);
}

hipError_t dev_analysis(int np, const AnalysisArgs& a, int grid, hipStream_t s, int* n_part) {
  switch (np) {
    case 7: return dev_analysis_np7(a, grid, s, n_part);     // kf_analysis7.hip
    case 10: return dev_analysis_np10(a, grid, s, n_part);   // kf_analysis10.hip
    case 1: l_analysis<1>(a, grid, s, n_part); break;
    case 2: l_analysis<2>(a, grid, s, n_part); break;
    case 3: l_analysis<3>(a, grid, s, n_part); break;
    case 4: l_analysis<4>(a, grid, s, n_part); break;
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
// Fixed-order f64 sum of a launch's norm partials: one workgroup (at most
// KF_MAX_BLOCKS = 65536 entries, 512 KiB: a few microseconds).  No scratch
// buffer, so reductions on different streams never share state.
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
