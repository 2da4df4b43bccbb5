// kf_core.h — per-pixel math shared by the gfx950 kernels and the host runner.
//
// Every routine here is written once as __host__ __device__ code: the HIP
// kernels in kf_kernels.hip run it one pixel per lane on MI355X, and
// kf_host.cpp runs the *same* source over an OpenMP loop on the CPU (the
// CPU path of the engine and the numerics harness for CI without a GPU).
//
// Reference semantics (QCDIS/KaFKA-InferenceEngine):
//   * analysis  = kafka/inference/solvers.py:100-145 (variational_kalman_multiband)
//                 with the Gauss-Newton linearisation of kafka/linear_kf.py:245-307
//   * operators = kafka/inference/utils.py:130-219 (GP emulator operators),
//                 kafka/observation_operators/sar_forward_model.py:13-106 (WCM)
//   * propagators = kafka/inference/kf_tools.py:174-353, blend :75-96
// The reference builds one (n_p N)x(n_p N) sparse system and factors it with
// SuperLU; every block is n_p x n_p, so here each pixel's
// block lives in registers as a packed upper triangle and is factored with an
// unrolled Cholesky.
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define KF_HD __host__ __device__ __forceinline__
#else
#define KF_HD inline __attribute__((always_inline))
#endif

// KF_PHASE_CLOCKS (measuring build, `_build.py --prof` -> module _kafka_hip_prof,
// selected with KAFKA_PROF=1): the matrix-core analysis kernels add the shader
// cycles (s_memtime) each wave spends in a phase to per-wave counters, summed
// into kf_phase_clk[slot] at the end of the kernel; ext.phase_clocks() reads
// them.  The clock reads drain lgkmcnt, so the build runs somewhat slower: it
// attributes time, it does not time the release kernel.
enum : int {
  KF_PH_PROLOGUE = 0,   // LDS table staging
  KF_PH_FORECAST = 1,   // fused forecast + prior right-hand side
  KF_PH_BAND_IN = 2,    // observation decode, GP inputs
  KF_PH_GP = 3,         // gp_mfma_sums: operands, chunk loop, extraction
  KF_PH_BAND_OUT = 4,   // value / Jacobian, normal equations
  KF_PH_SOLVE = 5,      // analysis_epilogue: factor, solve, stores
  KF_PH_GROUPS = 6,     // pixel groups (count)
  KF_PH_NSLOT = 8
};
#if defined(KF_PHASE_CLOCKS) && defined(__HIPCC__)
static __device__ unsigned long long kf_phase_clk[KF_PH_NSLOT];
#endif
#if defined(KF_PHASE_CLOCKS) && defined(__HIP_DEVICE_COMPILE__)
// per-wave accumulators in registers, added to kf_phase_clk once per wave at
// the end of the kernel (per-boundary atomics on 8 shared addresses serialise
// in one L2 channel and sit in vmcnt ahead of the wave's own loads)
struct KfPhaseAcc {
  uint64_t t0;
  uint64_t acc[KF_PH_NSLOT];
};
#define KF_PHASE_PARAM , ::KfPhaseAcc& kf_pc_
#define KF_PHASE_ARG , kf_pc_
#define KF_PHASE_KERNEL_BEGIN                                 \
  ::KfPhaseAcc kf_pc_;                                      \
  for (int s_ = 0; s_ < KF_PH_NSLOT; ++s_) kf_pc_.acc[s_] = 0; \
  kf_pc_.t0 = __builtin_amdgcn_s_memtime();
#define KF_PHASE(slot)                                  \
  {                                                     \
    const uint64_t t1_ = __builtin_amdgcn_s_memtime();  \
    kf_pc_.acc[slot] += t1_ - kf_pc_.t0;                \
    kf_pc_.t0 = t1_;                                    \
  }
#define KF_PHASE_COUNT(slot) kf_pc_.acc[slot] += 1;
#define KF_PHASE_KERNEL_END                                                                      \
  if ((threadIdx.x & 63) == 0)                                                                   \
    for (int s_ = 0; s_ < KF_PH_NSLOT; ++s_) atomicAdd(&kf_phase_clk[s_], (unsigned long long)kf_pc_.acc[s_]);
#else
#define KF_PHASE_PARAM
#define KF_PHASE_ARG
#define KF_PHASE_KERNEL_BEGIN
#define KF_PHASE(slot)
#define KF_PHASE_COUNT(slot)
#define KF_PHASE_KERNEL_END
#endif

// KF_CHECKED (debug build, `_build.py --checked` -> module _kafka_hip_checked,
// selected with KAFKA_CHECKED=1): index assertions on the gather / scatter /
// neighbour paths (SURVEY.md §5.2 "explicit bounds assertions in the debug
// build").  A failed check prints the condition and traps (device) or aborts
// (host runner); the release build compiles them away.
#ifdef KF_CHECKED
#include <stdio.h>
#include <stdlib.h>
#if defined(__HIPCC__)
#define KF_DCHECK(c)                                                          \
  do {                                                                        \
    if (!(c)) {                                                               \
      printf("KF_DCHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);        \
      __builtin_trap();                                                       \
    }                                                                         \
  } while (0)
#else
#define KF_DCHECK(c)                                                          \
  do {                                                                        \
    if (!(c)) {                                                               \
      fprintf(stderr, "KF_DCHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      abort();                                                                \
    }                                                                         \
  } while (0)
#endif
#else
#define KF_DCHECK(c) ((void)0)
#endif

namespace kf {

constexpr int MAX_D = 16;         // max mapped inputs per band / max state size
constexpr int MAX_NT = 136;       // ntri(16)
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
constexpr float LN10 = 2.302585092994046f;
constexpr float LOG2_10 = 3.321928094887362f;
constexpr float DEG2RAD = 0.017453292519943295f;

KF_HD constexpr int ntri(int n) { return n * (n + 1) / 2; }
constexpr int FD_PRECOMP = -1;    // AnalysisArgs.fast_d: all bands OP_PRECOMP
constexpr int FD_LINEAR = -2;     // AnalysisArgs.fast_d: all bands OP_LINEAR (identity / selection)
// packed upper triangle, row-major: (0,0) (0,1) .. (0,n-1) (1,1) ..
KF_HD constexpr int tri(int n, int i, int j) { return i * n - (i * (i - 1)) / 2 + (j - i); }
template <int NP> KF_HD constexpr int sym(int i, int j) { return i <= j ? tri(NP, i, j) : tri(NP, j, i); }

// ---------------------------------------------------------------------------
// enums shared with Python (kafka_inferenceengine_amd/ops/_abi.py)
enum ObsKind : int32_t { OBS_NONE = 0, OBS_F32 = 1, OBS_DN16 = 2, OBS_BF16 = 3, OBS_BF16Y = 4 };
enum OpKind : int32_t { OP_PRECOMP = 0, OP_LINEAR = 1, OP_GP = 2, OP_SAR = 3 };
enum PropMode : int32_t {
  PROP_PRIOR = 0,         // no_propagation: reset to prior (kf_tools.py:316-353)
  PROP_PRIOR_PARTIAL = 1, // LAI propagator generalised (kf_tools.py:292-314)
  PROP_INFO_APPROX = 2,   // diagonal information-filter approx (kf_tools.py:247-289)
  PROP_INFO_EXACT = 3,    // (I + P^-1 Q)^-1 P^-1 (kf_tools.py:208-245)
  PROP_STANDARD = 4,      // covariance form P + Q (kf_tools.py:174-205)
  PROP_IDENTITY = 5       // x_f = M x_a, P_f^-1 = P_a^-1 (no inflation)
};
enum StatusBits : uint8_t {
  ST_OK = 0, ST_NONSPD = 1, ST_NONFINITE = 2, ST_BAD_OP = 4, ST_NO_OBS = 8, ST_FALLBACK = 16,
  // a GP band's input (at the final iteration's linearisation point) lies
  // outside the emulator's training box (widened by models/operators.py GP_DOMAIN_MARGIN, BandDesc.dom_*):
  // the emulator extrapolates there -- the analytic operator of the reference
  // refuses such states (sar_forward_model.py:68-71,102-105: ValueError)
  ST_OUT_OF_DOMAIN = 32
};

// One observation band as seen by the fused analysis kernel.  Built on the
// host by kf_bindings (pack_band_descs) so the C++ layout is authoritative.
struct BandDesc {
  int32_t op, obs, d, T;
  int32_t Tp;                  // GP: the first Tp record pairs carry alpha > 0, the rest alpha < 0
  int32_t gpm_nchunk;          // GP on MFMA: 32-point chunks of the split-f16 table (0: VALU path only)
  int32_t map[MAX_D];          // state index feeding input d of the operator
  float scale, rel_unc, unc_floor, offset;
  float coef[MAX_D];           // LINEAR: c_j per state j; GP: lambda_d; SAR: A,B,C,D,E,theta
  float center[MAX_D];         // GP input centre (training mean), subtracted in-kernel
  const float* gp;             // GP records [T/2][d+1][2]: L + log2|alpha|, B[d] (models/gp.py)
  const float* y;              // OBS_F32 observation
  const float* w;              // OBS_F32 inverse variance (weight)
  const uint8_t* mask;         // optional validity
  const uint16_t* dn;          // OBS_DN16 digital numbers (0 = nodata)
  const float* aux;            // per-pixel auxiliary (SAR incidence angle, deg)
  const float* pre_h0;         // OP_PRECOMP H0 [N]
  const float* pre_h;          // OP_PRECOMP h [NP][ld]
  float* h0_out;               // optional diagnostics: H0 at the linearisation point
  int64_t pre_ld;              // leading dim of pre_h
  const void* gpm;             // GP split-f16 MFMA fragments (kf_gp_mfma.h, models/gp.py:mfma_tables)
  float gpm_scale;             // 2^sigma: undoes the f16-range shift folded into the table's L'
  int32_t map_identity;        // 1: map[d] == d for every input d (full-state GP: no gather / scatter)
  int32_t map_kind;            // GPM_MAP_*: a map known at compile time (JRC-TIP bands), 0: runtime map
  int32_t dom_check;           // GP: the training box of the centred inputs (+ GP_DOMAIN_MARGIN) is set:
  float dom_lo[MAX_D];         // the host folds the bands' boxes into AnalysisArgs.dom_* (state space)
  float dom_hi[MAX_D];
};


// JRC-TIP band mappers (kafka/inference/kf_tools.py:19-23, band_selecta): the
// matrix-core kernel gathers the GP inputs and updates only the 4 x 4 touched
// entries of A with these compiled in instead of the runtime map's selects.
constexpr int GPM_MAP_RUNTIME = 0, GPM_MAP_TIP_VIS = 2, GPM_MAP_TIP_NIR = 3;
// AnalysisArgs.band_layout: BAND_LAYOUT_TIP = exactly two bands, the JRC-TIP VIS
// then NIR maps (kafka/inference/utils.py:148-153), 7-parameter state
// BAND_LAYOUT_SHARED_X = every band a full-state GP (identity map, D = NP)
// with the same centre: the global-table matrix-core kernel builds the
// exponent operand once per Gauss-Newton iteration (kf_gp_mfma.h)
constexpr int BAND_LAYOUT_RUNTIME = 0, BAND_LAYOUT_TIP = 1, BAND_LAYOUT_SHARED_X = 2;

struct PropArgs {
  int64_t N, ld;
  int32_t mode, blend, quirk_blend, pad0;
  uint32_t prop_mask;    // PROP_PRIOR_PARTIAL: which parameters are propagated
  const float* x_a;      // [NP][ld]
  const float* p_a;      // [NT][ld] analysis precision (or covariance for STANDARD)
  float* x_f;            // [NP][ld]
  float* p_f;            // [NT][ld]
  float m[MAX_D];        // diagonal trajectory model
  float q[MAX_D];        // diagonal trajectory uncertainty
  const float* q_pix;    // optional per-pixel Q [NP][ld]
  float reset_mean[MAX_D];
  float reset_cinv[MAX_NT];
  float blend_mean[MAX_D];
  float blend_cinv[MAX_NT];
  const float* blend_mean_pix;   // optional per-pixel prior mean [NP][ld]
  const float* blend_cinv_pix;   // optional per-pixel prior precision [NT][ld]
  uint8_t* status;
  // Covariance-form consumers of a fused forecast (K1g).  cov_fast: reset_cov
  // holds reset_cinv^-1 (packed), so the forecast covariance is that constant
  // with one Sherman-Morrison rank-1 update per propagated parameter
  // (gain_forecast) instead of a Cholesky inverse per pixel.  pa_pdiag: the
  // analysis rows tri(j, j) of the propagated j hold the analysis PRECISION
  // diagonal (the gain form's stored rows), read as is instead of inverting p_a.
  int32_t cov_fast, pa_pdiag;
  float reset_cov[MAX_NT];
};

// Dense row-strip geometry (every pixel of the strip and of the halo rows
// active): neighbours and degrees follow from the pixel index, no [4][N]
// table read.  Local pixel p = r * w + c; halo-up pixel of column c at N + c,
// halo-down at N + n_up + c (parallel/partition.py:neighbour_table layout).
struct StripGeo {
  int64_t w, n_up;       // w = 0: not dense, use the neighbour table
  int32_t h, halo;       // rows; bit 0: halo row above, bit 1: halo row below
};

KF_HD int32_t geo_neighbour(const StripGeo& g, int64_t N, int64_t p, int k) {
  const uint32_t w = (uint32_t)g.w;
  const uint32_t r = (uint32_t)p / w, c = (uint32_t)p - r * w;
  switch (k) {
    case 0: return r > 0 ? (int32_t)(p - w) : ((g.halo & 1) ? (int32_t)(N + c) : -1);
    case 1: return r + 1 < (uint32_t)g.h ? (int32_t)(p + w) : ((g.halo & 2) ? (int32_t)(N + g.n_up + c) : -1);
    case 2: return c > 0 ? (int32_t)(p - 1) : -1;
    default: return c + 1 < w ? (int32_t)(p + 1) : -1;
  }
}

// Compile-time launch specialisations of the fused analysis (analysis_epilogue
// / pixel_analysis_mfma SPEC): with the forecast fused (AnalysisArgs.prop set)
// the explicit-forecast and band-chunk paths are dropped, and without the
// regulariser its prepare; the cold code no longer holds SGPRs across the
// hot path (TIP kernel: 89 -> 18 SGPR spill slots).
constexpr int SPEC_ANY = 0, SPEC_PROP = 1, SPEC_PROP_REG = 2;
// SPEC_PROP_PF: SPEC_PROP whose grid loop also loads the next pixel group's
// forecast inputs ahead (small emulators, kf_device.h:analysis_mfma_kernel)
constexpr int SPEC_PROP_PF = 3;

// AnalysisArgs.variant: the production kernel (AV_DEFAULT) or an alternate
// device path kept as a test oracle -- each is bit-identical to the default or
// pinned against it by a GPU test (tests/test_gpu*.py, test_oracles.py); no
// environment switch selects them in production runs.
enum AnalysisVariant : int32_t {
  AV_DEFAULT = 0,
  AV_VALU_ORACLE = 4,        // GP sums on the f32 VALU record loop instead of the matrix cores
  AV_GT_PREFETCH = 7,        // global tables: next chunk's fragments loaded under the current one
  AV_RUNTIME_LAYOUT = 10,    // JRC-TIP bands through the runtime-layout kernel (BAND_LAYOUT_TIP's oracle)
  AV_PER_BAND_OPERAND = 14,  // BAND_LAYOUT_SHARED_X: exponent operand rebuilt per band
  AV_BLOCK_ORDER = 16,       // exponent MFMAs block by block (gpm_il_default's other order)
  AV_GENERIC_SPEC = 18       // fused forecast through the generic launch instead of SPEC_PROP
};

struct AnalysisArgs {
  int64_t N, ld;
  int32_t n_bands, solve;
  int32_t fast_d, fast_obs;  // host hint: all bands GP with fast_d inputs, one encoding (0: generic)
  int32_t variant;           // AnalysisVariant (AV_DEFAULT; the others are test oracles)
  int32_t gpm_frags;         // > 0: every band has an MFMA table; LDS fragments (16 B) of all bands + 1 zero
  int32_t gpm_global;        // 1: every band has an MFMA table, read from global memory (too large for LDS)
  const BandDesc* bands;
  const float* x_prev;   // [NP][ld] linearisation point
  const float* x_f;      // [NP][ld] forecast mean
  const float* pf_inv;   // [NT][ld] forecast precision (packed)
  float* x_out;          // [NP][ld]
  float* a_out;          // [NT][ld] analysis precision (may be null)
  float* b_out;          // [NP][ld] rhs (regulariser / band-chunk path, may be null)
  const float* a_in;     // [NT][ld] band-chunk accumulation: start from (a_in, b_in) instead of the prior
  const float* b_in;     // [NP][ld]
  uint8_t* status;       // per-pixel flags (may be null)
  double* partials;      // per-block sum (x_out - x_prev)^2
  const PropArgs* prop;  // fused propagation (device copy; x_f / pf_inv unused, x_prev null = linearise at the forecast)
  float* out_mean;       // fused output (DeviceOutput): x and 1/sqrt(diag A) into [NP][out_plane] rasters
  float* out_unc;
  const int64_t* out_idx;  // raster position of each pixel (null: identity)
  int64_t out_plane;
  // K9 regulariser prepare fused into the epilogue (reg_v non-null): A_reg = A +
  // g deg E_R -> a_out, u = A_reg^-1 b -> x_out, V = A_reg^-1 E_R -> reg_v [k*NP][ld];
  // no convergence partial (the JACOBI_FINISH pass computes it)
  float reg_gamma;
  uint32_t reg_mask;
  const int32_t* reg_nbr;  // [4][N] neighbour table (degrees) unless reg_geo.w > 0
  float* reg_v;
  float* x0_out;           // the linearisation point (the fused forecast when x_prev is null)
  StripGeo reg_geo;
  // Gauss-Newton iterations run by this launch (1, or 2 = the first iteration,
  // which can never end the loop (min_iterations = 2, linear_kf.py:297-304),
  // kept in registers: solved, its norm partial to partials_first, and the
  // second linearised at its x; outputs as for one launch of the second)
  int32_t gn_fused;
  // host hint: the bands form a layout known at compile time (BAND_LAYOUT_*),
  // selecting a kernel with the band loop unrolled over fixed maps; 0: runtime
  int32_t band_layout;
  double* partials_first;  // per-block sum (x_1 - x_0)^2 of the first fused iteration
  // pixel visiting order (null: 0..N-1): the pixels with an observation first
  // (obs_order), so cloudy pixels fill whole waves that skip the GP -- the
  // emulator runs on observed pixels only, as in the reference's operator
  // (utils.py:130-170, run_emulator on x0[mask])
  const int32_t* order;
  // visiting slots of this launch (0: N): the per-chunk Gauss-Newton loop
  // (EngineConfig.convergence_chunk) visits only the pixels of the chunks that
  // have not converged, order[0 .. n_visit)
  int64_t n_visit;
  // null, or the count of slots to visit in device memory (<= n_visit, which
  // then only bounds the grid): a launch queued before the host has read the
  // count, the per-chunk loop's iterations past the first read decision
  const int32_t* n_visit_dev;
  // per-pixel |x - x0|^2 of the launch's last iteration (the per-chunk norms,
  // chunk_partials_kernel), stored at the pixel index; may be null
  float* dn_out;
  // packed precision rows stored to a_out (bit t: row t); 0 = every row.  The
  // engine's store_precision="auto" keeps only what the next forecast reads
  // (the LAI propagator: the TLAI diagonal entry, kf_tools.py:292-314)
  uint64_t a_rows;
  // GP domain box in state space (ST_OUT_OF_DOMAIN): the intersection over the
  // GP bands of their inputs' training boxes mapped to the state indices they
  // read (ops/kernels.py make_band_table); +-inf where no band constrains j
  int32_t dom_check;
  float dom_lo[MAX_D];
  float dom_hi[MAX_D];
  // Line tables (matrix-core kernels): the launch's first Gauss-Newton
  // iteration is linearised at a partial-reset forecast (x_prev null), whose
  // parameters other than the single propagated one (line_j; -1: none) are the
  // reset mean for every pixel.  Each GP band's value and input gradient there
  // are functions of x_f,j alone, tabulated on the host in float64 as cubic
  // Hermite pieces over line_n intervals from line_t0 (spacing 1 / line_inv_h):
  // [line_n][n_bands][D + 1][4] coefficients in s = (t - t_k) / h (value, then
  // d/d input d).  A wave whose observed pixels all lie inside the table
  // evaluates the polynomials instead of the GP sums (models/gp.py:line_table).
  const float* line_tab;
  float line_t0, line_inv_h;
  int32_t line_n, line_j;
};

// slots visited by a launch: n_visit (0: N), or the device count (<= that bound)
KF_HD int64_t visit_bounded(int64_t n_visit, int64_t N, const int32_t* n_dev) {
  const int64_t n = n_visit > 0 ? n_visit : N;
  if (!n_dev) return n;
  const int64_t d = *n_dev;
  return d < 0 ? 0 : (d < n ? d : n);
}
KF_HD int64_t visit_count(const AnalysisArgs& a) { return visit_bounded(a.n_visit, a.N, a.n_visit_dev); }

// the linearisation point outside the launch's GP domain box (NaN counts as
// outside); AP: the launch arguments in any address space
template <int NP, typename AP>
KF_HD bool state_out_of_domain(AP a, const float (&x)[NP]) {
  if (!a->dom_check) return false;
  bool o = false;
#pragma unroll
  for (int j = 0; j < NP; ++j) o = o || !(x[j] >= a->dom_lo[j] && x[j] <= a->dom_hi[j]);
  return o;
}
// packed precision row t stored under AnalysisArgs.a_rows
KF_HD bool a_row_on(uint64_t rows, int t) { return rows == 0 || ((rows >> t) & 1u); }


// ---------------------------------------------------------------------------
// small helpers

// Pixel of visiting slot q under AnalysisArgs.order (null: the identity).
KF_HD int64_t visit_px(const int32_t* order, int64_t q) { return order ? (int64_t)order[q] : q; }
template <int NP>
KF_HD float gather_state(const float (&x)[NP], int idx) {
  float v = x[0];
#pragma unroll
  for (int j = 1; j < NP; ++j) v = (idx == j) ? x[j] : v;
  return v;
}

// The same select with a wave-uniform index for the matrix-core kernels: the
// empty asm between the steps keeps the chain from being recognised as a
// dynamically indexed private array, which hipcc lowers to a 28-byte scratch
// store + per-input scratch loads per band (the round-2 "32 B scratch").
template <int NP>
KF_HD float gather_state_u(const float (&x)[NP], int idx) {
  float v = x[0];
#pragma unroll
  for (int j = 1; j < NP; ++j) {
    v = (idx == j) ? x[j] : v;
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(v));
#endif
  }
  return v;
}

KF_HD float kexp2(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_exp2f(x);
#else
  return exp2f(x);
#endif
}

// (not `v - v == 0`: with FP contraction the compiler rewrites a product's
// `v - v` into fma(a, b, -a*b), the product's rounding error, which is != 0)
KF_HD bool finitef(float v) { return __builtin_isfinite(v); }

// Hardware reciprocal / reciprocal square root (1 ulp) instead of the ~10-
// instruction IEEE division expansion; the per-pixel solves are f32 anyway.
KF_HD float kf_rcp(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rcpf(x);
#else
  return 1.f / x;
#endif
}
KF_HD float kf_rsqrt(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rsqf(x);
#else
  return 1.f / sqrtf(x);
#endif
}

// Wave-uniform read-only data (band descriptors, GP training records) is read
// through the constant address space so hipcc emits scalar s_load/s_buffer
// loads into SGPRs (one fetch per wave, no VGPRs, no vector-memory traffic).
#if defined(__HIP_DEVICE_COMPILE__)
#define KF_CONST_AS __attribute__((address_space(4)))
#else
#define KF_CONST_AS
#endif
template <typename T>
KF_HD const KF_CONST_AS T* cptr(const T* p) { return (const KF_CONST_AS T*)(p); }

// Opaque copy of a wave-uniform pointer: loads through the result cannot be
// hoisted out of the enclosing (pixel) loop, so rarely used constants are
// re-fetched with s_load where needed instead of pinning SGPRs (and spilling
// them to VGPR lanes) across the GP loop.
template <typename T>
KF_HD const KF_CONST_AS T* opaque(const KF_CONST_AS T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+s"(p));
#endif
  return p;
}

// Opaque copy of a per-lane value: address arithmetic derived from the result
// is recomputed where it is used instead of being hoisted out of an enclosing
// loop and kept live across it (the fused Gauss-Newton loop of
// pixel_analysis: ~60 hoisted 64-bit row addresses took 156 -> 256 VGPRs).
KF_HD int64_t opaque_lane(int64_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(v));
#endif
  return v;
}

// Pixel p of an SoA row: `row` (array + r * ld) is wave-uniform and p's byte
// offset is formed in 32 bits, so gfx950 addresses the element as SGPR base +
// 32-bit VGPR offset (global_load/store saddr form) -- one offset VGPR shared
// by every row instead of a 64-bit VGPR address (2 VALU, 2 VGPRs) per access.
// Valid while N * sizeof(T) < 2^32: the host wrappers (ops/kernels.py) bound
// N, out_plane < 2^30.
// The row base goes through an SGPR asm operand (as a global-address-space
// pointer, so the access stays a global_* instruction) so the optimiser cannot
// fold it and the lane offset into one 64-bit VGPR sum: every row passed here
// must be wave-uniform (kernel arguments, BandDesc fields, uniform row indices).
template <typename T>
KF_HD T* pxp(T* row, int64_t p) {
#if defined(__HIP_DEVICE_COMPILE__)
  __attribute__((address_space(1))) char* g = (__attribute__((address_space(1))) char*)row;
  asm volatile("" : "+s"(g));
  return (T*)(g + (uint32_t)((uint32_t)p * (uint32_t)sizeof(T)));
#else
  return (T*)((char*)row + (uint32_t)((uint32_t)p * (uint32_t)sizeof(T)));
#endif
}
template <typename T>
KF_HD const T* pxp(const T* row, int64_t p) {
#if defined(__HIP_DEVICE_COMPILE__)
  const __attribute__((address_space(1))) char* g = (const __attribute__((address_space(1))) char*)row;
  asm volatile("" : "+s"(g));
  return (const T*)(g + (uint32_t)((uint32_t)p * (uint32_t)sizeof(T)));
#else
  return (const T*)((const char*)row + (uint32_t)((uint32_t)p * (uint32_t)sizeof(T)));
#endif
}
// KF_PXS: the SGPR-base form (pxp); KF_PX: plain 64-bit indexing.  The SGPR
// form is used where the row bases are short-lived (the analysis epilogue's
// stores, after the GP loop): applied to every access it kept ~60 row bases
// live in SGPRs across the fused Gauss-Newton loop and spilled them to VGPR
// lanes (186 spill slots, 171 VGPRs: one wave per SIMD fewer).
#define KF_PXS(base, off, p) (*::kf::pxp((base) + (off), (p)))
#define KF_PX(base, off, p) ((base)[(off) + (p)])

// In-place packed Cholesky A = U^T U (U upper, stored in A's packed slots).
// Convention: the diagonal slots hold 1 / U_jj (what the solves multiply by);
// only chol_solve / chol_inverse read a factor.
template <int NP>
KF_HD bool chol_packed(float (&A)[ntri(NP)]) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    float s = A[tri(NP, j, j)];
#pragma unroll
    for (int k = 0; k < j; ++k) s = fmaf(-A[tri(NP, k, j)], A[tri(NP, k, j)], s);
    ok = ok && (s > 0.f) && finitef(s);
    s = s > 0.f ? s : 1.f;
    const float inv = kf_rsqrt(s);
    A[tri(NP, j, j)] = inv;
#pragma unroll
    for (int i = j + 1; i < NP; ++i) {
      float t = A[tri(NP, j, i)];
#pragma unroll
      for (int k = 0; k < j; ++k) t = fmaf(-A[tri(NP, k, j)], A[tri(NP, k, i)], t);
      A[tri(NP, j, i)] = t * inv;
    }
  }
  return ok;
}

// Solve U^T U x = b with U from chol_packed (b overwritten by x).
template <int NP>
KF_HD void chol_solve(const float (&U)[ntri(NP)], float (&b)[NP]) {
#pragma unroll
  for (int i = 0; i < NP; ++i) {  // U^T z = b
    float t = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) t = fmaf(-U[tri(NP, k, i)], b[k], t);
    b[i] = t * U[tri(NP, i, i)];
  }
#pragma unroll
  for (int i = NP - 1; i >= 0; --i) {  // U x = z
    float t = b[i];
#pragma unroll
    for (int k = i + 1; k < NP; ++k) t = fmaf(-U[tri(NP, i, k)], b[k], t);
    b[i] = t * U[tri(NP, i, i)];
  }
}

// Packed inverse of an SPD matrix from its Cholesky factor (column by column).
template <int NP>
KF_HD void chol_inverse(const float (&U)[ntri(NP)], float (&Ainv)[ntri(NP)]) {
#pragma unroll
  for (int c = 0; c < NP; ++c) {
    float e[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) e[i] = (i == c) ? 1.f : 0.f;
    chol_solve<NP>(U, e);
#pragma unroll
    for (int i = 0; i <= c; ++i) Ainv[tri(NP, i, c)] = e[i];
  }
}

template <int NP>
KF_HD void symv(const float (&A)[ntri(NP)], const float (&x)[NP], float (&y)[NP]) {
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < NP; ++j) t = fmaf(A[sym<NP>(i, j)], x[j], t);
    y[i] = t;
  }
}

KF_HD float bf16_to_f32(uint16_t b) {
  const uint32_t u = (uint32_t)b << 16;
  float f;
  __builtin_memcpy(&f, &u, 4);
  return f;
}

// ---------------------------------------------------------------------------
// observation decode: returns weight w (inverse variance, 0 when masked) and y
// FOBS != 0 compiles a single encoding (fast-path kernels).
template <int FOBS = 0>
KF_HD void decode_obs(const BandDesc& bd, int64_t p, float& y_out, float& w_out) {
  // locals, assigned once at the end: conditional stores through the output
  // references made the compiler spill (y, w) to scratch in generic kernels
  float y = 0.f, w = 0.f;
  if (FOBS == OBS_DN16 || (FOBS == 0 && bd.obs == OBS_DN16)) {
    const uint16_t dn = KF_PX(bd.dn, 0, p);
    const float yd = (float)dn * bd.scale;
    const float sig = fmaxf(bd.rel_unc * yd, bd.unc_floor);
    const bool ok = dn > 0 && sig > 0.f;
    w = ok ? kf_rcp(sig * sig) : 0.f;
    y = dn > 0 ? yd : 0.f;
  } else if (FOBS == OBS_F32 || FOBS == OBS_BF16 || (FOBS == 0 && (bd.obs == OBS_F32 || bd.obs == OBS_BF16))) {
    float yv, wv;
    if (FOBS == OBS_F32 || (FOBS == 0 && bd.obs == OBS_F32)) {
      yv = KF_PX(bd.y, 0, p);
      wv = KF_PX(bd.w, 0, p);
    } else {
      // bf16 (y, w) pairs: half the ingest bytes of f32; math stays f32
      yv = bf16_to_f32(reinterpret_cast<const uint16_t*>(bd.y)[p]);
      wv = bf16_to_f32(reinterpret_cast<const uint16_t*>(bd.w)[p]);
    }
    const bool keep = (!bd.mask || KF_PX(bd.mask, 0, p)) && (wv > 0.f) && finitef(wv) && finitef(yv);
    y = keep ? yv : 0.f;
    w = keep ? wv : 0.f;
  } else if (FOBS == OBS_BF16Y || (FOBS == 0 && bd.obs == OBS_BF16Y)) {
    // bf16 y only (half the ingest bytes of (y, w) pairs), NaN = no data; the
    // weight follows the relative-uncertainty model of the DN16 path
    const float yv = bf16_to_f32(reinterpret_cast<const uint16_t*>(bd.y)[p]);
    const float sig = fmaxf(bd.rel_unc * fabsf(yv), bd.unc_floor);
    const bool keep = (!bd.mask || KF_PX(bd.mask, 0, p)) && finitef(yv) && sig > 0.f;
    y = keep ? yv : 0.f;
    w = keep ? kf_rcp(sig * sig) : 0.f;
  }
  y_out = y;
  w_out = w;
}

// obs_order class of pixel p: the band groups (grp[b], null: one group) with
// an observation at p, as a bit mask, mapped so that class 0 is "observed in
// every group" and class 2^G - 1 "in none".
KF_HD int obs_class(const BandDesc* bands, const int32_t* grp, int nb, int G, int64_t p) {
  int key = 0;
  for (int b = 0; b < nb; ++b) {
    const int g = grp ? grp[b] : 0;
    if ((key >> g) & 1) continue;
    float y, w;
    decode_obs<0>(bands[b], p, y, w);
    if (w > 0.f) key |= 1 << g;
  }
  return ((1 << G) - 1) - key;
}

// ---------------------------------------------------------------------------
// Observation operators: value H0 and Jacobian row h (length NP) at x.

// RBF (ARD) Gaussian-process emulator, inputs centred on the training mean:
//   f(x) = offset + sum_i alpha_i s exp(-1/2 sum_d lambda_d (x_d - t_id)^2)
// Records (host-built, models/gp.py): per training point
//   L'_i = log2(s |alpha_i|) - 1/2 log2e sum_d lambda_d t_id^2,  B_id = log2e lambda_d t_id
// (t centred), so that with c = -1/2 log2e sum lambda x^2 (per pixel)
//   m_i = 2^(L'_i + c + B_i.x) = |alpha_i| k_i,
//   S0 = sum sgn(alpha_i) m_i = f - offset,
//   S'_d = sum sgn(alpha_i) m_i B_id = log2e lambda_d sum alpha_i k_i t_id,
//   df/dx_d = -lambda_d (x_d S0 - sum alpha k t_d) = -lambda_d x_d S0 + ln2 S'_d.
// B doubles as the exponent and the gradient weight, so a point costs D + 1
// record floats instead of 2D + 2 (alpha and alpha*t are folded away).  Points
// are grouped by the sign of alpha (first Tp pairs positive; each group padded
// to a pair with L' = -1e30, i.e. m = 0) and the sums are negated between the
// groups.  Stored as PAIRS, field-major: rec[pair][field][2]; on gfx950 one
// pair is one v_pk_fma_f32 per field with the pair as one 64-bit SGPR operand
// (2 points per lane per issue).  Replaces gp.predict + the lil_matrix scatter
// of utils.py:181-219.
KF_HD float gp_rec(const KF_CONST_AS float* r, int R, int i, int f) {
  return r[((int64_t)(i >> 1) * R + f) * 2 + (i & 1)];
}

#if defined(__HIP_DEVICE_COMPILE__)
typedef float kf_f2 __attribute__((ext_vector_type(2)));

// Streams training-point pairs (s_load into SGPRs) and accumulates S0 += m and
// S'_d += B_d m, two points per v_pk_fma_f32.
// ADDC: exponent = L' + c + B.x; without it L' + B.x and the caller rescales by 2^c.
template <int D, int UNR, bool ADDC>
__device__ __forceinline__ void gp_pairs(const KF_CONST_AS kf_f2* __restrict__ r2, int T2, const kf_f2 (&xv)[D],
                                         kf_f2 cv, kf_f2& S0v, kf_f2 (&Sv)[D]) {
  constexpr int R = D + 1;
#pragma unroll UNR
  for (int i = 0; i < T2; ++i) {
    const KF_CONST_AS kf_f2* __restrict__ ri = r2 + (int64_t)i * R;
    kf_f2 e;
    if constexpr (ADDC) {
      e = ri[0] + cv;
#pragma unroll
      for (int d = 0; d < D; ++d) e = __builtin_elementwise_fma(ri[1 + d], xv[d], e);
    } else {
      e = __builtin_elementwise_fma(ri[1], xv[0], ri[0]);
#pragma unroll
      for (int d = 1; d < D; ++d) e = __builtin_elementwise_fma(ri[1 + d], xv[d], e);
    }
    kf_f2 m;
    m.x = kexp2(e.x);
    m.y = kexp2(e.y);
    S0v += m;
#pragma unroll
    for (int d = 0; d < D; ++d) Sv[d] = __builtin_elementwise_fma(ri[1 + d], m, Sv[d]);
  }
}

// Both sign groups: S = S(alpha > 0) - S(alpha < 0).
template <int D, int UNR, bool ADDC>
__device__ __forceinline__ void gp_signed_pairs(const KF_CONST_AS kf_f2* __restrict__ r2, int T2, int Tp,
                                                const kf_f2 (&xv)[D], kf_f2 cv, kf_f2& S0v, kf_f2 (&Sv)[D]) {
  gp_pairs<D, UNR, ADDC>(r2, Tp, xv, cv, S0v, Sv);
  S0v = -S0v;
#pragma unroll
  for (int d = 0; d < D; ++d) Sv[d] = -Sv[d];
  gp_pairs<D, UNR, ADDC>(r2 + (int64_t)Tp * (D + 1), T2 - Tp, xv, cv, S0v, Sv);
  S0v = -S0v;
#pragma unroll
  for (int d = 0; d < D; ++d) Sv[d] = -Sv[d];
}
#endif

// FOLD: when every lane of the wave has -c <= GP_FOLD_MAX the per-point "+ c"
// is dropped from the exponent (one packed op of D + 2 per point pair) and the
// sums are rescaled by 2^c once; exponents then grow by at most GP_FOLD_MAX,
// i.e. <= ~1e-6 relative error in k.  Otherwise the wave takes the exact loop.
constexpr float GP_FOLD_MAX = 16.f;

// f = offset + S0,  df/dx_d = -lambda_d x_d S0 + ln2 S'_d, scattered to the state.
template <int NP, int D, typename F, typename I>
KF_HD void gp_epilogue(float offset, const F& coef, const I& map, const float (&xi)[D], float S0,
                       const float (&S)[D], float& H0, float (&h)[NP]) {
  H0 = offset + S0;
#pragma unroll
  for (int j = 0; j < NP; ++j) h[j] = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const float g = fmaf(-coef[d] * xi[d], S0, LN2 * S[d]);
#pragma unroll
    for (int j = 0; j < NP; ++j) h[j] += (map[d] == j) ? g : 0.f;
  }
}

// RELOAD + bdp (device fast paths): the descriptor's table entry; its epilogue fields
// are then re-read after the record stream through an opaque pointer instead
// of being kept live in SGPRs across it (which spills them to VGPR lanes:
// ~270 fewer v_readlane/v_writelane per pixel in analysis_kernel<7,4,DN16>).
template <int NP, int D, int UNR = 4, bool FOLD = false, bool RELOAD = false>
KF_HD void gp_eval(const BandDesc& bd, const float (&x)[NP], float& H0, float (&h)[NP],
                   const BandDesc* bdp = nullptr) {
  float xi[D];
  float c = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    xi[d] = gather_state<NP>(x, bd.map[d]) - bd.center[d];
    c = fmaf(bd.coef[d] * xi[d], xi[d], c);
  }
  c *= -0.5f * LOG2E;
  float S0, S[D];
  constexpr int R = D + 1;
#if defined(__HIP_DEVICE_COMPILE__)
  const KF_CONST_AS kf_f2* __restrict__ r2 = (const KF_CONST_AS kf_f2*)cptr(bd.gp);
  const int T2 = bd.T >> 1;
  const int Tp = bd.Tp;
  kf_f2 S0v = {0.f, 0.f}, Sv[D], xv[D];
  const kf_f2 cv = {c, c};
#pragma unroll
  for (int d = 0; d < D; ++d) { Sv[d] = kf_f2{0.f, 0.f}; xv[d] = kf_f2{xi[d], xi[d]}; }
  bool folded = false;
  if constexpr (FOLD) folded = __all(c >= -GP_FOLD_MAX);
  if (folded)
    gp_signed_pairs<D, UNR, false>(r2, T2, Tp, xv, cv, S0v, Sv);
  else
    gp_signed_pairs<D, UNR, true>(r2, T2, Tp, xv, cv, S0v, Sv);
  if (folded) {
    const float sc = kexp2(c);
    S0v *= sc;
#pragma unroll
    for (int d = 0; d < D; ++d) Sv[d] *= sc;
  }
  S0 = S0v.x + S0v.y;
#pragma unroll
  for (int d = 0; d < D; ++d) S[d] = Sv[d].x + Sv[d].y;
#else
  const float* r = bd.gp;
  float S0a[2] = {0.f, 0.f}, Sa[2][D];
#pragma unroll
  for (int d = 0; d < D; ++d) Sa[0][d] = Sa[1][d] = 0.f;
  for (int i = 0; i < bd.T; ++i) {
    const int l = i & 1;
    float e = gp_rec(r, R, i, 0) + c;
#pragma unroll
    for (int d = 0; d < D; ++d) e = fmaf(gp_rec(r, R, i, 1 + d), xi[d], e);
    const float m = ((i >> 1) < bd.Tp) ? kexp2(e) : -kexp2(e);
    S0a[l] += m;
#pragma unroll
    for (int d = 0; d < D; ++d) Sa[l][d] = fmaf(gp_rec(r, R, i, 1 + d), m, Sa[l][d]);
  }
  S0 = S0a[0] + S0a[1];
#pragma unroll
  for (int d = 0; d < D; ++d) S[d] = Sa[0][d] + Sa[1][d];
#endif
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (RELOAD) {
    const KF_CONST_AS BandDesc* q = opaque(cptr(bdp));
    gp_epilogue<NP, D>(q->offset, q->coef, q->map, xi, S0, S, H0, h);
    return;
  }
#endif
  gp_epilogue<NP, D>(bd.offset, bd.coef, bd.map, xi, S0, S, H0, h);
}

// Water Cloud Model (sar_forward_model.py:13-106), analytic gradient.
// Returns false for LAI<=0 / SM<=0 (the reference raises ValueError there).
template <int NP>
KF_HD bool sar_eval(const BandDesc& bd, int64_t p, const float (&x)[NP], float& H0, float (&h)[NP]) {
  const float V = gather_state<NP>(x, bd.map[0]);
  const float SM = gather_state<NP>(x, bd.map[1]);
  const float A = bd.coef[0], B = bd.coef[1], C = bd.coef[2], Dc = bd.coef[3], E = bd.coef[4];
  const float th = bd.aux ? KF_PX(bd.aux, 0, p) : bd.coef[5];
  const float mu = cosf(th * DEG2RAD);
  const bool ok = (V > 0.f) && (SM > 0.f);
  const float Vs = ok ? V : 1.f;
  const float tau = expf(-2.f * B / mu * Vs);
  float z = powf(Vs, E);
  if (!finitef(z)) z = 1.f;
  float z1 = powf(Vs, E - 1.f);
  if (!finitef(z1)) z1 = 1.f;
  const float ssoil = kexp2(LOG2_10 * (C + Dc * SM) * 0.1f);
  H0 = A * z * mu * (1.f - tau) + tau * ssoil;
  const float dV = A * E * mu * z1 * (1.f - tau) + 2.f * A * B * z * tau - 2.f * B * tau * ssoil / mu;
  const float dS = Dc * LN10 * 0.1f * tau * ssoil;
#pragma unroll
  for (int j = 0; j < NP; ++j) h[j] = (bd.map[0] == j ? dV : 0.f) + (bd.map[1] == j ? dS : 0.f);
  return ok;
}

template <int NP, int D = 1>
KF_HD void gp_dispatch(const BandDesc& bd, const float (&x)[NP], float& H0, float (&h)[NP]) {
  if constexpr (D <= NP && D <= 12) {
    if (bd.d == D) { gp_eval<NP, D>(bd, x, H0, h); return; }
    gp_dispatch<NP, D + 1>(bd, x, H0, h);
  } else {
    H0 = 0.f;
#pragma unroll
    for (int j = 0; j < NP; ++j) h[j] = 0.f;
  }
}

// Evaluate one band's operator.  Returns false when the operator is invalid here.
template <int NP>
KF_HD bool eval_operator(const BandDesc& bd, int64_t p, int64_t ld, const float (&x)[NP],
                         float& H0, float (&h)[NP]) {
  bool ok = true;
  switch (bd.op) {
    case OP_GP:
      gp_dispatch<NP>(bd, x, H0, h);
      break;
    case OP_SAR:
      ok = sar_eval<NP>(bd, p, x, H0, h);
      break;
    case OP_LINEAR: {
      float t = bd.offset;
#pragma unroll
      for (int j = 0; j < NP; ++j) { h[j] = bd.coef[j]; t = fmaf(h[j], x[j], t); }
      H0 = t;
    } break;
    default: {  // OP_PRECOMP
      H0 = KF_PX(bd.pre_h0, 0, p);
#pragma unroll
      for (int j = 0; j < NP; ++j) h[j] = KF_PX(bd.pre_h, j * bd.pre_ld, p);
    }
  }
  bool fin = finitef(H0);
#pragma unroll
  for (int j = 0; j < NP; ++j) fin = fin && finitef(h[j]);
  return ok && fin;
}

// ---------------------------------------------------------------------------
// K4/K5: propagation and prior blending for one pixel.
// Forecast fused into the analysis kernel: the partial prior reset, one
// compile-time formula (a runtime mode switch in the analysis prologue costs
// ~35 VGPRs across the GP loop).  The host maps PROP_PRIOR (mask 0) and
// PROP_INFO_APPROX (all propagated, zero reset precision) onto it:
//   xf_j = m_j x_a,j (propagated) | mu_j (reset)
//   Pf   = C^-1 with diag_j = 1 / (1 / P_a,jj + q_j) for propagated j.
template <int NP>
KF_HD void forecast_partial_mean(const KF_CONST_AS PropArgs* a, int64_t p, float (&xf)[NP]) {
#pragma unroll
  for (int j = 0; j < NP; ++j)
    xf[j] = ((a->prop_mask >> j) & 1u) ? a->m[j] * KF_PX(a->x_a, j * a->ld, p) : a->reset_mean[j];
}

template <int NP>
KF_HD void forecast_partial_precision(const KF_CONST_AS PropArgs* a, int64_t p, float (&P)[ntri(NP)]) {
  const int64_t ld = a->ld;
#pragma unroll
  for (int t = 0; t < ntri(NP); ++t) P[t] = a->reset_cinv[t];
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    if ((a->prop_mask >> j) & 1u) {
      const float q = a->q_pix ? KF_PX(a->q_pix, j * ld, p) : a->q[j];
      P[tri(NP, j, j)] = kf_rcp(kf_rcp(KF_PX(a->p_a, tri(NP, j, j) * ld, p)) + q);
    }
  }
}

template <int NP>
KF_HD void forecast_partial(const KF_CONST_AS PropArgs* a, int64_t p, float (&xf)[NP], float (&P)[ntri(NP)]) {
  forecast_partial_precision<NP>(a, p, P);
  forecast_partial_mean<NP>(a, p, xf);
}

// The propagated parameter when exactly one is (the LAI propagator: TLAI), else -1.
KF_HD int prop_single(uint32_t mask) { return (mask && !(mask & (mask - 1u))) ? __builtin_ctz(mask) : -1; }

// forecast_partial with that parameter's x_a and P_a,jj already loaded (the
// SPEC_PROP_PF kernels load the next pixel group's ahead): the same arithmetic.
template <int NP>
KF_HD void forecast_partial_pre(const KF_CONST_AS PropArgs* a, int64_t p, int j1, float xa1, float pa1,
                                float (&xf)[NP], float (&P)[ntri(NP)]) {
  const int64_t ld = a->ld;
#pragma unroll
  for (int t = 0; t < ntri(NP); ++t) P[t] = a->reset_cinv[t];
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    if (j == j1) {
      const float q = a->q_pix ? KF_PX(a->q_pix, j * ld, p) : a->q[j];
      P[tri(NP, j, j)] = kf_rcp(kf_rcp(pa1) + q);
      xf[j] = a->m[j] * xa1;
    } else {
      xf[j] = a->reset_mean[j];
    }
  }
}

// forecast_pixel computes the forecast (xf, P) of pixel p without storing it;
// the analysis kernel calls it directly when the propagation is fused.
template <int NP>
KF_HD uint8_t forecast_pixel(const PropArgs& a, int64_t p, float (&xf)[NP], float (&P)[ntri(NP)]) {
  constexpr int NT = ntri(NP);
  const int64_t ld = a.ld;
  uint8_t st = 0;
  float q[NP];
#pragma unroll
  for (int j = 0; j < NP; ++j) q[j] = a.q_pix ? KF_PX(a.q_pix, j * ld, p) : a.q[j];

  switch (a.mode) {
    case PROP_PRIOR: {
#pragma unroll
      for (int j = 0; j < NP; ++j) xf[j] = a.reset_mean[j];
#pragma unroll
      for (int t = 0; t < NT; ++t) P[t] = a.reset_cinv[t];
    } break;
    case PROP_PRIOR_PARTIAL: {
#pragma unroll
      for (int t = 0; t < NT; ++t) P[t] = a.reset_cinv[t];
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const bool pj = (a.prop_mask >> j) & 1u;
        xf[j] = pj ? a.m[j] * KF_PX(a.x_a, j * ld, p) : a.reset_mean[j];
        if (pj) {
          const float pa = KF_PX(a.p_a, tri(NP, j, j) * ld, p);
          P[tri(NP, j, j)] = kf_rcp(kf_rcp(pa) + q[j]);   // same rounding as forecast_partial
        }
      }
    } break;
    case PROP_INFO_APPROX: {
#pragma unroll
      for (int j = 0; j < NP; ++j) xf[j] = a.m[j] * KF_PX(a.x_a, j * ld, p);
#pragma unroll
      for (int t = 0; t < NT; ++t) P[t] = 0.f;
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const float d = KF_PX(a.p_a, tri(NP, j, j) * ld, p);
        P[tri(NP, j, j)] = d / (1.f + d * q[j]);
      }
    } break;
    case PROP_INFO_EXACT: {
      // P_f^-1 = (I + P_a^-1 Q)^-1 P_a^-1 = (P_a + Q)^-1
#pragma unroll
      for (int j = 0; j < NP; ++j) xf[j] = a.m[j] * KF_PX(a.x_a, j * ld, p);
      float U[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) U[t] = KF_PX(a.p_a, t * ld, p);
      bool ok = chol_packed<NP>(U);
      float C[NT];
      chol_inverse<NP>(U, C);
#pragma unroll
      for (int j = 0; j < NP; ++j) C[tri(NP, j, j)] += q[j];
      ok = chol_packed<NP>(C) && ok;
      chol_inverse<NP>(C, P);
      if (!ok) st |= ST_NONSPD;
    } break;
    case PROP_STANDARD: {
#pragma unroll
      for (int j = 0; j < NP; ++j) xf[j] = a.m[j] * KF_PX(a.x_a, j * ld, p);
#pragma unroll
      for (int t = 0; t < NT; ++t) P[t] = KF_PX(a.p_a, t * ld, p);
#pragma unroll
      for (int j = 0; j < NP; ++j) P[tri(NP, j, j)] += q[j];
    } break;
    default: {  // PROP_IDENTITY
#pragma unroll
      for (int j = 0; j < NP; ++j) xf[j] = a.m[j] * KF_PX(a.x_a, j * ld, p);
#pragma unroll
      for (int t = 0; t < NT; ++t) P[t] = KF_PX(a.p_a, t * ld, p);
    }
  }

  if (a.blend) {
    // Gaussian product of forecast (xf, P) with prior (mu, C^-1) (kf_tools.py:75-96).
    float mu[NP], Ci[NT];
#pragma unroll
    for (int j = 0; j < NP; ++j) mu[j] = a.blend_mean_pix ? KF_PX(a.blend_mean_pix, j * ld, p) : a.blend_mean[j];
#pragma unroll
    for (int t = 0; t < NT; ++t) Ci[t] = a.blend_cinv_pix ? KF_PX(a.blend_cinv_pix, t * ld, p) : a.blend_cinv[t];
    float b1[NP], b2[NP];
    if (a.quirk_blend) {  // reference operand swap (kf_tools.py:90)
      symv<NP>(P, mu, b1);
      symv<NP>(Ci, xf, b2);
    } else {
      symv<NP>(P, xf, b1);
      symv<NP>(Ci, mu, b2);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) P[t] += Ci[t];
    float U[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) U[t] = P[t];
#pragma unroll
    for (int j = 0; j < NP; ++j) xf[j] = b1[j] + b2[j];
    if (!chol_packed<NP>(U)) st |= ST_NONSPD;
    chol_solve<NP>(U, xf);
  }
  return st;
}

template <int NP>
KF_HD void pixel_propagate(const PropArgs& a, int64_t p) {
  constexpr int NT = ntri(NP);
  const int64_t ld = a.ld;
  float xf[NP], P[NT];
  const uint8_t st = forecast_pixel<NP>(a, p, xf, P);
#pragma unroll
  for (int j = 0; j < NP; ++j) KF_PX(a.x_f, j * ld, p) = xf[j];
#pragma unroll
  for (int t = 0; t < NT; ++t) KF_PX(a.p_f, t * ld, p) = P[t];
  if (a.status) KF_PX(a.status, 0, p) |= st;
}

// Full-form right-hand side b = r + A x0 from the correction form r (DELTA).
template <int NP>
KF_HD void delta_to_full(const float (&A)[ntri(NP)], const float (&x0)[NP], float (&b)[NP]) {
  float t[NP];
  symv<NP>(A, x0, t);
#pragma unroll
  for (int j = 0; j < NP; ++j) b[j] += t[j];
}

// K1 epilogue: store (A, b) if requested, factor and solve, health fallback
// to the forecast, store x and status; returns |x - x0|^2.  AP is a host or
// constant-address-space pointer to the launch arguments.
// DELTA: b holds the correction form r = P_f^-1 (x_f - x0) + sum w h (y - H0)
// and x = x0 + A^-1 r (the same analysis as x = A^-1 b with b = r + A x0, but
// the f32 solve error scales with |x - x0| instead of |x|); b_out and the
// regulariser get the full form.
// store = false: a fused intermediate Gauss-Newton iteration (AnalysisArgs.
// gn_fused) or a tail lane -- the same solve and health fallback, x left in b,
// nothing stored.  final_it = false: an intermediate iteration, which takes the
// plain solve even when the launch carries the regulariser (reg_v: the fused
// spatial launch, a plain first iteration and the regularised prepare of the
// second).
// The fused kernels reach this function from ONE call site for both kinds of
// iteration, so the intermediate x is bit-identical to a separate launch's
// (two inlined copies of the solve may be scheduled / contracted differently).
// SPEC (kf_device.h SPEC_*): the launch's forecast / regulariser known at
// compile time -- SPEC_PROP: fused forecast, no regulariser; SPEC_PROP_REG:
// fused forecast and regulariser; SPEC_ANY: decided from the arguments.
template <int NP, bool DELTA = false, int SPEC = SPEC_ANY, typename AP>
KF_HD float analysis_epilogue(AP a, int64_t p, float (&A)[ntri(NP)], float (&b)[NP], const float (&x0)[NP],
                              uint8_t st, bool store = true, bool final_it = true) {
  constexpr int NT = ntri(NP);
  const int64_t ld = a->ld;
  const bool has_prop = SPEC != SPEC_ANY || a->prop;
  if (store && a->x0_out) {
#pragma unroll
    for (int j = 0; j < NP; ++j) KF_PXS(a->x0_out, j * ld, p) = x0[j];
  }
  const bool reg = (SPEC == SPEC_PROP_REG || (SPEC == SPEC_ANY && a->reg_v)) && final_it;
  if (DELTA && (reg || a->b_out)) delta_to_full<NP>(A, x0, b);
  if (reg) {
    int deg = 0;
    if (a->reg_geo.w > 0) {
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) deg += geo_neighbour(a->reg_geo, a->N, p, q4) >= 0 ? 1 : 0;
    } else {
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) deg += a->reg_nbr[q4 * a->N + p] >= 0 ? 1 : 0;
    }
    const float gd = a->reg_gamma * (float)deg;
#pragma unroll
    for (int j = 0; j < NP; ++j)
      if ((a->reg_mask >> j) & 1u) A[tri(NP, j, j)] += gd;
    if (store && a->a_out) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
          if (a_row_on(a->a_rows, t)) KF_PXS(a->a_out, t * ld, p) = A[t];
    }
    float dA[NP];   // output uncertainty: 1/sqrt(diag) of the regularised precision
#pragma unroll
    for (int j = 0; j < NP; ++j) dA[j] = A[tri(NP, j, j)];
    const bool spd = chol_packed<NP>(A);
    chol_solve<NP>(A, b);
    bool fin = true;
#pragma unroll
    for (int j = 0; j < NP; ++j) fin = fin && finitef(b[j]);
    // Health fallback (same rule as the plain path below): a non-SPD or
    // non-finite pixel keeps its forecast and is decoupled (V = 0, so the
    // sweeps give x = u = x_f and only finite values reach its neighbours
    // and, through fill_halo, the adjacent ranks).
    const bool bad = !spd || !fin;
    if (bad) {
      st |= (!spd ? ST_NONSPD : 0) | (!fin ? ST_NONFINITE : 0) | ST_FALLBACK;
      float Af[NT];
      if (has_prop) {
        forecast_partial<NP>(opaque(cptr(a->prop)), p, b, Af);
      } else {
#pragma unroll
        for (int j = 0; j < NP; ++j) b[j] = KF_PXS(a->x_f, j * ld, p);
#pragma unroll
        for (int t = 0; t < NT; ++t) Af[t] = KF_PXS(a->pf_inv, t * ld, p);
      }
      if (store && a->a_out) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
          if (a_row_on(a->a_rows, t)) KF_PXS(a->a_out, t * ld, p) = Af[t];
      }
#pragma unroll
      for (int j = 0; j < NP; ++j) dA[j] = Af[tri(NP, j, j)];
    }
    if (store && a->out_unc) {
      // the uncertainty raster of the final iteration (the mean follows in
      // reg_finish): written here, where diag A is in registers, so the finish
      // pass does not re-read the precision
      const int64_t r = a->out_idx ? KF_PXS(a->out_idx, 0, p) : p;
      const int64_t pl = a->out_plane;
#pragma unroll
      for (int j = 0; j < NP; ++j) KF_PXS(a->out_unc, j * pl, r) = kf_rsqrt(dA[j]);
    }
    if (!store) return 0.f;
#pragma unroll
    for (int j = 0; j < NP; ++j) KF_PXS(a->x_out, j * ld, p) = b[j];
    int c = 0;
#pragma unroll
    for (int r = 0; r < NP; ++r) {
      if ((a->reg_mask >> r) & 1u) {
        float e[NP];
#pragma unroll
        for (int j = 0; j < NP; ++j) e[j] = (j == r) ? 1.f : 0.f;
        chol_solve<NP>(A, e);
#pragma unroll
        for (int j = 0; j < NP; ++j) KF_PXS(a->reg_v, ((int64_t)c * NP + j) * ld, p) = bad ? 0.f : e[j];
        ++c;
      }
    }
    if (a->status) KF_PXS(a->status, 0, p) = st;
    return 0.f;
  }
  if (store && a->a_out) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
          if (a_row_on(a->a_rows, t)) KF_PXS(a->a_out, t * ld, p) = A[t];
  }
  if (store && a->b_out) {
#pragma unroll
    for (int j = 0; j < NP; ++j) KF_PXS(a->b_out, j * ld, p) = b[j];
  }
  float dn = 0.f;
  if (a->solve) {
    float dA[NP];   // analysis precision diagonal (output uncertainty) before the in-place factorisation
#pragma unroll
    for (int j = 0; j < NP; ++j) dA[j] = A[tri(NP, j, j)];
    const bool spd = chol_packed<NP>(A);
    chol_solve<NP>(A, b);
    if (DELTA && !a->b_out) {
#pragma unroll
      for (int j = 0; j < NP; ++j) b[j] += x0[j];
    }
    bool fin = true;
#pragma unroll
    for (int j = 0; j < NP; ++j) fin = fin && finitef(b[j]);
    if (!spd || !fin) {
      // Health fallback: keep the forecast (prior) for this pixel.
      st |= (!spd ? ST_NONSPD : 0) | (!fin ? ST_NONFINITE : 0) | ST_FALLBACK;
      if (has_prop) {
        forecast_partial<NP>(opaque(cptr(a->prop)), p, b, A);   // rare path: recompute instead of keeping it live
      } else {
#pragma unroll
        for (int j = 0; j < NP; ++j) b[j] = KF_PXS(a->x_f, j * ld, p);
#pragma unroll
        for (int t = 0; t < NT; ++t) A[t] = KF_PXS(a->pf_inv, t * ld, p);
      }
#pragma unroll
      for (int j = 0; j < NP; ++j) dA[j] = A[tri(NP, j, j)];
      if (store && a->a_out) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
          if (a_row_on(a->a_rows, t)) KF_PXS(a->a_out, t * ld, p) = A[t];
      }
    }
    if (store) {
#pragma unroll
      for (int j = 0; j < NP; ++j) KF_PXS(a->x_out, j * ld, p) = b[j];
    }
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const float d = b[j] - x0[j];
      dn = fmaf(d, d, dn);
    }
    if (store && a->out_unc) {
      // fused output dump: the unpack pass's work without re-reading x and A.
      // out_mean null: the state's x is the mean raster (dense strip, identity
      // map: DeviceOutput aliases it), only the uncertainty is written
      const int64_t r = a->out_idx ? KF_PXS(a->out_idx, 0, p) : p;
      const int64_t pl = a->out_plane;
      if (a->out_mean) {
#pragma unroll
        for (int j = 0; j < NP; ++j) KF_PXS(a->out_mean, j * pl, r) = b[j];
      }
#pragma unroll
      for (int j = 0; j < NP; ++j) KF_PXS(a->out_unc, j * pl, r) = kf_rsqrt(dA[j]);
    }
  }
  if (store && a->status) KF_PXS(a->status, 0, p) = st;
  return dn;
}

// ---------------------------------------------------------------------------
// K1: fused Gauss-Newton analysis for one pixel (information form).
//   A = P_f^-1 + sum_b w_b h_b h_b^T,  b = P_f^-1 x_f + sum_b w_b h_b y'_b,
//   y'_b = y_b + h_b . x0 - H0_b,      x_a = A^-1 b
// Returns (x_a - x0)^2 summed over parameters.
// FD > 0: fast path where every band is a GP with FD inputs and FOBS encoding
// (the compiler then drops the SAR/linear/precomputed code and its registers);
// FD == FD_PRECOMP: every band has a precomputed operator (split GP path).
// Prior part of the right-hand side: P_f^-1 x_f (full form) or P_f^-1 (x_f - x0)
// (correction form, DELTA; 0 when linearising at the forecast).
template <int NP, bool DELTA>
KF_HD void prior_rhs(const float (&A)[ntri(NP)], const float (&xf)[NP], const float (&x0)[NP], float (&b)[NP]) {
  if (DELTA) {
    float d[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) d[j] = xf[j] - x0[j];
    symv<NP>(A, d, b);
  } else {
    symv<NP>(A, xf, b);
  }
}

// DELTA (correction form, analysis_epilogue) for the GP and precomputed
// operators; the linear operators keep the full form, whose y' = y - offset
// makes a repeated iteration exact (static convergence, linear_kf.py).
template <int NP, int FD = 0, int FOBS = 0, int UNR = 4, bool FOLD = false>
KF_HD float pixel_analysis(const AnalysisArgs& a, int64_t p, float& dn_first) {
  constexpr bool DELTA = FD > 0 || FD == FD_PRECOMP;
  constexpr int NT = ntri(NP);
  const int64_t ld = a.ld;
  float x0[NP], A[NT], b[NP];
  if (a.x_prev) {
#pragma unroll
    for (int j = 0; j < NP; ++j) x0[j] = KF_PX(a.x_prev, j * ld, p);
  }
  dn_first = 0.f;
  for (int it = 0;; ++it) {
  p = opaque_lane(p);
  uint8_t st = 0;
  if (a.prop) {
    // fused propagation: forecast of this pixel from the previous analysis,
    // never written to HBM (saves the propagate pass and its 2 x 140 B/px)
    float xf[NP];
    forecast_partial<NP>(opaque(cptr(a.prop)), p, xf, A);
    if (!a.x_prev && it == 0) {
#pragma unroll
      for (int j = 0; j < NP; ++j) x0[j] = xf[j];
    }
    if (DELTA && !a.x_prev && it == 0) {
      // correction form linearised at the forecast: P_f^-1 (x_f - x0) = 0
#pragma unroll
      for (int j = 0; j < NP; ++j) b[j] = 0.f;
    } else {
      prior_rhs<NP, DELTA>(A, xf, x0, b);
    }
  } else if (a.a_in) {
    // band-chunked accumulation: continue from a previous chunk's (A, b)
#pragma unroll
    for (int t = 0; t < NT; ++t) A[t] = KF_PX(a.a_in, t * ld, p);
#pragma unroll
    for (int j = 0; j < NP; ++j) b[j] = KF_PX(a.b_in, j * ld, p);
    if (DELTA) {
      float t[NP];
      symv<NP>(A, x0, t);
#pragma unroll
      for (int j = 0; j < NP; ++j) b[j] -= t[j];
    }
  } else {
    float xf[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) xf[j] = KF_PX(a.x_f, j * ld, p);
#pragma unroll
    for (int t = 0; t < NT; ++t) A[t] = KF_PX(a.pf_inv, t * ld, p);
    prior_rhs<NP, DELTA>(A, xf, x0, b);
  }
  int nobs = 0;
  for (int bi = 0; bi < a.n_bands; ++bi) {
    const BandDesc bd = cptr(a.bands)[bi];
    float y, w;
    decode_obs<FOBS>(bd, p, y, w);
    if (!(w > 0.f)) {
      if (bd.h0_out) KF_PX(bd.h0_out, 0, p) = 0.f;
      continue;
    }
    float H0, h[NP];
    bool ok;
    if constexpr (FD > 0) {
#if defined(__HIP_DEVICE_COMPILE__)
      gp_eval<NP, FD, UNR, FOLD, true>(bd, x0, H0, h, a.bands + bi);
#else
      gp_eval<NP, FD, UNR, FOLD>(bd, x0, H0, h);
#endif
      ok = finitef(H0);
#pragma unroll
      for (int j = 0; j < NP; ++j) ok = ok && finitef(h[j]);
    } else if constexpr (FD == FD_PRECOMP) {
      // precomputed operator (split GP path / host factories): H0, h from HBM
      H0 = KF_PX(bd.pre_h0, 0, p);
      ok = finitef(H0);
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        h[j] = KF_PX(bd.pre_h, j * bd.pre_ld, p);
        ok = ok && finitef(h[j]);
      }
    } else if constexpr (FD == FD_LINEAR) {
      // linear / identity operator (utils.py:119-126, fixed): h = c, H0 = offset + c . x0
      float t = bd.offset;
#pragma unroll
      for (int j = 0; j < NP; ++j) { h[j] = bd.coef[j]; t = fmaf(h[j], x0[j], t); }
      H0 = t;
      ok = finitef(H0);
    } else {
      ok = eval_operator<NP>(bd, p, ld, x0, H0, h);
    }
    float* h0o = bd.h0_out;
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (FD > 0) h0o = opaque(cptr(a.bands + bi))->h0_out;   // not live across the GP loop
#endif
    if (h0o) KF_PX(h0o, 0, p) = H0;
    if (!ok) { st |= ST_BAD_OP; continue; }
    ++nobs;
    float yp;
    if (DELTA) {
      yp = y - H0;   // correction form: the residual at x0
    } else if (FD == FD_LINEAR || (FD == 0 && bd.op == OP_LINEAR)) {
      // linear operator: y + h.x0 - (offset + h.x0) = y - offset exactly, so
      // the analysis does not depend on the linearisation point and a second
      // Gauss-Newton iteration reproduces the first bit for bit (norm 0)
      yp = y - bd.offset;
    } else {
      yp = y - H0;
#pragma unroll
      for (int j = 0; j < NP; ++j) yp = fmaf(h[j], x0[j], yp);
    }
    const float wy = w * yp;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const float wh = w * h[i];
      b[i] = fmaf(h[i], wy, b[i]);
#pragma unroll
      for (int j = i; j < NP; ++j) A[tri(NP, i, j)] = fmaf(wh, h[j], A[tri(NP, i, j)]);
    }
  }
  if (nobs == 0) st |= ST_NO_OBS;
  if (state_out_of_domain<NP>(&a, x0)) st |= ST_OUT_OF_DOMAIN;
  float dn;
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (FD != 0) {
    // fast kernels: re-read the launch arguments from the kernarg segment
    // through an opaque pointer, so they are not pinned in SGPRs across the
    // band / record loops above (analysis_kernel passes them at offset 0)
    const KF_CONST_AS AnalysisArgs* ka =
        opaque((const KF_CONST_AS AnalysisArgs*)__builtin_amdgcn_kernarg_segment_ptr());
    // linear operators (no regulariser): the second fused iteration would
    // rebuild the same (A, b) -- the absolute form does not read x0 -- and
    // reproduce x_1 bit for bit, so the first iteration's epilogue is final
    // (outputs stored, its norm the first one, the second's exactly 0)
    const bool lin2 = FD == FD_LINEAR && it + 1 < ka->gn_fused && !ka->reg_v && !ka->x0_out;
    const bool last = it + 1 >= ka->gn_fused || lin2;
    dn = analysis_epilogue<NP, DELTA>(ka, p, A, b, x0, st, last, last);
    if (lin2) {
      dn_first = dn;
      return 0.f;
    }
    if (last) return dn;
  } else
#endif
  {
    const bool lin2 = FD == FD_LINEAR && it + 1 < a.gn_fused && !a.reg_v && !a.x0_out;
    const bool last = it + 1 >= a.gn_fused || lin2;
    dn = analysis_epilogue<NP, DELTA>(&a, p, A, b, x0, st, last, last);
    if (lin2) {
      dn_first = dn;
      return 0.f;
    }
    if (last) return dn;
  }
  // fused intermediate iteration: x_1 (left in b) becomes the linearisation point
  dn_first = dn;
#pragma unroll
  for (int j = 0; j < NP; ++j) x0[j] = b[j];
  }
}

// Packed SPD inverse (covariance <-> precision conversion).
template <int NP>
KF_HD bool pixel_invert(const float* src, float* dst, int64_t ld, int64_t p) {
  constexpr int NT = ntri(NP);
  float U[NT], R[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) U[t] = KF_PX(src, t * ld, p);
  const bool ok = chol_packed<NP>(U);
  chol_inverse<NP>(U, R);
#pragma unroll
  for (int t = 0; t < NT; ++t) KF_PX(dst, t * ld, p) = R[t];
  return ok;
}

// ---------------------------------------------------------------------------
// K1g: covariance / gain form, bands processed as sequential scalar updates
// (equal to the joint update for diagonal R):
//   s = h^T P h + 1/w,  k = P h / s,  x += k (y' - h^T x),  P -= k (P h)^T
// with y' = y - H0 + h . x0 (iterated EKF linearised about x0).  Same fast
// paths as K1 (FD: all-GP bands with FD inputs, FOBS: one encoding), the
// forecast fused from the previous analysis (prop), the output rasters written
// by the last iteration (out_mean / out_unc), and K1's launch features: GN
// iterations 1 + 2 in one launch (gn_fused), the observed-first visiting order,
// the per-chunk visiting subset and |dx|^2 per pixel (order / n_visit / dn_out)
// and the stored-rows policy (pdiag_rows).
struct GainArgs {
  int64_t N, ld;
  int32_t n_bands, joseph;
  int32_t fast_d, fast_obs;  // host hint, as AnalysisArgs
  const BandDesc* bands;
  const float* x_prev;   // linearisation point (null with prop: the forecast)
  const float* x_f;
  const float* p_f;      // forecast covariance (packed)
  float* x_out;
  float* p_out;          // analysis covariance (packed, may be null)
  uint8_t* status;
  double* partials;
  const PropArgs* prop;  // fused forecast (device copy; p_a = analysis COVARIANCE); x_f / p_f unused
  float* out_mean;       // fused output: x and 1/sqrt(diag P^-1) into [NP][out_plane] rasters
  float* out_unc;        //   (out_mean null with out_unc set: the state's x is the mean raster)
  const int64_t* out_idx;
  int64_t out_plane;
  int32_t gpm_frags;     // > 0: GP on the matrix cores (LDS tables, as AnalysisArgs); gain_mfma_kernel
  int32_t gn_fused;      // 2: iterations 1 and 2 in one launch (as AnalysisArgs.gn_fused)
  double* partials_first;  // per-block sum (x_1 - x_0)^2 of the first fused iteration
  const int32_t* order;  // visiting order (null: 0..N-1)
  int64_t n_visit;       // visiting slots (0: N)
  const int32_t* n_visit_dev;  // null, or the device count of slots (<= n_visit), as AnalysisArgs
  float* dn_out;         // per-pixel |x - x0|^2 of the last iteration (per-chunk norms); may be null
  // stored rows: bit j set -> p_out row tri(j, j) receives the analysis
  // PRECISION diagonal entry (P^-1)_jj and no covariance row is stored (what a
  // fused forecast with PropArgs.pa_pdiag reads: the propagated parameters'
  // entries); 0: the full analysis covariance
  uint32_t pdiag_rows;
  int32_t pad_;
  // line tables of the first iteration at the fused forecast (as AnalysisArgs.line_*)
  const float* line_tab;
  float line_t0, line_inv_h;
  int32_t line_n, line_j;
};

KF_HD int64_t visit_count(const GainArgs& a) { return visit_bounded(a.n_visit, a.N, a.n_visit_dev); }

// The partial-prior-reset forecast (forecast_partial) of an analysis held as a
// covariance, returned as a covariance: Pa^-1 = inv(P_a) supplies the
// propagated diagonals (or p_a holds them, pa_pdiag), C = reset precision with
// those diagonals, P_f = C^-1.  PROP_PRIOR (mask 0) and PROP_INFO_APPROX (all
// propagated, C0 = 0) map onto it as for K1 (ops/kernels.py:prop_args).
template <int NP>
KF_HD uint8_t forecast_partial_cov(const KF_CONST_AS PropArgs* a, int64_t p, float (&xf)[NP],
                                   float (&P)[ntri(NP)]) {
  constexpr int NT = ntri(NP);
  const int64_t ld = a->ld;
  uint8_t st = 0;
  float C[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) C[t] = a->reset_cinv[t];
  if (a->prop_mask) {
    float Pi[NT];
    if (a->pa_pdiag) {
#pragma unroll
      for (int j = 0; j < NP; ++j)
        if ((a->prop_mask >> j) & 1u) Pi[tri(NP, j, j)] = KF_PX(a->p_a, tri(NP, j, j) * ld, p);
    } else {
      float U[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) U[t] = KF_PX(a->p_a, t * ld, p);
      if (!chol_packed<NP>(U)) st |= ST_NONSPD;
      chol_inverse<NP>(U, Pi);
    }
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      if ((a->prop_mask >> j) & 1u) {
        const float q = a->q_pix ? KF_PX(a->q_pix, j * ld, p) : a->q[j];
        C[tri(NP, j, j)] = kf_rcp(kf_rcp(Pi[tri(NP, j, j)]) + q);
      }
    }
  }
  forecast_partial_mean<NP>(a, p, xf);
  if (!chol_packed<NP>(C)) st |= ST_NONSPD;
  chol_inverse<NP>(C, P);
  return st;
}

// The same forecast without a Cholesky per pixel (PropArgs.cov_fast): C
// differs from the constant reset precision C0 only in the propagated
// diagonals, so P_f = C^-1 is the constant C0^-1 (reset_cov) updated by one
// Sherman-Morrison rank-1 term per propagated j,
//   (M + d e_j e_j^T)^-1 = M^-1 - d u u^T / (1 + d u_j),  u = M^-1 e_j.
// Also returns the forecast precision diagonal cd (the information identity
// diag(P_a^-1) = cd + sum_b w_b h_b^2 then gives the uncertainty raster and
// the stored rows without inverting P_a).
template <int NP>
KF_HD uint8_t gain_forecast(const KF_CONST_AS PropArgs* a, int64_t p, float (&xf)[NP], float (&P)[ntri(NP)],
                            float (&cd)[NP]) {
  constexpr int NT = ntri(NP);
  const int64_t ld = a->ld;
  uint8_t st = 0;
#pragma unroll
  for (int t = 0; t < NT; ++t) P[t] = a->reset_cov[t];
#pragma unroll
  for (int j = 0; j < NP; ++j) cd[j] = a->reset_cinv[tri(NP, j, j)];
  if (a->prop_mask) {
    float d[NP];
    if (a->pa_pdiag) {
#pragma unroll
      for (int j = 0; j < NP; ++j)
        d[j] = ((a->prop_mask >> j) & 1u) ? KF_PX(a->p_a, tri(NP, j, j) * ld, p) : 1.f;
    } else {
      float U[NT], Pi[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) U[t] = KF_PX(a->p_a, t * ld, p);
      if (!chol_packed<NP>(U)) st |= ST_NONSPD;
      chol_inverse<NP>(U, Pi);
#pragma unroll
      for (int j = 0; j < NP; ++j) d[j] = Pi[tri(NP, j, j)];
    }
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      if (!((a->prop_mask >> j) & 1u)) continue;
      const float q = a->q_pix ? KF_PX(a->q_pix, j * ld, p) : a->q[j];
      const float c = kf_rcp(kf_rcp(d[j]) + q);
      const float delta = c - cd[j];
      cd[j] = c;
      float u[NP];
#pragma unroll
      for (int i = 0; i < NP; ++i) u[i] = P[sym<NP>(i, j)];
      const float den = fmaf(delta, u[j], 1.f);
      if (!(den > 0.f)) st |= ST_NONSPD;
      const float f = delta * kf_rcp(den);
#pragma unroll
      for (int i = 0; i < NP; ++i)
#pragma unroll
        for (int k = i; k < NP; ++k) P[tri(NP, i, k)] = fmaf(-f * u[i], u[k], P[tri(NP, i, k)]);
    }
  }
  forecast_partial_mean<NP>(a, p, xf);
  return st;
}

// One scalar-band Kalman update of (x, P) (covariance form, diagonal R):
// S = h^T P h + r, K = P h / S, x += K (y - H0 - h^T (x - x0)), P -= K (P h)^T
// (Joseph: P = (I - K h^T) P (I - K h^T)^T + K K^T r).
template <int NP>
KF_HD void gain_band_update(float (&P)[ntri(NP)], float (&x)[NP], const float (&x0)[NP], const float (&h)[NP],
                            float H0, float y, float w, bool joseph) {
  float ph[NP];
  symv<NP>(P, h, ph);
  const float r = kf_rcp(w);                  // observation variance
  float s = r, innov = y - H0;
#pragma unroll
  for (int j = 0; j < NP; ++j) { s = fmaf(h[j], ph[j], s); innov = fmaf(h[j], x0[j] - x[j], innov); }
  const float is = kf_rcp(s);
  float k[NP];
#pragma unroll
  for (int j = 0; j < NP; ++j) { k[j] = ph[j] * is; x[j] = fmaf(k[j], innov, x[j]); }
  if (joseph) {
    // P = (I - k h^T) P (I - k h^T)^T + k k^T r = P - k ph^T - ph k^T + k k^T (h^T P h + r)
#pragma unroll
    for (int i = 0; i < NP; ++i)
#pragma unroll
      for (int j = i; j < NP; ++j)
        P[tri(NP, i, j)] = P[tri(NP, i, j)] - k[i] * ph[j] - ph[i] * k[j] + k[i] * k[j] * s;
  } else {
#pragma unroll
    for (int i = 0; i < NP; ++i)
#pragma unroll
      for (int j = i; j < NP; ++j) P[tri(NP, i, j)] = fmaf(-k[i], ph[j], P[tri(NP, i, j)]);
  }
}

// The forecast (x_f, P_f) of pixel p: fused (fast or Cholesky form) or read.
// Returns the status bits; cd_ok: cd holds the forecast precision diagonal.
template <int NP, typename GA>
KF_HD uint8_t gain_load_forecast(const GA& a, int64_t p, float (&xf)[NP], float (&P)[ntri(NP)], float (&cd)[NP],
                                 bool& cd_ok) {
  constexpr int NT = ntri(NP);
  const int64_t ld = a.ld;
  cd_ok = false;
  if (a.prop) {
    const KF_CONST_AS PropArgs* pa = opaque(cptr(a.prop));
    if (pa->cov_fast) {
      cd_ok = true;
      return gain_forecast<NP>(pa, p, xf, P, cd);
    }
    return forecast_partial_cov<NP>(pa, p, xf, P);
  }
#pragma unroll
  for (int j = 0; j < NP; ++j) xf[j] = KF_PX(a.x_f, j * ld, p);
#pragma unroll
  for (int t = 0; t < NT; ++t) P[t] = KF_PX(a.p_f, t * ld, p);
  return 0;
}

template <int NP, typename GA>
KF_HD float gain_finish(const GA& a, int64_t p, float (&x)[NP], float (&P)[ntri(NP)], const float (&x0)[NP],
                        uint8_t st, int nobs, const float* dA);

// One pixel of K1g over a.gn_fused (1 or 2) Gauss-Newton iterations.
// EVAL(bi, it, x0, y, w, H0, h, ok) -> bool use: decodes band bi and, where it
// is used, evaluates its operator at x0 (iteration it of the launch) (the matrix-core evaluator runs for the
// whole wave: every lane calls it, act = false lanes included).  Iteration 2
// restarts from the forecast linearised at iteration 1's x; the returned
// |x - x0|^2 is the last iteration's, dn1 the first's.
template <int NP, typename GA, typename EVAL>
KF_HD float gain_pixel(const GA& a, int64_t p, bool act, float& dn1, EVAL&& eval) {
  constexpr int NT = ntri(NP);
  const int64_t ld = a.ld;
  float xf[NP], x0[NP], x[NP], P[NT], cd[NP];
  bool cd_ok;
  const uint8_t st_fc = gain_load_forecast<NP>(a, p, xf, P, cd, cd_ok);
  if (a.x_prev) {
#pragma unroll
    for (int j = 0; j < NP; ++j) x0[j] = KF_PX(a.x_prev, j * ld, p);
  } else {
#pragma unroll
    for (int j = 0; j < NP; ++j) x0[j] = xf[j];
  }
  const int gn = a.gn_fused > 1 ? 2 : 1;
  dn1 = 0.f;
  uint8_t st = st_fc;
  int nobs = 0;
  float dA[NP];
  for (int it = 0; it < gn; ++it) {
    if (it > 0) {
      // iteration 2 linearises at iteration 1's analysis, from the forecast again
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const float d = x[j] - x0[j];
        dn1 = fmaf(d, d, dn1);
        x0[j] = x[j];
      }
      // through an opaque pixel index: recomputed, not kept live across iteration 1 (CSE)
      gain_load_forecast<NP>(a, opaque_lane(p), xf, P, cd, cd_ok);
      st = st_fc;
      nobs = 0;
    }
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      x[j] = xf[j];
      dA[j] = cd[j];
    }
    for (int bi = 0; bi < a.n_bands; ++bi) {
      float y, w, H0, h[NP];
      bool ok;
      const bool use = eval(bi, it, x0, y, w, H0, h, ok);
      if (use && !ok) st |= ST_BAD_OP;
      if (use && ok) {
        ++nobs;
#pragma unroll
        for (int j = 0; j < NP; ++j) dA[j] = fmaf(w * h[j], h[j], dA[j]);
        gain_band_update<NP>(P, x, x0, h, H0, y, w, a.joseph != 0);
      }
    }
  }
  if (!act) return 0.f;
  return gain_finish<NP>(a, p, x, P, x0, st, nobs, cd_ok ? dA : nullptr);
}

template <int NP, int FD = 0, int FOBS = 0>
KF_HD float pixel_gain(const GainArgs& a, int64_t p, float& dn1) {
  const int64_t ld = a.ld;
  return gain_pixel<NP>(a, p, true, dn1, [&](int bi, int, const float (&x0)[NP], float& y, float& w, float& H0,
                                             float (&h)[NP], bool& ok) -> bool {
    const BandDesc bd = cptr(a.bands)[bi];
    decode_obs<FOBS>(bd, p, y, w);
    if (!(w > 0.f)) {
      if (bd.h0_out) KF_PX(bd.h0_out, 0, p) = 0.f;
      return false;
    }
    if constexpr (FD > 0) {
#if defined(__HIP_DEVICE_COMPILE__)
      gp_eval<NP, FD, 4, false, true>(bd, x0, H0, h, a.bands + bi);
#else
      gp_eval<NP, FD>(bd, x0, H0, h);
#endif
      ok = finitef(H0);
#pragma unroll
      for (int j = 0; j < NP; ++j) ok = ok && finitef(h[j]);
    } else {
      ok = eval_operator<NP>(bd, p, ld, x0, H0, h);
    }
    float* h0o = bd.h0_out;
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (FD > 0) h0o = opaque(cptr(a.bands + bi))->h0_out;
#endif
    if (h0o) KF_PX(h0o, 0, p) = H0;
    return true;
  });
}

// K1g tail (shared with the matrix-core gain kernel, kf_gp_mfma.h): health
// fallback, state / covariance (or precision-diagonal) stores, fused output;
// returns |x - x0|^2.  dA: the analysis precision diagonal by the information
// identity (fast forecasts), else null (inverted from P where needed).
template <int NP, typename GA>
KF_HD float gain_finish(const GA& a, int64_t p, float (&x)[NP], float (&P)[ntri(NP)], const float (&x0)[NP],
                        uint8_t st, int nobs, const float* dA) {
  constexpr int NT = ntri(NP);
  const int64_t ld = a.ld;
  if (nobs == 0) st |= ST_NO_OBS;
  bool fin = true;
#pragma unroll
  for (int j = 0; j < NP; ++j) fin = fin && finitef(x[j]);
  float dfb[NP];
  if (!fin) {
    // health fallback: keep the forecast for this pixel
    st |= ST_NONFINITE | ST_FALLBACK;
    bool cd_ok;
    gain_load_forecast<NP>(a, p, x, P, dfb, cd_ok);
    dA = cd_ok ? dfb : nullptr;
  }
  float dn = 0.f;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    KF_PX(a.x_out, j * ld, p) = x[j];
    const float d = x[j] - x0[j];
    dn = fmaf(d, d, dn);
  }
  const bool need_pi = a.out_unc || (a.p_out && a.pdiag_rows);
  float pid[NP];
  if (need_pi) {
    if (dA) {
#pragma unroll
      for (int j = 0; j < NP; ++j) pid[j] = dA[j];
    } else {
      float U[NT], Pi[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) U[t] = P[t];
      if (!chol_packed<NP>(U)) st |= ST_NONSPD;
      chol_inverse<NP>(U, Pi);
#pragma unroll
      for (int j = 0; j < NP; ++j) pid[j] = Pi[tri(NP, j, j)];
    }
  }
  if (a.p_out) {
    if (a.pdiag_rows) {
#pragma unroll
      for (int j = 0; j < NP; ++j)
        if ((a.pdiag_rows >> j) & 1u) KF_PX(a.p_out, tri(NP, j, j) * ld, p) = pid[j];
    } else {
#pragma unroll
      for (int t = 0; t < NT; ++t) KF_PX(a.p_out, t * ld, p) = P[t];
    }
  }
  if (a.out_unc) {
    // fused output: 1/sqrt(diag P^-1), the information form's uncertainty raster
    const int64_t r = a.out_idx ? KF_PX(a.out_idx, 0, p) : p;
    const int64_t pl = a.out_plane;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      if (a.out_mean) KF_PX(a.out_mean, j * pl, r) = x[j];
      KF_PX(a.out_unc, j * pl, r) = kf_rsqrt(pid[j]);
    }
  }
  if (a.status) KF_PX(a.status, 0, p) = st;
  if (a.dn_out) KF_PX(a.dn_out, 0, p) = dn;
  return dn;
}

// ---------------------------------------------------------------------------
// K9: block-Jacobi sweep for the GMRF spatial regulariser (new capability):
//   (A_p + g deg_p E_R) x_p = b_p + g E_R sum_q x_q
// neighbours index an extended x (local pixels, then halo pixels).
struct JacobiArgs {
  int64_t N, ld, ld_ext;
  float gamma;
  uint32_t reg_mask;
  const float* a_in;     // [NT][ld]
  const float* b_in;     // [NP][ld]
  const float* x_ext;    // [NP][ld_ext]
  const int32_t* nbr;    // [4][N] index into x_ext, -1 if none
  const float* x_ref;    // [NP][ld] linearisation point (for the norm)
  float* x_out;          // [NP][ld]
  float* a_out;          // optional: regularised precision written back
  double* partials;
  // Affine form of the same sweeps (JACOBI_PREPARE / _SWEEP / _FINISH): with
  // A_reg = A + g deg E_R factored once per GN iteration, u = A_reg^-1 b and
  // V = A_reg^-1 E_R (NP x k), a sweep is x = u + g V s(x_R), s = sum of the
  // neighbours' regularised components, so only the k regularised fields z
  // are iterated (and exchanged); the full state is formed once at the end.
  int32_t mode, k;
  const float* u;        // [NP][ld]    A_reg^-1 b            (SWEEP, FINISH)
  float* v;              // [k*NP][ld]  column c of V = A_reg^-1 e_{R_c} (PREPARE writes)
  float* z_out;          // [k][ld_ext] regularised components (SWEEP writes the local part)
  StripGeo geo;          // dense strip: neighbours from the index (nbr unused)
  int64_t p0, pn;        // pixel range [p0, p0 + pn) of this launch (pn = 0: all N); C2 overlap
  // Chebyshev acceleration of the sweeps (SWEEP only): z_new = z_prev +
  // omega (jacobi(z) - z_prev) with the semi-iterative weights of a Jacobi
  // matrix whose spectrum lies in [-rho, rho] (linear_kf.py); z_prev = null:
  // the plain Jacobi sweep
  const float* z_prev;   // [k][ld_ext] the iterate before z (local part)
  float omega;
  // FINISH only, optional: fused output dump (unpack_kernel's work) of x and
  // 1/sqrt(diag A) with A = a_in (the analysis precision of this iteration)
  float* out_mean;       // [NP][out_plane]
  float* out_unc;        // [NP][out_plane]
  const int64_t* out_idx;   // raster position of pixel p (nullptr: p)
  int64_t out_plane;
};

template <typename JA>
KF_HD int32_t jacobi_neighbour(const JA& a, int64_t p, int k) {
  const int32_t q = a.geo.w > 0 ? geo_neighbour(a.geo, a.N, p, k) : a.nbr[k * a.N + p];
  KF_DCHECK(q >= -1 && q < a.ld_ext);
  return q;
}

constexpr int JACOBI_CLASSIC = 0, JACOBI_PREPARE = 1, JACOBI_SWEEP = 2, JACOBI_FINISH = 3;

// neighbour sums of the k fields of an extended array (x_ext rows 0..k-1)
template <int NP>
KF_HD void reg_neighbour_sums(const JacobiArgs& a, int64_t p, float (&s)[NP], int& deg) {
#pragma unroll
  for (int c = 0; c < NP; ++c) s[c] = 0.f;
  deg = 0;
#pragma unroll
  for (int q4 = 0; q4 < 4; ++q4) {
    const int32_t q = jacobi_neighbour(a, p, q4);
    if (q >= 0) {
      ++deg;
#pragma unroll
      for (int c = 0; c < NP; ++c)
        if (c < a.k) s[c] += a.x_ext[c * a.ld_ext + q];
    }
  }
}

template <int NP>
KF_HD float pixel_reg_prepare(const JacobiArgs& a, int64_t p) {
  constexpr int NT = ntri(NP);
  const int64_t ld = a.ld;
  float A[NT], b[NP];
#pragma unroll
  for (int t = 0; t < NT; ++t) A[t] = KF_PX(a.a_in, t * ld, p);
#pragma unroll
  for (int j = 0; j < NP; ++j) b[j] = KF_PX(a.b_in, j * ld, p);
  int deg = 0;
#pragma unroll
  for (int q4 = 0; q4 < 4; ++q4) deg += jacobi_neighbour(a, p, q4) >= 0 ? 1 : 0;
#pragma unroll
  for (int j = 0; j < NP; ++j)
    if ((a.reg_mask >> j) & 1u) A[tri(NP, j, j)] += a.gamma * (float)deg;
  if (a.a_out) {
#pragma unroll
    for (int t = 0; t < NT; ++t) KF_PX(a.a_out, t * ld, p) = A[t];
  }
  const bool spd = chol_packed<NP>(A);
  chol_solve<NP>(A, b);
  bool bad = !spd;
#pragma unroll
  for (int j = 0; j < NP; ++j) bad = bad || !finitef(b[j]);
  // unhealthy pixel: decoupled (V = 0) at the reference point (x_ref when
  // given, else 0), so no non-finite value enters the neighbour sums
#pragma unroll
  for (int j = 0; j < NP; ++j) KF_PX(a.x_out, j * ld, p) = bad ? (a.x_ref ? KF_PX(a.x_ref, j * ld, p) : 0.f) : b[j];
  int c = 0;
#pragma unroll
  for (int r = 0; r < NP; ++r) {
    if ((a.reg_mask >> r) & 1u) {
      float e[NP];
#pragma unroll
      for (int j = 0; j < NP; ++j) e[j] = (j == r) ? 1.f : 0.f;
      chol_solve<NP>(A, e);
#pragma unroll
      for (int j = 0; j < NP; ++j) KF_PX(a.v, ((int64_t)c * NP + j) * ld, p) = bad ? 0.f : e[j];
      ++c;
    }
  }
  return 0.f;
}

template <int NP>
KF_HD float pixel_reg_sweep(const JacobiArgs& a, int64_t p) {
  const int64_t ld = a.ld;
  float s[NP];
  int deg;
  reg_neighbour_sums<NP>(a, p, s, deg);
  int r = 0;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    if ((a.reg_mask >> j) & 1u) {
      float z = 0.f;
#pragma unroll
      for (int c = 0; c < NP; ++c)
        if (c < a.k) z = fmaf(KF_PX(a.v, ((int64_t)c * NP + j) * ld, p), s[c], z);
      float zn = fmaf(a.gamma, z, KF_PX(a.u, j * ld, p));
      if (a.z_prev) {
        const float zp = a.z_prev[r * a.ld_ext + p];
        zn = fmaf(a.omega, zn - zp, zp);
      }
      a.z_out[r * a.ld_ext + p] = zn;
      ++r;
    }
  }
  return 0.f;
}

template <int NP>
KF_HD float pixel_reg_finish(const JacobiArgs& a, int64_t p) {
  const int64_t ld = a.ld;
  float s[NP];
  int deg;
  reg_neighbour_sums<NP>(a, p, s, deg);
  float dn = 0.f;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    float z = 0.f;
#pragma unroll
    for (int c = 0; c < NP; ++c)
      if (c < a.k) z = fmaf(KF_PX(a.v, ((int64_t)c * NP + j) * ld, p), s[c], z);
    const float x = fmaf(a.gamma, z, KF_PX(a.u, j * ld, p));
    KF_PX(a.x_out, j * ld, p) = x;
    const float d = x - KF_PX(a.x_ref, j * ld, p);
    dn = fmaf(d, d, dn);
    if (a.out_mean) {
      const int64_t r = a.out_idx ? KF_PX(a.out_idx, 0, p) : p;
      KF_DCHECK(r >= 0 && r < a.out_plane);
      KF_PX(a.out_mean, j * a.out_plane, r) = x;
      if (a.out_unc) KF_PX(a.out_unc, j * a.out_plane, r) = kf_rsqrt(KF_PX(a.a_in, tri(NP, j, j) * ld, p));
    }
  }
  return dn;
}

// One regularised field (k = 1, the GMRF-on-LAI configuration): the sweep and
// finish passes for U pixels per thread (i0, i0 + stride, ...), every load
// issued before the first store.  These passes stream ~16 and ~120 B/px; one
// pixel per thread and iteration left them latency-bound (one HBM round trip
// per grid-stride step).  Neighbours are read branch-free (a missing one
// reads the pixel itself and is weighted 0).
constexpr int JACOBI_SWEEP1 = 4, JACOBI_FINISH1 = 5, JACOBI_U = 4;

template <typename JA>
KF_HD float reg_nsum1(const JA& a, int64_t p) {
  float s = 0.f;
#pragma unroll
  for (int q4 = 0; q4 < 4; ++q4) {
    const int32_t q = jacobi_neighbour(a, p, q4);
    const float zq = a.x_ext[q >= 0 ? (int64_t)q : p];
    s += q >= 0 ? zq : 0.f;
  }
  return s;
}

template <int NP, int U>
KF_HD float reg_sweep1(const JacobiArgs& a, int64_t i0, int64_t stride, int64_t n) {
  const int64_t ld = a.ld;
  const int j0 = __builtin_ctz(a.reg_mask);
  float z[U];
  int64_t pp[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = i0 + u * stride;
    pp[u] = a.p0 + (i < n ? i : i0);
    const float s = reg_nsum1(a, pp[u]);
    z[u] = fmaf(a.gamma, a.v[j0 * ld + pp[u]] * s, a.u[j0 * ld + pp[u]]);
    if (a.z_prev) {
      const float zp = a.z_prev[pp[u]];
      z[u] = fmaf(a.omega, z[u] - zp, zp);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (i0 + u * stride < n) a.z_out[pp[u]] = z[u];
  return 0.f;
}

template <int NP, int U>
KF_HD float reg_finish1(const JacobiArgs& a, int64_t i0, int64_t stride, int64_t n) {
  const int64_t ld = a.ld;
  float x[U][NP];
  int64_t pp[U];
  float dn = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = i0 + u * stride;
    pp[u] = a.p0 + (i < n ? i : i0);
    const float s = reg_nsum1(a, pp[u]);
    float du = 0.f;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      x[u][j] = fmaf(a.gamma, a.v[j * ld + pp[u]] * s, a.u[j * ld + pp[u]]);
      const float d = x[u][j] - a.x_ref[j * ld + pp[u]];
      du = fmaf(d, d, du);
    }
    dn += i < n ? du : 0.f;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (i0 + u * stride >= n) continue;
    const int64_t p = pp[u];
#pragma unroll
    for (int j = 0; j < NP; ++j) KF_PX(a.x_out, j * ld, p) = x[u][j];
    if (a.out_mean) {
      const int64_t r = a.out_idx ? KF_PX(a.out_idx, 0, p) : p;
      KF_DCHECK(r >= 0 && r < a.out_plane);
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        KF_PX(a.out_mean, j * a.out_plane, r) = x[u][j];
        if (a.out_unc) KF_PX(a.out_unc, j * a.out_plane, r) = kf_rsqrt(KF_PX(a.a_in, tri(NP, j, j) * ld, p));
      }
    }
  }
  return dn;
}

// Dense strips (StripGeo) with one regularised field: the row-loop forms of
// reg_sweep1 / reg_finish1.  A block walks whole rows, its threads the
// columns, so (row, column) are loop indices -- no per-neighbour integer
// division of the pixel index (geo_neighbour) -- and the neighbour sum adds
// up / down / left / right in reg_nsum1's order (bit-identical results).
constexpr int JACOBI_SWEEP1D = 6, JACOBI_FINISH1D = 7;

template <typename JA>
KF_HD float reg_nsum_dense(const JA& a, uint32_t r, uint32_t c, int64_t p) {
  const uint32_t w = (uint32_t)a.geo.w;
  float s = 0.f;
  if (r > 0) s += a.x_ext[p - w];
  else if (a.geo.halo & 1) s += a.x_ext[a.N + c];
  if (r + 1 < (uint32_t)a.geo.h) s += a.x_ext[p + w];
  else if (a.geo.halo & 2) s += a.x_ext[a.N + a.geo.n_up + c];
  if (c > 0) s += a.x_ext[p - 1];
  if (c + 1 < w) s += a.x_ext[p + 1];
  return s;
}

// U pixels of row r at columns c0 + u * BLOCK (u < U): every load of the U
// pixels is issued before the first store (the stores may alias the inputs
// as far as the compiler knows, which would serialise a per-pixel order).
template <int NP, int U, int BS>
KF_HD void reg_sweep1d(const JacobiArgs& a, uint32_t r, uint32_t c0, int j0) {
  const uint32_t w = (uint32_t)a.geo.w;
  const int64_t ld = a.ld;
  float z[U];
  int64_t pp[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t c = c0 + u * BS < w ? c0 + u * BS : c0;
    const int64_t p = (int64_t)r * w + c;
    pp[u] = p;
    z[u] = fmaf(a.gamma, KF_PX(a.v, j0 * ld, p) * reg_nsum_dense(a, r, c, p), KF_PX(a.u, j0 * ld, p));
    if (a.z_prev) {
      const float zp = KF_PX(a.z_prev, 0, p);
      z[u] = fmaf(a.omega, z[u] - zp, zp);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (c0 + u * BS < w) a.z_out[pp[u]] = z[u];
}

template <int NP, int U, int BS>
KF_HD float reg_finish1d(const JacobiArgs& a, uint32_t r, uint32_t c0) {
  const uint32_t w = (uint32_t)a.geo.w;
  const int64_t ld = a.ld;
  float x[U][NP];
  int64_t pp[U];
  float dn = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool in = c0 + u * BS < w;
    const uint32_t c = in ? c0 + u * BS : c0;
    const int64_t p = (int64_t)r * w + c;
    pp[u] = p;
    const float s = reg_nsum_dense(a, r, c, p);
    float du = 0.f;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      x[u][j] = fmaf(a.gamma, KF_PX(a.v, j * ld, p) * s, KF_PX(a.u, j * ld, p));
      const float d = x[u][j] - KF_PX(a.x_ref, j * ld, p);
      du = fmaf(d, d, du);
    }
    dn += in ? du : 0.f;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (c0 + u * BS >= w) continue;
    const int64_t p = pp[u];
#pragma unroll
    for (int j = 0; j < NP; ++j) KF_PX(a.x_out, j * ld, p) = x[u][j];
    if (a.out_mean) {
      const int64_t ro = a.out_idx ? KF_PX(a.out_idx, 0, p) : p;
      KF_DCHECK(ro >= 0 && ro < a.out_plane);
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        KF_PX(a.out_mean, j * a.out_plane, ro) = x[u][j];
        if (a.out_unc) KF_PX(a.out_unc, j * a.out_plane, ro) = kf_rsqrt(KF_PX(a.a_in, tri(NP, j, j) * ld, p));
      }
    }
  }
  return dn;
}

// The finish over 4 adjacent pixels of one row (w % 4 == 0, so a 4-aligned
// pixel index never straddles rows) with 16-byte loads and stores: the pass
// streams ~116 B/px (~200 with the output dump), and per-pixel 4-byte
// accesses left it at about half the HBM rate.  Same operations per pixel as
// reg_finish1d (neighbour order up, down, left, right).  The launcher checks
// the alignment of every operand (kf_kernels.hip).
constexpr int JACOBI_FINISH4 = 8;

struct alignas(16) F4 {
  float x, y, z, w;
};
KF_HD F4 ld4(const float* p) { return *reinterpret_cast<const F4*>(p); }
KF_HD void st4(float* p, F4 v) { *reinterpret_cast<F4*>(p) = v; }
KF_HD float f4_at(const F4& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }

template <int NP>
KF_HD float reg_finish4(const JacobiArgs& a, int64_t p) {
  const int64_t w = a.geo.w, ld = a.ld, N = a.N;
  const int64_t r = p / w, c = p - r * w;
  const float* z = a.x_ext;
  const bool up = r > 0 || (a.geo.halo & 1), dn = r + 1 < a.geo.h || (a.geo.halo & 2);
  const F4 zu = up ? ld4(r > 0 ? z + p - w : z + N + c) : F4{0.f, 0.f, 0.f, 0.f};
  const F4 zd = dn ? ld4(r + 1 < a.geo.h ? z + p + w : z + N + a.geo.n_up + c) : F4{0.f, 0.f, 0.f, 0.f};
  const F4 zc = ld4(z + p);
  const float zl = c > 0 ? z[p - 1] : 0.f;
  const float zr = c + 4 < w ? z[p + 4] : 0.f;
  float s[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float t = 0.f;
    if (up) t += f4_at(zu, i);
    if (dn) t += f4_at(zd, i);
    if (c + i > 0) t += i == 0 ? zl : f4_at(zc, i - 1);
    if (c + i + 1 < w) t += i == 3 ? zr : f4_at(zc, i + 1);
    s[i] = t;
  }
  F4 x[NP];
  float du4[4] = {0.f, 0.f, 0.f, 0.f};   // per pixel, as reg_finish1d
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const F4 u = ld4(a.u + j * ld + p), v = ld4(a.v + j * ld + p), xr = ld4(a.x_ref + j * ld + p);
    x[j] = F4{fmaf(a.gamma, v.x * s[0], u.x), fmaf(a.gamma, v.y * s[1], u.y), fmaf(a.gamma, v.z * s[2], u.z),
              fmaf(a.gamma, v.w * s[3], u.w)};
    const float d0 = x[j].x - xr.x, d1 = x[j].y - xr.y, d2 = x[j].z - xr.z, d3 = x[j].w - xr.w;
    du4[0] = fmaf(d0, d0, du4[0]);
    du4[1] = fmaf(d1, d1, du4[1]);
    du4[2] = fmaf(d2, d2, du4[2]);
    du4[3] = fmaf(d3, d3, du4[3]);
  }
  F4 dg[NP];
  if (a.out_unc) {
#pragma unroll
    for (int j = 0; j < NP; ++j) dg[j] = ld4(a.a_in + tri(NP, j, j) * ld + p);
  }
#pragma unroll
  for (int j = 0; j < NP; ++j) st4(a.x_out + j * ld + p, x[j]);
  if (a.out_mean) {
#pragma unroll
    for (int j = 0; j < NP; ++j) st4(a.out_mean + j * a.out_plane + p, x[j]);
  }
  if (a.out_unc) {
#pragma unroll
    for (int j = 0; j < NP; ++j)
      st4(a.out_unc + j * a.out_plane + p,
          F4{kf_rsqrt(dg[j].x), kf_rsqrt(dg[j].y), kf_rsqrt(dg[j].z), kf_rsqrt(dg[j].w)});
  }
  return ((du4[0] + du4[1]) + du4[2]) + du4[3];
}

// Several sweeps of one regularised field in one pass over a dense strip with
// no halo rows (world = 1, or a strip with no neighbours): temporal blocking.
// A workgroup loads a tile plus a ring `nsweep` pixels wide into LDS, runs
// every sweep there (the ring's values go stale one pixel per sweep, the
// interior never reads a stale one) and writes the interior's last two
// iterates.  Sweep s is reg_sweep1d's update with omega[s], Chebyshev against
// the previous iterate when bit s of prev_mask is set (plain Jacobi
// otherwise); the same operations in the same order, so the result is
// bit-identical to nsweep launches of JACOBI_SWEEP1D.
constexpr int REG_TILE_MAX_SWEEPS = 8;
struct RegTileArgs {
  int64_t ld;                // u / v leading dimension
  int32_t w, h;              // strip geometry (w * h local pixels)
  int32_t j0, nsweep;        // regularised row of u / v; sweeps in this pass (at most)
  uint32_t prev_mask;        // bit s: sweep s is a Chebyshev step against the iterate before
  float gamma;
  float omega[REG_TILE_MAX_SWEEPS];
  const float* u;            // [NP][ld]  (row j0 used)
  const float* v;            // [k*NP][ld] (row j0 used)
  const float* z;            // [w*h] current iterate
  const float* zp;           // [w*h] the iterate before (read when the first sweep is a Chebyshev step)
  float* z_out;              // iterate after the pass's sweeps
  float* zp_out;             // the iterate before that
  // Deep halo (tile-DP strips with neighbours; C2 once per pass instead of once
  // per sweep): rows -hu..-1 above and h..h+hd-1 below the strip, each side 4
  // planes of halo_plane floats -- u, v, z, zp -- row-major from its first row
  // (row -hu, row h).  The ring of the strip's edge tiles reads them; a pass of
  // ns <= min(hu, hd) sweeps (hu / hd > 0) leaves every strip row exact because
  // the values that go stale at the halo's outer edge move one row per sweep.
  int32_t hu, hd;
  const float* halo_up;
  const float* halo_dn;
  int64_t halo_plane;
  int32_t ty0, ty1;          // tile rows [ty0, ty1) of this launch (ty1 = 0: every tile row)
  // Device-resident schedule (RegSchedule, no host read-back before the pass):
  // sched[0] = sweeps of this GN iteration's coupled solve before the finish,
  // omega_tab[s] = the Chebyshev weight of sweep s (0: a plain Jacobi sweep).
  // This pass runs sweeps s_base .. s_base + min(nsweep, sched[0] - s_base) - 1
  // (none: the outputs are copies of the inputs).  Null: nsweep / prev_mask / omega.
  const int32_t* sched;
  const float* omega_tab;
  int32_t s_base;
};

// sweeps this pass runs and the weight of its sweep s (cheb: a Chebyshev step)
KF_HD int reg_tile_nsweep(const RegTileArgs& a) {
  if (!a.sched) return a.nsweep;
  const int left = a.sched[0] - a.s_base;
  return left < 0 ? 0 : (left < a.nsweep ? left : a.nsweep);
}
KF_HD float reg_tile_omega(const RegTileArgs& a, int s, bool& cheb) {
  if (a.sched) {
    const float om = a.omega_tab[a.s_base + s];
    cheb = om != 0.f;
    return om;
  }
  cheb = (a.prev_mask >> s) & 1u;
  return a.omega[s];
}

// Chebyshev schedule of a GN iteration's coupled solve (K9) from the all-rank
// Jacobi bound rho (Gershgorin, linear_kf.py:_reg_schedule): S sweeps in all
// (the last is the finish) cut the error by tol at the Chebyshev rate
// sigma = rho / (1 + sqrt(1 - rho^2)); rho >= 1 (or NaN): max_sweeps plain
// Jacobi sweeps; rho <= 0: one.  omega[it] for it < S - 1 (0: plain Jacobi,
// the first sweep always).  Double precision, one thread: the device kernel
// and the host runner evaluate the same expressions.
KF_HD int reg_cheb_schedule(double rho, double tol, int max_sweeps, float* omega, double* rho_used) {
  int S;
  double r = rho;
  if (!(r < 1.0)) {
    r = 0.0;
    S = max_sweeps;
  } else if (r <= 0.0) {
    r = 0.0;
    S = 1;
  } else {
    const double sigma = r / (1.0 + sqrt(fmax(0.0, 1.0 - r * r)));
    const double need = ceil(log(2.0 / tol) / log(1.0 / sigma));
    S = (int)fmin(fmax(1.0, need), (double)max_sweeps);
  }
  double om = 1.0;
  for (int it = 0; it < S - 1; ++it) {
    const bool cheb = r > 0.0 && it > 0;
    if (cheb) om = it == 1 ? 1.0 / (1.0 - 0.5 * r * r) : 1.0 / (1.0 - 0.25 * r * r * om);
    omega[it] = cheb ? (float)om : 0.f;
  }
  *rho_used = r;
  return S;
}

struct RegScheduleArgs {
  const float* pmax;         // per-block maxima of v_RR * deg (reg_rho pass), npart of them
  int32_t npart;
  float gamma;
  double* rho;               // [1] g * max: written by the rho pass, all-reduced (max) over ranks in between
  double tol;
  int32_t max_sweeps;
  int32_t* sched;            // [1] sweeps before the finish (S - 1)
  float* omega_tab;          // [max_sweeps]
  double* info;              // [2] rho used, S (read back by the host, asynchronously)
};

// per-pixel term of the Jacobi bound for one regularised field on a dense strip:
// V_RR * deg (deg from the index, halo rows included)
KF_HD float reg_rho_term(const float* vrow, const StripGeo& g, int64_t p) {
  const uint32_t w = (uint32_t)g.w;
  const uint32_t r = (uint32_t)p / w, c = (uint32_t)p - r * w;
  const int deg = ((r > 0 || (g.halo & 1)) ? 1 : 0) + ((r + 1 < (uint32_t)g.h || (g.halo & 2)) ? 1 : 0) +
                  (c > 0 ? 1 : 0) + (c + 1 < w ? 1 : 0);
  return vrow[p] * (float)deg;
}

// neighbour sum in reg_nsum_dense's order (up, down, left, right; missing ones skipped)
KF_HD float reg_tile_nsum(const float* z, int64_t p, int64_t w, bool up, bool dn, bool lf, bool rt) {
  float s = 0.f;
  if (up) s += z[p - w];
  if (dn) s += z[p + w];
  if (lf) s += z[p - 1];
  if (rt) s += z[p + 1];
  return s;
}

KF_HD float reg_tile_step(const RegTileArgs& a, int s, float s_nb, float u, float v, float zp) {
  float z = fmaf(a.gamma, v * s_nb, u);
  bool cheb;
  const float om = reg_tile_omega(a, s, cheb);
  if (cheb) z = fmaf(om, z - zp, zp);
  return z;
}

template <int NP>
KF_HD float pixel_jacobi_classic(const JacobiArgs& a, int64_t p);

template <int NP>
KF_HD float pixel_jacobi(const JacobiArgs& a, int64_t p) {
  switch (a.mode) {
    case JACOBI_PREPARE: return pixel_reg_prepare<NP>(a, p);
    case JACOBI_SWEEP: return pixel_reg_sweep<NP>(a, p);
    case JACOBI_FINISH: return pixel_reg_finish<NP>(a, p);
    default: return pixel_jacobi_classic<NP>(a, p);
  }
}

template <int NP>
KF_HD float pixel_jacobi_classic(const JacobiArgs& a, int64_t p) {
  constexpr int NT = ntri(NP);
  const int64_t ld = a.ld;
  float A[NT], b[NP];
#pragma unroll
  for (int t = 0; t < NT; ++t) A[t] = KF_PX(a.a_in, t * ld, p);
#pragma unroll
  for (int j = 0; j < NP; ++j) b[j] = KF_PX(a.b_in, j * ld, p);
  int deg = 0;
  float sx[NP];
#pragma unroll
  for (int j = 0; j < NP; ++j) sx[j] = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int32_t q = jacobi_neighbour(a, p, k);
    if (q >= 0) {
      ++deg;
#pragma unroll
      for (int j = 0; j < NP; ++j) sx[j] += a.x_ext[j * a.ld_ext + q];
    }
  }
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    if ((a.reg_mask >> j) & 1u) {
      A[tri(NP, j, j)] += a.gamma * (float)deg;
      b[j] = fmaf(a.gamma, sx[j], b[j]);
    }
  }
  if (a.a_out) {
#pragma unroll
    for (int t = 0; t < NT; ++t) KF_PX(a.a_out, t * ld, p) = A[t];
  }
  chol_packed<NP>(A);
  chol_solve<NP>(A, b);
  float dn = 0.f;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    KF_PX(a.x_out, j * ld, p) = b[j];
    const float d = b[j] - KF_PX(a.x_ref, j * ld, p);
    dn = fmaf(d, d, dn);
  }
  return dn;
}

// ---------------------------------------------------------------------------
// Per-chunk Gauss-Newton convergence (EngineConfig.convergence_chunk).  The
// reference never runs a whole tile as one filter: its drivers cut the raster
// into get_chunks tiles (kafka_test_Py36.py:241, 256^2) and each chunk's own
// LinearKalman tests ||x_a - x_prev||_2 / len(x_a) over that chunk alone
// (linear_kf.py:293-304).  The engine keeps one filter per rank and evaluates
// that test per chunk: the analysis writes each pixel's |x - x0|^2 (dn_out),
// chunk_partials sums a chunk's pixels in a fixed order (bit-reproducible,
// independent of the visiting order), the ranks' per-chunk partials are
// all-gathered and summed in rank order (chunk_decide, identical on every
// rank), and converged chunks leave the visiting order (chunk_compact).

// this rank's pixels of a chunk: runs of consecutive local indices, one per
// (chunk, raster row) -- the active pixels of a row inside a chunk's column
// range are contiguous in the strip's row-major numbering.  The summation
// order: runs in groups of CHUNK_GROUP_RUNS (row order); within a group, a
// thread-strided f64 sum per column slot, the xor shuffle tree of wave_sum and
// the wave sums in order; the group totals then in group order.
constexpr int CHUNK_GROUP_RUNS = 16;
struct ChunkPartialArgs {
  const float* dn;           // [N] |x - x0|^2 per pixel (AnalysisArgs.dn_out)
  const int32_t* seg_start;  // [S] first local pixel of each run
  const int32_t* seg_len;    // [S] run length
  const int32_t* lc_ptr;     // [n_local + 1]: runs of local chunk c are [lc_ptr[c], lc_ptr[c + 1]), row order
  const int32_t* lc_gid;     // [n_local] global chunk id (get_chunks order, 0-based)
  int32_t n_local;
  const uint8_t* active;     // [nc] chunks still iterating (frozen ones are skipped)
  int64_t* part;             // [nc] this rank's sum per global chunk, in quanta (chunk_quant)
  int64_t* gpart;            // [n_local * groups] scratch: the group totals
  int32_t groups;            // >= ceil(runs / CHUNK_GROUP_RUNS) of every local chunk
  const double* qinv;        // [nc] quanta per unit of |dx|^2 of each chunk (engine/chunks.py:quantum)
  int64_t clamp;             // largest quanta one pixel contributes (twice the exit threshold)
};

// One pixel's |dx|^2 in integer quanta of its chunk's squared norm: the sums
// are exact, so a chunk's total (and its exit test) does not depend on how
// the strips of the ranks cut it, nor on the order of the adds -- 1, 4 and 8
// ranks decide alike by construction.  A pixel at or above the clamp (twice
// the chunk's threshold on its own), or NaN, counts as the clamp: the chunk
// does not stop, as the reference's ``norm < tol`` is false for it.
KF_HD int64_t chunk_quant(float dn, double qinv, int64_t clamp) {
  const double v = (double)dn * qinv;
  if (!(v < (double)clamp)) return clamp;
  return (int64_t)(v + 0.5);
}

struct ChunkDecideArgs {
  const int64_t* part_all;   // [world][nc] all ranks' partials in quanta (all-gathered)
  int32_t world, nc;
  const double* len_x;       // [nc] n_params x active pixels of the chunk (all ranks)
  const int32_t* local_count;  // [nc] this rank's pixels of the chunk
  double tol;
  int32_t n_iter, min_iter, max_iter;
  uint8_t* active;           // [nc] in/out
  uint8_t* newly;            // [nc] out: converged (or bailed out) at this iteration
  int32_t* iters;            // [nc] out: Gauss-Newton iterations of the chunk (set when it stops)
  double* info;              // [4] chunks still active (all ranks), largest norm tested, this rank's active
                             // pixels, chunks stopped at this iteration
  int32_t* px_out;           // null, or this rank's active pixels as an int (the next launch's device count)
  double unit;               // squared chunk norm ||dx||^2 / len_x^2 of one quantum
};

// the reference's exit test (linear_kf.py:297-304) for one chunk
KF_HD bool chunk_stops(double norm, int n_iter, int min_iter, int max_iter, double tol) {
  return (norm < tol && n_iter >= min_iter) || n_iter > max_iter;
}

struct ChunkCompactArgs {
  const int32_t* order_in;   // visiting order of the last launch (null: 0..n_in-1)
  int64_t n_in;
  const int32_t* n_in_dev;   // null, or the device count of order_in's slots (<= n_in, the grid bound)
  const int32_t* chunk_of;   // [N] global chunk of each local pixel
  const uint8_t* active;
  const uint8_t* newly;
  int32_t* counts;           // [blocks + 1] scratch (device)
  int32_t* order_out;        // the active chunks' pixels, in order_in's order (stable)
  const float* x_src;        // frozen copy: x of the newly stopped chunks' pixels from x_src ...
  float* x_dst;              // ... into x_dst (the next launch's output buffer keeps their final x)
  int32_t np;
  int64_t ld;
};

// ---------------------------------------------------------------------------
// K6: second-order (Hessian) correction for GP bands (kf_tools.py:26-72):
//   A -= w r d2f/dx2,  r = y - H0 at x.
template <int NP, int D>
KF_HD void gp_hessian(const BandDesc& bd, const float (&x)[NP], float& f, float (&Hs)[ntri(NP)]) {
  float xi[D];
  float c = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    xi[d] = gather_state<NP>(x, bd.map[d]) - bd.center[d];
    c = fmaf(bd.coef[d] * xi[d], xi[d], c);
  }
  c *= -0.5f * LOG2E;
  float S0 = 0.f, S[D], S2[ntri(D)];
#pragma unroll
  for (int d = 0; d < D; ++d) S[d] = 0.f;
#pragma unroll
  for (int t = 0; t < ntri(D); ++t) S2[t] = 0.f;
  constexpr int R = D + 1;
  const KF_CONST_AS float* rr = cptr(bd.gp);
  for (int i = 0; i < bd.T; ++i) {
    float e = gp_rec(rr, R, i, 0) + c;
#pragma unroll
    for (int d = 0; d < D; ++d) e = fmaf(gp_rec(rr, R, i, 1 + d), xi[d], e);
    const float m = kexp2(e);                       // |alpha_i| k_i
    const float ak = ((i >> 1) < bd.Tp) ? m : -m;   // alpha_i k_i
    S0 += ak;
    float t[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      t[d] = gp_rec(rr, R, i, 1 + d) / (LOG2E * bd.coef[d]);
      S[d] = fmaf(ak, t[d], S[d]);
    }
#pragma unroll
    for (int u = 0; u < D; ++u)
#pragma unroll
      for (int v = u; v < D; ++v) S2[tri(D, u, v)] = fmaf(ak * t[u], t[v], S2[tri(D, u, v)]);
  }
  f = bd.offset + S0;
  // d2f/dxu dxv = lu lv [xu xv S0 - xu Sv - xv Su + Suv] - lu delta_uv S0
#pragma unroll
  for (int t = 0; t < ntri(NP); ++t) Hs[t] = 0.f;
#pragma unroll
  for (int u = 0; u < D; ++u)
#pragma unroll
    for (int v = u; v < D; ++v) {
      const float lu = bd.coef[u], lv = bd.coef[v];
      float val = lu * lv * (xi[u] * xi[v] * S0 - xi[u] * S[v] - xi[v] * S[u] + S2[tri(D, u, v)]);
      if (u == v) val -= lu * S0;
      const int ju = bd.map[u], jv = bd.map[v];
#pragma unroll
      for (int i = 0; i < NP; ++i)
#pragma unroll
        for (int j = i; j < NP; ++j) {
          const bool hit = (ju == i && jv == j) || (ju == j && jv == i);
          const bool dup = (u != v) && (ju == jv) && (ju == i) && (i == j);
          Hs[tri(NP, i, j)] += hit ? (dup ? 2.f * val : val) : 0.f;
        }
    }
}

template <int NP, int D = 1>
KF_HD bool gp_hessian_dispatch(const BandDesc& bd, const float (&x)[NP], float& f, float (&Hs)[ntri(NP)]) {
  if constexpr (D <= NP && D <= 12) {
    if (bd.d == D) { gp_hessian<NP, D>(bd, x, f, Hs); return true; }
    return gp_hessian_dispatch<NP, D + 1>(bd, x, f, Hs);
  } else {
    return false;
  }
}

}  // namespace kf
