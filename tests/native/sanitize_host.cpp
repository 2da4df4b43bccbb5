// sanitize_host.cpp — AddressSanitizer / UBSan driver for the host runner.
//
// GPU sanitizers are not available on the MI355X pool, so memory-safety of the
// per-pixel code (kf_core.h, shared verbatim with the gfx950 kernels) is
// checked here on the CPU: every host entry point runs on a small problem with
// exactly-sized buffers (no padding), so an out-of-bounds index in the shared
// code faults under -fsanitize=address.  Built and run by
// tests/test_sanitizers.py:
//   g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer
//       -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Icsrc -fopenmp
//       tests/native/sanitize_host.cpp csrc/kf_host.cpp
#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "kf_launch.h"

using namespace kf;

namespace {

std::mt19937 rng(1234);
float unif(float a, float b) { return std::uniform_real_distribution<float>(a, b)(rng); }

int failures = 0;
void check(bool ok, const char* what) {
  if (!ok) {
    std::fprintf(stderr, "FAIL: %s\n", what);
    ++failures;
  }
}
bool all_finite(const std::vector<float>& v) {
  for (float f : v)
    if (!std::isfinite(f)) return false;
  return true;
}

// GP records, pair layout [T/2][D+1][2] (models/gp.py: records()): L', B[D];
// the first half of the pairs is the alpha > 0 group (BandDesc.Tp = T/4).
std::vector<float> gp_records(int D, int T) {
  const int R = D + 1;
  std::vector<float> r((size_t)T / 2 * R * 2);
  for (int i = 0; i < T; ++i) {
    const float t_scale = 0.3f;
    for (int f = 0; f < R; ++f) {
      const float v = (f == 0) ? unif(-6.f, -3.f)                 // L' = L + log2|alpha|
                               : unif(-1.f, 1.f) * t_scale;      // B
      r[((size_t)(i >> 1) * R + f) * 2 + (i & 1)] = v;
    }
  }
  return r;
}

template <int NP>
void spd_packed(std::vector<float>& P, int64_t N, float diag) {
  constexpr int NT = NP * (NP + 1) / 2;
  P.assign((size_t)NT * N, 0.f);
  for (int64_t p = 0; p < N; ++p)
    for (int i = 0; i < NP; ++i)
      for (int j = i; j < NP; ++j)
        P[(size_t)tri(NP, i, j) * N + p] = (i == j) ? diag + unif(0.f, 1.f) : unif(-0.1f, 0.1f);
}

}  // namespace

int main() {
  constexpr int NP = 7, NT = NP * (NP + 1) / 2, D = 4, T = 64;
  const int64_t N = 1000;              // not a multiple of 256: exercises the ragged tail
  const int grid = (int)((N + 255) / 256);

  std::vector<float> x((size_t)NP * N), xf((size_t)NP * N), Pf, xo((size_t)NP * N), ao((size_t)NT * N);
  std::vector<float> bo((size_t)NP * N);
  for (auto& v : x) v = unif(0.1f, 0.9f);
  for (auto& v : xf) v = unif(0.1f, 0.9f);
  spd_packed<NP>(Pf, N, 10.f);
  std::vector<uint8_t> status((size_t)N);
  std::vector<double> partials((size_t)grid);

  // two GP bands on uint16 DN observations (0 = masked)
  std::vector<std::vector<float>> recs = {gp_records(D, T), gp_records(D, T)};
  std::vector<std::vector<uint16_t>> dn(2, std::vector<uint16_t>((size_t)N));
  std::vector<std::vector<float>> h0o(2, std::vector<float>((size_t)N));
  for (auto& d : dn)
    for (auto& v : d) v = (unif(0.f, 1.f) < 0.2f) ? 0 : (uint16_t)unif(100.f, 5000.f);
  BandDesc bands[2];
  for (int b = 0; b < 2; ++b) {
    BandDesc& bd = bands[b];
    std::memset(&bd, 0, sizeof(bd));
    bd.op = OP_GP;
    bd.obs = OBS_DN16;
    bd.d = D;
    bd.T = T;
    bd.Tp = T / 4;
    const int mp[2][4] = {{0, 1, 6, 2}, {3, 4, 6, 5}};
    for (int d = 0; d < D; ++d) {
      bd.map[d] = mp[b][d];
      bd.coef[d] = unif(0.5f, 5.f);
      bd.center[d] = 0.5f;
    }
    bd.scale = 1e-4f;
    bd.rel_unc = 0.05f;
    bd.unc_floor = 2.5e-3f;
    bd.gp = recs[b].data();
    bd.dn = dn[b].data();
    bd.h0_out = h0o[b].data();
  }

  // K1 information-form analysis
  AnalysisArgs a;
  std::memset(&a, 0, sizeof(a));
  a.N = N; a.ld = N; a.n_bands = 2; a.solve = 1;
  a.bands = bands; a.x_prev = x.data(); a.x_f = xf.data(); a.pf_inv = Pf.data();
  a.x_out = xo.data(); a.a_out = ao.data(); a.b_out = bo.data(); a.status = status.data();
  a.partials = partials.data();
  check(host_analysis(NP, a, grid) == 0, "host_analysis rc");
  check(all_finite(xo) && all_finite(ao), "analysis outputs finite");

  // K1 with the propagation fused (partial prior reset, linearised at the forecast)
  std::vector<float> ao2((size_t)NT * N);
  PropArgs pr;
  std::memset(&pr, 0, sizeof(pr));
  pr.N = N; pr.ld = N; pr.mode = PROP_PRIOR_PARTIAL; pr.prop_mask = 1u << 6;
  for (int j = 0; j < NP; ++j) { pr.m[j] = 1.f; pr.q[j] = 0.04f; pr.reset_mean[j] = 0.5f; }
  for (int t = 0; t < NT; ++t) pr.reset_cinv[t] = 0.f;
  for (int j = 0; j < NP; ++j) pr.reset_cinv[tri(NP, j, j)] = 4.f;
  pr.x_a = x.data(); pr.p_a = Pf.data();
  AnalysisArgs af = a;
  af.x_prev = nullptr; af.x_f = nullptr; af.pf_inv = nullptr; af.a_out = ao2.data(); af.b_out = nullptr;
  af.prop = &pr;
  check(host_analysis(NP, af, grid) == 0, "host_analysis fused rc");
  check(all_finite(xo) && all_finite(ao2), "fused analysis outputs finite");

  // band-chunk accumulation (a_in/b_in) without a solve
  AnalysisArgs ac = a;
  ac.solve = 0; ac.a_in = ao.data(); ac.b_in = bo.data(); ac.a_out = ao2.data(); ac.b_out = bo.data();
  ac.x_out = nullptr; ac.partials = nullptr;
  check(host_analysis(NP, ac, grid) == 0, "host_analysis chunk rc");

  // K4/K5 propagators (every mode, with and without blend)
  std::vector<float> pxf((size_t)NP * N), ppf((size_t)NT * N);
  for (int mode = PROP_PRIOR; mode <= PROP_IDENTITY; ++mode)
    for (int blend = 0; blend < 2; ++blend) {
      PropArgs pp = pr;
      pp.mode = mode; pp.blend = blend; pp.quirk_blend = blend;
      for (int j = 0; j < NP; ++j) pp.blend_mean[j] = 0.4f;
      for (int j = 0; j < NP; ++j) pp.blend_cinv[tri(NP, j, j)] = 2.f;
      pp.x_f = pxf.data(); pp.p_f = ppf.data(); pp.status = status.data();
      check(host_propagate(NP, pp) == 0, "host_propagate rc");
      check(all_finite(pxf), "propagate mean finite");
    }

  // K1g gain form (covariance input = inverse of the precision above)
  std::vector<float> cov((size_t)NT * N), po((size_t)NT * N);
  check(host_invert(NP, Pf.data(), cov.data(), N, N, status.data()) == 0, "host_invert rc");
  GainArgs g;
  std::memset(&g, 0, sizeof(g));
  g.N = N; g.ld = N; g.n_bands = 2; g.joseph = 1; g.bands = bands;
  g.x_prev = x.data(); g.x_f = xf.data(); g.p_f = cov.data(); g.x_out = xo.data(); g.p_out = po.data();
  g.status = status.data(); g.partials = partials.data();
  check(host_gain(NP, g, grid) == 0, "host_gain rc");
  check(all_finite(xo) && all_finite(po), "gain outputs finite");

  // K2 split operator (7 params, 4 inputs) and K6 Hessian correction
  std::vector<float> h0((size_t)2 * N), hh((size_t)2 * NP * N);
  check(host_gp_operator(NP, bands, 2, x.data(), N, N, h0.data(), hh.data(), N) == 0, "host_gp_operator rc");
  check(all_finite(h0) && all_finite(hh), "gp operator finite");
  std::vector<float> ah = ao;
  check(host_hessian(NP, bands, 2, x.data(), ah.data(), N, N) == 0, "host_hessian rc");

  // K9 Jacobi sweep on a 40 x 25 raster (4-neighbour table, no halo)
  const int H = 40, W = 25;
  std::vector<int32_t> nbr((size_t)4 * N);
  for (int64_t p = 0; p < N; ++p) {
    const int r = (int)(p / W), c = (int)(p % W);
    nbr[0 * N + p] = r > 0 ? (int32_t)(p - W) : -1;
    nbr[1 * N + p] = r < H - 1 ? (int32_t)(p + W) : -1;
    nbr[2 * N + p] = c > 0 ? (int32_t)(p - 1) : -1;
    nbr[3 * N + p] = c < W - 1 ? (int32_t)(p + 1) : -1;
  }
  JacobiArgs j;
  std::memset(&j, 0, sizeof(j));
  j.N = N; j.ld = N; j.ld_ext = N; j.gamma = 5.f; j.reg_mask = 1u << 6;
  j.a_in = ao.data(); j.b_in = bo.data(); j.x_ext = x.data(); j.nbr = nbr.data(); j.x_ref = x.data();
  j.x_out = xo.data(); j.a_out = ao2.data(); j.partials = partials.data();
  check(host_jacobi(NP, j, grid) == 0, "host_jacobi rc");
  check(all_finite(xo), "jacobi output finite");

  // K8 unpack into a raster with holes
  const int64_t plane = N + 17;
  std::vector<int64_t> idx((size_t)N);
  for (int64_t p = 0; p < N; ++p) idx[p] = p + (p > 500 ? 17 : 0);
  std::vector<float> mean((size_t)NP * plane), unc((size_t)NP * plane);
  check(host_unpack(NP, x.data(), Pf.data(), N, N, idx.data(), mean.data(), unc.data(), plane) == 0,
        "host_unpack rc");

  // K7 LUT nearest
  const int M = 33;
  std::vector<float> lut((size_t)M * NP);
  for (auto& v : lut) v = unif(0.f, 1.f);
  std::vector<int32_t> near((size_t)N);
  check(host_lut_nearest(lut.data(), M, NP, x.data(), N, N, near.data()) == 0, "host_lut_nearest rc");
  for (int32_t v : near) check(v >= 0 && v < M, "lut index in range");

  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("sanitize_host ok\n");
  return 0;
}
