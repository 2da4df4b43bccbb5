// kf_bindings.cpp — pybind11 module `_kafka_hip`.
// Pointers cross the boundary as integers (torch data_ptr()); streams as
// torch.cuda.current_stream().cuda_stream.  `device=True` launches the gfx950
// kernel on the given stream, `device=False` runs the identical per-pixel
// code on the host (kf_host.cpp).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <stdexcept>
#include <string>
#include <vector>
#include "kf_launch.h"
#include "kf_deflate.h"
#include "kf_stream.h"

namespace py = pybind11;
using namespace kf;
namespace kf {
void bind_tiff(py::module_& m);   // kf_tiff.cpp
}

template <typename T>
static T* P(uintptr_t v) { return reinterpret_cast<T*>(v); }

static void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
static void check_host(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string(what) + ": unsupported n_params on host runner");
}

template <typename A, size_t N>
static void set_arr(A (&dst)[N], const std::vector<A>& v, const char* name) {
  if (v.size() > N) throw std::runtime_error(std::string(name) + " too long");
  for (size_t i = 0; i < N; ++i) dst[i] = i < v.size() ? v[i] : A(0);
}
template <typename A, size_t N>
static std::vector<A> get_arr(const A (&src)[N]) { return std::vector<A>(src, src + N); }

#define PTR_FIELD(cls, name, T)                                                                     \
  def_property(#name, [](const cls& s) { return (uintptr_t)s.name; },                              \
               [](cls& s, uintptr_t v) { s.name = reinterpret_cast<T>(v); })
#define GEO_FIELDS(cls, g)                                                                          \
  def_property("geo_w", [](const cls& s) { return s.g.w; }, [](cls& s, int64_t v) { s.g.w = v; })        \
      .def_property("geo_n_up", [](const cls& s) { return s.g.n_up; }, [](cls& s, int64_t v) { s.g.n_up = v; }) \
      .def_property("geo_h", [](const cls& s) { return s.g.h; }, [](cls& s, int32_t v) { s.g.h = v; })   \
      .def_property("geo_halo", [](const cls& s) { return s.g.halo; }, [](cls& s, int32_t v) { s.g.halo = v; })
#define ARR_FIELD(cls, name, T)                                                                     \
  def_property(#name, [](const cls& s) { return get_arr(s.name); },                                \
               [](cls& s, const std::vector<T>& v) { set_arr(s.name, v, #name); })

#ifndef KF_MODULE_NAME
#define KF_MODULE_NAME _kafka_hip
#endif
PYBIND11_MODULE(KF_MODULE_NAME, m) {
  m.doc() = "KaFKA MI355X kernels (gfx950) + host runner of the same per-pixel code";
  m.attr("MAX_D") = MAX_D;
  m.attr("MAX_BLOCKS") = KF_MAX_BLOCKS;
  m.attr("SIZEOF_BANDDESC") = (int)sizeof(BandDesc);

  py::class_<BandDesc>(m, "BandDesc")
      .def(py::init([]() { BandDesc b; memset(&b, 0, sizeof(b)); return b; }))
      .def_readwrite("op", &BandDesc::op)
      .def_readwrite("obs", &BandDesc::obs)
      .def_readwrite("d", &BandDesc::d)
      .def_readwrite("T", &BandDesc::T)
      .def_readwrite("Tp", &BandDesc::Tp)
      .ARR_FIELD(BandDesc, map, int32_t)
      .def_readwrite("map_identity", &BandDesc::map_identity)
      .def_readwrite("map_kind", &BandDesc::map_kind)
      .def_readwrite("dom_check", &BandDesc::dom_check)
      .ARR_FIELD(BandDesc, dom_lo, float)
      .ARR_FIELD(BandDesc, dom_hi, float)
      .def_readwrite("scale", &BandDesc::scale)
      .def_readwrite("rel_unc", &BandDesc::rel_unc)
      .def_readwrite("unc_floor", &BandDesc::unc_floor)
      .def_readwrite("offset", &BandDesc::offset)
      .ARR_FIELD(BandDesc, coef, float)
      .ARR_FIELD(BandDesc, center, float)
      .PTR_FIELD(BandDesc, gp, const float*)
      .PTR_FIELD(BandDesc, y, const float*)
      .PTR_FIELD(BandDesc, w, const float*)
      .PTR_FIELD(BandDesc, mask, const uint8_t*)
      .PTR_FIELD(BandDesc, dn, const uint16_t*)
      .PTR_FIELD(BandDesc, aux, const float*)
      .PTR_FIELD(BandDesc, pre_h0, const float*)
      .PTR_FIELD(BandDesc, pre_h, const float*)
      .PTR_FIELD(BandDesc, h0_out, float*)
      .def_readwrite("pre_ld", &BandDesc::pre_ld)
      .def_readwrite("gpm_nchunk", &BandDesc::gpm_nchunk)
      .def_readwrite("gpm_scale", &BandDesc::gpm_scale)
      .PTR_FIELD(BandDesc, gpm, const void*);

  m.def("pack_band_descs", [](const std::vector<BandDesc>& v) {
    return py::bytes(reinterpret_cast<const char*>(v.data()), v.size() * sizeof(BandDesc));
  });

  m.def("pack_prop_args", [](const PropArgs& a) {
    return py::bytes(reinterpret_cast<const char*>(&a), sizeof(PropArgs));
  });

  py::class_<AnalysisArgs>(m, "AnalysisArgs")
      .def(py::init([]() { AnalysisArgs a; memset(&a, 0, sizeof(a)); return a; }))
      .def_readwrite("N", &AnalysisArgs::N)
      .def_readwrite("ld", &AnalysisArgs::ld)
      .def_readwrite("n_bands", &AnalysisArgs::n_bands)
      .def_readwrite("solve", &AnalysisArgs::solve)
      .def_readwrite("fast_d", &AnalysisArgs::fast_d)
      .def_readwrite("fast_obs", &AnalysisArgs::fast_obs)
      .def_readwrite("variant", &AnalysisArgs::variant)
      .def_readwrite("gpm_frags", &AnalysisArgs::gpm_frags)
      .def_readwrite("gpm_global", &AnalysisArgs::gpm_global)
      .PTR_FIELD(AnalysisArgs, bands, const BandDesc*)
      .PTR_FIELD(AnalysisArgs, x_prev, const float*)
      .PTR_FIELD(AnalysisArgs, x_f, const float*)
      .PTR_FIELD(AnalysisArgs, pf_inv, const float*)
      .PTR_FIELD(AnalysisArgs, x_out, float*)
      .PTR_FIELD(AnalysisArgs, a_out, float*)
      .PTR_FIELD(AnalysisArgs, b_out, float*)
      .PTR_FIELD(AnalysisArgs, a_in, const float*)
      .PTR_FIELD(AnalysisArgs, b_in, const float*)
      .PTR_FIELD(AnalysisArgs, status, uint8_t*)
      .PTR_FIELD(AnalysisArgs, partials, double*)
      .PTR_FIELD(AnalysisArgs, partials_first, double*)
      .PTR_FIELD(AnalysisArgs, order, const int32_t*)
      .def_readwrite("n_visit", &AnalysisArgs::n_visit)
      .PTR_FIELD(AnalysisArgs, n_visit_dev, const int32_t*)
      .PTR_FIELD(AnalysisArgs, dn_out, float*)
      .def_readwrite("a_rows", &AnalysisArgs::a_rows)
      .def_readwrite("dom_check", &AnalysisArgs::dom_check)
      .ARR_FIELD(AnalysisArgs, dom_lo, float)
      .ARR_FIELD(AnalysisArgs, dom_hi, float)
      .def_readwrite("gn_fused", &AnalysisArgs::gn_fused)
      .def_readwrite("band_layout", &AnalysisArgs::band_layout)
      .PTR_FIELD(AnalysisArgs, prop, const PropArgs*)
      .PTR_FIELD(AnalysisArgs, out_mean, float*)
      .PTR_FIELD(AnalysisArgs, out_unc, float*)
      .PTR_FIELD(AnalysisArgs, out_idx, const int64_t*)
      .def_readwrite("out_plane", &AnalysisArgs::out_plane)
      .def_readwrite("reg_gamma", &AnalysisArgs::reg_gamma)
      .def_readwrite("reg_mask", &AnalysisArgs::reg_mask)
      .PTR_FIELD(AnalysisArgs, reg_nbr, const int32_t*)
      .PTR_FIELD(AnalysisArgs, reg_v, float*)
      .PTR_FIELD(AnalysisArgs, x0_out, float*)
      .PTR_FIELD(AnalysisArgs, line_tab, const float*)
      .def_readwrite("line_t0", &AnalysisArgs::line_t0)
      .def_readwrite("line_inv_h", &AnalysisArgs::line_inv_h)
      .def_readwrite("line_n", &AnalysisArgs::line_n)
      .def_readwrite("line_j", &AnalysisArgs::line_j)
      .GEO_FIELDS(AnalysisArgs, reg_geo);

  py::class_<GainArgs>(m, "GainArgs")
      .def(py::init([]() { GainArgs a; memset(&a, 0, sizeof(a)); return a; }))
      .def_readwrite("N", &GainArgs::N)
      .def_readwrite("ld", &GainArgs::ld)
      .def_readwrite("n_bands", &GainArgs::n_bands)
      .def_readwrite("joseph", &GainArgs::joseph)
      .def_readwrite("fast_d", &GainArgs::fast_d)
      .def_readwrite("fast_obs", &GainArgs::fast_obs)
      .def_readwrite("out_plane", &GainArgs::out_plane)
      .def_readwrite("gpm_frags", &GainArgs::gpm_frags)
      .def_readwrite("gn_fused", &GainArgs::gn_fused)
      .def_readwrite("n_visit", &GainArgs::n_visit)
      .PTR_FIELD(GainArgs, n_visit_dev, const int32_t*)
      .def_readwrite("pdiag_rows", &GainArgs::pdiag_rows)
      .PTR_FIELD(GainArgs, partials_first, double*)
      .PTR_FIELD(GainArgs, line_tab, const float*)
      .def_readwrite("line_t0", &GainArgs::line_t0)
      .def_readwrite("line_inv_h", &GainArgs::line_inv_h)
      .def_readwrite("line_n", &GainArgs::line_n)
      .def_readwrite("line_j", &GainArgs::line_j)
      .PTR_FIELD(GainArgs, order, const int32_t*)
      .PTR_FIELD(GainArgs, dn_out, float*)
      .PTR_FIELD(GainArgs, prop, const PropArgs*)
      .PTR_FIELD(GainArgs, out_mean, float*)
      .PTR_FIELD(GainArgs, out_unc, float*)
      .PTR_FIELD(GainArgs, out_idx, const int64_t*)
      .PTR_FIELD(GainArgs, bands, const BandDesc*)
      .PTR_FIELD(GainArgs, x_prev, const float*)
      .PTR_FIELD(GainArgs, x_f, const float*)
      .PTR_FIELD(GainArgs, p_f, const float*)
      .PTR_FIELD(GainArgs, x_out, float*)
      .PTR_FIELD(GainArgs, p_out, float*)
      .PTR_FIELD(GainArgs, status, uint8_t*)
      .PTR_FIELD(GainArgs, partials, double*);

  py::class_<JacobiArgs>(m, "JacobiArgs")
      .def(py::init([]() { JacobiArgs a; memset(&a, 0, sizeof(a)); return a; }))
      .def_readwrite("N", &JacobiArgs::N)
      .def_readwrite("ld", &JacobiArgs::ld)
      .def_readwrite("ld_ext", &JacobiArgs::ld_ext)
      .def_readwrite("gamma", &JacobiArgs::gamma)
      .def_readwrite("reg_mask", &JacobiArgs::reg_mask)
      .PTR_FIELD(JacobiArgs, a_in, const float*)
      .PTR_FIELD(JacobiArgs, b_in, const float*)
      .PTR_FIELD(JacobiArgs, x_ext, const float*)
      .PTR_FIELD(JacobiArgs, nbr, const int32_t*)
      .PTR_FIELD(JacobiArgs, x_ref, const float*)
      .PTR_FIELD(JacobiArgs, x_out, float*)
      .PTR_FIELD(JacobiArgs, a_out, float*)
      .PTR_FIELD(JacobiArgs, partials, double*)
      .def_readwrite("mode", &JacobiArgs::mode)
      .def_readwrite("p0", &JacobiArgs::p0)
      .def_readwrite("pn", &JacobiArgs::pn)
      .def_readwrite("k", &JacobiArgs::k)
      .PTR_FIELD(JacobiArgs, u, const float*)
      .PTR_FIELD(JacobiArgs, v, float*)
      .PTR_FIELD(JacobiArgs, z_out, float*)
      .PTR_FIELD(JacobiArgs, z_prev, const float*)
      .def_readwrite("omega", &JacobiArgs::omega)
      .PTR_FIELD(JacobiArgs, out_mean, float*)
      .PTR_FIELD(JacobiArgs, out_unc, float*)
      .PTR_FIELD(JacobiArgs, out_idx, const int64_t*)
      .def_readwrite("out_plane", &JacobiArgs::out_plane)
      .GEO_FIELDS(JacobiArgs, geo);

  py::class_<PropArgs>(m, "PropArgs")
      .def(py::init([]() { PropArgs a; memset(&a, 0, sizeof(a)); return a; }))
      .def_readwrite("N", &PropArgs::N)
      .def_readwrite("ld", &PropArgs::ld)
      .def_readwrite("mode", &PropArgs::mode)
      .def_readwrite("blend", &PropArgs::blend)
      .def_readwrite("quirk_blend", &PropArgs::quirk_blend)
      .def_readwrite("prop_mask", &PropArgs::prop_mask)
      .PTR_FIELD(PropArgs, x_a, const float*)
      .PTR_FIELD(PropArgs, p_a, const float*)
      .PTR_FIELD(PropArgs, x_f, float*)
      .PTR_FIELD(PropArgs, p_f, float*)
      .ARR_FIELD(PropArgs, m, float)
      .ARR_FIELD(PropArgs, q, float)
      .PTR_FIELD(PropArgs, q_pix, const float*)
      .ARR_FIELD(PropArgs, reset_mean, float)
      .ARR_FIELD(PropArgs, reset_cinv, float)
      .ARR_FIELD(PropArgs, blend_mean, float)
      .ARR_FIELD(PropArgs, blend_cinv, float)
      .PTR_FIELD(PropArgs, blend_mean_pix, const float*)
      .PTR_FIELD(PropArgs, blend_cinv_pix, const float*)
      .PTR_FIELD(PropArgs, status, uint8_t*)
      .def_readwrite("cov_fast", &PropArgs::cov_fast)
      .def_readwrite("pa_pdiag", &PropArgs::pa_pdiag)
      .ARR_FIELD(PropArgs, reset_cov, float);

  m.def("supported_np", [](int np) { return host_supported(np); });
  m.def("grid", [](int64_t N) { return dev_grid(N); });
  m.def("set_max_blocks", [](int n) { set_max_blocks(n); });
  m.def("get_max_blocks", []() { return get_max_blocks(); });
#ifdef KF_PHASE_CLOCKS
  // shader cycles per phase of the 7- or 10-parameter matrix-core analysis kernels,
  // summed over waves (kf_core.h KF_PH_*); reset=True zeroes them after reading
  m.def("phase_clocks", [](int np, bool reset) {
    unsigned long long v[KF_PH_NSLOT];
    check_hip(np == 10 ? phase_clocks_np10(v, reset) : phase_clocks_np7(v, reset), "phase_clocks");
    return std::vector<unsigned long long>(v, v + KF_PH_NSLOT);
  }, py::arg("n_params") = 7, py::arg("reset") = false);
#endif
  m.def("set_gp_unroll", [](int n) { set_gp_unroll(n); });

  // -> norm partial entries written (device: workgroups or 64-slot tiles; host: workgroups)
  m.def("analysis", [](int np, const AnalysisArgs& a, int grid, bool device, uintptr_t stream) {
    int n_part = grid;
    if (device) check_hip(dev_analysis(np, a, grid, (hipStream_t)stream, &n_part), "analysis");
    else check_host(host_analysis(np, a, grid), "analysis");
    return n_part;
  });
  m.def("gain", [](int np, const GainArgs& a, int grid, bool device, uintptr_t stream) {
    if (device) check_hip(dev_gain(np, a, grid, (hipStream_t)stream), "gain");
    else check_host(host_gain(np, a, grid), "gain");
  });
  m.def("jacobi", [](int np, const JacobiArgs& a, int grid, bool device, uintptr_t stream) {
    if (device) check_hip(dev_jacobi(np, a, grid, (hipStream_t)stream), "jacobi");
    else check_host(host_jacobi(np, a, grid), "jacobi");
  });
  m.def("propagate", [](int np, const PropArgs& a, bool device, uintptr_t stream) {
    if (device) check_hip(dev_propagate(np, a, (hipStream_t)stream), "propagate");
    else check_host(host_propagate(np, a), "propagate");
  });
  m.def("invert", [](int np, uintptr_t src, uintptr_t dst, int64_t N, int64_t ld, uintptr_t st, bool device,
                     uintptr_t stream) {
    if (device) check_hip(dev_invert(np, P<const float>(src), P<float>(dst), N, ld, P<uint8_t>(st),
                                     (hipStream_t)stream), "invert");
    else check_host(host_invert(np, P<const float>(src), P<float>(dst), N, ld, P<uint8_t>(st)), "invert");
  });
  m.def("operator_eval", [](int np, uintptr_t bands, int band, uintptr_t x, int64_t N, int64_t ld, uintptr_t h0,
                            uintptr_t h, int64_t h_ld, uintptr_t ok, bool device, uintptr_t stream) {
    if (device) check_hip(dev_operator(np, P<const BandDesc>(bands), band, P<const float>(x), N, ld, P<float>(h0),
                                       P<float>(h), h_ld, P<uint8_t>(ok), (hipStream_t)stream), "operator_eval");
    else check_host(host_operator(np, P<const BandDesc>(bands), band, P<const float>(x), N, ld, P<float>(h0),
                                  P<float>(h), h_ld, P<uint8_t>(ok)), "operator_eval");
  });
  m.def("gp_operator_supported", [](int np, int d) { return gp_operator_supported(np, d); });
  m.def("gp_operator", [](int np, int d, uintptr_t bands, int nb, uintptr_t x, int64_t N, int64_t ld, uintptr_t h0,
                          uintptr_t h, int64_t ldh, bool device, uintptr_t stream) {
    if (device) check_hip(dev_gp_operator(np, d, P<const BandDesc>(bands), nb, P<const float>(x), N, ld, P<float>(h0),
                                          P<float>(h), ldh, (hipStream_t)stream), "gp_operator");
    else check_host(host_gp_operator(np, P<const BandDesc>(bands), nb, P<const float>(x), N, ld, P<float>(h0),
                                     P<float>(h), ldh), "gp_operator");
  });
  m.def("hessian", [](int np, uintptr_t bands, int nb, uintptr_t x, uintptr_t a, int64_t N, int64_t ld,
                      bool device, uintptr_t stream) {
    if (device) check_hip(dev_hessian(np, P<const BandDesc>(bands), nb, P<const float>(x), P<float>(a), N, ld,
                                      (hipStream_t)stream), "hessian");
    else check_host(host_hessian(np, P<const BandDesc>(bands), nb, P<const float>(x), P<float>(a), N, ld),
                    "hessian");
  });
  m.def("unpack", [](int np, uintptr_t x, uintptr_t a, int64_t N, int64_t ld, uintptr_t idx, uintptr_t mean,
                     uintptr_t unc, int64_t plane, bool device, uintptr_t stream) {
    if (device) check_hip(dev_unpack(np, P<const float>(x), P<const float>(a), N, ld, P<const int64_t>(idx),
                                     P<float>(mean), P<float>(unc), plane, (hipStream_t)stream), "unpack");
    else check_host(host_unpack(np, P<const float>(x), P<const float>(a), N, ld, P<const int64_t>(idx),
                                P<float>(mean), P<float>(unc), plane), "unpack");
  });
  // GeoTIFF tile encoder (predictor 3 + fixed-Huffman zlib per 256^2 tile)
  m.attr("DFL_TILE") = DFL_TILE;
  m.attr("DFL_BOUND") = DFL_BOUND;
  m.attr("DFL_ROW_SCRATCH") = (int64_t)DFL_TILE * DFL_ROW_WORDS * 4;   // scratch bytes per tile (device)
  m.def("deflate_tiles", [](uintptr_t src, int64_t plane_ld, int H, int W, int nplanes, uintptr_t out,
                            uintptr_t sizes, bool device, uintptr_t stream, uintptr_t scratch) {
    DflArgs a{};
    a.src = P<const float>(src);
    a.plane_ld = plane_ld;
    a.H = H;
    a.W = W;
    a.nplanes = nplanes;
    a.tiles_x = (W + DFL_TILE - 1) / DFL_TILE;
    a.tiles_y = (H + DFL_TILE - 1) / DFL_TILE;
    a.out = P<uint8_t>(out);
    a.sizes = P<uint32_t>(sizes);
    a.scratch = P<uint8_t>(scratch);
    if (device && !scratch) throw std::runtime_error("deflate_tiles: the device encoder needs its row scratch");
    if ((int64_t)H * W > plane_ld) throw std::runtime_error("deflate_tiles: plane_ld < H * W");
    if (device) check_hip(dev_deflate_tiles(a, (hipStream_t)stream), "deflate_tiles");
    else {
      py::gil_scoped_release nogil;
      check_host(host_deflate_tiles(a), "deflate_tiles");
    }
  });
  m.def("deflate_pack", [](uintptr_t scratch, uintptr_t sizes, uintptr_t offs, uintptr_t packed, int ntiles,
                           uintptr_t stream) {
    check_hip(dev_deflate_pack(P<const uint8_t>(scratch), P<const uint32_t>(sizes), P<const int64_t>(offs),
                               P<uint8_t>(packed), ntiles, (hipStream_t)stream), "deflate_pack");
  });
  m.def("reduce_partials", [](uintptr_t partials, int n, uintptr_t out, uintptr_t stream) {
    check_hip(dev_reduce(P<const double>(partials), n, P<double>(out), (hipStream_t)stream), "reduce_partials");
  });
  m.def("gather", [](int elem_bytes, uintptr_t src, uintptr_t idx, uintptr_t dst, int64_t n, int rows,
                     int64_t src_ld, int64_t dst_ld, uintptr_t stream) {
    check_hip(dev_gather(elem_bytes, P<const void>(src), P<const int64_t>(idx), P<void>(dst), n, rows, src_ld,
                         dst_ld, (hipStream_t)stream), "gather");
  });
  // stable partition by observation class (AnalysisArgs.order); grp: band
  // group per band (null: one group), G groups (1..3); counts: ((chunks + 1)
  // * 2^G) int32 scratch (device, global partition only); local: each
  // KF_ORD_CHUNK-pixel chunk partitioned in place
  m.def("obs_order_chunks", &obs_order_chunks);
  m.def("obs_order", [](uintptr_t bands, uintptr_t grp, int nb, int G, int64_t N, uintptr_t counts, uintptr_t order,
                        bool local, bool device, uintptr_t stream) {
    if (N > (int64_t)INT32_MAX) throw std::runtime_error("obs_order: N exceeds int32");
    if (G < 1 || G > 3) throw std::runtime_error("obs_order: 1 to 3 band groups");
    if (device) check_hip(dev_obs_order(P<const BandDesc>(bands), P<const int32_t>(grp), nb, G, N, P<int32_t>(counts),
                                        P<int32_t>(order), local, (hipStream_t)stream), "obs_order");
    else if (host_obs_order(P<const BandDesc>(bands), P<const int32_t>(grp), nb, G, N, P<int32_t>(order), local) != 0)
      throw std::runtime_error("obs_order failed");
  });
  // per-chunk Gauss-Newton convergence (kf_core.h ChunkPartialArgs ...)
  m.def("chunk_partials", [](uintptr_t dn, uintptr_t seg_start, uintptr_t seg_len, uintptr_t lc_ptr, uintptr_t lc_gid,
                             int n_local, uintptr_t active, uintptr_t part, uintptr_t gpart, int groups,
                             uintptr_t qinv, int64_t clamp, bool device, uintptr_t stream) {
    ChunkPartialArgs a{};
    a.dn = P<const float>(dn);
    a.seg_start = P<const int32_t>(seg_start);
    a.seg_len = P<const int32_t>(seg_len);
    a.lc_ptr = P<const int32_t>(lc_ptr);
    a.lc_gid = P<const int32_t>(lc_gid);
    a.n_local = n_local;
    a.active = P<const uint8_t>(active);
    a.part = P<int64_t>(part);
    a.gpart = P<int64_t>(gpart);
    a.groups = groups;
    a.qinv = P<const double>(qinv);
    a.clamp = clamp;
    if (device) check_hip(dev_chunk_partials(a, (hipStream_t)stream), "chunk_partials");
    else host_chunk_partials(a);
  });
  m.def("chunk_decide", [](uintptr_t part_all, int world, int nc, uintptr_t len_x, uintptr_t local_count, double tol,
                           int n_iter, int min_iter, int max_iter, uintptr_t active, uintptr_t newly, uintptr_t iters,
                           uintptr_t info, uintptr_t px_out, double unit, bool device, uintptr_t stream) {
    ChunkDecideArgs a{};
    a.part_all = P<const int64_t>(part_all);
    a.unit = unit;
    a.world = world;
    a.nc = nc;
    a.len_x = P<const double>(len_x);
    a.local_count = P<const int32_t>(local_count);
    a.tol = tol;
    a.n_iter = n_iter;
    a.min_iter = min_iter;
    a.max_iter = max_iter;
    a.active = P<uint8_t>(active);
    a.newly = P<uint8_t>(newly);
    a.iters = P<int32_t>(iters);
    a.info = P<double>(info);
    a.px_out = P<int32_t>(px_out);
    if (device) check_hip(dev_chunk_decide(a, (hipStream_t)stream), "chunk_decide");
    else host_chunk_decide(a);
  });
  m.def("chunk_compact_blocks", &chunk_compact_blocks);
  // -> kept slots on the host runner, -1 on the device (the count is known from chunk_decide's info)
  m.def("chunk_compact", [](uintptr_t order_in, int64_t n_in, uintptr_t chunk_of, uintptr_t active, uintptr_t newly,
                            uintptr_t counts, uintptr_t order_out, uintptr_t x_src, uintptr_t x_dst, int np, int64_t ld,
                            uintptr_t n_in_dev, bool device, uintptr_t stream) -> int64_t {
    if (n_in > (int64_t)INT32_MAX) throw std::runtime_error("chunk_compact: more than 2^31 slots");
    ChunkCompactArgs a{};
    a.order_in = P<const int32_t>(order_in);
    a.n_in = n_in;
    a.n_in_dev = P<const int32_t>(n_in_dev);
    a.chunk_of = P<const int32_t>(chunk_of);
    a.active = P<const uint8_t>(active);
    a.newly = P<const uint8_t>(newly);
    a.counts = P<int32_t>(counts);
    a.order_out = P<int32_t>(order_out);
    a.x_src = P<const float>(x_src);
    a.x_dst = P<float>(x_dst);
    a.np = np;
    a.ld = ld;
    if (device) {
      check_hip(dev_chunk_compact(a, (hipStream_t)stream), "chunk_compact");
      return -1;
    }
    return host_chunk_compact(a);
  });
  m.def("lut_nearest", [](uintptr_t lut, int M, int D, uintptr_t x, int64_t N, int64_t ld, uintptr_t out,
                          bool device, uintptr_t stream) {
    if (device) check_hip(dev_lut_nearest(P<const float>(lut), M, D, P<const float>(x), N, ld, P<int32_t>(out),
                                          (hipStream_t)stream), "lut_nearest");
    else host_lut_nearest(P<const float>(lut), M, D, P<const float>(x), N, ld, P<int32_t>(out));
  });

  // omega non-empty: host schedule (nsweep = len(omega)); else the device
  // schedule (sched / omega_tab, at most nsweep sweeps from s_base)
  m.def("reg_tiled", [](int64_t ld, int w, int h, int j0, uint32_t prev_mask, float gamma,
                        const std::vector<float>& omega, uintptr_t u, uintptr_t v, uintptr_t z, uintptr_t zp,
                        uintptr_t z_out, uintptr_t zp_out, bool device, uintptr_t stream, int nsweep, int hu, int hd,
                        uintptr_t halo_up, uintptr_t halo_dn, int64_t halo_plane, int ty0, int ty1, uintptr_t sched,
                        uintptr_t omega_tab, int s_base) {
    RegTileArgs a{};
    a.ld = ld;
    a.w = w;
    a.h = h;
    a.j0 = j0;
    if (!omega.empty()) {
      a.nsweep = (int32_t)omega.size();
      if (sched) throw std::runtime_error("reg_tiled: host omegas and a device schedule");
      set_arr(a.omega, omega, "omega");
    } else {
      a.nsweep = nsweep;
      if (!sched || !omega_tab) throw std::runtime_error("reg_tiled: no omegas and no device schedule");
    }
    if (a.nsweep < 1 || a.nsweep > REG_TILE_MAX_SWEEPS) throw std::runtime_error("reg_tiled: 1..8 sweeps");
    a.prev_mask = prev_mask;
    a.gamma = gamma;
    a.u = P<const float>(u);
    a.v = P<const float>(v);
    a.z = P<const float>(z);
    a.zp = P<const float>(zp);
    a.z_out = P<float>(z_out);
    a.zp_out = P<float>(zp_out);
    a.hu = hu;
    a.hd = hd;
    a.halo_up = P<const float>(halo_up);
    a.halo_dn = P<const float>(halo_dn);
    a.halo_plane = halo_plane;
    a.ty0 = ty0;
    a.ty1 = ty1;
    a.sched = P<const int32_t>(sched);
    a.omega_tab = P<const float>(omega_tab);
    a.s_base = s_base;
    if (device) check_hip(dev_reg_tiled(a, (hipStream_t)stream), "reg_tiled");
    else if (host_reg_tiled(a) != 0) throw std::runtime_error("reg_tiled: bad arguments");
  }, py::arg("ld"), py::arg("w"), py::arg("h"), py::arg("j0"), py::arg("prev_mask"), py::arg("gamma"),
     py::arg("omega"), py::arg("u"), py::arg("v"), py::arg("z"), py::arg("zp"), py::arg("z_out"),
     py::arg("zp_out"), py::arg("device"), py::arg("stream"), py::arg("nsweep") = 0, py::arg("hu") = 0,
     py::arg("hd") = 0, py::arg("halo_up") = 0, py::arg("halo_dn") = 0, py::arg("halo_plane") = 0,
     py::arg("ty0") = 0, py::arg("ty1") = 0, py::arg("sched") = 0, py::arg("omega_tab") = 0,
     py::arg("s_base") = 0);
  m.def("reg_rho_blocks", [](int64_t N) { return reg_rho_blocks(N); });
  // rho = gamma * max_p v_RR(p) deg(p) of one field on a dense strip -> rho[0] (f64)
  m.def("reg_rho", [](uintptr_t vrow, int64_t w, int h, int halo, int64_t N, uintptr_t pmax, int npart, float gamma,
                      uintptr_t rho, bool device, uintptr_t stream) {
    StripGeo g{};
    g.w = w;
    g.h = h;
    g.halo = halo;
    g.n_up = (halo & 1) ? w : 0;
    if (w <= 0 || (int64_t)h * w != N) throw std::runtime_error("reg_rho: dense geometry w * h != N");
    RegScheduleArgs a{};
    a.pmax = P<const float>(pmax);
    a.npart = npart;
    a.gamma = gamma;
    a.rho = P<double>(rho);
    if (device) check_hip(dev_reg_rho(P<const float>(vrow), g, N, a, (hipStream_t)stream), "reg_rho");
    else if (host_reg_rho(P<const float>(vrow), g, N, a) != 0) throw std::runtime_error("reg_rho: bad arguments");
  });
  m.def("reg_schedule", [](uintptr_t rho, double tol, int max_sweeps, uintptr_t sched, uintptr_t omega_tab,
                           uintptr_t info, bool device, uintptr_t stream) {
    RegScheduleArgs a{};
    a.rho = P<double>(rho);
    a.tol = tol;
    a.max_sweeps = max_sweeps;
    a.sched = P<int32_t>(sched);
    a.omega_tab = P<float>(omega_tab);
    a.info = P<double>(info);
    if (device) check_hip(dev_reg_schedule(a, (hipStream_t)stream), "reg_schedule");
    else if (host_reg_schedule(a) != 0) throw std::runtime_error("reg_schedule: bad arguments");
  });

  bind_stream(m);
  bind_tiff(m);
}
