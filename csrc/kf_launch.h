// kf_launch.h — launcher entry points (device: kf_kernels.hip + kf_analysis{7,10}.hip,
// host: kf_host.cpp).
#pragma once
#include <stdint.h>
#include "kf_core.h"
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#else
#include <hip/hip_runtime_api.h>
#endif

// Grid cap for the grid-stride kernels (A/B, scripts/gpu_grid.sh: 16384 is 3 %
// faster than 4096 at 15M and 120M px; round 4, scripts/gpu_r4_v22.sh at 120M
// px: 768 persistent blocks 45.6 ms, 16384 42.2, 32768-131072 41.9, one pixel
// per thread 42.8 -- the cloud skip makes blocks uneven, so more blocks finish
// closer together, up to the point where the per-block LDS table staging and
// dispatch cost more).
#define KF_MAX_BLOCKS 65536

namespace kf {

int dev_grid(int64_t N);
void set_max_blocks(int n);
void set_gp_unroll(int n);
int get_max_blocks();
// *n_part: norm partial entries written (workgroups of the grid-stride launch)
hipError_t dev_analysis(int np, const AnalysisArgs& a, int grid, hipStream_t s, int* n_part);
hipError_t dev_analysis_np7(const AnalysisArgs& a, int grid, hipStream_t s, int* n_part);
hipError_t dev_analysis_np10(const AnalysisArgs& a, int grid, hipStream_t s, int* n_part);
#ifdef KF_PHASE_CLOCKS
hipError_t phase_clocks_np7(unsigned long long* out, bool reset);
hipError_t phase_clocks_np10(unsigned long long* out, bool reset);
#endif
hipError_t dev_gain(int np, const GainArgs& a, int grid, hipStream_t s);
hipError_t dev_jacobi(int np, const JacobiArgs& a, int grid, hipStream_t s);
hipError_t dev_propagate(int np, const PropArgs& a, hipStream_t s);
hipError_t dev_invert(int np, const float* src, float* dst, int64_t N, int64_t ld, uint8_t* st, hipStream_t s);
hipError_t dev_operator(int np, const BandDesc* b, int band, const float* x, int64_t N, int64_t ld, float* h0,
                        float* h, int64_t h_ld, uint8_t* ok, hipStream_t s);
hipError_t dev_hessian(int np, const BandDesc* b, int nb, const float* x, float* a, int64_t N, int64_t ld,
                       hipStream_t s);
hipError_t dev_gp_operator(int np, int d, const BandDesc* b, int nb, const float* x, int64_t N, int64_t ld,
                           float* h0, float* h, int64_t ldh, hipStream_t s);
bool gp_operator_supported(int np, int d);
hipError_t dev_unpack(int np, const float* x, const float* a, int64_t N, int64_t ld, const int64_t* idx,
                      float* mean, float* unc, int64_t plane, hipStream_t s);
hipError_t dev_reduce(const double* partials, int n, double* out, hipStream_t s);
hipError_t dev_gather(int elem_bytes, const void* src, const int64_t* idx, void* dst, int64_t n, int rows,
                      int64_t src_ld, int64_t dst_ld, hipStream_t s);
hipError_t dev_lut_nearest(const float* lut, int M, int D, const float* x, int64_t N, int64_t ld, int32_t* out,
                           hipStream_t s);
hipError_t dev_reg_tiled(const RegTileArgs& a, hipStream_t s);
int reg_rho_blocks(int64_t N);
hipError_t dev_reg_rho(const float* vrow, const StripGeo& g, int64_t N, const RegScheduleArgs& a, hipStream_t s);
hipError_t dev_reg_schedule(const RegScheduleArgs& a, hipStream_t s);

// per-chunk Gauss-Newton convergence (kf_core.h ChunkPartialArgs ...)
constexpr int KF_CMP_CHUNK = 4096;   // visiting slots per compaction workgroup
int chunk_compact_blocks(int64_t n);
hipError_t dev_chunk_partials(const ChunkPartialArgs& a, hipStream_t s);
hipError_t dev_chunk_decide(const ChunkDecideArgs& a, hipStream_t s);
hipError_t dev_chunk_compact(const ChunkCompactArgs& a, hipStream_t s);
int host_chunk_partials(const ChunkPartialArgs& a);
int host_chunk_decide(const ChunkDecideArgs& a);
int64_t host_chunk_compact(const ChunkCompactArgs& a);

// Host runner: the same per-pixel code over OpenMP; the block partition
// mirrors the device grid-stride mapping so partials have the same meaning.
bool host_supported(int np);
int host_analysis(int np, const AnalysisArgs& a, int grid);
int host_gain(int np, const GainArgs& a, int grid);
int host_jacobi(int np, const JacobiArgs& a, int grid);
int host_propagate(int np, const PropArgs& a);
int host_invert(int np, const float* src, float* dst, int64_t N, int64_t ld, uint8_t* st);
int host_operator(int np, const BandDesc* b, int band, const float* x, int64_t N, int64_t ld, float* h0, float* h,
                  int64_t h_ld, uint8_t* ok);
int host_hessian(int np, const BandDesc* b, int nb, const float* x, float* a, int64_t N, int64_t ld);
int host_gp_operator(int np, const BandDesc* b, int nb, const float* x, int64_t N, int64_t ld, float* h0, float* h,
                     int64_t ldh);
int host_unpack(int np, const float* x, const float* a, int64_t N, int64_t ld, const int64_t* idx, float* mean,
                float* unc, int64_t plane);
// obs_order chunk: pixels per scatter workgroup; local = 1 partitions each
// chunk on its own (no count / scan passes, chunk-aligned, see kf_kernels.hip)
constexpr int KF_ORD_CHUNK = 4096;
int obs_order_chunks(int64_t N);
hipError_t dev_obs_order(const BandDesc* bands, const int32_t* grp, int nb, int G, int64_t N, int32_t* counts,
                         int32_t* order, bool local, hipStream_t s);
int host_obs_order(const BandDesc* bands, const int32_t* grp, int nb, int G, int64_t N, int32_t* order, bool local);
int host_lut_nearest(const float* lut, int M, int D, const float* x, int64_t N, int64_t ld, int32_t* out);
int host_reg_tiled(const RegTileArgs& a);
int host_reg_rho(const float* vrow, const StripGeo& g, int64_t N, const RegScheduleArgs& a);
int host_reg_schedule(const RegScheduleArgs& a);

// GeoTIFF tile encoder (kf_deflate.h / kf_deflate.hip): planes [nplanes][plane_ld]
// of H x W float32 rasters -> one zlib stream per 256 x 256 tile at
// out + tile * DFL_BOUND, its byte count in sizes[tile] (tiles plane-major,
// row-major within a plane)
struct DflArgs {
  const float* src;
  int64_t plane_ld;
  int32_t H, W, nplanes, tiles_x, tiles_y, pad_;
  uint8_t* out;
  uint32_t* sizes;
  uint8_t* scratch;   // device: DFL_TILE * DFL_ROW_WORDS words per tile (row bit strings before the shift)
};
hipError_t dev_deflate_tiles(const DflArgs& a, hipStream_t s);
hipError_t dev_deflate_pack(const uint8_t* scratch, const uint32_t* sizes, const int64_t* offs, uint8_t* packed,
                            int ntiles, hipStream_t s);
int host_deflate_tiles(const DflArgs& a);

}  // namespace kf
