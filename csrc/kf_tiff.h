// kf_tiff.h — native GeoTIFF window decode (kf_tiff.cpp), shared with the
// ingest ring (kf_stream.cpp) so granule bands decode straight into pinned slots.
#pragma once
#include <cstdint>
#include <string>

namespace kf {
namespace tiff {
// rows [r0, r1) x columns [c0, c1) of sample `band` into dst (dense, row-major)
void read_window(const std::string& path, int band, void* dst, uint64_t r0, uint64_t r1, uint64_t c0, uint64_t c1,
                 int nthreads);
}  // namespace tiff
}  // namespace kf
