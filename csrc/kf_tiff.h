// kf_tiff.h — native GeoTIFF window decode (kf_tiff.cpp), shared with the
// ingest ring (kf_stream.cpp) so granule bands decode straight into pinned slots.
#pragma once
#include <cstdint>
#include <string>

namespace kf {
namespace tiff {
// rows [r0, r1) x columns [c0, c1) of sample `band` into dst (dense, row-major);
// elem_bytes > 0: throw unless the file's samples are exactly that size
void read_window(const std::string& path, int band, void* dst, uint64_t r0, uint64_t r1, uint64_t c0, uint64_t c1,
                 int nthreads, int elem_bytes = 0);
}  // namespace tiff
}  // namespace kf
