// kf_analysis10.hip — analysis-kernel instantiations for 10-parameter states
// (PROSAIL / SAIL), a translation unit of its own so the GP-loop
// variants compile in parallel with the rest (_build.py).
#include "kf_device.h"

namespace kf {

hipError_t dev_analysis_np10(const AnalysisArgs& a, int grid, hipStream_t s) {
  l_analysis<10>(a, grid, s);
  return hipGetLastError();
}

}  // namespace kf
