// kf_analysis7.hip — analysis-kernel instantiations for 7-parameter states
// (JRC-TIP), a translation unit of its own so the GP-loop
// variants compile in parallel with the rest (_build.py).
#include "kf_device.h"

namespace kf {

hipError_t dev_analysis_np7(const AnalysisArgs& a, int grid, hipStream_t s) {
  l_analysis<7>(a, grid, s);
  return hipGetLastError();
}

}  // namespace kf
