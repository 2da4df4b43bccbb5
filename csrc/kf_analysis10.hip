// kf_analysis10.hip — analysis-kernel instantiations for 10-parameter states
// (PROSAIL / SAIL), a translation unit of its own so the GP-loop
// variants compile in parallel with the rest (_build.py).
#include "kf_device.h"

namespace kf {

hipError_t dev_analysis_np10(const AnalysisArgs& a, int grid, hipStream_t s, int* n_part) {
  l_analysis<10>(a, grid, s, n_part);
  return hipGetLastError();
}

#ifdef KF_PHASE_CLOCKS
// the phase counters of this translation unit's (10-parameter) analysis kernels
hipError_t phase_clocks_np10(unsigned long long* out, bool reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(kf_phase_clk), sizeof(kf_phase_clk));
  if (e == hipSuccess && reset) {
    const unsigned long long z[KF_PH_NSLOT] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(kf_phase_clk), z, sizeof(z));
  }
  return e;
}
#endif

}  // namespace kf
