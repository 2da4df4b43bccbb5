// Semantics probe of __builtin_amdgcn_permlane32_swap on gfx950: prints, for
// lanes 0, 1, 32, 33, the two returned words when both inputs are the lane id.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o) {
  const unsigned l = threadIdx.x;
  const auto r = __builtin_amdgcn_permlane32_swap(l, l + 100u, false, false);
  o[2 * l] = r[0];
  o[2 * l + 1] = r[1];
}
int main() {
  unsigned* d;
  unsigned h[128];
  (void)hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l : {0, 1, 31, 32, 33, 63}) printf("lane %d: r0=%u r1=%u\n", l, h[2 * l], h[2 * l + 1]);
  return 0;
}
