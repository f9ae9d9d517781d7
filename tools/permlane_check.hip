// permlane_check.hip -- prints v_permlane32_swap / v_permlane16_swap results
// for lane-id inputs (semantics check for the k_stream transpose).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *o) {
  const unsigned l = threadIdx.x;
  auto r = __builtin_amdgcn_permlane32_swap(l, 100 + l, false, false);
  o[l] = r[0]; o[64 + l] = r[1];
  auto s = __builtin_amdgcn_permlane16_swap(l, 100 + l, false, false);
  o[128 + l] = s[0]; o[192 + l] = s[1];
}
int main() {
  unsigned *d, h[256];
  hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char *nm[4] = {"p32 vdst", "p32 vsrc", "p16 vdst", "p16 vsrc"};
  for (int t = 0; t < 4; ++t) {
    printf("%s:", nm[t]);
    for (int l = 0; l < 64; l += 8) printf(" [%d]=%u", l, h[64 * t + l]);
    printf(" [63]=%u\n", h[64 * t + 63]);
  }
  return 0;
}
