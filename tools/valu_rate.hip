// Microbenchmark: wave64 VALU issue rate on gfx950 for the instruction mix of
// k_stream (v_perm_b32, v_bitop3_b32, v_alignbyte_b32, v_add_u32, v_xor_b32),
// with W waves per SIMD.  Prints cycles per instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
template <int OP>
__global__ __launch_bounds__(1024) void k(uint32_t *out, int iters) {
  uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (OP == 0) {   // v_perm_b32
        a0 = __builtin_amdgcn_perm(a0, a1, 0x0c020100u); a1 = __builtin_amdgcn_perm(a1, a2, 0x0c020100u);
        a2 = __builtin_amdgcn_perm(a2, a3, 0x0c020100u); a3 = __builtin_amdgcn_perm(a3, a4, 0x0c020100u);
        a4 = __builtin_amdgcn_perm(a4, a5, 0x0c020100u); a5 = __builtin_amdgcn_perm(a5, a6, 0x0c020100u);
        a6 = __builtin_amdgcn_perm(a6, a7, 0x0c020100u); a7 = __builtin_amdgcn_perm(a7, a0, 0x0c020100u);
      } else if (OP == 1) {   // v_bitop3_b32
        a0 = __builtin_amdgcn_bitop3_b32(a0, a1, a2, 0x96); a1 = __builtin_amdgcn_bitop3_b32(a1, a2, a3, 0x96);
        a2 = __builtin_amdgcn_bitop3_b32(a2, a3, a4, 0x96); a3 = __builtin_amdgcn_bitop3_b32(a3, a4, a5, 0x96);
        a4 = __builtin_amdgcn_bitop3_b32(a4, a5, a6, 0x96); a5 = __builtin_amdgcn_bitop3_b32(a5, a6, a7, 0x96);
        a6 = __builtin_amdgcn_bitop3_b32(a6, a7, a0, 0x96); a7 = __builtin_amdgcn_bitop3_b32(a7, a0, a1, 0x96);
      } else if (OP == 2) {   // v_alignbyte_b32
        a0 = __builtin_amdgcn_alignbyte(a0, a1, 2); a1 = __builtin_amdgcn_alignbyte(a1, a2, 2);
        a2 = __builtin_amdgcn_alignbyte(a2, a3, 2); a3 = __builtin_amdgcn_alignbyte(a3, a4, 2);
        a4 = __builtin_amdgcn_alignbyte(a4, a5, 2); a5 = __builtin_amdgcn_alignbyte(a5, a6, 2);
        a6 = __builtin_amdgcn_alignbyte(a6, a7, 2); a7 = __builtin_amdgcn_alignbyte(a7, a0, 2);
      } else {   // v_add_u32 / v_xor_b32
        a0 += a1; a1 ^= a2; a2 += a3; a3 ^= a4; a4 += a5; a5 ^= a6; a6 += a7; a7 ^= a0;
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
int main() {
  int dev = 0, ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
  uint32_t *out;
  hipMalloc(&out, 64 << 20);
  const int iters = 2000;
  const char *names[4] = {"v_perm_b32", "v_bitop3_b32", "v_alignbyte", "v_add/xor"};
  for (int wps = 1; wps <= 4; wps *= 2) {   // waves per SIMD: block of 256*wps threads, one block per CU
    for (int op = 0; op < 4; ++op) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0); hipEventCreate(&e1);
      dim3 g(ncu), b(256 * wps);
      auto launch = [&]() {
        if (op == 0) hipLaunchKernelGGL(k<0>, g, b, 0, 0, out, iters);
        if (op == 1) hipLaunchKernelGGL(k<1>, g, b, 0, 0, out, iters);
        if (op == 2) hipLaunchKernelGGL(k<2>, g, b, 0, 0, out, iters);
        if (op == 3) hipLaunchKernelGGL(k<3>, g, b, 0, 0, out, iters);
      };
      launch();
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double instr_per_wave = (double)iters * 16 * 8;
      const double cyc = ms * 1e-3 * clk * 1e3;   // at the reported clock
      printf("waves/SIMD %d %-14s %.3f ms  %.2f cycles per instr per SIMD (clock %d MHz)\n", wps, names[op], ms,
             cyc / (instr_per_wave * wps), clk / 1000);
    }
  }
  return 0;
}
