// FETCH_SIZE calibration for the frame pass's per-lane gathers:
// every lane reads K x 16 B from its own random 16-B aligned position of a
// 4 GiB buffer (far past the Infinity Cache), the access shape of k_frames'
// head / piece / tail loads.  Prints the requested bytes and the 128-B lines
// the gathers touch; rocprofv3 --pmc FETCH_SIZE of the same run gives what
// the counter reports for them (tools/gpu_s5.sh -> profiles/r05/).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/gather_cal tools/gather_cal.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("hip %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <int K>
__global__ __launch_bounds__(256) void k_gather(const uint4 *__restrict__ buf, uint64_t n16, uint64_t nlanes,
                                                uint32_t seed, uint4 *__restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nlanes) return;
  const uint64_t p = mix(i * 0x100000001b3ull + seed) % (n16 - K);
  uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint4 w = buf[p + k];
    acc.x ^= w.x; acc.y ^= w.y; acc.z ^= w.z; acc.w ^= w.w;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[i & 1023] = acc;   // keeps the loads
}

static uint64_t host_mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main() {
  const uint64_t bytes = 4ull << 30, n16 = bytes / 16;
  uint4 *buf = nullptr, *out = nullptr;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 1024 * sizeof(uint4)));
  CK(hipMemset(buf, 0x5a, bytes));
  const uint64_t nlanes = 4ull << 20;   // 4 Mi gathers per launch
  for (int K : {4, 5}) {
    // the lines the gathers touch (host replay of the same positions)
    std::vector<uint64_t> lines;
    lines.reserve(nlanes * 2);
    for (uint64_t i = 0; i < nlanes; ++i) {
      const uint64_t p = host_mix(i * 0x100000001b3ull + 7) % (n16 - K);
      for (uint64_t l = (p * 16) / 128; l <= ((p + K) * 16 - 1) / 128; ++l) lines.push_back(l);
    }
    std::sort(lines.begin(), lines.end());
    const uint64_t uniq = (uint64_t)(std::unique(lines.begin(), lines.end()) - lines.begin());
    for (int rep = 0; rep < 3; ++rep) {
      if (K == 4) hipLaunchKernelGGL(k_gather<4>, dim3((unsigned)(nlanes / 256)), dim3(256), 0, 0, buf, n16, nlanes, 7u, out);
      else hipLaunchKernelGGL(k_gather<5>, dim3((unsigned)(nlanes / 256)), dim3(256), 0, 0, buf, n16, nlanes, 7u, out);
      CK(hipDeviceSynchronize());
    }
    std::printf("gather K=%d (%d B per lane): lanes %llu requested %llu B, distinct 128-B lines %llu = %llu B\n", K,
                16 * K, (unsigned long long)nlanes, (unsigned long long)(nlanes * 16 * K), (unsigned long long)uniq,
                (unsigned long long)(uniq * 128));
  }
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
