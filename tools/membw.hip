// membw.hip -- read-pattern microbenchmark for the k_stream design space.
// Every variant reads the whole buffer once (persistent 1024-thread blocks,
// one per CU, grid-stride over 4 KiB units) and folds the bytes into a
// per-lane XOR so nothing is dead-code eliminated.
//   0 strided : lane owns 64 contiguous bytes, 4 x dwordx4 at 64-B lane stride
//   1 coalesced: lane reads 16 B at 16*lane + 1024*i (i = 0..3)
//   2 strided, prefetch depth 2
//   3 LDS-DMA : global_load_lds_dwordx4 of the unit into LDS, then
//               ds_read_b128 of the lane's 64 B (rotated, conflict-free)
//   4 coalesced + nontemporal loads
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ __launch_bounds__(1024, 1) void k_strided(const uint8_t *buf, uint32_t nunits, uint32_t *out) {
  const int lane = threadIdx.x & 63;
  const uint32_t W = gridDim.x * 16;
  uint32_t acc = 0;
  uint32_t u = blockIdx.x * 16 + (threadIdx.x >> 6);
  uint4 a0, a1, a2, a3;
  if (u < nunits) {
    const uint4 *p = (const uint4 *)(buf + (uint64_t)u * 4096 + lane * 64);
    a0 = p[0]; a1 = p[1]; a2 = p[2]; a3 = p[3];
  }
  for (; u < nunits; u += W) {
    uint4 b0, b1, b2, b3;
    if (u + W < nunits) {
      const uint4 *p = (const uint4 *)(buf + (uint64_t)(u + W) * 4096 + lane * 64);
      b0 = p[0]; b1 = p[1]; b2 = p[2]; b3 = p[3];
    }
    acc ^= a0.x ^ a0.y ^ a0.z ^ a0.w ^ a1.x ^ a1.y ^ a1.z ^ a1.w ^ a2.x ^ a2.y ^ a2.z ^ a2.w ^ a3.x ^ a3.y ^ a3.z ^ a3.w;
    a0 = b0; a1 = b1; a2 = b2; a3 = b3;
  }
  out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

template <bool NT>
__global__ __launch_bounds__(1024, 1) void k_coalesced(const uint8_t *buf, uint32_t nunits, uint32_t *out) {
  const int lane = threadIdx.x & 63;
  const uint32_t W = gridDim.x * 16;
  uint32_t acc = 0;
  uint32_t u = blockIdx.x * 16 + (threadIdx.x >> 6);
  v4u a[4];
  auto ld = [&](uint32_t uu, v4u (&r)[4]) {
    const v4u *p = (const v4u *)(buf + (uint64_t)uu * 4096) + lane;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = NT ? __builtin_nontemporal_load(p + 64 * i) : p[64 * i];
  };
  if (u < nunits) ld(u, a);
  for (; u < nunits; u += W) {
    v4u b[4];
    if (u + W < nunits) ld(u + W, b);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc ^= a[i].x ^ a[i].y ^ a[i].z ^ a[i].w;
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = b[i];
  }
  out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

__global__ __launch_bounds__(1024, 1) void k_strided2(const uint8_t *buf, uint32_t nunits, uint32_t *out) {
  const int lane = threadIdx.x & 63;
  const uint32_t W = gridDim.x * 16;
  uint32_t acc = 0;
  uint32_t u = blockIdx.x * 16 + (threadIdx.x >> 6);
  uint4 a[4], b[4];
  auto ld = [&](uint32_t uu, uint4 (&r)[4]) {
    const uint4 *p = (const uint4 *)(buf + (uint64_t)uu * 4096 + lane * 64);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = p[i];
  };
  if (u < nunits) ld(u, a);
  if (u + W < nunits) ld(u + W, b);
  for (; u < nunits; u += W) {
    uint4 c[4];
    if (u + 2 * W < nunits) ld(u + 2 * W, c);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc ^= a[i].x ^ a[i].y ^ a[i].z ^ a[i].w;
#pragma unroll
    for (int i = 0; i < 4; ++i) { a[i] = b[i]; b[i] = c[i]; }
  }
  out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

// LDS-DMA: each wave DMA-loads its 4 KiB unit into its own 2 x 4 KiB LDS
// ring (double buffered), then reads its 64-B piece per lane with rotated
// ds_read_b128 (conflict-free for the b128 lane groups).
__global__ __launch_bounds__(1024, 1) void k_ldsdma(const uint8_t *buf, uint32_t nunits, uint32_t *out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint8_t *ring = smem + wv * 8192;
  const uint32_t W = gridDim.x * 16;
  uint32_t acc = 0;
  uint32_t u = blockIdx.x * 16 + wv;
  auto dma = [&](uint32_t uu, int slot) {
    const uint8_t *g = buf + (uint64_t)uu * 4096 + lane * 16;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((const void *)(g + 1024 * i),
                                       (__attribute__((address_space(3))) void *)(ring + slot * 4096 + 1024 * i), 16, 0, 0);
  };
  int slot = 0;
  if (u < nunits) dma(u, 0);
  for (; u < nunits; u += W) {
    if (u + W < nunits) {
      dma(u + W, slot ^ 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const uint8_t *base = ring + slot * 4096 + lane * 64;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = (i + (lane >> 2)) & 3;
      const uint4 q = *(const uint4 *)(base + 16 * c);
      acc ^= q.x ^ q.y ^ q.z ^ q.w;
    }
    slot ^= 1;
  }
  out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

int main(int argc, char **argv) {
  const uint64_t gib = argc > 1 ? atoll(argv[1]) : 4;
  const uint64_t B = gib << 30;
  const uint32_t nunits = (uint32_t)(B / 4096);
  uint8_t *d;
  uint32_t *o;
  CK(hipMalloc(&d, B));
  CK(hipMalloc(&o, 1 << 22));
  CK(hipMemset(d, 0x5a, B));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int grid = prop.multiProcessorCount;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char *names[] = {"strided64", "coalesced", "strided64-pf2", "ldsdma-b128", "coalesced-nt"};
  for (int round = 0; round < 3; ++round) {
    for (int v = 0; v < 5; ++v) {
      float best = 1e9;
      for (int it = 0; it < 5; ++it) {
        CK(hipEventRecord(e0));
        if (v == 0) hipLaunchKernelGGL(k_strided, dim3(grid), dim3(1024), 0, 0, d, nunits, o);
        if (v == 1) hipLaunchKernelGGL(k_coalesced<false>, dim3(grid), dim3(1024), 0, 0, d, nunits, o);
        if (v == 2) hipLaunchKernelGGL(k_strided2, dim3(grid), dim3(1024), 0, 0, d, nunits, o);
        if (v == 3) hipLaunchKernelGGL(k_ldsdma, dim3(grid), dim3(1024), 16 * 8192, 0, d, nunits, o);
        if (v == 4) hipLaunchKernelGGL(k_coalesced<true>, dim3(grid), dim3(1024), 0, 0, d, nunits, o);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      if (round == 2) printf("%-16s %8.3f ms  %7.1f GB/s\n", names[v], best, B / best / 1e6);
    }
  }
  return 0;
}
