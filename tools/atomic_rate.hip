// Development microbenchmark: scattered 64-bit CAS / OR / load rates on one
// MI355X over a 512 MiB table (the K3 table's size class).  Not part of the
// product.  Build: hipcc --offload-arch=gfx950 -O3 tools/atomic_rate.hip -o atomic_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}

template <int MODE>
__global__ void k(unsigned long long* t, uint64_t mask, int per, uint64_t seed, unsigned long long* sink) {
  uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  unsigned long long acc = 0;
  for (int j = 0; j < per; ++j) {
    const uint64_t a = mix(seed + i * 131 + j) & mask;
    if (MODE == 0) acc += atomicCAS(t + a, 0ull, a + 1);                       // device scope
    if (MODE == 1) acc += __hip_atomic_compare_exchange_strong(t + a, &acc, a + 1, __ATOMIC_RELAXED,
                                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (MODE == 2) atomicOr(t + a, 1ull);                                       // no return
    if (MODE == 3) acc += t[a];                                                 // plain load
    if (MODE == 4) acc += atomicOr(t + a, 1ull);                                // with return
  }
  if (acc == 0x123456789ull) sink[0] = acc;
}

int main() {
  const uint64_t words = 64ull << 20;                 // 512 MiB
  unsigned long long *t, *sink;
  hipMalloc(&t, words * 8);
  hipMalloc(&sink, 8);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const int per = 16, threads = 256;
  const unsigned blocks = 4096;
  const double ops = (double)blocks * threads * per;
  const char* names[] = {"CAS device", "CAS workgroup", "OR noret device", "load", "OR ret device"};
  for (int mode = 0; mode < 5; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      hipMemset(t, 0, words * 8);
      hipEventRecord(a);
      switch (mode) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(threads), 0, 0, t, words - 1, per, rep * 7919ull, sink); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(threads), 0, 0, t, words - 1, per, rep * 7919ull, sink); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(threads), 0, 0, t, words - 1, per, rep * 7919ull, sink); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(threads), 0, 0, t, words - 1, per, rep * 7919ull, sink); break;
        case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(threads), 0, 0, t, words - 1, per, rep * 7919ull, sink); break;
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      printf("%-16s rep %d: %.3f ms  %.2f G ops/s\n", names[mode], rep, ms, ops / ms / 1e6);
    }
  }
  return 0;
}
