// Development microbenchmark (not part of the product): rates that decide K3's
// design on one MI355X.
//  1. one returning atomicAdd per block on a single address (the coverage
//     pass's queue counter) vs spread over 64 lines, 122 880 blocks;
//  2. random 16-byte loads, 64-bit CAS and non-returning atomicOr against
//     the table size (32 MiB .. 2 GiB): what a compact, Infinity-Cache
//     resident table would buy.
// Build: hipcc --offload-arch=gfx950 -O3 tools/rates.hip -o tools/bin/rates
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}

template <int SPREAD>
__global__ void q_count(unsigned long long* ctr, unsigned long long* out) {
  __shared__ unsigned long long base;
  if (threadIdx.x == 0) base = atomicAdd(ctr + 8 * (blockIdx.x % SPREAD), 3ull);
  __syncthreads();
  if (base == 0xFFFFFFFFFFFFull) out[threadIdx.x] = base;
}

__global__ void r_load16(const uint4* __restrict__ p, uint64_t mask16, int per, unsigned* sink) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  unsigned acc = 0;
  for (int j = 0; j < per; ++j) {
    const uint4 v = p[mix(i * 977 + j) & mask16];
    acc ^= v.x ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

__global__ void r_cas(unsigned long long* p, uint64_t mask8, int per, uint64_t seed, unsigned* sink) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  unsigned long long acc = 0;
  for (int j = 0; j < per; ++j) {
    const uint64_t a = mix(i * 977 + j + seed) & mask8;
    acc += atomicCAS(p + a, 0ull, a | 1);
  }
  if (acc == 0x9e3779b9ull) sink[0] = (unsigned)acc;
}

__global__ void r_or(unsigned long long* p, uint64_t mask8, int per, uint64_t seed) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  for (int j = 0; j < per; ++j) atomicOr(p + (mix(i * 977 + j + seed) & mask8), 2ull);
}

int main() {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto ms_of = [&](auto launch) {
    hipEventRecord(a);
    launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
  };
  unsigned long long *ctr, *out;
  hipMalloc(&ctr, 64 * 64 * 8);
  hipMalloc(&out, 256 * 8);
  const unsigned nb = 122880;
  for (int rep = 0; rep < 3; ++rep) {
    hipMemset(ctr, 0, 64 * 64 * 8);
    float m1 = ms_of([&] { hipLaunchKernelGGL(q_count<1>, dim3(nb), dim3(256), 0, 0, ctr, out); });
    float m8 = ms_of([&] { hipLaunchKernelGGL(q_count<8>, dim3(nb), dim3(256), 0, 0, ctr, out); });
    float m64 = ms_of([&] { hipLaunchKernelGGL(q_count<64>, dim3(nb), dim3(256), 0, 0, ctr, out); });
    printf("queue counter, %u blocks: 1 address %.3f ms, 8 lines %.3f ms, 64 lines %.3f ms\n", nb, m1, m8, m64);
  }
  const uint64_t maxb = 2ull << 30;
  void* buf = nullptr;
  unsigned* sink = nullptr;
  hipMalloc(&buf, maxb);
  hipMalloc(&sink, 64);
  const int per = 16, T = 256;
  const unsigned blocks = 8192;
  const double ops = (double)blocks * T * per;
  for (uint64_t sz = 32ull << 20; sz <= maxb; sz *= 2) {
    hipMemset(buf, 0, sz);
    float ml = 0, mc = 0, mo = 0;
    for (int rep = 0; rep < 2; ++rep) {
      ml = ms_of([&] { hipLaunchKernelGGL(r_load16, dim3(blocks), dim3(T), 0, 0, (const uint4*)buf, sz / 16 - 1, per,
                                          sink); });
      hipMemset(buf, 0, sz);
      mc = ms_of([&] { hipLaunchKernelGGL(r_cas, dim3(blocks), dim3(T), 0, 0, (unsigned long long*)buf, sz / 8 - 1,
                                          per, (uint64_t)rep << 40, sink); });
      mo = ms_of([&] { hipLaunchKernelGGL(r_or, dim3(blocks), dim3(T), 0, 0, (unsigned long long*)buf, sz / 8 - 1,
                                          per, (uint64_t)rep << 41); });
    }
    printf("table %5llu MiB: load16 %.1f G/s  cas %.1f G/s  or %.1f G/s\n", (unsigned long long)(sz >> 20),
           ops / ml / 1e6, ops / mc / 1e6, ops / mo / 1e6);
  }
  hipDeviceSynchronize();
  return 0;
}
