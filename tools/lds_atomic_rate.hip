// Development microbenchmark: LDS operation rates at random addresses in a
// 64 KiB table per block (k_build_range's range copy: 4096 buckets x 2
// words), 2 blocks of 512 threads per CU as k_build_range runs.  Not part of
// the product.  Build: hipcc --offload-arch=gfx950 -O3 tools/lds_atomic_rate.hip -o lds_atomic_rate
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

constexpr int WORDS = 8192;                    // 64 KiB of 8-byte words
constexpr int PER = 64;                        // operations per thread

template <int MODE>
__global__ void __launch_bounds__(512, 4) k(uint32_t seed, unsigned long long* sink) {
  __shared__ unsigned long long W[WORDS];
  for (int i = threadIdx.x; i < WORDS; i += 512) W[i] = 0ull;
  __syncthreads();
  unsigned long long acc = 0;
  uint32_t* W32 = reinterpret_cast<uint32_t*>(W);
  const uint32_t base = seed + (blockIdx.x * 512u + threadIdx.x) * 977u;
#pragma unroll 8
  for (int j = 0; j < PER; ++j) {
    const uint32_t a = mix32(base + (uint32_t)j) & (WORDS - 1);
    const unsigned long long v = ((unsigned long long)(a + 1) << 26) | (j & 63);
    if (MODE == 0) acc += atomicCAS(W + a, 0ull, v);                              // ds_cmpst_rtn_b64
    if (MODE == 1) __hip_atomic_fetch_max(W + a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);   // ds_max_u64
    if (MODE == 2) __hip_atomic_fetch_or(W + a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);    // ds_or_b64
    if (MODE == 3) W[a] = v;                                                       // ds_write_b64
    if (MODE == 4) acc += W[a];                                                    // ds_read_b64
    if (MODE == 5) acc += atomicCAS(W32 + 2 * a, 0u, (uint32_t)v);                // ds_cmpst_rtn_b32
    if (MODE == 6) __hip_atomic_fetch_add(W32 + 2 * a, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // ds_add_u32
    if (MODE == 7) acc += __hip_atomic_fetch_max(W + a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // ds_max_rtn_u64
    if (MODE == 8) acc += __hip_atomic_fetch_add(W32 + 2 * a, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // ds_add_rtn_u32
    if (MODE == 9) __hip_atomic_fetch_or(W32 + 2 * a, (uint32_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // ds_or_b32
  }
  __syncthreads();
  acc += W[threadIdx.x];
  if (acc == 0x123456789ull) sink[0] = acc;
}

int main() {
  unsigned long long* sink;
  hipMalloc(&sink, 8);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const unsigned blocks = 2u * cus * 16u;      // 16 rounds of 2 blocks per CU
  const double ops = (double)blocks * 512 * PER;
  const char* names[] = {"cmpst_rtn_b64", "max_u64 noret", "or_b64 noret", "write_b64", "read_b64",
                         "cmpst_rtn_b32", "add_u32 noret", "max_rtn_u64", "add_rtn_u32", "or_b32 noret"};
  void (*ks[])(uint32_t, unsigned long long*) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>, k<8>, k<9>};
  for (int m = 0; m < 10; ++m) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(a);
      hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(512), 0, 0, 12345u + rep, sink);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    // lane-ops per CU per ns, and cycles per wave-instruction per CU at 2.4 GHz
    const double per_cu_ns = ops / cus / (best * 1e6);
    std::printf("%-16s %8.3f ms  %7.2f lane-ops/ns/CU  %6.1f cycles per wave-op per CU\n", names[m], best,
                per_cu_ns, 64.0 * 2.4 / per_cu_ns);
  }
  return 0;
}
