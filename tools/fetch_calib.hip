// Development microbenchmark: calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE
// against known byte counts for the access patterns the K3 / K5 kernels use
// (MI355X_MICROARCH.md: "other access widths are uncalibrated").  Not part of
// the product.  Each pattern is one kernel; the buffer (2 GiB) is far beyond
// the 256 MiB Infinity Cache, so random accesses miss on-die caches.
// Build: hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/bin/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}

// 16 B per lane, coalesced, whole buffer prefix of n16 elements
__global__ void c_stream16(const uint4* __restrict__ p, uint64_t n16, unsigned* sink) {
  unsigned acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

// the same stream with non-temporal loads (K1's FASTA passes, the split and
// range passes' records)
__global__ void c_stream16nt(const uint4* __restrict__ p, uint64_t n16, unsigned* sink) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  unsigned acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p) + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}
// 8 B per lane, non-temporal (the split / range passes' keys)
__global__ void c_stream8nt(const unsigned long long* __restrict__ p, uint64_t n8, unsigned* sink) {
  unsigned long long acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n8; i += (uint64_t)gridDim.x * blockDim.x)
    acc ^= __builtin_nontemporal_load(p + i);
  if (acc == 0x9e3779b9ull) sink[0] = (unsigned)acc;
}

// random aligned 16-byte loads (one per lane per iteration)
__global__ void c_rand16(const uint4* __restrict__ p, uint64_t mask16, int per, unsigned* sink) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  unsigned acc = 0;
  for (int j = 0; j < per; ++j) {
    const uint4 v = p[mix(i * 977 + j) & mask16];
    acc ^= v.x ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

// random aligned 8-byte loads
__global__ void c_rand8(const unsigned long long* __restrict__ p, uint64_t mask8, int per, unsigned* sink) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  unsigned long long acc = 0;
  for (int j = 0; j < per; ++j) acc ^= p[mix(i * 977 + j) & mask8];
  if (acc == 0x9e3779b9ull) sink[0] = (unsigned)acc;
}

// random 64-bit CAS on zeroed words (every CAS succeeds: one 8-byte write each)
__global__ void c_cas8(unsigned long long* p, uint64_t mask8, int per, unsigned* sink) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  unsigned long long acc = 0;
  for (int j = 0; j < per; ++j) {
    const uint64_t a = mix(i * 977 + j + 0x51ed) & mask8;
    acc += atomicCAS(p + a, 0ull, a | 1);
  }
  if (acc == 0x9e3779b9ull) sink[0] = (unsigned)acc;
}

// random 64-bit atomicOr without return
__global__ void c_or8(unsigned long long* p, uint64_t mask8, int per) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  for (int j = 0; j < per; ++j) atomicOr(p + (mix(i * 977 + j + 0xabc) & mask8), 2ull);
}

// 16 B per lane coalesced stores
__global__ void c_store16(uint4* __restrict__ p, uint64_t n16) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = make_uint4((unsigned)i, 0, 0, 0);
}

int main() {
  const uint64_t bytes = 2ull << 30;
  void* buf = nullptr;
  unsigned* sink = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
  hipMemset(buf, 0, bytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int per = 16, T = 256;
  const unsigned blocks = 16384;                        // 64 M accesses per random kernel
  const double acc = (double)blocks * T * per;
  auto timed = [&](const char* name, double req_bytes, auto launch) {
    hipEventRecord(a);
    launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    printf("%-10s requested %.3f GB  %.3f ms  %.1f GB/s\n", name, req_bytes / 1e9, ms, req_bytes / ms / 1e6);
  };
  for (int rep = 0; rep < 2; ++rep) {
    timed("stream16", 1.0 * (1ull << 30), [&] {
      hipLaunchKernelGGL(c_stream16, dim3(8192), dim3(T), 0, 0, (const uint4*)buf, (1ull << 30) / 16, sink);
    });
    timed("stream16nt", 1.0 * (1ull << 30), [&] {
      hipLaunchKernelGGL(c_stream16nt, dim3(8192), dim3(T), 0, 0, (const uint4*)buf, (1ull << 30) / 16, sink);
    });
    timed("stream8nt", 1.0 * (1ull << 30), [&] {
      hipLaunchKernelGGL(c_stream8nt, dim3(8192), dim3(T), 0, 0, (const unsigned long long*)buf, (1ull << 30) / 8,
                         sink);
    });
    timed("rand16", acc * 16, [&] {
      hipLaunchKernelGGL(c_rand16, dim3(blocks), dim3(T), 0, 0, (const uint4*)buf, bytes / 16 - 1, per, sink);
    });
    timed("rand8", acc * 8, [&] {
      hipLaunchKernelGGL(c_rand8, dim3(blocks), dim3(T), 0, 0, (const unsigned long long*)buf, bytes / 8 - 1, per,
                         sink);
    });
    hipMemset(buf, 0, bytes);
    timed("cas8", acc * 8, [&] {
      hipLaunchKernelGGL(c_cas8, dim3(blocks), dim3(T), 0, 0, (unsigned long long*)buf, bytes / 8 - 1, per, sink);
    });
    timed("or8", acc * 8, [&] {
      hipLaunchKernelGGL(c_or8, dim3(blocks), dim3(T), 0, 0, (unsigned long long*)buf, bytes / 8 - 1, per);
    });
    timed("store16", 1.0 * (1ull << 30), [&] {
      hipLaunchKernelGGL(c_store16, dim3(8192), dim3(T), 0, 0, (uint4*)buf, (1ull << 30) / 16);
    });
  }
  hipDeviceSynchronize();
  hipFree(buf);
  hipFree(sink);
  return 0;
}
