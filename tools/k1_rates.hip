// Development microbenchmark (not part of the product): streaming-read rates
// for K1's geometry on one MI355X.  A 508 MB buffer (FASTA-like: 60 bases
// and '\n'), read by
//   w16k    one wave per 16 KiB, all 16 loads issued first (k_span_sum's shape)
//   w16k_s  one wave per 16 KiB, one load in flight ahead (k_emit's shape)
//   w4k     one wave per 4 KiB, 4 loads up front
//   gs      grid-stride, 2048 blocks x 256, 16 B per lane per step, 4 deep
//   copy    w16k reading + writing the same bytes to a second buffer
//   rw14    w16k reading + writing 5/16 of the bytes (K1's packed outputs)
// Build: hipcc --offload-arch=gfx950 -O3 tools/k1_rates.hip -o tools/bin/k1_rates
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>
#include <unistd.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int STEPS>
__global__ void __launch_bounds__(256) w_front(const uint8_t* __restrict__ buf, uint64_t n, unsigned* sink) {
  const int lane = threadIdx.x & 63;
  const uint64_t span = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t p0 = span * (uint64_t)(STEPS * 1024);
  if (p0 >= n) return;
  uint4 v[STEPS];
#pragma unroll
  for (int s = 0; s < STEPS; ++s) {
    const uint64_t p = p0 + (uint64_t)s * 1024 + lane * 16;
    v[s] = p + 16 <= n ? *reinterpret_cast<const uint4*>(buf + p) : make_uint4(0, 0, 0, 0);
  }
  unsigned acc = 0;
#pragma unroll
  for (int s = 0; s < STEPS; ++s) acc = acc * 31u + (v[s].x ^ v[s].y ^ v[s].z ^ v[s].w);
  if (acc == 0x7FFFFFFFu) sink[0] = acc;
}

__global__ void __launch_bounds__(256) w_stream(const uint8_t* __restrict__ buf, uint64_t n, unsigned* sink) {
  const int lane = threadIdx.x & 63;
  const uint64_t span = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t p0 = span * 16384ull;
  if (p0 >= n) return;
  uint64_t p = p0 + lane * 16;
  uint4 v = p + 16 <= n ? *reinterpret_cast<const uint4*>(buf + p) : make_uint4(0, 0, 0, 0);
  unsigned acc = 0;
  for (int s = 0; s < 16; ++s) {
    const uint64_t pn = p + 1024;
    const uint4 vn = (s + 1 < 16 && pn + 16 <= n) ? *reinterpret_cast<const uint4*>(buf + pn) : make_uint4(0, 0, 0, 0);
    acc = acc * 31u + (v.x ^ v.y ^ v.z ^ v.w);
    v = vn;
    p = pn;
  }
  if (acc == 0x7FFFFFFFu) sink[0] = acc;
}

__global__ void __launch_bounds__(256) w_gs(const uint4* __restrict__ p, uint64_t n16, unsigned* sink) {
  unsigned acc = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
    acc += a.x ^ b.y ^ c.z ^ d.w;
  }
  for (; i < n16; i += stride) acc += p[i].x;
  if (acc == 0x7FFFFFFFu) sink[0] = acc;
}

template <int WDEN>   // write 16 / WDEN bytes per 16 read (WDEN = 1: copy)
__global__ void __launch_bounds__(256) w_rw(const uint8_t* __restrict__ buf, uint64_t n, uint8_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const uint64_t span = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t p0 = span * 16384ull;
  if (p0 >= n) return;
  uint4 v[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const uint64_t p = p0 + (uint64_t)s * 1024 + lane * 16;
    v[s] = p + 16 <= n ? *reinterpret_cast<const uint4*>(buf + p) : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const uint64_t p = p0 + (uint64_t)s * 1024 + lane * 16;
    if (p + 16 > n) continue;
    if (WDEN == 1) {
      *reinterpret_cast<uint4*>(out + p) = v[s];
    } else {
      // 4 B packed word + 1 B exception per 16 read (5/16)
      reinterpret_cast<uint32_t*>(out)[p >> 4] = v[s].x ^ v[s].y ^ v[s].z ^ v[s].w;
      out[(n >> 2) + (p >> 4)] = (uint8_t)v[s].x;
    }
  }
}

int main() {
  const uint64_t n = 508334450ull;
  std::vector<uint8_t> h(n);
  const char* acgt = "ACGT";
  uint64_t x = 88172645463325252ull;
  for (uint64_t i = 0; i < n; ++i) {
    if (i % 61 == 60) { h[i] = '\n'; continue; }
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    h[i] = (uint8_t)acgt[x & 3];
  }
  uint8_t *d, *o;
  unsigned* sink;
  CK(hipMalloc(&d, n + 64));
  CK(hipMalloc(&o, n + 64));
  CK(hipMalloc(&sink, 64));
  CK(hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const unsigned spans16 = (unsigned)((n + 16383) / 16384), spans4 = (unsigned)((n + 4095) / 4096);
  auto run = [&](const char* name, double bytes, auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    float best = 1e9f, sum = 0.f;
    for (int r = 0; r < 20; ++r) {
      (void)hipEventRecord(a, 0);
      launch();
      (void)hipEventRecord(b, 0);
      (void)hipEventSynchronize(b);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, a, b);
      best = ms < best ? ms : best;
      sum += ms;
    }
    CK(hipGetLastError());
    std::printf("%-8s best %.4f ms avg %.4f ms  %.1f GB/s (best)\n", name, best, sum / 20, bytes / best / 1e6);
    return 0;
  };
  run("w16k", n, [&] { hipLaunchKernelGGL(w_front<16>, dim3((spans16 + 3) / 4), dim3(256), 0, 0, d, n, sink); });
  run("w16k_s", n, [&] { hipLaunchKernelGGL(w_stream, dim3((spans16 + 3) / 4), dim3(256), 0, 0, d, n, sink); });
  run("w4k", n, [&] { hipLaunchKernelGGL(w_front<4>, dim3((spans4 + 3) / 4), dim3(256), 0, 0, d, n, sink); });
  run("gs", n, [&] { hipLaunchKernelGGL(w_gs, dim3(2048), dim3(256), 0, 0, reinterpret_cast<const uint4*>(d), n / 16, sink); });
  run("copy", 2.0 * n, [&] { hipLaunchKernelGGL(w_rw<1>, dim3((spans16 + 3) / 4), dim3(256), 0, 0, d, n, o); });
  run("rw5_16", n * 21.0 / 16, [&] { hipLaunchKernelGGL(w_rw<4>, dim3((spans16 + 3) / 4), dim3(256), 0, 0, d, n, o); });
  // each launch after the GPU idled ~0.3 ms (as a build's first kernel does)
  {
    float best = 1e9f, sum = 0.f;
    for (int r = 0; r < 20; ++r) {
      CK(hipDeviceSynchronize());
      usleep(300);
      (void)hipEventRecord(a, 0);
      hipLaunchKernelGGL(w_front<16>, dim3((spans16 + 3) / 4), dim3(256), 0, 0, d, n, sink);
      (void)hipEventRecord(b, 0);
      (void)hipEventSynchronize(b);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, a, b);
      best = ms < best ? ms : best;
      sum += ms;
    }
    std::printf("%-8s best %.4f ms avg %.4f ms  %.1f GB/s (best)\n", "w16k_idle", best, sum / 20, n / best / 1e6);
  }
  // each launch right after a kernel that wrote 480 MiB elsewhere (the
  // previous build's table: dirty lines in the Infinity Cache / L2)
  {
    // (480 MiB copied from the 508 MB input buffer into a 480 MiB one: both in bounds)
    const uint64_t jn = 480ull << 20;
    static_assert((480ull << 20) < 508334450ull, "the copy's source is the input buffer");
    uint8_t* junk;
    CK(hipMalloc(&junk, jn + 64));
    const unsigned jsp = (unsigned)((jn + 16383) / 16384);
    float best = 1e9f, sum = 0.f;
    for (int r = 0; r < 20; ++r) {
      hipLaunchKernelGGL(w_rw<1>, dim3((jsp + 3) / 4), dim3(256), 0, 0, d, jn, junk);
      (void)hipEventRecord(a, 0);
      hipLaunchKernelGGL(w_front<16>, dim3((spans16 + 3) / 4), dim3(256), 0, 0, d, n, sink);
      (void)hipEventRecord(b, 0);
      (void)hipEventSynchronize(b);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, a, b);
      best = ms < best ? ms : best;
      sum += ms;
    }
    CK(hipGetLastError());
    std::printf("%-8s best %.4f ms avg %.4f ms  %.1f GB/s (best)\n", "w16k_dirty", best, sum / 20, n / best / 1e6);
  }
  // the Infinity Cache: a 128 MB / 64 MB piece read once, then twice in a row
  for (uint64_t mb : {64ull, 128ull}) {
    const uint64_t m = mb << 20;
    const unsigned sp = (unsigned)((m + 16383) / 16384);
    run(mb == 64 ? "p64x1" : "p128x1", (double)m, [&] { hipLaunchKernelGGL(w_front<16>, dim3((sp + 3) / 4), dim3(256), 0, 0, d, m, sink); });
    run(mb == 64 ? "p64x2" : "p128x2", 2.0 * m, [&] {
      hipLaunchKernelGGL(w_front<16>, dim3((sp + 3) / 4), dim3(256), 0, 0, d, m, sink);
      hipLaunchKernelGGL(w_front<16>, dim3((sp + 3) / 4), dim3(256), 0, 0, d, m, sink);
    });
  }
  return 0;
}
