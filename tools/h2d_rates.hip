// Development microbenchmark (not part of the product): what it costs to move
// a page-cache-warm, memory-mapped FASTA (what seq2bytes hands the hot path,
// kmer_numba.py:117-119) into HBM on one MI355X box.
//   1. pinned hipMemcpy H2D (the PCIe bound);
//   2. hipMemcpy straight from the read-only mapping (HIP's own staging);
//   3. hipHostRegister of the mapping (+ ReadOnly flag), H2D from it, unregister;
//   4. memcpy mapping -> pinned with T host threads (T = 1, 2, 4, 8, 12, 16);
//   5. a fresh mapping's first touch (page faults), with and without MAP_POPULATE.
// Build: hipcc --offload-arch=gfx950 -O3 -pthread tools/h2d_rates.hip -o tools/bin/h2d_rates
// Run:   tools/bin/h2d_rates /tmp/x.bin 508334450
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) printf("%s: %s\n", #x, hipGetErrorString(e_));               \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void par_copy(uint8_t* dst, const uint8_t* src, size_t n, int T) {
  std::vector<std::thread> th;
  const size_t part = (n / T + 4095) & ~(size_t)4095;
  for (int t = 0; t < T; ++t) {
    const size_t a = std::min(n, t * part), b = std::min(n, a + part);
    th.emplace_back([=] { if (b > a) memcpy(dst + a, src + a, b - a); });
  }
  for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "/tmp/h2d_rates.bin";
  const size_t n = argc > 2 ? strtoull(argv[2], nullptr, 10) : 508334450ull;
  {  // the file, then one read for page-cache warmth
    int fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0644);
    std::vector<uint8_t> blk(1 << 24);
    for (size_t i = 0; i < blk.size(); ++i) blk[i] = "ACGT\n"[i % 5];
    for (size_t o = 0; o < n; o += blk.size()) {
      const size_t l = std::min(blk.size(), n - o);
      if (write(fd, blk.data(), l) != (ssize_t)l) { printf("write failed\n"); return 1; }
    }
    close(fd);
  }
  int fd = open(path, O_RDONLY);
  uint8_t *dev = nullptr, *pin = nullptr;
  CK(hipMalloc(&dev, n));
  CK(hipHostMalloc((void**)&pin, n, hipHostMallocDefault));
  memset(pin, 1, n);
  auto h2d = [&](const void* src, const char* what, int reps) {
    for (int r = 0; r < reps; ++r) {
      CK(hipDeviceSynchronize());
      const double t = now();
      CK(hipMemcpy(dev, src, n, hipMemcpyHostToDevice));
      const double dt = now() - t;
      printf("%-44s rep %d: %8.3f ms  %6.2f GB/s\n", what, r, dt * 1e3, n / dt / 1e9);
    }
  };
  h2d(pin, "pinned hipMemcpy", 3);

  // 5: first touch of a fresh mapping
  for (int pop = 0; pop < 2; ++pop) {
    const double t = now();
    void* m = mmap(nullptr, n, PROT_READ, MAP_SHARED | (pop ? MAP_POPULATE : 0), fd, 0);
    const double t1 = now();
    volatile uint64_t s = 0;
    for (size_t o = 0; o < n; o += 4096) s += ((const uint8_t*)m)[o];
    const double t2 = now();
    printf("fresh mmap%s: mmap %.3f ms, touch every page %.3f ms\n", pop ? " MAP_POPULATE" : "", (t1 - t) * 1e3,
           (t2 - t1) * 1e3);
    munmap(m, n);
  }
  // first touch by 8 threads
  {
    void* m = mmap(nullptr, n, PROT_READ, MAP_SHARED, fd, 0);
    const double t = now();
    par_copy(pin, (const uint8_t*)m, n, 8);
    printf("fresh mmap, 8-thread memcpy to pinned (faults included): %.3f ms\n", (now() - t) * 1e3);
    munmap(m, n);
  }

  const uint8_t* m = (const uint8_t*)mmap(nullptr, n, PROT_READ, MAP_SHARED, fd, 0);
  volatile uint64_t s = 0;
  for (size_t o = 0; o < n; o += 4096) s += m[o];             // map every page once
  h2d(m, "pageable (mmap) hipMemcpy", 3);
  {
    std::vector<uint8_t> heap(n);
    memcpy(heap.data(), m, n);
    h2d(heap.data(), "pageable (heap) hipMemcpy", 2);
  }
  // 4: host memcpy into pinned
  for (int T : {1, 2, 4, 8, 12, 16, 24}) {
    double best = 1e9;
    for (int r = 0; r < 3; ++r) {
      const double t = now();
      par_copy(pin, m, n, T);
      best = std::min(best, now() - t);
    }
    printf("memcpy mmap -> pinned, %2d threads: %8.3f ms  %6.2f GB/s\n", T, best * 1e3, n / best / 1e9);
  }
  // 3: registration of the mapping
  for (unsigned fl : {(unsigned)hipHostRegisterDefault, (unsigned)hipHostRegisterReadOnly}) {
    for (int r = 0; r < 2; ++r) {
      double t = now();
      hipError_t e = hipHostRegister((void*)m, n, fl);
      const double treg = now() - t;
      if (e != hipSuccess) {
        printf("hipHostRegister(flags %u): %s (%.3f ms)\n", fl, hipGetErrorString(e), treg * 1e3);
        (void)hipGetLastError();
        break;
      }
      t = now();
      CK(hipMemcpy(dev, m, n, hipMemcpyHostToDevice));
      const double tc = now() - t;
      t = now();
      CK(hipHostUnregister((void*)m));
      const double tu = now() - t;
      printf("hipHostRegister(flags %u) rep %d: register %.3f ms, H2D %.3f ms (%.2f GB/s), unregister %.3f ms\n", fl, r,
             treg * 1e3, tc * 1e3, n / tc / 1e9, tu * 1e3);
    }
  }
  int ncpu = (int)std::thread::hardware_concurrency();
  printf("hardware_concurrency %d\n", ncpu);
  munmap((void*)m, n);
  close(fd);
  unlink(path);
  return 0;
}
