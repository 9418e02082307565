// pg_stage.hip — host FASTA bytes to HBM for pg_parse_host / pg_build_host.
//
// The reference reads its input through np.memmap (seq2bytes,
// kmer_numba.py:117-119): pageable, page-cache-backed memory.  A
// hipMemcpyAsync from such a pointer is staged by the HIP runtime one buffer at
// a time and returns only when the bytes are gone, so nothing overlaps it.
// Here a pageable source goes through a ring of pinned slots instead: a stager
// thread copies chunk i in 8 MiB pieces into free slots with a small pool of
// memcpy threads (one host core moves ~23 GB/s from a warm mapping, 8 ~100
// GB/s, the PCIe link 57.5 GB/s; tools/h2d_rates.hip), queues each piece's
// DMA on the copy stream and records the chunk's event, while the caller's
// thread keeps launching K1 (and, in pg_build_host, stage A) behind the chunks
// that have landed.  A pinned source (hipHostMalloc / registered) is DMA'd
// directly, as before.  By default the stager first tries to register each
// page-aligned chunk of a pageable source for the duration of the upload
// (hipHostRegister, read-only) and DMA it directly - one pass over host DRAM
// instead of three, which matters when 8 GPUs of a node load at once; a chunk
// that cannot be registered (an unaligned pointer, memory the driver refuses)
// sends it and every later chunk through the ring.
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <sched.h>
#include <thread>

#include "pg_internal.h"

namespace pg {

constexpr uint64_t NSLOT = 8;            // pinned slots of the ring (at most)

struct HostPool {
  int device = 0;
  unsigned nworkers = 0;                 // memcpy threads besides the stager
  std::vector<std::thread> workers;
  std::thread stager;
  std::mutex mu;
  std::condition_variable cv;            // workers and stager: new work, consumption, stop
  std::condition_variable cv_main;       // the caller: chunks queued, job done
  bool stop = false;

  // one parallel memcpy at a time (the stager's), tagged by generation
  uint8_t* cp_dst = nullptr;
  const uint8_t* cp_src = nullptr;
  uint64_t cp_len = 0, cp_part = 0;
  uint32_t cp_parts = 0, cp_gen = 0;
  std::atomic<uint64_t> cp_next{0};      // (generation << 32) | next part
  std::atomic<uint32_t> cp_done{0};

  // the current upload
  bool job = false, abort = false, failed = false;
  uint8_t* dst = nullptr;
  const uint8_t* src = nullptr;
  uint64_t n = 0, nch = 0, nslots = 0, S = 0;          // S: bytes per slot (one piece)
  std::vector<uint64_t> bounds;          // chunk i = [bounds[i], bounds[i+1])
  uint8_t* slots = nullptr;              // the ring (allocated when a chunk is staged)
  PinBuf* pin = nullptr;
  bool reg = false;                      // register chunks and DMA them directly
  std::vector<uint8_t*> registered;
  hipEvent_t slot_ev[NSLOT] = {};        // each slot's last DMA
  hipStream_t stream = nullptr;
  hipEvent_t* cev = nullptr;
  uint64_t queued = 0, consumed = 0;
  std::string err;

  void run_parts(uint32_t gen, uint8_t* d, const uint8_t* s, uint64_t len, uint64_t part, uint32_t parts) {
    for (;;) {
      uint64_t v = cp_next.load(std::memory_order_acquire);
      if ((uint32_t)(v >> 32) != gen || (uint32_t)v >= parts) return;
      if (!cp_next.compare_exchange_weak(v, v + 1, std::memory_order_acq_rel)) continue;
      const uint64_t a = (uint64_t)(uint32_t)v * part, b = std::min(len, a + part);
      if (b > a) std::memcpy(d + a, s + a, b - a);
      cp_done.fetch_add(1, std::memory_order_release);
    }
  }

  void worker_main() {
    uint32_t seen = 0;
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return stop || cp_gen != seen; });
      if (stop) return;
      seen = cp_gen;
      uint8_t* d = cp_dst;
      const uint8_t* s = cp_src;
      const uint64_t len = cp_len, part = cp_part;
      const uint32_t parts = cp_parts;
      lk.unlock();
      run_parts(seen, d, s, len, part, parts);
      lk.lock();
    }
  }

  // memcpy of len bytes by the stager and every worker (called by the stager only)
  void par_copy(uint8_t* d, const uint8_t* s, uint64_t len) {
    const uint64_t unit = 1ull << 20;
    uint32_t parts = (uint32_t)std::min<uint64_t>(4ull * (nworkers + 1), (len + unit - 1) / unit);
    if (parts < 1) parts = 1;
    const uint64_t part = ((len + parts - 1) / parts + 4095) & ~4095ull;
    uint32_t gen;
    {
      std::lock_guard<std::mutex> g(mu);
      cp_dst = d; cp_src = s; cp_len = len; cp_part = part; cp_parts = parts;
      cp_done.store(0, std::memory_order_relaxed);
      gen = ++cp_gen;
      cp_next.store((uint64_t)gen << 32, std::memory_order_release);
    }
    if (nworkers) cv.notify_all();
    run_parts(gen, d, s, len, part, parts);
    while (cp_done.load(std::memory_order_acquire) < parts) std::this_thread::yield();
  }

  void stager_main() {
    (void)hipSetDevice(device);
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return stop || job; });
      if (stop) return;
      uint64_t piece = 0;                // pieces queued so far (slot = piece % nslots)
      // (a slot may still feed a DMA of an upload that was abandoned)
      for (auto ev : slot_ev) (void)hipEventSynchronize(ev);
      for (uint64_t i = 0; i < nch; ++i) {
        // cev[i & 15] is recorded again only after the caller queued its wait
        // on chunk i - 16
        cv.wait(lk, [&] { return stop || abort || i < consumed + 16; });
        if (stop || abort) break;
        lk.unlock();
        std::string e;
        try {
          // the chunk in pieces of one slot: the DMA of a piece starts as
          // soon as it is in pinned memory, so the ring fills in one piece's
          // copy time and the link never waits for a whole chunk
          const uint64_t off = bounds[i], len = bounds[i + 1] - bounds[i];
          bool direct = false;
          if (reg) {
            // register the chunk's pages for this upload and DMA them directly:
            // one pass over host memory instead of three, and no copy ahead of
            // the link; re-registering pages the runtime has seen is nearly free
            uint8_t* p = const_cast<uint8_t*>(src + off);
            const uint64_t rl = (len + 4095) & ~4095ull;
            if (((uintptr_t)p & 4095) == 0 && hipHostRegister(p, rl, hipHostRegisterReadOnly) == hipSuccess) {
              registered.push_back(p);
              PG_HIP(hipMemcpyAsync(dst + off, p, len, hipMemcpyHostToDevice, stream));
              direct = true;
            } else {
              (void)hipGetLastError();
              reg = false;                 // the rest goes through the ring
            }
          }
          if (!direct && !slots) {
            pin->reserve(nslots * S);
            slots = pin->as<uint8_t>();
          }
          for (uint64_t po = 0, pl; !direct && po < len; po += pl, ++piece) {
            // the first pieces small (2, 4, 8 ... MiB up to a slot): the link
            // starts after one small copy instead of a whole slot's
            pl = std::min<uint64_t>(std::min<uint64_t>(S, len - po), piece < 8 ? (uint64_t)(2ull << 20) << piece : S);
            const uint64_t slot = piece % nslots;
            if (piece >= nslots) PG_HIP(hipEventSynchronize(slot_ev[slot]));   // the slot's last DMA
            par_copy(slots + slot * S, src + off + po, pl);
            PG_HIP(hipMemcpyAsync(dst + off + po, slots + slot * S, pl, hipMemcpyHostToDevice, stream));
            PG_HIP(hipEventRecord(slot_ev[slot], stream));
          }
          PG_HIP(hipEventRecord(cev[i & 15], stream));
        } catch (const std::exception& x) {
          e = x.what();
        }
        lk.lock();
        if (!e.empty()) {
          failed = true;
          err = e;
          break;
        }
        queued = i + 1;
        cv_main.notify_all();
      }
      if (!registered.empty()) {         // the DMAs done, the pages released
        lk.unlock();
        (void)hipStreamSynchronize(stream);
        for (auto p : registered) (void)hipHostUnregister(p);
        registered.clear();
        lk.lock();
      }
      job = false;                       // the source is no longer read
      cv_main.notify_all();
    }
  }
};

static unsigned default_threads() {
  cpu_set_t set;
  CPU_ZERO(&set);
  unsigned cpus = 8;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) cpus = (unsigned)CPU_COUNT(&set);
  return std::max(1u, std::min(8u, cpus / 2));
}

static HostPool* pool_of(Ctx& c) {
  const unsigned want = c.host_threads ? (unsigned)c.host_threads : default_threads();
  if (c.pool && c.pool->nworkers + 1 == want) return c.pool;
  pool_destroy(c);
  auto* P = new HostPool();
  P->device = c.device;
  for (auto& e : P->slot_ev) PG_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  P->nworkers = want - 1;
  for (unsigned t = 0; t < P->nworkers; ++t) P->workers.emplace_back([P] { P->worker_main(); });
  P->stager = std::thread([P] { P->stager_main(); });
  c.pool = P;
  return P;
}

void pool_destroy(Ctx& c) {
  HostPool* P = c.pool;
  if (!P) return;
  {
    std::lock_guard<std::mutex> g(P->mu);
    P->stop = true;
  }
  P->cv.notify_all();
  for (auto& t : P->workers) t.join();
  P->stager.join();
  for (auto e : P->slot_ev)
    if (e) (void)hipEventDestroy(e);
  delete P;
  c.pool = nullptr;
}

static bool is_pinned(const void* p) {
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

static std::vector<uint64_t> uniform_bounds(uint64_t n, uint64_t chunk) {
  std::vector<uint64_t> b{0};
  for (uint64_t o = 0; o < n; o += chunk) b.push_back(std::min(n, o + chunk));
  return b;
}

Upload::Upload(Ctx& c, uint8_t* dst, const uint8_t* src, uint64_t n, uint64_t chunk)
    : Upload(c, dst, src, n, uniform_bounds(n, chunk)) {}

Upload::Upload(Ctx& c, uint8_t* dst, const uint8_t* src, uint64_t n, std::vector<uint64_t> bounds)
    : c_(c), dst_(dst), src_(src), nch_(n ? bounds.size() - 1 : 0), bounds_(std::move(bounds)) {
  staged = nch_ && !(is_pinned(src) && is_pinned(src + n - 1));
  if (!staged) return;
  const uint64_t S = std::min(c.stage_piece, n);
  const uint64_t nslots = std::min<uint64_t>(std::min<uint64_t>(NSLOT, c.stage_slots),
                                             (n + S - 1) / S);
  if (!c.host_register) c.stage_pin.reserve(nslots * S);
  P_ = pool_of(c);
  std::lock_guard<std::mutex> g(P_->mu);
  P_->dst = dst; P_->src = src; P_->n = n; P_->bounds = bounds_; P_->nch = nch_;
  P_->nslots = nslots;
  P_->S = S;
  P_->slots = c.host_register ? nullptr : c.stage_pin.as<uint8_t>();
  P_->pin = &c.stage_pin;
  P_->reg = c.host_register != 0;
  P_->stream = c.stream3;
  P_->cev = c.cev;
  P_->queued = P_->consumed = 0;
  P_->abort = P_->failed = false;
  P_->err.clear();
  P_->job = true;
  P_->cv.notify_all();
}

void Upload::wait_queued(uint64_t i) {
  if (!staged) {
    // copies run up to 8 chunks ahead of the caller (an event is recorded
    // again only after the caller's wait on it was queued)
    while (issued_ < nch_ && issued_ < i + 8) {
      const uint64_t off = bounds_[issued_], len = bounds_[issued_ + 1] - off;
      PG_HIP(hipMemcpyAsync(dst_ + off, src_ + off, len, hipMemcpyHostToDevice, c_.stream3));
      PG_HIP(hipEventRecord(c_.cev[issued_ & 15], c_.stream3));
      ++issued_;
    }
    return;
  }
  std::unique_lock<std::mutex> lk(P_->mu);
  P_->cv_main.wait(lk, [&] { return P_->failed || P_->queued > i; });
  if (P_->failed) throw Error(-5, "host upload: " + P_->err);
}

void Upload::consumed(uint64_t i) {
  if (!staged) return;
  {
    std::lock_guard<std::mutex> g(P_->mu);
    P_->consumed = i + 1;
  }
  P_->cv.notify_all();
}

void Upload::finish() {
  if (!staged || done_) return;
  std::unique_lock<std::mutex> lk(P_->mu);
  P_->cv_main.wait(lk, [&] { return !P_->job; });
  done_ = true;
  if (P_->failed) throw Error(-5, "host upload: " + P_->err);
}

Upload::~Upload() {
  if (!staged || done_) return;
  std::unique_lock<std::mutex> lk(P_->mu);
  P_->abort = true;
  P_->cv.notify_all();
  P_->cv_main.wait(lk, [&] { return !P_->job; });
}

}  // namespace pg
