// pg_internal.h — host-side context shared by the pangenome HIP translation
// units.  Not part of the public ABI (include/pangenome.h is).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <functional>
#include <vector>

#include "pg_common.h"

namespace pg {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define PG_HIP(x)                                                                       \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess)                                                               \
      throw ::pg::Error(-5, std::string(#x) + ": " + hipGetErrorString(e_));            \
  } while (0)

// Device bytes held by every DevBuf of the process, their peak, and an
// optional cap (pg_tune PG_TUNE_DEVICE_CAP: tests of the memory budget of a
// path at a scaled-down size; 0 = none).
struct DevBytes {
  static std::atomic<uint64_t>& cur() { static std::atomic<uint64_t> v{0}; return v; }
  static std::atomic<uint64_t>& peak() { static std::atomic<uint64_t> v{0}; return v; }
  static std::atomic<uint64_t>& cap() { static std::atomic<uint64_t> v{0}; return v; }
  static void add(uint64_t b) {
    const uint64_t now = cur().fetch_add(b) + b;
    uint64_t pk = peak().load();
    while (now > pk && !peak().compare_exchange_weak(pk, now)) {}
  }
  // pg_tune PG_TUNE_POISON (debug): every new allocation is filled with this
  // byte (-1 = off), so a read of memory no kernel wrote shows up as a
  // different result instead of inheriting an earlier run's bytes
  static std::atomic<int>& poison() { static std::atomic<int> v{-1}; return v; }
};

// A growable device buffer (never shrinks; reused across calls so the steady
// state does no hipMalloc).
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }                // (function-local scratch buffers free themselves)
  void reserve(size_t bytes) {
    if (bytes <= cap) return;
    release();
    size_t nb = bytes + bytes / 8 + 256;
    const uint64_t lim = DevBytes::cap().load();
    if (lim && DevBytes::cur().load() + nb > lim)
      throw Error(-12, "device memory cap: " + std::to_string(DevBytes::cur().load() + nb) + " > " +
                           std::to_string(lim) + " bytes");
    const hipError_t e = hipMalloc(&p, nb);
    if (e != hipSuccess) {
      p = nullptr;
      (void)hipGetLastError();
      throw Error(e == hipErrorOutOfMemory ? -12 : -5,
                  std::string("hipMalloc of ") + std::to_string(nb) + " bytes (" +
                      std::to_string(DevBytes::cur().load()) + " held by the library): " + hipGetErrorString(e));
    }
    cap = nb;
    DevBytes::add(nb);
    const int pv = DevBytes::poison().load();
    if (pv >= 0) {
      PG_HIP(hipMemset(p, pv, nb));
      PG_HIP(hipDeviceSynchronize());
    }
  }
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
  void release() {
    if (p) {
      (void)hipFree(p);
      DevBytes::cur().fetch_sub(cap);
    }
    p = nullptr;
    cap = 0;
  }
};

// A growable pinned host buffer: device-to-host copies into it are plain DMA
// on the stream (a pageable destination costs a staged, synchronous copy).
struct PinBuf {
  void* p = nullptr;
  void* dp = nullptr;             // device view (coherent buffers written by kernels)
  size_t cap = 0;
  unsigned flags = hipHostMallocDefault;
  void reserve(size_t bytes) {
    if (bytes <= cap) return;
    if (p) PG_HIP(hipHostFree(p));
    p = dp = nullptr;
    size_t nb = bytes + bytes / 8 + 256;
    PG_HIP(hipHostMalloc(&p, nb, flags));
    if (flags & hipHostMallocMapped) PG_HIP(hipHostGetDevicePointer(&dp, p, 0));
    cap = nb;
  }
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Per-kernel timing on the context's stream (HIP events), so callers can
// price the dominant kernel against the HBM roofline.
// (off: no event is recorded and ms() is 0 - PG_TUNE_TIMERS 0, to price the
// timing events themselves)
struct Timer {
  hipEvent_t a = nullptr, b = nullptr;
  bool off = false;
  void init() {
    if (!a) { PG_HIP(hipEventCreate(&a)); PG_HIP(hipEventCreate(&b)); }
  }
  void start(hipStream_t s) { if (!off) PG_HIP(hipEventRecord(a, s)); }
  void stop(hipStream_t s) { if (!off) PG_HIP(hipEventRecord(b, s)); }
  double ms() {
    if (off) return 0.0;
    float t = 0;
    PG_HIP(hipEventSynchronize(b));
    PG_HIP(hipEventElapsedTime(&t, a, b));
    return (double)t;
  }
  void destroy() {
    if (a) { (void)hipEventDestroy(a); (void)hipEventDestroy(b); }
    a = b = nullptr;
  }
};

struct HostPool;                  // pg_stage.hip: the pinned staging ring's threads

struct Ctx {
  int device = 0;
  int k = 27;
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;  // side stream: K3 work passes overlap the next coverage pass
  hipStream_t stream3 = nullptr;  // copy stream: chunked host uploads (pg_parse_host, pg_build_host)
  hipStream_t stream_hi = nullptr; // high priority: K1's header pass and record table beside the emission
  hipEvent_t ev[16] = {};         // ordering events between the two streams
  hipEvent_t ext_ev = nullptr;    // pg_stream_wait: the caller's stream's queued work, waited on by ours
  hipEvent_t rec_ev = nullptr;    // the record table's copy to the host (K1)
  hipEvent_t cev[16] = {};        // chunk-landed events of the copy stream
  int n_cu = 256;                 // compute units (persistent-kernel grids)
  int k3_chunks = 0;              // pg_tune: K3 chunks (0 = by tile count)
  int k3_wblk = 0;                // pg_tune: work blocks per CU, low 4 bits; last chunk's, high 4 bits (0 = 2)
  int k3_emit = 0;                // pg_tune: work pass (0 = two halves per segment, 1 = one)
  int k1_form = 0;                // pg_tune: K1 form bits (PG_TUNE_K1; default: the per-step span pass)
  int k3_tail = 0;                // pg_tune: last K3 chunk in 16ths of the others (0 = 10)
  int k3_head = 0;                // pg_tune: first K3 chunk in 16ths of the others (0 = 16)
  int k3_cover = 0;               // pg_tune: coverage pass (0 = packed form, 1 = LDS-staged members, 2 = quad form)
  int k3_anchors = 0;             // pg_tune: packed coverage pass anchors per tile and reference (0 = 4)
  int early_split = 1;            // pg_tune: pg_build_host splits each landed chunk's records (stage B under the upload)
  uint64_t h2d_chunk = 64ull << 20;   // pg_tune: bytes per H2D chunk of pg_parse_host
  uint64_t h2d_tail = 0;              // pg_tune: bytes of pg_build_host's last H2D chunk (0: uniform chunks)
  int host_threads = 0;           // pg_tune: memcpy threads of the staging ring (0 = by CPU affinity)
  uint64_t stage_piece = 32ull << 20;  // pg_tune: bytes per staging-ring slot (one DMA)
  uint64_t stage_slots = 4;       // pg_tune: staging-ring slots (2..8)
  int host_register = 1;          // pg_tune: register pageable chunks and DMA them (0: staging ring only)
  HostPool* pool = nullptr;       // staging ring threads (created on the first pageable upload)
  PinBuf stage_pin;               // staging ring slots
  int bb_shift = 0;               // pg_tune: table bits below the sized ones (tests of the overflow paths)
  uint64_t region_cap_force = 0;  // pg_tune: first stage A region size (tests of the re-run path)

  // ---- input FASTA (device-resident; either owned or borrowed)
  DevBuf fasta_own;
  const uint8_t* d_fasta = nullptr;
  uint64_t n_bytes = 0;

  // ---- parse products (K1)
  DevBuf span_sum, span_start;    // per 16 KiB wave span: function / inclusive prefix (K1)
  DevBuf n_sel;                   // device counters
  DevBuf rec_start, rec_len;      // int64 per record: compacted offset / length
  DevBuf rec_hdr, rec_ptr;        // int64 per record: header byte span packed, `ptr` emulation
  DevBuf rec_flag;                // uint8 per record: take part in the current pass
  DevBuf cls;                     // uint8 per base: class code (records concatenated); K1 writes only
                                  // the 16-base chunks with an exception or shared by two spans
  DevBuf p2;                      // uint32 per 16 bases: 2-bit codes (class & 3), the packed base stream
  DevBuf e16;                     // uint8 per 16 bases: nonzero if any is not ACGT
  bool cls_full = false;          // every chunk of `cls` written (ensure_cls)
  // ---- routed exchange (pg_route_*): the last build's stage A records held
  // in their regions for their owners instead of stages B/C
  bool route_req = false;         // the next build_dbg stops after stage A
  bool route_ready = false;       // stage A records held (route_reg: per region, clipped)
  uint64_t route_total = 0, route_maxreg = 0, route_maxbin = 0;
  unsigned route_sentinel = 0;
  std::vector<uint64_t> route_reg;
  DevBuf route_buf;               // region offsets and owner sums of pg_route_scatter
  PinBuf route_pin;
  uint64_t n_cls = 0;             // length of the compacted stream (bases before the first header too)
  DevBuf scratch;                 // rocPRIM temp storage
  DevBuf rec_pack;                // the scan total + int64 [5][rec_cap]: the record table for one copy
  uint64_t rec_cap = 0;           // record arrays sized for the last parse's record count
  PinBuf h_pin;                   // pinned staging for small device-to-host reads
  uint64_t n_lines = 0, n_records = 0, n_bases = 0, n_nl = 0;
  std::vector<int64_t> h_rec_start, h_rec_len, h_rec_hdr_start, h_rec_hdr_len, h_rec_ptr;
  bool parsed = false;

  // ---- dBG table (K3 stage C) and rdBG (fused K5)
  DevBuf table;                   // primary buckets (2 x 64-bit words each)
  DevBuf ovf;                     // overflow slots (16 B)
  TableView tv{};                 // hash (fixed by k) and current geometry (pg_common.h)
  int kb = 0, cbits = 0, hash_k = 0, bb = 0;   // key bits, coarse bin bits, k of tv's hash, bucket bits
  uint64_t cap = 0;               // primary buckets (power of two)
  uint64_t ovf_cap = 0;           // overflow slots (power of two)
  PinBuf h_out{nullptr, nullptr, 0, hipHostMallocMapped | hipHostMallocCoherent};   // k_gather_out's target
  std::vector<uint8_t> dev_flag;  // the record flags last uploaded to rec_flag (at dev_flag_p)
  const void* dev_flag_p = nullptr;
  bool t1_open = false;           // stage A queued, its side stream not yet joined (finish_build joins)
  DevBuf flags;                   // [0] sentinel seen, [1] stage A bits, [4] stage B/C bits
  uint64_t n_dbg = 0, n_rdbg = 0, n_canon = 0, sentinel = 0;
  bool built = false, reduced = false;
  int rc0 = 1;
  uint64_t windows_fw = 0, windows_total = 0;

  // ---- partitioned build (pg_dbg.hip)
  DevBuf recA_key, recA_mw, ctrA;     // stage A: records per (coarse bin, XCD) region and cursors
  uint64_t capA = 0;                  // records per stage A region
  DevBuf recS_key[2], recS_mw[2];     // stage B outputs (ping-pong)
  DevBuf ctrS;                        // stage B cursors, all levels
  DevBuf snapA;                       // pg_build_host's early split: stage A cursors already split
  double w_ratio = 0;                 // last host build: forward windows per input byte
  bool early_split_used = false;      // the last pg_build_host's stage C read the early split's partitions
  int bc_attempts = 0;                // stages B/C runs of the last build (1: no re-run)
  int split_passes = 0;               // stage B k_split passes of the last build (0: split under the upload)
  // the largest partition of each split level that a build had to re-run
  // for (at table bits lv_keep_bb): later builds' plans start from them
  std::vector<uint64_t> lv_keep;
  int lv_keep_bb = -1;
  DevBuf rseg;                        // rdBG keys: one segment of rseg_cap per stage C block
  DevBuf k5_ctr;                      // per stage C block: key / dBG / member counts
  uint64_t rseg_cap = 0, rseg_nseg = 0;
  std::vector<uint64_t> rseg_cnt;     // members per segment
  uint64_t n_records_a = 0;           // stage A records of the last build
  double u_ratio = 0, r_ratio = 0;    // last build: records per forward window, rdBG keys per record

  // ---- K3 tiles
  DevBuf tile_sched;              // per-stripe tile offsets + record order (k_tiles input)
  PinBuf tile_pin;
  uint64_t n_tiles = 0;
  int tile_k = 0;
  int k3_ref = -1;                // k_cover's dedup reference record (the lead), -1: none
  int k3_ref2 = -1;               // k_cover's second reference record, -1: none
  DevBuf part_cnt;                // multi-GPU partition: owner counts and cursors
  uint64_t part_counts[64] = {};  // counts of the last count pass
  uint64_t part_sums[64] = {};    // row_check sums of the last scatter's runs
  uint64_t merge_sum = 0, merge_rows = 0;   // the last merge: row_check sum / non-empty records it read
  uint64_t work_items = 0;        // the last build's work-pass items (segments the coverage pass left)
  uint64_t part_total = 0;
  int part_nparts = 0;
  uint64_t part_gen = ~0ull;      // build_gen of the table the counts are for
  uint64_t build_gen = 0;         // bumped by every table build / merge
  DevBuf k3_hint;                 // int32 [8 XCDs][2 references][R]: last drift k_cover found
  DevBuf tile_desc;               // tile descriptors (record start / length / index / stripe)
  DevBuf k3_queue;                // segments left with work after the coverage pass, + counters
  std::vector<int64_t> tile_sig_len;   // record lengths / flags the tile list was built for
  std::vector<uint8_t> tile_sig_flag;

  // ---- walk passes (edges / labels)
  DevBuf tile_cnt, tile_off;      // per tile x strand counts / offsets
  DevBuf occ;                     // member / hit occurrences, walk ordered
  DevBuf edge_tab, pair_tab;      // edge table and (edge, walk) dedup set
  DevBuf edge_out;                // compacted edge slots
  DevBuf edge_exp;                // edges in first-occurrence order: [n][4] tuple, [n] count, [n] first walk
  uint64_t edge_cap = 0, pair_cap = 0, n_edges = 0;
  DevBuf lab_tab;                 // label table (hash of (key, value) -> label)
  uint64_t lab_cap = 0;
  DevBuf lab_list;                // the labels in order: [n] key, [n] value, [n] label
  uint64_t n_labels = 0;
  DevBuf rows_buf;                // rows of the last row pass: [n][5] int64
  uint64_t n_rows = 0;
  // text of the last edge or row pass (pg_edges_format / pg_rows_format)
  DevBuf text_len, text_off, text_buf, text_names;
  uint64_t text_total = 0;
  bool text_xyz = false, text_rows = false;

  // ---- npz persistence (pg_persist.hip)
  DevBuf preload;                 // staged PreEnt pairs, OR-merged by every build
  uint64_t n_preload = 0;
  std::vector<uint8_t> last_flag; // record flags / extra empties / strands of the last build
  int last_extra = 0;
  DevBuf dump_cnt;                // uint32 occurrence count per (entry, orientation) of the last build
  std::vector<PinBuf> dump_pin;   // pg_dbg_dump_fd: one pinned piece buffer per writer thread
  bool dump_ready = false;
  uint64_t dump_size = 0, dump_sentinel = 0;

  // timings of the last calls (ms, HIP events on `stream`)
  Timer t0, t1, t6;
  double ms_parse = 0, ms_clear = 0, ms_insert = 0, ms_short = 0, ms_scan = 0, ms_split = 0, ms_range = 0;
  double ms_total_build = 0;

  // Wait for the stream by polling it: the blocking wait's wake-up costs
  // ~20-30 us per host round trip on the build's critical path (two per
  // build).  After 50 ms of polling it blocks (long waits, and errors come
  // back through the blocking call).
  void sync() {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const hipError_t e = hipStreamQuery(stream);
      if (e == hipSuccess) return;
      if (e != hipErrorNotReady) break;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) break;
    }
    PG_HIP(hipStreamSynchronize(stream));
  }
};

// pg_stage.hip
// One chunked upload of n host bytes to dst on c.stream3: chunk i's copy is
// marked by c.cev[i & 15] on stream3 once wait_queued(i) returns.  A
// pageable source goes through the pinned staging ring (a stager thread and
// its memcpy pool); a pinned one is DMA'd directly, up to 8 chunks ahead.
// The source is read until finish() (or the destructor) returns.
class Upload {
 public:
  Upload(Ctx& c, uint8_t* dst, const uint8_t* src, uint64_t n, uint64_t chunk);
  // chunk i = bytes [bounds[i], bounds[i+1]) (bounds[0] = 0, back() = n)
  Upload(Ctx& c, uint8_t* dst, const uint8_t* src, uint64_t n, std::vector<uint64_t> bounds);
  uint64_t off(uint64_t i) const { return bounds_[i]; }
  uint64_t len(uint64_t i) const { return bounds_[i + 1] - bounds_[i]; }
  ~Upload();
  Upload(const Upload&) = delete;
  Upload& operator=(const Upload&) = delete;
  uint64_t chunks() const { return nch_; }
  void wait_queued(uint64_t i);   // chunk i's copy is queued and c.cev[i & 15] recorded
  void consumed(uint64_t i);      // the caller has queued its wait on c.cev[i & 15]
  void finish();                  // every chunk queued; rethrows a stager error
  bool staged = false;            // through the pinned ring

 private:
  Ctx& c_;
  uint8_t* dst_;
  const uint8_t* src_;
  uint64_t nch_;
  std::vector<uint64_t> bounds_;
  HostPool* P_ = nullptr;
  uint64_t issued_ = 0;
  bool done_ = false;
};
void pool_destroy(Ctx& c);

// pg_parse.hip
// h_src: host bytes, uploaded in chunks pipelined with K1.  on_chunk (host
// input only): called after each chunk with the number of records complete
// so far (their lengths in c.h_rec_len, c.n_records = that count), and once
// at the end with all of them; it may enqueue work on c.stream.
void parse_fasta(Ctx& c, const uint8_t* h_src = nullptr, const std::function<void(uint64_t)>* on_chunk = nullptr);
// the class bytes of every chunk K1 left packed (e16 == 0), once per parse,
// on c.stream: for the passes that read `cls` directly (walks, checkpoints)
void ensure_cls(Ctx& c);
inline PackedCls packed_cls(Ctx& c) { return PackedCls{c.cls.as<uint8_t>(), c.p2.as<uint32_t>(), c.e16.as<uint8_t>()}; }
// pg_build_host: parse of host bytes with stage A of the build streamed under
// the upload (every record, no -n / checkpoint plan), then stages B and C
void build_host(Ctx& c, const uint8_t* h_src, uint64_t n, int rc0);
// pg_dbg.hip
void build_dbg(Ctx& c, const uint8_t* h_rec_flag, int extra_empty, int rc0);
void build_rdbg(Ctx& c);
uint64_t export_dbg(Ctx& c, uint64_t* h_keys, uint16_t* h_masks, uint64_t cap);
uint64_t export_rdbg(Ctx& c, uint64_t* h_keys, uint64_t cap);
uint64_t partition_dbg(Ctx& c, int nparts, void* d_out, uint64_t out_cap, uint64_t* h_counts);
void merge_dbg(Ctx& c, const void* d_pairs, uint64_t n, uint64_t cap_hint, int sentinel, int rot = -1);
void merge_dbg_segs(Ctx& c, const void* const* segs, const uint64_t* ns, int nseg, int sentinel, int rot);
// routed exchange: owners of the held stage A records (2^lg owners)
void route_counts(Ctx& c, int lg, uint64_t* counts);
void route_scatter(Ctx& c, int lg, void* d_out, uint64_t out_cap, uint64_t* sums);
void route_finish(Ctx& c);
void rows_checksum(Ctx& c, const void* d_rows, const uint64_t* off, uint64_t nseg, uint64_t* sums, bool row12 = false);
// pg_persist.hip
struct PreEnt {                   // one staged oakht slot: oriented key, 12-bit mask, count
  unsigned long long key;
  uint32_t mask, count;
};
void dbg_load(Ctx& c, const uint64_t* keys, const uint16_t* masks, const uint8_t* counts, uint64_t n);
uint64_t dbg_dump(Ctx& c, uint64_t& capacity, uint64_t* keys, uint16_t* values, uint8_t* counts);
uint64_t dbg_dump_fd(Ctx& c, uint64_t& capacity, int fd, const uint64_t* off, uint32_t* crc);
// n device bytes to descriptor fd at its position (pg_edges_format_fd, pg_rows_format_fd)
void text_to_fd(Ctx& c, const uint8_t* src, uint64_t n, int fd, const char* what);
uint64_t oakht_capacity(uint64_t size);
// pg_walk.hip
uint64_t walk_edges(Ctx& c, const uint8_t* h_rec_flag, int rc1);
void export_edges(Ctx& c, uint64_t* tuples, int64_t* counts, int64_t* first_walk, uint64_t cap);
void set_labels(Ctx& c, const int64_t* key, const int64_t* val, const int64_t* id, uint64_t n);
uint64_t walk_rows(Ctx& c, const uint8_t* h_rec_flag, int rc1);
void export_rows(Ctx& c, int64_t* rows5, uint64_t cap);
uint64_t format_edges(Ctx& c, char* out, uint64_t cap, int fd = -1);
uint64_t labels_from_edges(Ctx& c, const uint64_t* h_tuples, uint64_t n_edges, const int64_t* mk, const int64_t* mv,
                           const int64_t* mi, uint64_t n_mcl, int64_t next_id);
void export_labels(Ctx& c, int64_t* key, int64_t* val, int64_t* id, uint64_t cap);
uint64_t format_rows_text(Ctx& c, const char* names, const int64_t* name_off, uint64_t n_names, char* out,
                          uint64_t cap, int fd = -1);

// helpers
inline uint64_t next_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}
inline int log2u(uint64_t p) {
  int b = 0;
  while ((1ull << b) < p) ++b;
  return b;
}

// Bits of a k-mer key: keys < 5^k <= 2^kb.
inline int key_bits(int k) {
  uint64_t maxkey = 1;
  for (int i = 0; i < k; ++i) maxkey *= 5;
  return std::max(1, log2u(maxkey));
}

// The hash of a table for k-mers of length k (a bijection of kb-bit keys,
// fixed by k: records carry h = perm(c) before the table is sized) and the
// reverse-complement constants; the bucket geometry comes from set_geometry.
inline TableView make_hash(int k, int& kb) {
  kb = key_bits(k);
  TableView t{};
  t.kmask = kb >= 64 ? ~0ull : ((1ull << kb) - 1ull);
  t.sh1 = std::max(1, kb / 2);
  t.sh2 = std::max(1, kb / 3);
  auto inv = [](uint64_t m) {                                 // inverse of odd m mod 2^64
    uint64_t x = m;
    for (int i = 0; i < 6; ++i) x *= 2 - m * x;
    return x;
  };
  t.m1 = (0x9E3779B97F4A7C15ull & t.kmask) | 1ull;
  t.m2 = (0xC2B2AE3D27D4EB4Full & t.kmask) | 1ull;
  t.m1i = inv(t.m1) & t.kmask;
  t.m2i = inv(t.m2) & t.kmask;
  rc_constants(k, t.rc_pad, t.rc_inv);
  return t;
}
// 2^bb buckets (kb - 38 <= bb <= kb: the quotient kb - bb plus the 26 mask
// bits fit one 64-bit word) and `ovf_slots` (a power of two) overflow slots.
inline void set_geometry(TableView& t, int kb, int bb, uint64_t ovf_slots) {
  t.bmask = (1ull << bb) - 1ull;
  t.qbits = (uint32_t)(kb - bb);
  t.omask = ovf_slots - 1;
}
inline unsigned grid_for(uint64_t n, unsigned block, unsigned cap = 65536u) {
  uint64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

}  // namespace pg
