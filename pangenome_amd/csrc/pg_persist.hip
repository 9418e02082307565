// pg_persist.hip — the dBG's npz side file: dump() / load_on_disk()
// (kmer_numba.py:243-335), written as a slot layout the reference's oakht
// accepts, and loaded back as staged pairs the next build OR-merges.
//
// Dump = three passes over the last build, outside the timed K3 path:
//   k_count_windows / k_count_short   every window of the build again: one
//       atomicAdd on its (table entry, orientation) counter — the oakht's
//       `counts` are occurrences per oriented key (__setitem__ :556),
//       something the OR-table does not keep;
//   k_count_staged   staged npz slots add their own counts (-r resume);
//   k_dump_list / k_dump_propose / k_dump_claim   each present oriented key
//       takes a free slot of oakht.pointer's probe sequence (:521-538): j =
//       FNV-1a(low 4 key bytes) mod capacity, then j, j+1, j+4, j+9, ... .
//       Any insertion order gives a layout lookups accept (a key's earlier
//       probes were occupied when it was placed and nothing is ever removed);
//       rounds in which the smallest proposing key takes each slot make it
//       the same layout on every run.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>

#include "pg_internal.h"

namespace pg {

constexpr int PBLK = 256;
constexpr int CW = 16;                              // windows per thread
constexpr uint64_t CCHUNK = (uint64_t)PBLK * CW;   // windows per block

__device__ __forceinline__ void count_at(const TableView& T, unsigned* cnt, uint64_t c, int orient, unsigned add) {
  const uint64_t e = tab_find(T, c);
  if (e != ~0ull) atomicAdd(cnt + 2 * e + orient, add);
}
// both orientation counters of c's entry at once (one lookup, one 64-bit
// atomic: the low word is orientation 0, the high word orientation 1; a
// counter stays far below 2^32, so no carry crosses into the other)
__device__ __forceinline__ void count_pair(const TableView& T, unsigned* cnt, uint64_t c, unsigned long long add) {
  const uint64_t e = tab_find(T, c);
  if (e != ~0ull) atomicAdd(reinterpret_cast<unsigned long long*>(cnt) + e, add);
}

// windows [j*CCHUNK, (j+1)*CCHUNK) of record r (n >= k+2): the forward
// occurrence of key K and, with rc, the reverse strand's occurrence of its
// twin Kr (seq2dbg_jit_ :1215-1221 walks both strands).
template <bool RC>
__global__ void __launch_bounds__(PBLK)
k_count_windows(const uint8_t* __restrict__ cls, const unsigned long long* __restrict__ chunks,
                const long long* __restrict__ rec_start, const long long* __restrict__ rec_len, int k,
                uint64_t shift, TableView T, unsigned* __restrict__ cnt) {
  const unsigned long long ch = chunks[blockIdx.x];
  const int r = (int)(ch >> 32);
  const long long rs = rec_start[r], last = rec_len[r] - k;
  const long long q0 = (long long)(ch & 0xFFFFFFFFull) * (long long)CCHUNK + (long long)threadIdx.x * CW;
  const long long q1 = q0 + CW <= last + 1 ? q0 + CW : last + 1;
  if (q0 >= q1) return;
  const uint8_t* s = cls + rs;
  uint64_t K = 0, Kr = 0, pw = 1;
  for (int j = 0; j < k; ++j) {
    const uint32_t cj = s[q0 + j];
    K += (uint64_t)digit_fw(cj) * pw;
    Kr = Kr * 5 + digit_rc(cj);
    pw *= 5;
  }
  for (long long q = q0; q < q1; ++q) {
    if (q != q0) {
      const uint32_t dout = s[q - 1], din = s[q + k - 1];
      K = (K - digit_fw(dout)) * INV5 + (uint64_t)digit_fw(din) * shift;
      Kr = (Kr - (uint64_t)digit_rc(dout) * shift) * 5 + digit_rc(din);
    }
    const uint64_t c = K <= Kr ? K : Kr;
    // with rc a window and its twin add one to each orientation of c (a
    // palindrome: two to orientation 0); without, its own orientation
    const unsigned long long one = K <= Kr ? 1ull : 1ull << 32;
    count_pair(T, cnt, c, RC ? (K == Kr ? 2ull : 1ull | 1ull << 32) : one);
  }
}

__global__ void k_count_short(const uint8_t* __restrict__ cls, const long long* __restrict__ rec_start,
                              const long long* __restrict__ rec_len, const uint8_t* __restrict__ rec_flag,
                              uint64_t R, int k, uint64_t shift, int rc, TableView T, unsigned* __restrict__ cnt) {
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < R;
       r += (uint64_t)gridDim.x * blockDim.x) {
    const long long n = rec_len[r];
    if (!rec_flag[r] || n < k || n > k + 1) continue;
    auto emit = [&](uint64_t x, uint32_t) {
      const uint64_t xr = T.rc(x);
      count_at(T, cnt, x <= xr ? x : xr, x <= xr ? 0 : 1, 1u);
    };
    short_strand(cls, rec_start[r], n, 0, k, shift, emit);
    if (rc) short_strand(cls, rec_start[r], n, 1, k, shift, emit);
  }
}

__global__ void k_count_staged(const PreEnt* __restrict__ e, uint64_t n, TableView T, unsigned* __restrict__ cnt) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t x = e[i].key;
    if (x == SENTINEL) continue;
    const uint64_t xr = T.rc(x);
    count_at(T, cnt, x <= xr ? x : xr, x <= xr ? 0 : 1, e[i].count);
  }
}

__global__ void k_count_present(TableView T, uint64_t nw, uint64_t ntot, unsigned long long* __restrict__ out) {
  unsigned long long n = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < ntot;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t m = entry_mask(T, nw, i);
    n += (unsigned long long)((m & PRES_A) != 0) + (unsigned long long)((m & PRES_B) != 0);
  }
  for (int o = 32; o > 0; o >>= 1) n += __shfl_down(n, o, 64);
  if ((threadIdx.x & 63) == 0 && n) atomicAdd(out, n);
}

// oakht.fnv for ksize 1 (:400-418): FNV-1a over the key's low 4 bytes
__host__ __device__ __forceinline__ uint64_t oak_fnv(uint64_t x) {
  uint64_t a = 0xcbf29ce484222325ull;
  for (int i = 0; i < 4; ++i) {
    a ^= (x >> (8 * i)) & 0xFFull;
    a *= 0x100000001b3ull;
  }
  return a;
}

// The slot placement, deterministic: in rounds, every oriented key not yet
// placed proposes the first slot of its probe sequence that no earlier round
// filled (atomicMin of key + 1 on the slot's proposal word), and the
// smallest proposer takes each proposed slot; the others go on from there
// next round.  Which slot a key ends in depends only on the set of keys, not
// on the order threads run (one racing pass gave a different, equally valid
// layout per run), so two dumps of one build are byte-equal.
struct PendEnt {                                   // an oriented key waiting for its slot
  unsigned long long x;
  uint32_t vc;                                     // value | count << 16
  uint32_t probe;                                  // probe index kk of its next try
};
__global__ void k_dump_list(TableView T, uint64_t nw, uint64_t ntot, const unsigned* __restrict__ cnt,
                            PendEnt* __restrict__ out, unsigned long long* __restrict__ nout) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < ntot;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t m = entry_mask(T, nw, i);
    const uint32_t np = ((m & PRES_A) ? 1u : 0u) + ((m & PRES_B) ? 1u : 0u);
    if (!np) continue;
    const uint64_t c = entry_key(T, nw, i);
    unsigned long long at = atomicAdd(nout, (unsigned long long)np);
    for (int o = 0; o < 2; ++o) {
      if (!(m & (o ? PRES_B : PRES_A))) continue;
      const unsigned n = cnt[2 * i + o];
      const uint32_t v = (o ? (m >> B_SHIFT) : m) & MASK12;
      const uint32_t cn = n > 255u ? 255u : (n ? n : 1u);
      out[at++] = PendEnt{o ? T.rc(c) : c, v | (cn << 16), 0u};
    }
  }
}
__device__ __forceinline__ uint64_t oak_probe(uint64_t j0, uint64_t kk, uint64_t M) { return (j0 + kk * kk) % M; }

__global__ void k_dump_propose(PendEnt* __restrict__ e, uint64_t n, uint64_t M, const unsigned char* __restrict__ ocnts,
                               unsigned long long* __restrict__ prop, unsigned* __restrict__ fail) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    PendEnt p = e[i];
    const uint64_t j0 = oak_fnv(p.x) % M;
    uint64_t kk = p.probe;
    while (kk < M && ocnts[oak_probe(j0, kk, M)]) ++kk;     // (filled slots are final)
    if (kk >= M) { atomicOr(fail, 1u); continue; }
    e[i].probe = (uint32_t)kk;
    atomicMin(prop + oak_probe(j0, kk, M), p.x + 1ull);
  }
}
__global__ void k_dump_claim(const PendEnt* __restrict__ e, uint64_t n, uint64_t M,
                             const unsigned long long* __restrict__ prop, unsigned long long* __restrict__ okeys,
                             unsigned short* __restrict__ ovals, unsigned char* __restrict__ ocnts,
                             PendEnt* __restrict__ left, unsigned long long* __restrict__ nleft) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const PendEnt p = e[i];
    const uint64_t s = oak_probe(oak_fnv(p.x) % M, p.probe, M);
    if (prop[s] == p.x + 1ull) {                  // the smallest key that proposed s
      okeys[s] = p.x;
      ovals[s] = (unsigned short)(p.vc & 0xFFFFu);
      ocnts[s] = (unsigned char)(p.vc >> 16);
    } else {
      left[atomicAdd(nleft, 1ull)] = PendEnt{p.x, p.vc, p.probe + 1u};
    }
  }
}

// ---------------------------------------------------------------- host
// oakht.isprime / find_prime (:355-372), including 2 and 3 not being "prime"
static bool ref_isprime(uint64_t n) {
  if (n <= 1 || n % 2 == 0 || n % 3 == 0) return false;
  for (uint64_t i = 5; i * i <= n; i += 6)
    if (n % i == 0 || n % (i + 2) == 0) return false;
  return true;
}
static uint64_t ref_find_prime(uint64_t n) {
  for (uint64_t i = n; i < n + 70000000ull; ++i)
    if (ref_isprime(i)) return i;
  throw Error(-34, "find_prime: no prime in range");
}

uint64_t oakht_capacity(uint64_t size) {
  // init_dict(capacity=2**20) (:1242), then a resize to find_prime(int(N*1.62))
  // each time size / capacity exceeds the 0.75 load (:433, :551-558)
  uint64_t cap = ref_find_prime(1ull << 20);
  while ((double)size * 1.0 / (double)cap > 0.75) cap = ref_find_prime((uint64_t)((double)cap * 1.62));
  return cap;
}

void dbg_load(Ctx& c, const uint64_t* keys, const uint16_t* masks, const uint8_t* counts, uint64_t n) {
  c.n_preload = 0;
  if (!n) return;
  const uint64_t kmax = pow5(c.k);
  std::vector<PreEnt> h(n);
  for (uint64_t i = 0; i < n; ++i) {
    if (keys[i] != SENTINEL && keys[i] >= kmax)
      throw Error(-22, "pg_dbg_load: key " + std::to_string(keys[i]) + " is not a k=" + std::to_string(c.k) +
                           " k-mer");
    h[i] = PreEnt{keys[i], (uint32_t)(masks ? masks[i] & MASK12 : 0u), counts ? (uint32_t)counts[i] : 1u};
  }
  c.preload.reserve(sizeof(PreEnt) * n);
  PG_HIP(hipMemcpyAsync(c.preload.p, h.data(), sizeof(PreEnt) * n, hipMemcpyHostToDevice, c.stream));
  c.sync();
  c.n_preload = n;
}

static void dump_counts(Ctx& c) {
  const uint64_t nw = 2 * c.cap, ntot = nw + c.ovf_cap;
  c.dump_cnt.reserve(8 * ntot);
  unsigned* cnt = c.dump_cnt.as<unsigned>();
  PG_HIP(hipMemsetAsync(cnt, 0, 8 * ntot, c.stream));
  const uint64_t R = c.n_records;
  const uint64_t shift = pow5(c.k - 1);
  std::vector<unsigned long long> chunks;
  uint64_t sentinel = 0;
  for (uint64_t r = 0; r < R; ++r) {
    if (!c.last_flag[r]) continue;
    const int64_t n = c.h_rec_len[r];
    if (n < c.k) { ++sentinel; continue; }
    if (n < c.k + 2) continue;
    const uint64_t nch = ((uint64_t)(n - c.k + 1) + CCHUNK - 1) / CCHUNK;
    for (uint64_t j = 0; j < nch; ++j) chunks.push_back(((unsigned long long)r << 32) | j);
  }
  DevBuf dch;
  ensure_cls(c);                              // (the window counts read class bytes)
  if (!chunks.empty()) {
    dch.reserve(8 * chunks.size());
    PG_HIP(hipMemcpyAsync(dch.p, chunks.data(), 8 * chunks.size(), hipMemcpyHostToDevice, c.stream));
    if (c.rc0)
      hipLaunchKernelGGL(k_count_windows<true>, dim3((unsigned)chunks.size()), dim3(PBLK), 0, c.stream,
                         c.cls.as<uint8_t>(), dch.as<unsigned long long>(), c.rec_start.as<long long>(),
                         c.rec_len.as<long long>(), c.k, shift, c.tv, cnt);
    else
      hipLaunchKernelGGL(k_count_windows<false>, dim3((unsigned)chunks.size()), dim3(PBLK), 0, c.stream,
                         c.cls.as<uint8_t>(), dch.as<unsigned long long>(), c.rec_start.as<long long>(),
                         c.rec_len.as<long long>(), c.k, shift, c.tv, cnt);
    PG_HIP(hipGetLastError());
  }
  if (R) {
    hipLaunchKernelGGL(k_count_short, dim3(grid_for(R, PBLK, 1024)), dim3(PBLK), 0, c.stream, c.cls.as<uint8_t>(),
                       c.rec_start.as<long long>(), c.rec_len.as<long long>(), c.rec_flag.as<uint8_t>(), R, c.k,
                       shift, c.rc0, c.tv, cnt);
    PG_HIP(hipGetLastError());
  }
  uint64_t staged_sentinel = 0;
  if (c.n_preload) {
    hipLaunchKernelGGL(k_count_staged, dim3(grid_for(c.n_preload, PBLK, 4096)), dim3(PBLK), 0, c.stream,
                       c.preload.as<PreEnt>(), c.n_preload, c.tv, cnt);
    PG_HIP(hipGetLastError());
    std::vector<PreEnt> h(c.n_preload);
    PG_HIP(hipMemcpyAsync(h.data(), c.preload.p, sizeof(PreEnt) * c.n_preload, hipMemcpyDeviceToHost, c.stream));
    c.sync();
    for (const PreEnt& e : h)
      if (e.key == SENTINEL) staged_sentinel += e.count;
  }
  DevBuf npres;
  npres.reserve(8);
  PG_HIP(hipMemsetAsync(npres.p, 0, 8, c.stream));
  hipLaunchKernelGGL(k_count_present, dim3(grid_for(ntot, 256, 8192)), dim3(256), 0, c.stream, c.tv, nw, ntot,
                     npres.as<unsigned long long>());
  PG_HIP(hipGetLastError());
  unsigned long long present = 0;
  PG_HIP(hipMemcpyAsync(&present, npres.p, 8, hipMemcpyDeviceToHost, c.stream));
  c.sync();
  dch.release();
  npres.release();
  // n<k records and extra empty records: one sentinel occurrence per strand
  c.dump_sentinel = c.sentinel ? (sentinel + (uint64_t)c.last_extra) * (c.rc0 ? 2 : 1) + staged_sentinel : 0;
  c.dump_size = present + (c.sentinel ? 1 : 0);
  c.dump_ready = true;
}

// the oakht slot arrays of capacity M on the device (keys 8 B, values 2 B,
// counts 1 B per slot), the n<k sentinel included
struct DumpSlots {
  DevBuf ok, ov, oc;
};
static void dump_place(Ctx& c, uint64_t M, DumpSlots& d) {
  const uint64_t nw = 2 * c.cap, ntot = nw + c.ovf_cap;
  const uint64_t npend = c.dump_size - (c.sentinel ? 1 : 0);
  DevBuf prop, fail, lst[2], cnt;
  prop.reserve(8 * M); d.ok.reserve(8 * M); d.ov.reserve(2 * M); d.oc.reserve(M); fail.reserve(4);
  cnt.reserve(16);
  for (auto& b : lst) b.reserve(sizeof(PendEnt) * std::max<uint64_t>(npend, 1));
  PG_HIP(hipMemsetAsync(prop.p, 0xFF, 8 * M, c.stream));
  PG_HIP(hipMemsetAsync(d.ok.p, 0, 8 * M, c.stream));
  PG_HIP(hipMemsetAsync(d.ov.p, 0, 2 * M, c.stream));
  PG_HIP(hipMemsetAsync(d.oc.p, 0, M, c.stream));
  PG_HIP(hipMemsetAsync(fail.p, 0, 4, c.stream));
  PG_HIP(hipMemsetAsync(cnt.p, 0, 16, c.stream));
  auto* nc = cnt.as<unsigned long long>();
  hipLaunchKernelGGL(k_dump_list, dim3(grid_for(ntot, 256, 8192)), dim3(256), 0, c.stream, c.tv, nw, ntot,
                     c.dump_cnt.as<unsigned>(), lst[0].as<PendEnt>(), nc);
  PG_HIP(hipGetLastError());
  unsigned long long n = 0;
  PG_HIP(hipMemcpyAsync(&n, nc, 8, hipMemcpyDeviceToHost, c.stream));
  c.sync();
  if (n != npend) throw Error(-5, "pg_dbg_dump: " + std::to_string(n) + " present keys, counted " + std::to_string(npend));
  for (int round = 0, a = 0; n; ++round, a ^= 1) {
    if (round > 100000) throw Error(-5, "pg_dbg_dump: slot placement does not converge");
    const unsigned g = grid_for(n, 256, 8192);
    hipLaunchKernelGGL(k_dump_propose, dim3(g), dim3(256), 0, c.stream, lst[a].as<PendEnt>(), n, M,
                       d.oc.as<unsigned char>(), prop.as<unsigned long long>(), fail.as<unsigned>());
    PG_HIP(hipGetLastError());
    PG_HIP(hipMemsetAsync(nc + 1, 0, 8, c.stream));
    hipLaunchKernelGGL(k_dump_claim, dim3(g), dim3(256), 0, c.stream, lst[a].as<PendEnt>(), n, M,
                       prop.as<unsigned long long>(), d.ok.as<unsigned long long>(), d.ov.as<unsigned short>(),
                       d.oc.as<unsigned char>(), lst[a ^ 1].as<PendEnt>(), nc + 1);
    PG_HIP(hipGetLastError());
    unsigned h[2] = {0u, 0u};
    unsigned long long left = 0;
    PG_HIP(hipMemcpyAsync(&left, nc + 1, 8, hipMemcpyDeviceToHost, c.stream));
    PG_HIP(hipMemcpyAsync(h, fail.p, 4, hipMemcpyDeviceToHost, c.stream));
    c.sync();
    if (h[0]) throw Error(-34, "pg_dbg_dump: a key found no free slot on its probe sequence");
    n = left;
  }
  prop.release();
  fail.release();
  for (auto& b : lst) b.release();
  if (c.sentinel) {                                  // key 2^64-1, mask '$' (:1087-1088)
    const uint64_t j0 = oak_fnv(SENTINEL) % M;
    uint64_t kk = 0, s = j0;
    for (; kk < M; ++kk) {                           // (a probe or two at load <= 0.75)
      s = (j0 + kk * kk) % M;
      uint8_t taken = 0;
      PG_HIP(hipMemcpy(&taken, d.oc.as<uint8_t>() + s, 1, hipMemcpyDeviceToHost));
      if (taken == 0) break;
    }
    if (kk == M) throw Error(-34, "pg_dbg_dump: no free slot for the n<k sentinel");
    const uint64_t key = SENTINEL;
    const uint16_t val = 32;
    const uint8_t cnt = (uint8_t)(c.dump_sentinel > 255 ? 255 : (c.dump_sentinel ? c.dump_sentinel : 1));
    PG_HIP(hipMemcpy(d.ok.as<uint64_t>() + s, &key, 8, hipMemcpyHostToDevice));
    PG_HIP(hipMemcpy(d.ov.as<uint16_t>() + s, &val, 2, hipMemcpyHostToDevice));
    PG_HIP(hipMemcpy(d.oc.as<uint8_t>() + s, &cnt, 1, hipMemcpyHostToDevice));
  }
}

static uint64_t dump_capacity(Ctx& c, uint64_t& capacity) {
  if (!c.built) throw Error(-22, "pg_dbg_dump: no dBG (call pg_build_dbg first)");
  if (!c.dump_ready) dump_counts(c);
  const uint64_t M = capacity ? capacity : oakht_capacity(c.dump_size);
  if (M < c.dump_size) throw Error(-34, "pg_dbg_dump: capacity below the key count");
  capacity = M;
  return M;
}

uint64_t dbg_dump(Ctx& c, uint64_t& capacity, uint64_t* keys, uint16_t* values, uint8_t* counts) {
  const uint64_t M = dump_capacity(c, capacity);
  if (!keys) return c.dump_size;
  if (!values || !counts) throw Error(-22, "pg_dbg_dump: values and counts are required with keys");
  DumpSlots d;
  dump_place(c, M, d);
  PG_HIP(hipMemcpyAsync(keys, d.ok.p, 8 * M, hipMemcpyDeviceToHost, c.stream));
  PG_HIP(hipMemcpyAsync(values, d.ov.p, 2 * M, hipMemcpyDeviceToHost, c.stream));
  PG_HIP(hipMemcpyAsync(counts, d.oc.p, M, hipMemcpyDeviceToHost, c.stream));
  c.sync();
  return c.dump_size;
}

// Device bytes to a descriptor: member m (src[m], len[m] bytes) in
// FD_PIECE pieces, each piece through a worker thread's own pinned buffer
// and stream, so the copies, the CRCs and the page-cache writes of different
// pieces overlap and no host array of the whole member is ever allocated.
// pos: the file offset of each member (pwrite, pieces landing in any order),
// or nullptr: the members in order at the descriptor's position (write, each
// piece waiting for the one before it: pipes, terminals, O_APPEND files).
// crc: each member's CRC-32, or nullptr.
constexpr uint64_t FD_PIECE = 16ull << 20;
constexpr size_t FD_KEEP = 4;
static void stream_to_fd(Ctx& c, int nm, const uint8_t* const* src, const uint64_t* len, int fd,
                         const uint64_t* pos, uint32_t* crc, const char* what) {
  struct Piece { int m; uint64_t at, n; };
  std::vector<Piece> jobs;
  for (int m = 0; m < nm; ++m)
    for (uint64_t a = 0; a < len[m]; a += FD_PIECE) jobs.push_back(Piece{m, a, std::min(FD_PIECE, len[m] - a)});
  if (jobs.empty()) {
    for (int m = 0; crc && m < nm; ++m) crc[m] = 0u;
    return;
  }
  std::vector<uint32_t> pc(jobs.size(), 0u);
  std::atomic<size_t> next{0};
  std::atomic<bool> bad{false};
  std::mutex em, om;
  std::condition_variable ocv;
  size_t turn = 0;                                     // (ordered writes) the piece whose write is next
  std::string err;
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const size_t nt = std::min<size_t>(std::min<size_t>(16, hw), jobs.size());
  if (c.dump_pin.size() < nt) c.dump_pin.resize(nt);
  for (size_t t = 0; t < nt; ++t) c.dump_pin[t].reserve(FD_PIECE);
  auto put = [&](const uint8_t* b, uint64_t n, int64_t at) {
    for (uint64_t w = 0; w < n;) {
      const ssize_t r = at >= 0 ? pwrite(fd, b + w, n - w, (off_t)(at + (int64_t)w)) : write(fd, b + w, n - w);
      if (r < 0) {
        if (errno == EINTR) continue;
        throw Error(-5, std::string(what) + ": write failed: " + std::strerror(errno));
      }
      w += (uint64_t)r;
    }
  };
  auto worker = [&](size_t t) {
    hipStream_t st = nullptr;
    try {
      PG_HIP(hipSetDevice(c.device));
      PG_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
      uint8_t* buf = c.dump_pin[t].as<uint8_t>();
      for (size_t j; !bad && (j = next++) < jobs.size();) {
        const Piece& p = jobs[j];
        PG_HIP(hipMemcpyAsync(buf, src[p.m] + p.at, p.n, hipMemcpyDeviceToHost, st));
        PG_HIP(hipStreamSynchronize(st));
        if (crc) pc[j] = (uint32_t)crc32(0ul, buf, (uInt)p.n);
        if (pos) {
          put(buf, p.n, (int64_t)(pos[p.m] + p.at));
          continue;
        }
        {
          std::unique_lock<std::mutex> lk(om);      // (pieces are claimed in order, so the lowest
          ocv.wait(lk, [&] { return turn == j || bad.load(); });   // unwritten one never waits)
        }
        if (bad) break;
        put(buf, p.n, -1);
        {
          std::lock_guard<std::mutex> lk(om);
          ++turn;
        }
        ocv.notify_all();
      }
    } catch (const std::exception& e) {
      {
        std::lock_guard<std::mutex> g(em);
        if (!bad.exchange(true)) err = e.what();
      }
      std::lock_guard<std::mutex> lk(om);
      ocv.notify_all();
    }
    if (st) (void)hipStreamDestroy(st);
  };
  std::vector<std::thread> th;
  for (size_t t = 1; t < nt; ++t) th.emplace_back(worker, t);
  worker(0);
  for (auto& x : th) x.join();
  // the context keeps FD_KEEP piece buffers for its next dump / text write
  // (pinning them costs ~1 ms each); the rest go back now, so a context holds
  // at most FD_KEEP x 18 MiB of pinned host memory between calls
  for (size_t t = FD_KEEP; t < c.dump_pin.size(); ++t) c.dump_pin[t].release();
  if (c.dump_pin.size() > FD_KEEP) c.dump_pin.resize(FD_KEEP);
  if (bad) throw Error(-5, err);
  if (!crc) return;
  for (int m = 0; m < nm; ++m) crc[m] = 0u;
  std::vector<bool> first(nm, true);
  for (size_t j = 0; j < jobs.size(); ++j) {          // pieces are in member order, ascending
    const int m = jobs[j].m;
    crc[m] = first[m] ? pc[j] : (uint32_t)crc32_combine(crc[m], pc[j], (z_off_t)jobs[j].n);
    first[m] = false;
  }
}

// dump() straight into a file: the slot arrays (keys, values, counts) at
// off[0..2], their CRC-32s in crc[0..2] (C3: 886 MB; C4: ~5 GB, never in a
// host array)
uint64_t dbg_dump_fd(Ctx& c, uint64_t& capacity, int fd, const uint64_t* off, uint32_t* crc) {
  const uint64_t M = dump_capacity(c, capacity);
  if (fd < 0) return c.dump_size;
  if (!off || !crc) throw Error(-22, "pg_dbg_dump_fd: offsets and crcs are required with a descriptor");
  DumpSlots d;
  dump_place(c, M, d);
  const uint8_t* src[3] = {d.ok.as<uint8_t>(), d.ov.as<uint8_t>(), d.oc.as<uint8_t>()};
  const uint64_t len[3] = {8 * M, 2 * M, M};
  stream_to_fd(c, 3, src, len, fd, off, crc, "pg_dbg_dump_fd");
  return c.dump_size;
}

// n device bytes written to fd at its position, which then follows them: a
// regular file opened without O_APPEND takes the pieces in parallel
// (pwrite), anything else in order
void text_to_fd(Ctx& c, const uint8_t* src, uint64_t n, int fd, const char* what) {
  struct stat sb;
  if (fstat(fd, &sb) != 0) throw Error(-9, std::string(what) + ": bad descriptor: " + std::strerror(errno));
  const int fl = fcntl(fd, F_GETFL);
  const off_t cur = lseek(fd, 0, SEEK_CUR);
  if (S_ISREG(sb.st_mode) && fl >= 0 && !(fl & O_APPEND) && cur >= 0) {
    const uint64_t at = (uint64_t)cur;
    stream_to_fd(c, 1, &src, &n, fd, &at, nullptr, what);
    if (lseek(fd, cur + (off_t)n, SEEK_SET) < 0)
      throw Error(-5, std::string(what) + ": seek failed: " + std::strerror(errno));
  } else {
    stream_to_fd(c, 1, &src, &n, fd, nullptr, nullptr, what);
  }
}

}  // namespace pg
