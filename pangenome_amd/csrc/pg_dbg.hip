// pg_dbg.hip — K3: k-mer windows -> open-addressed HBM table (atomic OR of
// neighbour masks); K5: degree scan + rdBG compaction; exports and the
// owner-partitioned exchange used by the multi-GPU build.
//
// Reference path: seq2rdbg (kmer_numba.py:1234-1268) -> seq2dbg_jit_
// (:1202-1230) -> build_dbg (:1052-1090) -> add_kmer (:1036-1047), then
// dbg2rdbg (:1313-1321) -> build_rdbg_jit_ (:1292-1309).
//
// Every forward-strand window q of a record carries its reverse-strand twin
// (window n-k-q of tab_rev(reversed(s)), :1215-1221), so one thread visit per
// position inserts both: the canonical key c = min(K, K') gets the forward
// mask in one 12-bit field and the reverse mask in the other (pg_common.h).
// That halves the random HBM probes against inserting the two strands as the
// reference does, while the exported dBG stays exactly the reference's.
//
// Homology-aware order.  A pangenome repeats each k-mer once per genome at
// nearly the same offset, so K3 walks tiles of TILE windows stripe-major
// (stripe j of every record, then stripe j+1, ...) and remaps blocks so one
// stripe's tiles run on one XCD: the first genome's probe of a slot misses,
// the other genomes' probes of it hit that XCD's L2 / the Infinity Cache.
#include <algorithm>
#include <cstring>
#include <numeric>
#include <rocprim/rocprim.hpp>

#include "pg_internal.h"

namespace pg {

constexpr int IBLOCK = 256;
constexpr int IW = 16;                        // windows per thread
constexpr int TILE = IBLOCK * IW;             // windows per tile (one block)
constexpr int MAX_PROBE = 4096;
constexpr int N_CNT = 64;                     // spread counters (one 64-byte line each)

// flags layout (uint32 words): [0] sentinel seen, [1] overflow, [16*(1+i)] counter i
__device__ __forceinline__ unsigned* counter(unsigned* flags, int i) { return flags + 16 * (1 + i); }

// Insert/OR one canonical key.  Returns 1 if this call created the slot.
// Plain loads may be stale (atomics run beyond the XCD's L2), but a slot only
// ever goes empty -> key and masks only gain bits: a stale empty is settled
// by the CAS's return value, a stale mask only costs a redundant atomicOr.
__device__ __forceinline__ int table_or(Slot* __restrict__ table, uint64_t capmask, uint64_t c,
                                        uint32_t mw, unsigned* flags) {
  const unsigned long long key1 = (unsigned long long)c + 1ull;
  uint64_t slot = fmix64(c) & capmask;
  for (int probe = 0; probe < MAX_PROBE; ++probe) {
    Slot* s = table + slot;
    const uint4 v = *reinterpret_cast<const uint4*>(s);
    const unsigned long long kk = (unsigned long long)v.x | ((unsigned long long)v.y << 32);
    if (kk == key1) {
      if ((v.z & mw) != mw) atomicOr(&s->mask, mw);
      return 0;
    }
    if (kk == 0ull) {
      const unsigned long long old = atomicCAS(&s->key1, 0ull, key1);
      if (old == 0ull || old == key1) {
        atomicOr(&s->mask, mw);
        return old == 0ull;
      }
    }
    slot = (slot + 1) & capmask;
  }
  atomicOr(flags + 1, 1u);
  return 0;
}

__device__ __forceinline__ void block_count(unsigned created, unsigned* flags) {
  __shared__ unsigned red[IBLOCK / 64];
  unsigned x = created;
  for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned t = 0;
    for (int w = 0; w < IBLOCK / 64; ++w) t += red[w];
    if (t) atomicAdd(counter(flags, blockIdx.x % N_CNT), t);
  }
}

// K3.  One block per tile (record, stripe j): windows [j*TILE, (j+1)*TILE) of
// a record with n >= k+2; thread t takes IW consecutive windows and rolls the
// keys of both strands across them.
template <bool RC>
__global__ void __launch_bounds__(IBLOCK)
k_insert(const uint8_t* __restrict__ cls, const unsigned long long* __restrict__ tiles,
         const long long* __restrict__ rec_start, const long long* __restrict__ rec_len, int k, uint64_t shift,
         Slot* __restrict__ table, uint64_t capmask, unsigned* __restrict__ flags) {
  const unsigned long long tile = tiles[xcd_swizzle(blockIdx.x, gridDim.x)];
  const int r = (int)(tile >> 32);
  const long long rs = rec_start[r], rn = rec_len[r];
  const long long last = rn - k;                              // last window index
  const long long q0 = (long long)(tile & 0xFFFFFFFFull) * TILE + (long long)threadIdx.x * IW;
  const long long q1 = q0 + IW <= last + 1 ? q0 + IW : last + 1;
  unsigned created = 0;
  uint64_t K = 0, Kr = 0;
  for (long long q = q0; q < q1; ++q) {
    const uint64_t p = (uint64_t)(rs + q);
    if (q == q0) {
      uint64_t pw = 1;
      for (int j = 0; j < k; ++j) {                // k2n_jit (:975-985), both strands
        const uint32_t cj = cls[p + j];
        K += (uint64_t)digit_fw(cj) * pw;
        Kr = Kr * 5 + digit_rc(cj);
        pw *= 5;
      }
    } else {                                       // Nu // 5 + alpha * 5^(k-1) (:1072)
      const uint32_t dout = cls[p - 1], din = cls[p + k - 1];
      K = (K - digit_fw(dout)) * INV5 + (uint64_t)digit_fw(din) * shift;
      Kr = (Kr - (uint64_t)digit_rc(dout) * shift) * 5 + digit_rc(din);
    }
    // forward window q: pred '#' at q==0, s[q-2] at the last window (:1080 quirk), else s[q-1]
    const uint32_t fpred = q == 0 ? LAM_HASH : lam_fw(cls[p - (q == last ? 2 : 1)]);
    const uint32_t fsucc = q == last ? LAM_DOLLAR : lam_fw(cls[p + k]);
    const uint32_t mf = (fpred << OFFBIT) | fsucc | PRES_A;
    uint64_t c;
    uint32_t mw;
    if (RC) {
      // its twin: reverse-strand window n-k-q, same boundary rules on that strand
      const uint32_t rpred = q == last ? LAM_HASH : lam_rc(cls[p + k + (q == 0 ? 1 : 0)]);
      const uint32_t rsucc = q == 0 ? LAM_DOLLAR : lam_rc(cls[p - 1]);
      const uint32_t mr = (rpred << OFFBIT) | rsucc | PRES_A;
      if (K < Kr)      { c = K;  mw = mf | (mr << 16); }
      else if (K > Kr) { c = Kr; mw = mr | (mf << 16); }
      else             { c = K;  mw = mf | mr; }
    } else {
      if (K <= Kr) { c = K; mw = mf; } else { c = Kr; mw = mf << 16; }
    }
    created += (unsigned)table_or(table, capmask, c, mw, flags);
  }
  block_count(created, flags);
}

// one reference window of an explicit strand (used for records with n <= k+1)
__device__ __forceinline__ void oriented_or(Slot* table, uint64_t capmask, int k, uint64_t x,
                                            uint32_t m12, unsigned* flags, unsigned& created) {
  const uint64_t xr = rc_key(x, k);
  const uint32_t m = m12 | PRES_A;
  if (x <= xr) created += (unsigned)table_or(table, capmask, x, m, flags);
  else created += (unsigned)table_or(table, capmask, xr, m << 16, flags);
}

// build_dbg for one strand of length n in {k, k+1}.  strand 0: s[i] = cls[rs+i];
// strand 1: s[i] = comp_class(cls[rs+n-1-i]) (tab_rev(reversed(s)), :1217).
__device__ void short_strand(const uint8_t* cls, long long rs, long long n, int strand, int k,
                             uint64_t shift, Slot* table, uint64_t capmask, unsigned* flags, unsigned& created) {
  auto S = [&](long long i) -> uint32_t {
    return strand == 0 ? (uint32_t)cls[rs + i] : comp_class(cls[rs + n - 1 - i]);
  };
  uint64_t K0 = 0, pw = 1;
  for (int j = 0; j < k; ++j) { K0 += (uint64_t)digit_fw(S(j)) * pw; pw *= 5; }
  if (n == k) {                                            // :1084-1085
    oriented_or(table, capmask, k, K0, (LAM_HASH << OFFBIT) | LAM_DOLLAR, flags, created);
    return;
  }
  // n == k+1 (:1061-1082): the loop never runs and numba reads its variable as 0
  oriented_or(table, capmask, k, K0, (LAM_HASH << OFFBIT) | lam_fw(S(k)), flags, created);
  const uint64_t K1 = K0 / 5 + (uint64_t)digit_fw(S(1)) * shift;   // alpha[seq[0+1]]
  oriented_or(table, capmask, k, K1, (lam_fw(S(1)) << OFFBIT) | LAM_DOLLAR, flags, created);  // seq[0-k] == s[1]
}

__global__ void __launch_bounds__(IBLOCK)
k_short(const uint8_t* __restrict__ cls, const long long* __restrict__ rec_start,
        const long long* __restrict__ rec_len, const uint8_t* __restrict__ rec_flag, uint64_t R, int k,
        uint64_t shift, int rc, Slot* table, uint64_t capmask, unsigned* flags) {
  unsigned created = 0;
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < R;
       r += (uint64_t)gridDim.x * blockDim.x) {
    if (!rec_flag[r]) continue;
    const long long n = rec_len[r];
    if (n > k + 1) continue;
    if (n < k) { atomicOr(flags, 1u); continue; }          // key -1, mask '$' (:1087-1088)
    short_strand(cls, rec_start[r], n, 0, k, shift, table, capmask, flags, created);
    if (rc) short_strand(cls, rec_start[r], n, 1, k, shift, table, capmask, flags, created);
  }
  block_count(created, flags);
}

// Extra empty records that the reference's checkpoint/resume yields (see
// pangenome_amd/host.py): each adds the n<k sentinel.
__global__ void k_set_flag(unsigned* flags) { atomicOr(flags, 1u); }

// K5: degree scan.  One block per 4096-slot tile (slot = tile*4096 + j*256 +
// tid, coalesced 16-byte loads); members are counted, block-scanned and placed
// with one global atomic per tile, then written by a second sweep that
// re-reads only member slots.  Marks rdBG membership in the slot for the walks.
constexpr int RJ = 16;
constexpr uint64_t RTILE = 256 * RJ;

__global__ void __launch_bounds__(256)
k_reduce(Slot* __restrict__ table, uint64_t cap, int k, unsigned long long* __restrict__ out,
         unsigned long long* __restrict__ counters) {
  __shared__ uint32_t lds[4];
  __shared__ unsigned long long tile_base;
  __shared__ unsigned long long red[4];
  const uint64_t ntile = cap / RTILE;
  unsigned long long ndbg = 0;
  for (uint64_t t = blockIdx.x; t < ntile; t += gridDim.x) {
    const uint64_t base = t * RTILE + threadIdx.x;
    uint32_t cnt = 0, bits = 0;
#pragma unroll
    for (int j = 0; j < RJ; ++j) {
      Slot* s = table + base + (uint64_t)j * 256;
      const uint4 v = *reinterpret_cast<const uint4*>(s);
      const bool occ = (v.x | v.y) != 0u;
      const uint32_t m = v.z;
      const bool pa = occ && (m & PRES_A), pb = occ && (m & PRES_B);
      const bool ma = pa && rdbg_member(m & MASK12);
      const bool mb = pb && rdbg_member((m >> 16) & MASK12);
      ndbg += (unsigned long long)pa + (unsigned long long)pb;
      cnt += (uint32_t)ma + (uint32_t)mb;
      bits |= ((uint32_t)ma | ((uint32_t)mb << 1)) << (2 * j);
      if (ma || mb) s->mask = m | (ma ? RDBG_A : 0u) | (mb ? RDBG_B : 0u);
    }
    uint32_t tot;
    const uint32_t pre = block_excl_scan<256>(cnt, lds, tot);
    if (threadIdx.x == 0) tile_base = tot ? atomicAdd(counters, (unsigned long long)tot) : 0ull;
    __syncthreads();
    unsigned long long o = tile_base + pre;
    while (bits) {
      const int b = __builtin_ctz(bits);
      const uint64_t c = table[base + (uint64_t)(b >> 1) * 256].key1 - 1ull;
      out[o++] = (b & 1) ? rc_key(c, k) : c;
      bits &= bits - 1u;
    }
    __syncthreads();                               // tile_base is reused next tile
  }
  for (int o = 32; o > 0; o >>= 1) ndbg += __shfl_down(ndbg, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ndbg;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = red[0] + red[1] + red[2] + red[3];
    if (t) atomicAdd(counters + 8, t);
  }
}

// dBG export: (key, 12-bit mask) of both orientations of every slot
__global__ void k_export_dbg(const Slot* __restrict__ table, uint64_t cap, int k,
                             unsigned long long* __restrict__ keys, unsigned short* __restrict__ masks,
                             unsigned long long* __restrict__ counter) {
  const int lane = threadIdx.x & 63;
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const Slot s = table[i];
    const bool pa = s.key1 && (s.mask & PRES_A), pb = s.key1 && (s.mask & PRES_B);
    const unsigned long long ba = __ballot(pa), bb = __ballot(pb);
    const unsigned na = __builtin_popcountll(ba), nbb = __builtin_popcountll(bb);
    if (na + nbb == 0) continue;
    const int leader = __builtin_ctzll(ba | bb);
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(counter, (unsigned long long)(na + nbb));
    base = __shfl(base, leader, 64);
    const uint64_t c = s.key1 - 1ull;
    if (pa) { uint64_t o = base + __builtin_popcountll(ba & lt); keys[o] = c; masks[o] = s.mask & MASK12; }
    if (pb) {
      uint64_t o = base + na + __builtin_popcountll(bb & lt);
      keys[o] = rc_key(c, k); masks[o] = (s.mask >> 16) & MASK12;
    }
  }
}

// ---- multi-GPU exchange: owner = high bits of the slot hash mod nparts
__device__ __forceinline__ int owner_of(uint64_t c, int nparts) {
  return (int)((fmix64(c) >> 40) % (uint64_t)nparts);
}

__global__ void k_part_count(const Slot* __restrict__ table, uint64_t cap, int nparts,
                             unsigned long long* __restrict__ counts) {
  __shared__ unsigned long long hist[64];
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long key1 = table[i].key1;
    if (key1) atomicAdd(&hist[owner_of(key1 - 1ull, nparts)], 1ull);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nparts; i += blockDim.x)
    if (hist[i]) atomicAdd(&counts[i], hist[i]);
}

__global__ void k_part_scatter(const Slot* __restrict__ table, uint64_t cap, int nparts,
                               unsigned long long* __restrict__ cursor, Slot* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
       i += (uint64_t)gridDim.x * blockDim.x) {
    Slot s = table[i];
    const int own = s.key1 ? owner_of(s.key1 - 1ull, nparts) : -1;
    for (int o = 0; o < nparts; ++o) {
      const unsigned long long b = __ballot(own == o);
      if (!b) continue;
      const int leader = __builtin_ctzll(b);
      unsigned long long base = 0;
      if (lane == leader) base = atomicAdd(&cursor[o], (unsigned long long)__builtin_popcountll(b));
      base = __shfl(base, leader, 64);
      if (own == o) {
        s.mask &= ~(RDBG_A | RDBG_B);
        s.aux = 0;
        out[base + __builtin_popcountll(b & lt)] = s;
      }
    }
  }
}

__global__ void __launch_bounds__(IBLOCK)
k_merge(const Slot* __restrict__ pairs, uint64_t n, Slot* __restrict__ table, uint64_t capmask,
        unsigned* __restrict__ flags) {
  unsigned created = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const Slot s = pairs[i];
    if (!s.key1) continue;
    created += (unsigned)table_or(table, capmask, s.key1 - 1ull, s.mask & ~(RDBG_A | RDBG_B), flags);
  }
  block_count(created, flags);
}

// ------------------------------------------------------------------ host
static void alloc_table(Ctx& c, uint64_t cap) {
  c.cap = cap;
  c.table.reserve(cap * sizeof(Slot));
  c.flags.reserve(4 * 16 * (N_CNT + 2));
}

static void clear_table(Ctx& c) {
  PG_HIP(hipMemsetAsync(c.table.p, 0, c.cap * sizeof(Slot), c.stream));
  PG_HIP(hipMemsetAsync(c.flags.p, 0, 4 * 16 * (N_CNT + 2), c.stream));
}

// read back [sentinel, overflow, sum of spread counters]
static void read_flags(Ctx& c, unsigned& sentinel, unsigned& overflow, uint64_t& created) {
  std::vector<unsigned> f(16 * (N_CNT + 2));
  PG_HIP(hipMemcpyAsync(f.data(), c.flags.p, 4 * f.size(), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  sentinel = f[0];
  overflow = f[1];
  created = 0;
  for (int i = 0; i < N_CNT; ++i) created += f[16 * (1 + i)];
}

// Tiles of records with n >= k+2, stripe-major: stripe 0 of every record, then
// stripe 1, ...  (records with more stripes first within a stripe).  Packed as
// record << 32 | stripe.  Cached while the record table and flags repeat.
static uint64_t make_tiles(Ctx& c, const std::vector<uint8_t>& flag) {
  const uint64_t R = c.n_records;
  if (c.tile_sig_len == c.h_rec_len && c.tile_sig_flag == flag && c.tile_k == c.k) return c.n_tiles;
  std::vector<std::pair<uint64_t, int>> nt;           // (stripes, record)
  uint64_t total = 0, maxs = 0;
  for (uint64_t r = 0; r < R; ++r) {
    const int64_t n = c.h_rec_len[r];
    if (!flag[r] || n < c.k + 2) continue;
    const uint64_t s = (uint64_t)((n - c.k + 1 + TILE - 1) / TILE);
    nt.push_back({s, (int)r});
    total += s;
    maxs = std::max(maxs, s);
  }
  std::stable_sort(nt.begin(), nt.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
  std::vector<unsigned long long> tiles;
  tiles.reserve(total);
  size_t live = nt.size();
  for (uint64_t j = 0; j < maxs; ++j) {
    while (live && nt[live - 1].first <= j) --live;
    for (size_t i = 0; i < live; ++i) tiles.push_back(((unsigned long long)nt[i].second << 32) | j);
  }
  c.tiles.reserve(8 * (total + 1));
  if (total) PG_HIP(hipMemcpyAsync(c.tiles.p, tiles.data(), 8 * total, hipMemcpyHostToDevice, c.stream));
  c.sync();
  c.tile_sig_len = c.h_rec_len;
  c.tile_sig_flag = flag;
  c.tile_k = c.k;
  c.n_tiles = total;
  return total;
}

void build_dbg(Ctx& c, const uint8_t* h_rec_flag, int extra_empty, int rc0) {
  if (!c.parsed) throw Error(-22, "build_dbg: no parsed FASTA (call pg_parse first)");
  const uint64_t R = c.n_records;
  c.rc0 = rc0;
  c.built = c.reduced = false;
  c.n_dbg = c.n_rdbg = c.n_canon = 0;
  c.windows_fw = 0;
  std::vector<uint8_t> flag(R, 1);
  if (h_rec_flag)
    for (uint64_t r = 0; r < R; ++r) flag[r] = h_rec_flag[r] & 1;
  if (R) PG_HIP(hipMemcpyAsync(c.rec_flag.p, flag.data(), R, hipMemcpyHostToDevice, c.stream));
  for (uint64_t r = 0; r < R; ++r)
    if (flag[r]) {
      const int64_t n = c.h_rec_len[r];
      c.windows_fw += n > c.k ? (uint64_t)(n - c.k + 1) : 1;
    }
  c.windows_total = c.windows_fw * (rc0 ? 2 : 1);
  const uint64_t ntiles = make_tiles(c, flag);
  // table size: learned capacity, else a conservative guess; rebuilt on overflow
  uint64_t cap = c.cap_hint ? c.cap_hint : next_pow2(std::max<uint64_t>(1ull << 20, c.windows_fw));
  const uint64_t shift = pow5(c.k - 1);
  c.t0.init(); c.t1.init();
  for (int attempt = 0; attempt < 8; ++attempt) {
    alloc_table(c, cap);
    c.t0.start(c.stream);
    clear_table(c);
    c.t0.stop(c.stream);
    Slot* tab = c.table.as<Slot>();
    unsigned* flags = c.flags.as<unsigned>();
    c.t1.start(c.stream);
    if (ntiles) {
      if (rc0)
        hipLaunchKernelGGL(k_insert<true>, dim3((unsigned)ntiles), dim3(IBLOCK), 0, c.stream, c.cls.as<uint8_t>(),
                           c.tiles.as<unsigned long long>(), c.rec_start.as<long long>(), c.rec_len.as<long long>(),
                           c.k, shift, tab, cap - 1, flags);
      else
        hipLaunchKernelGGL(k_insert<false>, dim3((unsigned)ntiles), dim3(IBLOCK), 0, c.stream, c.cls.as<uint8_t>(),
                           c.tiles.as<unsigned long long>(), c.rec_start.as<long long>(), c.rec_len.as<long long>(),
                           c.k, shift, tab, cap - 1, flags);
      PG_HIP(hipGetLastError());
    }
    c.t1.stop(c.stream);
    if (R) {
      hipLaunchKernelGGL(k_short, dim3(grid_for(R, IBLOCK, 1024)), dim3(IBLOCK), 0, c.stream,
                         c.cls.as<uint8_t>(), c.rec_start.as<long long>(), c.rec_len.as<long long>(),
                         c.rec_flag.as<uint8_t>(), R, c.k, shift, rc0, tab, cap - 1, flags);
      PG_HIP(hipGetLastError());
    }
    if (extra_empty) hipLaunchKernelGGL(k_set_flag, dim3(1), dim3(1), 0, c.stream, flags);
    unsigned sentinel = 0, overflow = 0;
    uint64_t created = 0;
    read_flags(c, sentinel, overflow, created);
    c.ms_clear = c.t0.ms();
    c.ms_insert = c.t1.ms();
    if (!overflow && created * 10 <= cap * 7) {
      c.n_canon = created;
      c.sentinel = sentinel ? 1 : 0;
      c.cap_hint = next_pow2(std::max<uint64_t>(1ull << 16, created * 2));
      c.built = true;
      return;
    }
    cap = next_pow2(std::max<uint64_t>(cap * 2, created * 3));
  }
  throw Error(-12, "build_dbg: hash table overflow after resizing");
}

void build_rdbg(Ctx& c) {
  if (!c.built) throw Error(-22, "build_rdbg: no dBG (call pg_build_dbg first)");
  c.rdbg_keys.reserve(8 * (2 * c.n_canon + 2));
  DevBuf& cnt = c.n_sel;
  cnt.reserve(128);
  PG_HIP(hipMemsetAsync(cnt.p, 0, 128, c.stream));
  c.t0.start(c.stream);
  hipLaunchKernelGGL(k_reduce, dim3(grid_for(c.cap / RTILE, 1, 8192)), dim3(256), 0, c.stream,
                     c.table.as<Slot>(), c.cap, c.k, c.rdbg_keys.as<unsigned long long>(),
                     cnt.as<unsigned long long>());
  PG_HIP(hipGetLastError());
  c.t0.stop(c.stream);
  unsigned long long res[9];
  PG_HIP(hipMemcpyAsync(res, cnt.p, sizeof(res), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  c.ms_scan = c.t0.ms();
  c.n_rdbg = res[0];
  c.n_dbg = res[8];
  if (c.sentinel) {         // key 2^64-1, mask 32: always an rdBG member
    unsigned long long s = SENTINEL;
    PG_HIP(hipMemcpyAsync(c.rdbg_keys.as<unsigned long long>() + c.n_rdbg, &s, 8, hipMemcpyHostToDevice,
                          c.stream));
    c.sync();
    c.n_rdbg += 1;
    c.n_dbg += 1;
  }
  c.reduced = true;
}

uint64_t export_dbg(Ctx& c, uint64_t* h_keys, uint16_t* h_masks, uint64_t cap) {
  if (!c.built) throw Error(-22, "export_dbg: no dBG");
  const uint64_t nmax = 2 * c.n_canon + 1;
  DevBuf keys, masks, cnt;
  keys.reserve(8 * nmax);
  masks.reserve(2 * nmax);
  cnt.reserve(8);
  PG_HIP(hipMemsetAsync(cnt.p, 0, 8, c.stream));
  hipLaunchKernelGGL(k_export_dbg, dim3(grid_for(c.cap, 256, 8192)), dim3(256), 0, c.stream,
                     c.table.as<Slot>(), c.cap, c.k, keys.as<unsigned long long>(),
                     masks.as<unsigned short>(), cnt.as<unsigned long long>());
  PG_HIP(hipGetLastError());
  unsigned long long n = 0;
  PG_HIP(hipMemcpyAsync(&n, cnt.p, 8, hipMemcpyDeviceToHost, c.stream));
  c.sync();
  const uint64_t total = n + (c.sentinel ? 1 : 0);
  if (h_keys && cap >= total) {
    PG_HIP(hipMemcpy(h_keys, keys.p, 8 * n, hipMemcpyDeviceToHost));
    PG_HIP(hipMemcpy(h_masks, masks.p, 2 * n, hipMemcpyDeviceToHost));
    if (c.sentinel) { h_keys[n] = SENTINEL; h_masks[n] = 32; }
  }
  keys.release(); masks.release(); cnt.release();
  return total;
}

uint64_t export_rdbg(Ctx& c, uint64_t* h_keys, uint64_t cap) {
  if (!c.reduced) throw Error(-22, "export_rdbg: no rdBG (call pg_build_rdbg first)");
  if (h_keys && cap >= c.n_rdbg)
    PG_HIP(hipMemcpy(h_keys, c.rdbg_keys.p, 8 * c.n_rdbg, hipMemcpyDeviceToHost));
  return c.n_rdbg;
}

uint64_t partition_dbg(Ctx& c, int nparts, void* d_out, uint64_t out_cap, uint64_t* h_counts) {
  if (!c.built) throw Error(-22, "partition_dbg: no dBG");
  if (nparts < 1 || nparts > 64) throw Error(-22, "partition_dbg: nparts must be in [1, 64]");
  DevBuf cnt;
  cnt.reserve(16 * 64);
  PG_HIP(hipMemsetAsync(cnt.p, 0, 16 * 64, c.stream));
  auto* counts = cnt.as<unsigned long long>();
  hipLaunchKernelGGL(k_part_count, dim3(grid_for(c.cap, 256, 4096)), dim3(256), 0, c.stream,
                     c.table.as<Slot>(), c.cap, nparts, counts);
  PG_HIP(hipGetLastError());
  std::vector<unsigned long long> h(nparts), off(nparts);
  PG_HIP(hipMemcpyAsync(h.data(), counts, 8 * nparts, hipMemcpyDeviceToHost, c.stream));
  c.sync();
  uint64_t total = 0;
  for (int i = 0; i < nparts; ++i) { off[i] = total; total += h[i]; h_counts[i] = h[i]; }
  if (d_out && out_cap >= total && total) {
    PG_HIP(hipMemcpyAsync(counts + 64, off.data(), 8 * nparts, hipMemcpyHostToDevice, c.stream));
    hipLaunchKernelGGL(k_part_scatter, dim3(grid_for(c.cap, 256, 4096)), dim3(256), 0, c.stream,
                       c.table.as<Slot>(), c.cap, nparts, counts + 64, reinterpret_cast<Slot*>(d_out));
    PG_HIP(hipGetLastError());
    c.sync();
  }
  cnt.release();
  return total;
}

void merge_dbg(Ctx& c, const void* d_pairs, uint64_t n, uint64_t cap_hint, int sentinel) {
  uint64_t cap = cap_hint ? next_pow2(cap_hint) : next_pow2(std::max<uint64_t>(1ull << 16, 2 * n));
  c.t1.init();
  for (int attempt = 0; attempt < 8; ++attempt) {
    alloc_table(c, cap);
    clear_table(c);
    if (sentinel) hipLaunchKernelGGL(k_set_flag, dim3(1), dim3(1), 0, c.stream, c.flags.as<unsigned>());
    c.t1.start(c.stream);
    if (n)
      hipLaunchKernelGGL(k_merge, dim3(grid_for(n, IBLOCK, 8192)), dim3(IBLOCK), 0, c.stream,
                         reinterpret_cast<const Slot*>(d_pairs), n, c.table.as<Slot>(), cap - 1,
                         c.flags.as<unsigned>());
    PG_HIP(hipGetLastError());
    c.t1.stop(c.stream);
    unsigned s = 0, overflow = 0;
    uint64_t created = 0;
    read_flags(c, s, overflow, created);
    c.ms_insert = c.t1.ms();
    if (!overflow && created * 10 <= cap * 7) {
      c.n_canon = created;
      c.sentinel = s ? 1 : 0;
      c.built = true;
      c.reduced = false;
      return;
    }
    cap = next_pow2(std::max<uint64_t>(cap * 2, created * 3));
  }
  throw Error(-12, "merge_dbg: hash table overflow after resizing");
}

}  // namespace pg
