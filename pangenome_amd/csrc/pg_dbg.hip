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
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "pg_internal.h"

namespace pg {

constexpr int IBLOCK = 256;
constexpr int MAX_PROBE = 4096;
constexpr int N_CNT = 64;          // spread counters (one 64-byte line each)

// flags layout (uint32 words): [0] sentinel seen, [1] overflow, [16*(1+i)] counter i
__device__ __forceinline__ unsigned* counter(unsigned* flags, int i) { return flags + 16 * (1 + i); }

// Insert/OR one canonical key.  Returns 1 if this call created the slot.
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

__device__ __forceinline__ uint64_t find_record(const long long* __restrict__ rec_start, uint64_t R, uint64_t p) {
  // last r with rec_start[r] <= p; 0 when p precedes record 0 (the caller
  // skips positions before rec_start[r])
  uint64_t lo = 0, hi = R;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if ((uint64_t)rec_start[mid] <= p) lo = mid + 1; else hi = mid;
  }
  return lo == 0 ? 0 : lo - 1;
}

// K3: one thread per run of W consecutive positions of the compacted stream.
template <int W, bool RC>
__global__ void __launch_bounds__(IBLOCK)
k_insert(const uint8_t* __restrict__ cls, uint64_t total,
         const long long* __restrict__ rec_start, const long long* __restrict__ rec_len,
         const uint8_t* __restrict__ rec_flag, uint64_t R, int k, uint64_t shift,
         Slot* __restrict__ table, uint64_t capmask, unsigned* __restrict__ flags) {
  __shared__ unsigned red[IBLOCK / 64];
  const uint64_t nruns = (total + W - 1) / W;
  unsigned created = 0;
  for (uint64_t run = blockIdx.x * (uint64_t)IBLOCK + threadIdx.x; run < nruns;
       run += (uint64_t)gridDim.x * IBLOCK) {
    const uint64_t p0 = run * W;
    const uint64_t p1 = p0 + W < total ? p0 + W : total;
    uint64_t r = find_record(rec_start, R, p0);
    long long rs = 0, rn = -1; bool rf = false;
    if (r < R) { rs = rec_start[r]; rn = rec_len[r]; rf = rec_flag[r] != 0; }
    bool have = false;
    uint64_t K = 0, Kr = 0;
    for (uint64_t p = p0; p < p1; ++p) {
      while (r < R && (long long)p >= rs + rn) {
        ++r;
        if (r < R) { rs = rec_start[r]; rn = rec_len[r]; rf = rec_flag[r] != 0; }
        have = false;
      }
      if (r >= R || (long long)p < rs) { have = false; continue; }
      const long long q = (long long)p - rs;
      if (!rf || rn < k + 2 || q > rn - k) { have = false; continue; }
      if (!have) {
        K = 0; Kr = 0;
        uint64_t pw = 1;
        for (int j = 0; j < k; ++j) {              // k2n_jit (:975-985), both strands
          const uint32_t cj = cls[p + j];
          K += (uint64_t)digit_fw(cj) * pw;
          Kr = Kr * 5 + digit_rc(cj);
          pw *= 5;
        }
        have = true;
      } else {                                     // Nu // 5 + alpha * 5^(k-1) (:1072)
        const uint32_t dout = cls[p - 1], din = cls[p + k - 1];
        K = (K - digit_fw(dout)) * INV5 + (uint64_t)digit_fw(din) * shift;
        Kr = (Kr - (uint64_t)digit_rc(dout) * shift) * 5 + digit_rc(din);
      }
      const long long last = rn - k;
      // forward window q: pred '#' at q==0, s[q-2] at the last window (:1080 quirk), else s[q-1]
      const uint32_t fpred = q == 0 ? LAM_HASH : lam_fw(cls[p - (q == last ? 2 : 1)]);
      const uint32_t fsucc = q == last ? LAM_DOLLAR : lam_fw(cls[p + k]);
      uint32_t mf = (fpred << OFFBIT) | fsucc | PRES_A;
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
  }
  // block-reduce the new-slot count, one atomic per block on a spread counter
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

// one reference window of an explicit strand (used for records with n <= k+1)
__device__ __forceinline__ void oriented_or(Slot* table, uint64_t capmask, int k, uint64_t x,
                                            uint32_t m12, unsigned* flags) {
  const uint64_t xr = rc_key(x, k);
  const uint32_t m = m12 | PRES_A;
  if (x <= xr) (void)table_or(table, capmask, x, m, flags);
  else (void)table_or(table, capmask, xr, m << 16, flags);
}

// build_dbg for one strand of length n in {k, k+1}.  strand 0: s[i] = cls[rs+i];
// strand 1: s[i] = comp_class(cls[rs+n-1-i]) (tab_rev(reversed(s)), :1217).
__device__ void short_strand(const uint8_t* cls, long long rs, long long n, int strand, int k,
                             uint64_t shift, Slot* table, uint64_t capmask, unsigned* flags) {
  auto S = [&](long long i) -> uint32_t {
    return strand == 0 ? (uint32_t)cls[rs + i] : comp_class(cls[rs + n - 1 - i]);
  };
  uint64_t K0 = 0, pw = 1;
  for (int j = 0; j < k; ++j) { K0 += (uint64_t)digit_fw(S(j)) * pw; pw *= 5; }
  if (n == k) {                                            // :1084-1085
    oriented_or(table, capmask, k, K0, (LAM_HASH << OFFBIT) | LAM_DOLLAR, flags);
    return;
  }
  // n == k+1 (:1061-1082): the loop never runs and numba reads its variable as 0
  oriented_or(table, capmask, k, K0, (LAM_HASH << OFFBIT) | lam_fw(S(k)), flags);
  const uint64_t K1 = K0 / 5 + (uint64_t)digit_fw(S(1)) * shift;   // alpha[seq[0+1]]
  oriented_or(table, capmask, k, K1, (lam_fw(S(1)) << OFFBIT) | LAM_DOLLAR, flags);  // seq[0-k] == s[1]
}

__global__ void k_short(const uint8_t* __restrict__ cls, const long long* __restrict__ rec_start,
                        const long long* __restrict__ rec_len, const uint8_t* __restrict__ rec_flag,
                        uint64_t R, int k, uint64_t shift, int rc, Slot* table, uint64_t capmask,
                        unsigned* flags) {
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < R;
       r += (uint64_t)gridDim.x * blockDim.x) {
    if (!rec_flag[r]) continue;
    const long long n = rec_len[r];
    if (n > k + 1) continue;
    if (n < k) { atomicOr(flags, 1u); continue; }          // key -1, mask '$' (:1087-1088)
    short_strand(cls, rec_start[r], n, 0, k, shift, table, capmask, flags);
    if (rc) short_strand(cls, rec_start[r], n, 1, k, shift, table, capmask, flags);
  }
}

// Extra empty records that the reference's checkpoint/resume yields (see
// DESIGN.md): each adds the n<k sentinel.
__global__ void k_set_flag(unsigned* flags) { atomicOr(flags, 1u); }

// K5: degree scan.  Marks rdBG membership in the slot and compacts the rdBG
// keys (forward orientation c, reverse orientation rc(c)).
__global__ void __launch_bounds__(256)
k_reduce(Slot* __restrict__ table, uint64_t cap, int k, unsigned long long* __restrict__ out,
         unsigned long long* __restrict__ counters) {
  __shared__ unsigned long long red[4];
  const int lane = threadIdx.x & 63;
  const unsigned long long lt = (1ull << lane) - 1ull;
  unsigned long long ndbg = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = *reinterpret_cast<const uint4*>(table + i);
    const unsigned long long key1 = (unsigned long long)v.x | ((unsigned long long)v.y << 32);
    const uint32_t m = v.z;
    const bool occ = key1 != 0ull;
    const bool pa = occ && (m & PRES_A), pb = occ && (m & PRES_B);
    const bool ma = pa && rdbg_member(m & MASK12);
    const bool mb = pb && rdbg_member((m >> 16) & MASK12);
    ndbg += (unsigned long long)pa + (unsigned long long)pb;
    if (ma || mb) table[i].mask = m | (ma ? RDBG_A : 0u) | (mb ? RDBG_B : 0u);
    const unsigned long long ba = __ballot(ma), bb = __ballot(mb);
    const unsigned na = __builtin_popcountll(ba), nbb = __builtin_popcountll(bb);
    if (na + nbb == 0) continue;
    unsigned long long base = 0;
    if (lane == __builtin_ctzll(ba | bb)) base = atomicAdd(counters, (unsigned long long)(na + nbb));
    base = __shfl(base, __builtin_ctzll(ba | bb), 64);
    const uint64_t c = key1 - 1ull;
    if (ma) out[base + __builtin_popcountll(ba & lt)] = c;
    if (mb) out[base + na + __builtin_popcountll(bb & lt)] = rc_key(c, k);
  }
  for (int o = 32; o > 0; o >>= 1) ndbg += __shfl_down(ndbg, o, 64);
  if (lane == 0) red[threadIdx.x >> 6] = ndbg;
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

__global__ void k_merge(const Slot* __restrict__ pairs, uint64_t n, Slot* __restrict__ table,
                        uint64_t capmask, unsigned* __restrict__ flags) {
  unsigned created = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const Slot s = pairs[i];
    if (!s.key1) continue;
    created += (unsigned)table_or(table, capmask, s.key1 - 1ull, s.mask & ~(RDBG_A | RDBG_B), flags);
  }
  for (int o = 32; o > 0; o >>= 1) created += __shfl_down(created, o, 64);
  if ((threadIdx.x & 63) == 0 && created) atomicAdd(counter(flags, blockIdx.x % N_CNT), created);
}

// ------------------------------------------------------------------ host
static unsigned insert_grid() {
  static unsigned g = 0;
  if (!g) {
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
    g = (unsigned)cus * 8u;
  }
  return g;
}

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

void build_dbg(Ctx& c, const uint8_t* h_rec_flag, int extra_empty, int rc0) {
  if (!c.parsed) throw Error(-22, "build_dbg: no parsed FASTA (call pg_parse first)");
  const uint64_t R = c.n_records;
  c.rc0 = rc0;
  c.built = c.reduced = false;
  c.n_dbg = c.n_rdbg = c.n_canon = 0;
  c.windows_fw = 0;
  if (R) {
    std::vector<uint8_t> flag(R, 1);
    if (h_rec_flag)
      for (uint64_t r = 0; r < R; ++r) flag[r] = h_rec_flag[r] & 1;
    PG_HIP(hipMemcpyAsync(c.rec_flag.p, flag.data(), R, hipMemcpyHostToDevice, c.stream));
    for (uint64_t r = 0; r < R; ++r)
      if (flag[r]) {
        const int64_t n = c.h_rec_len[r];
        c.windows_fw += n > c.k ? (uint64_t)(n - c.k + 1) : 1;
      }
  }
  c.windows_total = c.windows_fw * (rc0 ? 2 : 1);
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
    if (c.n_bases) {
      if (rc0)
        hipLaunchKernelGGL((k_insert<16, true>), dim3(insert_grid()), dim3(IBLOCK), 0, c.stream,
                           c.cls.as<uint8_t>(), c.n_bases + (uint64_t)c.h_rec_start[0],
                           c.rec_start.as<long long>(), c.rec_len.as<long long>(), c.rec_flag.as<uint8_t>(),
                           R, c.k, shift, tab, cap - 1, flags);
      else
        hipLaunchKernelGGL((k_insert<16, false>), dim3(insert_grid()), dim3(IBLOCK), 0, c.stream,
                           c.cls.as<uint8_t>(), c.n_bases + (uint64_t)c.h_rec_start[0],
                           c.rec_start.as<long long>(), c.rec_len.as<long long>(), c.rec_flag.as<uint8_t>(),
                           R, c.k, shift, tab, cap - 1, flags);
      PG_HIP(hipGetLastError());
    }
    c.t1.stop(c.stream);
    if (R) {
      hipLaunchKernelGGL(k_short, dim3(grid_for(R, 256, 1024)), dim3(256), 0, c.stream,
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
  unsigned sentinel = 0, overflow = 0;
  uint64_t created = 0;
  read_flags(c, sentinel, overflow, created);
  c.rdbg_keys.reserve(8 * (2 * c.n_canon + 2));
  DevBuf& cnt = c.n_sel;
  cnt.reserve(128);
  PG_HIP(hipMemsetAsync(cnt.p, 0, 128, c.stream));
  c.t0.start(c.stream);
  hipLaunchKernelGGL(k_reduce, dim3(grid_for(c.cap, 256, 8192)), dim3(256), 0, c.stream,
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
  if (sentinel) {           // key 2^64-1, mask 32: always an rdBG member
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
  unsigned sentinel = 0, overflow = 0;
  uint64_t created = 0;
  read_flags(c, sentinel, overflow, created);
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
  const uint64_t total = n + (sentinel ? 1 : 0);
  if (h_keys && cap >= total) {
    PG_HIP(hipMemcpy(h_keys, keys.p, 8 * n, hipMemcpyDeviceToHost));
    PG_HIP(hipMemcpy(h_masks, masks.p, 2 * n, hipMemcpyDeviceToHost));
    if (sentinel) { h_keys[n] = SENTINEL; h_masks[n] = 32; }
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
  for (int attempt = 0; attempt < 8; ++attempt) {
    alloc_table(c, cap);
    clear_table(c);
    if (sentinel) hipLaunchKernelGGL(k_set_flag, dim3(1), dim3(1), 0, c.stream, c.flags.as<unsigned>());
    c.t1.init();
    c.t1.start(c.stream);
    if (n)
      hipLaunchKernelGGL(k_merge, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c.stream,
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
