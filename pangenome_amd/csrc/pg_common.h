// pg_common.h — device-side encoding, table layout and hashing shared by the
// pangenome HIP kernels (gfx950 / CDNA4, wave64).
//
// Byte classes.  The reference looks every sequence byte up in three 256-entry
// tables: the base-5 digit `alpha` (kmer_numba.py:763-768), the neighbour mask
// `lastc` (:736-743) and, for the reverse strand, `lastc[tab_rev_bytes[b]]`
// (:191-195).  All three are functions of seven byte classes, so the parse
// kernel rewrites the FASTA into one class code per base and every later
// kernel derives digits and masks from the code with packed-constant shifts
// (no table loads on the hot path).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace pg {

enum : uint8_t {
  CLS_A = 0,      // A a
  CLS_C = 1,      // C c
  CLS_G = 2,      // G g
  CLS_T = 3,      // T t
  CLS_N = 4,      // N n
  CLS_DOLLAR = 5, // '$'  (lastc 32; its reverse complement is 'N')
  CLS_OTHER = 6,  // anything else: IUPAC, '\r', '#', ... (lastc 0, digit 4, RC 'N')
};

// alpha digit per class: A0 C2 G1 T3, others 4
__host__ __device__ __forceinline__ uint32_t digit_fw(uint32_t c) { return (0x04443120u >> (4u * c)) & 0xFu; }
// alpha of tab_rev(byte): A->T 3, C->G 1, G->C 2, T->A 0, others 4
__host__ __device__ __forceinline__ uint32_t digit_rc(uint32_t c) { return (0x04440213u >> (4u * c)) & 0xFu; }
// lastc per class: A1 C8 G4 T2 N16 $32 other0
__host__ __device__ __forceinline__ uint32_t lam_fw(uint32_t c) {
  return (uint32_t)((0x0000201002040801ull >> (8u * c)) & 0xFFu);
}
// lastc of tab_rev(byte): A->T 2, C->G 4, G->C 8, T->A 1, N/$/other -> N 16
__host__ __device__ __forceinline__ uint32_t lam_rc(uint32_t c) {
  return (uint32_t)((0x0010101001080402ull >> (8u * c)) & 0xFFu);
}
// class of tab_rev(byte) (used for the explicit reverse strand of short records)
__host__ __device__ __forceinline__ uint32_t comp_class(uint32_t c) {
  return (0x04440123u >> (4u * c)) & 0xFu;   // A->T C->G G->C T->A, N/$/other -> N
}

constexpr int OFFBIT = 6;        // offbit (:745): dBG masks and label lookups
constexpr int EDGE_OFFBIT = 5;   // :1814 passes bits(=5) into rdbg_edge_weight's offbit
constexpr uint32_t LAM_DOLLAR = 32;   // '$' end marker
constexpr uint32_t LAM_HASH = 0;      // '#' start marker
constexpr uint64_t SENTINEL = ~0ull;  // the n<k key (-1 stored in a uint64 array, :1038)

// ------------------------------------------------------------------ table
// One canonical k-mer per entry.  A key X and its reverse complement rc(X)
// share the entry of c = min(X, rc(X)); the entry keeps the reference's 12-bit
// OR-mask of each orientation separately (A for c, B for rc(c)), so the dBG
// exported from it is exactly the reference's non-canonical dBG
// (kmer_numba.py:1036-1047, :1215-1221).
//
// Mask word (26 bits): [0,12) A | 1<<12 presA | [13,25) B | 1<<25 presB.
// A presence bit is needed because a key's mask can be 0 (e.g. '#' before,
// IUPAC after).
constexpr uint32_t PRES_A = 1u << 12;
constexpr int B_SHIFT = 13;
constexpr uint32_t PRES_B = PRES_A << B_SHIFT;
constexpr uint32_t MASK12 = 0xFFFu;
constexpr int MW_BITS = 26;
constexpr uint64_t MW_MASK = (1ull << MW_BITS) - 1;

__host__ __device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// 16-byte entry: the overflow table's slots and the multi-GPU exchange record.
// key1 = c + 1 (0 = empty).
struct alignas(16) Slot {
  unsigned long long key1;
  unsigned int mask;   // 26-bit mask word
  unsigned int aux;
};
// A routed stage A record on the wire (pg_route_scatter / pg_route_merge):
// h (low word, high word) and the 26-bit mask word, 12 bytes, 4-byte aligned.
// Its integrity hash is row_check(h, mask word), the hash of the 16-byte
// {h, mask word, 0} form.
struct Row12 {
  unsigned int w[3];
};

// Integrity check of one 16-byte exchange record (words w0 = key1, w1 = mask |
// aux << 32).  Sums of it (mod 2^64) over a run of records are order-free, so
// the sender's per-owner sums, the receiver's per-source sums and what the
// owner's merge reads can be compared (pg_dbg_partition_sums,
// pg_rows_checksum, pg_dbg_merge_check; dist.py raises on a mismatch).
__host__ __device__ __forceinline__ uint64_t row_check(uint64_t w0, uint64_t w1) {
  return fmix64(w0 ^ fmix64(w1 ^ 0x9E3779B97F4A7C15ull));
}

// The primary table is quotiented: a bijective hash h = perm(c) of the kb-bit
// key splits into a bucket index (high bits) and a quotient (low qbits <= 38
// bits), so [quotient | 26-bit mask word] is one 64-bit word and a new key is
// created, masks included, by a single 64-bit CAS.  A bucket is 2 words (one
// 16-byte load per probe); a key whose bucket is full goes to the small
// overflow table of 16-byte slots (linear probing).  Entries only ever go
// empty -> key and masks only gain bits, which is what lets readers tolerate
// stale plain loads (device atomics execute beyond the XCD's L2).
struct TableView {
  unsigned long long* prim;    // 2 words per bucket
  uint64_t bmask;              // buckets - 1
  uint32_t qbits, sh1, sh2;
  uint32_t rot;                // the owner domain of a routed exchange: h rotated left by rot bits (0: none)
  uint64_t kmask, m1, m2, m1i, m2i;
  Slot* ovf;
  uint64_t omask;              // overflow slots - 1
  uint64_t rc_pad, rc_inv;     // rc(): 3(5^(27-k)-1)/4 and 5^-(27-k) mod 2^64 (see rc_key27)

  // rotate left by 0 < r < kb within the kb key bits
  __host__ __device__ __forceinline__ uint64_t rotk(uint64_t h, uint32_t r) const {
    const uint32_t kb = 64u - (uint32_t)__builtin_clzll(kmask);
    return ((h << r) | (h >> (kb - r))) & kmask;
  }
  __host__ __device__ __forceinline__ uint64_t perm(uint64_t c) const {
    uint64_t h = (c * m1) & kmask;
    h ^= h >> sh1;
    h = (h * m2) & kmask;
    h ^= h >> sh2;
    return rot ? rotk(h, rot) : h;
  }
  __host__ __device__ __forceinline__ static uint64_t unxs(uint64_t y, uint32_t s) {
    uint64_t x = y;
    for (uint32_t i = s; i < 64; i += s) x = y ^ (x >> s);
    return x;
  }
  __host__ __device__ __forceinline__ uint64_t unperm(uint64_t h) const {
    if (rot) h = rotk(h, 64u - (uint32_t)__builtin_clzll(kmask) - rot);
    h = unxs(h, sh2);
    h = (h * m2i) & kmask;
    h = unxs(h, sh1);
    return (h * m1i) & kmask;
  }
  // reverse complement of a k-digit key (== rc_key(x, k)), ~10x fewer
  // instructions than the digit loop
  __host__ __device__ __forceinline__ uint64_t rc(uint64_t x) const;
  // key of the primary word w of bucket b
  __host__ __device__ __forceinline__ uint64_t key_of(uint64_t b, unsigned long long w) const {
    return unperm((b << qbits) | (uint64_t)(w >> MW_BITS));
  }
};

// Read-only lookup (kernels after the build): the 26-bit mask word of c, or 0.
// A bucket's second word is only ever filled after its first, and the overflow
// table only after both, so an empty word ends the search.
__device__ __forceinline__ uint32_t tab_get(const TableView& T, uint64_t c) {
  const uint64_t h = T.perm(c);
  const uint64_t b = h >> T.qbits, q = h & ((1ull << T.qbits) - 1ull);
  const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(T.prim + 2 * b);
  if (v.x == 0ull) return 0u;
  if ((v.x >> MW_BITS) == q) return (uint32_t)(v.x & MW_MASK);
  if (v.y == 0ull) return 0u;
  if ((v.y >> MW_BITS) == q) return (uint32_t)(v.y & MW_MASK);
  const unsigned long long key1 = c + 1ull;
  uint64_t slot = fmix64(c) & T.omask;
  for (uint64_t probe = 0; probe <= T.omask; ++probe) {
    const Slot s = T.ovf[slot];
    if (s.key1 == key1) return s.mask;
    if (s.key1 == 0ull) return 0u;
    slot = (slot + 1) & T.omask;
  }
  return 0u;
}

// modular inverse of 5 mod 2^64: (K - d) is a multiple of 5 when d is K's low
// base-5 digit, so K / 5 == (K - d) * INV5 exactly, with one 64-bit multiply
constexpr uint64_t INV5 = 0xCCCCCCCCCCCCCCCDull;

__host__ __device__ __forceinline__ uint64_t pow5(int e) {
  uint64_t r = 1;
  for (int i = 0; i < e; ++i) r *= 5;
  return r;
}

// reverse complement of a base-5 key of k digits (digit j has weight 5^j)
__host__ __device__ __forceinline__ uint64_t rc_key(uint64_t x, int k) {
  uint64_t r = 0;
  for (int j = 0; j < k; ++j) {
    uint64_t q = x / 5;
    uint32_t d = (uint32_t)(x - q * 5);
    x = q;
    uint32_t rd = d < 4 ? 3u - d : 4u;
    r = r * 5 + rd;
  }
  return r;
}

// Reverse complement through 27 digits, three 9-digit chunks at a time in
// 32-bit arithmetic (v * 0xCCCCCCCD >> 34 == v / 5 for every 32-bit v).
// Reversing a k-digit key as 27 digits puts 27-k complemented zero digits
// (3 = 'T') below it: rc_key(x, k) == (R27 - 3(5^(27-k)-1)/4) / 5^(27-k),
// an exact division, done as a multiply by 5's inverse mod 2^64.
__host__ __device__ __forceinline__ uint32_t rc_digits9(uint32_t v) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint32_t q = (uint32_t)(((uint64_t)v * 0xCCCCCCCDull) >> 34);
    const uint32_t d = v - 5u * q;
    r = r * 5u + (d < 4u ? 3u - d : 4u);
    v = q;
  }
  return r;
}
__host__ __device__ __forceinline__ uint64_t rc_key27(uint64_t x) {
  constexpr uint64_t P9 = 1953125ull, P18 = P9 * P9;
  const uint64_t a = x / P18, r = x - a * P18;
  const uint32_t b = (uint32_t)(r / P9), c = (uint32_t)(r - (uint64_t)b * P9);
  return (uint64_t)rc_digits9(c) * P18 + (uint64_t)rc_digits9(b) * P9 + rc_digits9((uint32_t)a);
}
__host__ __device__ __forceinline__ uint64_t TableView::rc(uint64_t x) const {
  return (rc_key27(x) - rc_pad) * rc_inv;
}
inline void rc_constants(int k, uint64_t& pad, uint64_t& inv) {
  uint64_t p = 1, iv = 1;
  for (int i = k; i < 27; ++i) { p *= 5; iv *= INV5; }
  pad = 3 * ((p - 1) / 4);
  inv = iv;
}

// rdBG rule (build_rdbg_jit_ :1300-1305): drop iff exactly one predecessor
// bit and exactly one successor bit
__host__ __device__ __forceinline__ bool rdbg_member(uint32_t m12) {
  return !(__builtin_popcount(m12 >> OFFBIT) == 1 && __builtin_popcount(m12 & 63u) == 1);
}

// exclusive scan over a block of BLOCK threads (BLOCK/64 waves); lds holds
// BLOCK/64 words; every thread must call it
template <int BLOCK>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* lds, uint32_t& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) lds[wid] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < BLOCK / 64; ++w) {
    uint32_t s = lds[w];
    pre += (w < wid) ? s : 0u;
    tot += s;
  }
  __syncthreads();
  total = tot;
  return pre + x - v;
}

// The class stream as K1 leaves it: the packed words (16 bases x 2 bits per
// 32-bit word) and one exception byte per 16 bases, and the class bytes only
// of the 16-base chunks with an exception (N, '$', other) or shared by two
// parse spans.  ensure_cls fills in the rest for the passes that read bytes.
struct PackedCls {
  const uint8_t* cls;
  const uint32_t* p2;
  const uint8_t* e16;
  __device__ __forceinline__ uint32_t operator[](long long i) const {
    return e16[i >> 4] ? (uint32_t)cls[i] : (p2[i >> 4] >> (2 * (i & 15))) & 3u;
  }
};
// the 4 class bytes of bases 4d .. 4d+3 of a packed word
__device__ __forceinline__ uint32_t unpack4(uint32_t w, int d) {
  const uint32_t b = (w >> (8 * d)) & 0xFFu;
  return (b | (b << 6) | (b << 12) | (b << 18)) & 0x03030303u;
}

// build_dbg for one strand of length n in {k, k+1}: emit(key, 12-bit mask)
// per window.  strand 0: s[i] = cls[rs+i]; strand 1: s[i] =
// comp_class(cls[rs+n-1-i]) (tab_rev(reversed(s)), :1217).
template <class Src, class Emit>
__device__ void short_strand(const Src& cls, long long rs, long long n, int strand, int k, uint64_t shift,
                             Emit&& emit) {
  auto S = [&](long long i) -> uint32_t {
    return strand == 0 ? (uint32_t)cls[rs + i] : comp_class(cls[rs + n - 1 - i]);
  };
  uint64_t K0 = 0, pw = 1;
  for (int j = 0; j < k; ++j) { K0 += (uint64_t)digit_fw(S(j)) * pw; pw *= 5; }
  if (n == k) {                                            // :1084-1085
    emit(K0, (LAM_HASH << OFFBIT) | LAM_DOLLAR);
    return;
  }
  // n == k+1 (:1061-1082): the loop never runs and numba reads its variable as 0
  emit(K0, (LAM_HASH << OFFBIT) | lam_fw(S(k)));
  const uint64_t K1 = K0 / 5 + (uint64_t)digit_fw(S(1)) * shift;   // alpha[seq[0+1]]
  emit(K1, (lam_fw(S(1)) << OFFBIT) | LAM_DOLLAR);                 // seq[0-k] == s[1]
}

// ---- table entries.  Entry index space: [0, nw = 2*buckets) primary words,
// then [nw, nw + overflow slots) overflow slots.
__device__ __forceinline__ uint32_t entry_mask(const TableView& T, uint64_t nw, uint64_t i) {
  if (i < nw) {
    const unsigned long long w = T.prim[i];
    return w ? (uint32_t)(w & MW_MASK) : 0u;
  }
  const Slot s = T.ovf[i - nw];
  return s.key1 ? s.mask : 0u;
}
__device__ __forceinline__ uint64_t entry_key(const TableView& T, uint64_t nw, uint64_t i) {
  if (i < nw) return T.key_of(i >> 1, T.prim[i]);
  return T.ovf[i - nw].key1 - 1ull;
}
// entry index of canonical key c (tab_get's search), or ~0 when absent
__device__ __forceinline__ uint64_t tab_find(const TableView& T, uint64_t c) {
  const uint64_t h = T.perm(c);
  const uint64_t b = h >> T.qbits, q = h & ((1ull << T.qbits) - 1ull);
  const unsigned long long* w = T.prim + 2 * b;
  if (w[0] == 0ull) return ~0ull;
  if ((w[0] >> MW_BITS) == q) return 2 * b;
  if (w[1] == 0ull) return ~0ull;
  if ((w[1] >> MW_BITS) == q) return 2 * b + 1;
  const unsigned long long key1 = c + 1ull;
  uint64_t slot = fmix64(c) & T.omask;
  for (uint64_t probe = 0; probe <= T.omask; ++probe) {
    const unsigned long long k1 = T.ovf[slot].key1;
    if (k1 == key1) return 2 * (T.bmask + 1) + slot;
    if (k1 == 0ull) return ~0ull;
    slot = (slot + 1) & T.omask;
  }
  return ~0ull;
}

// bijective XCD-aware remap (cdna_hip_programming.md §5.5 T1): blocks b,
// b+8, b+16, ... share an XCD under round-robin dispatch; give them
// consecutive work items so an XCD's L2 sees contiguous work
__device__ __forceinline__ uint64_t xcd_swizzle(uint64_t b, uint64_t nb) {
  const uint64_t q = nb / 8, r = nb % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

}  // namespace pg
