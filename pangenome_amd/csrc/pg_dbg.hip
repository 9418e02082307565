// pg_dbg.hip — K3: k-mer windows -> quotiented HBM hash table (atomic OR of
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
// stripe's tiles run on one XCD: the first genome's probe of a bucket misses,
// the other genomes' probes of it hit that XCD's L2 / the Infinity Cache.
#include <algorithm>
#include <type_traits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "pg_internal.h"

namespace pg {

constexpr int IBLOCK = 256;
constexpr int IW = 16;                        // windows per thread
constexpr int TILE = IBLOCK * IW;             // windows per tile (one block)
constexpr int IB = 8;                         // windows per probe batch
constexpr int SPAN = TILE + 64;               // staged bytes (k <= 27: TILE + k + 3 <= SPAN - 16)
constexpr int N_CNT = 64;                     // spread counters (one 64-byte line each)

// flags layout (uint32 words): [0] sentinel seen, [1] overflow, [16*(1+i)] counter i
__device__ __forceinline__ unsigned* counter(unsigned* flags, int i) { return flags + 16 * (1 + i); }

// overflow table: linear probing on 16-byte slots (CAS on key1, then OR)
__device__ int ovf_or(const TableView& T, uint64_t c, uint32_t mw, unsigned* flags) {
  const unsigned long long key1 = (unsigned long long)c + 1ull;
  uint64_t slot = fmix64(c) & T.omask;
  for (uint64_t probe = 0; probe <= T.omask && probe < 65536; ++probe) {
    Slot* s = T.ovf + slot;
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
    slot = (slot + 1) & T.omask;
  }
  atomicOr(flags + 1, 1u);
  return 0;
}

#ifdef PG_DIAG
// diagnostic build only: per-path event counters at flags[16*(2+N_CNT)+i]
#define DIAG(i) atomicAdd(flags + 16 * (2 + N_CNT) + (i), 1u)
#else
#define DIAG(i) ((void)0)
#endif

// Insert/OR one canonical key given its bucket words v (possibly stale: a
// stale empty is settled by the CAS result, a stale mask only costs a
// redundant atomicOr).  Returns 1 if this call created the entry.
__device__ __forceinline__ int tab_or_at(const TableView& T, uint64_t c, uint64_t b, uint64_t q, uint32_t mw,
                                         ulonglong2 v, unsigned* flags) {
  unsigned long long* w = T.prim + 2 * b;
  unsigned long long x = v.x;
  DIAG(0);
  if (x == 0ull) {
    DIAG(1);
    x = atomicCAS(w, 0ull, (q << MW_BITS) | mw);
    if (x == 0ull) { DIAG(2); return 1; }
  }
  if ((x >> MW_BITS) == q) {
    if ((x & mw) != mw) { DIAG(3); atomicOr(w, (unsigned long long)mw); }
    return 0;
  }
  x = v.y;
  if (x == 0ull) {
    DIAG(4);
    x = atomicCAS(w + 1, 0ull, (q << MW_BITS) | mw);
    if (x == 0ull) { DIAG(5); return 1; }
  }
  if ((x >> MW_BITS) == q) {
    if ((x & mw) != mw) { DIAG(6); atomicOr(w + 1, (unsigned long long)mw); }
    return 0;
  }
  DIAG(7);
  return ovf_or(T, c, mw, flags);
}

// tab_or_at for a batch of N windows with their (possibly stale) bucket words,
// in rounds: every CAS of a round is issued before any result is used, so a
// lane waits for about two memory-side round trips per batch instead of one
// per window.  mm[i] == 0 skips entry i.
template <int N>
__device__ __forceinline__ void tab_or_batch(const TableView& T, const uint64_t (&cc)[N], const uint64_t (&hh)[N],
                                             const uint32_t (&mm)[N], const ulonglong2 (&v)[N], unsigned* flags,
                                             unsigned& created, int dbg = 0) {
  const uint64_t qmask = (1ull << T.qbits) - 1ull;
  unsigned long long res[N];
  uint32_t need = 0, on1 = 0;                    // CAS in flight; on word 1
#pragma unroll
  for (int i = 0; i < N; ++i) {
    res[i] = 0ull;
    if (!mm[i]) continue;
    const uint64_t b = hh[i] >> T.qbits, q = hh[i] & qmask;
    unsigned long long* w = T.prim + 2 * b;
    const unsigned long long x = v[i].x, y = v[i].y;
    const unsigned long long mine = (q << MW_BITS) | mm[i];
    if (x != 0ull && (x >> MW_BITS) == q) {
      if ((x & mm[i]) != mm[i] && !(dbg & 16)) atomicOr(w, (unsigned long long)mm[i]);
    } else if (x == 0ull) {
      if (dbg & 8) { *w = mine; ++created; continue; }   // dev knob: create by plain store (racy)
      res[i] = atomicCAS(w, 0ull, mine);
      need |= 1u << i;
    } else if (y != 0ull && (y >> MW_BITS) == q) {
      if ((y & mm[i]) != mm[i]) atomicOr(w + 1, (unsigned long long)mm[i]);
    } else if (y == 0ull) {
      res[i] = atomicCAS(w + 1, 0ull, mine);
      need |= 1u << i;
      on1 |= 1u << i;
    } else {
      created += (unsigned)ovf_or(T, cc[i], mm[i], flags);
    }
  }
  for (int round = 0; round < 2 && need; ++round) {
    uint32_t next = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      if (!((need >> i) & 1u)) continue;
      const uint64_t b = hh[i] >> T.qbits, q = hh[i] & qmask;
      unsigned long long* w = T.prim + 2 * b;
      const unsigned long long old = res[i];
      const bool w1 = (on1 >> i) & 1u;
      if (old == 0ull) { ++created; continue; }
      if ((old >> MW_BITS) == q) {               // another lane created it first
        if ((old & mm[i]) != mm[i]) atomicOr(w1 ? w + 1 : w, (unsigned long long)mm[i]);
        continue;
      }
      if (!w1) {                                 // word 0 holds another key: word 1
        const unsigned long long y = v[i].y;     // non-zero words are final
        if (y != 0ull && (y >> MW_BITS) == q) {
          if ((y & mm[i]) != mm[i]) atomicOr(w + 1, (unsigned long long)mm[i]);
        } else if (y == 0ull) {
          res[i] = atomicCAS(w + 1, 0ull, (q << MW_BITS) | mm[i]);
          next |= 1u << i;
          on1 |= 1u << i;
        } else {
          created += (unsigned)ovf_or(T, cc[i], mm[i], flags);
        }
      } else {
        created += (unsigned)ovf_or(T, cc[i], mm[i], flags);
      }
    }
    need = next;
  }
}

__device__ __forceinline__ int tab_or(const TableView& T, uint64_t c, uint32_t mw, unsigned* flags) {
  const uint64_t h = T.perm(c);
  const uint64_t b = h >> T.qbits, q = h & ((1ull << T.qbits) - 1ull);
  const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(T.prim + 2 * b);
  return tab_or_at(T, c, b, q, mw, v, flags);
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

// 4*ND bytes of LDS starting at byte index idx, realigned into dwords
template <int ND>
__device__ __forceinline__ void lds_bytes(const uint8_t* s, uint32_t idx, uint32_t (&out)[ND]) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(s + (idx & ~3u));
  const uint32_t sh = (idx & 3u) * 8u;
  uint32_t raw[ND + 1];
#pragma unroll
  for (int i = 0; i <= ND; ++i) raw[i] = w[i];
#pragma unroll
  for (int i = 0; i < ND; ++i)
    out[i] = sh ? (raw[i] >> sh) | (raw[i + 1] << (32u - sh)) : raw[i];
}
template <int ND>
__device__ __forceinline__ uint32_t byte_at(const uint32_t (&w)[ND], int j) {
  return (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
}

// k2n_jit (:975-985) for both strands of the window whose first base is LDS
// byte o: K = sum alpha(s[j]) 5^j, Kr = sum alpha'(s[j]) 5^(k-1-j).  The low
// 13 digits accumulate in 32 bits (5^13 < 2^32), the rest (<= 14) in 64.
__device__ __forceinline__ void init_keys(const uint8_t* sc, uint32_t o, int k, uint64_t& K, uint64_t& Kr) {
  uint32_t lo = 0, rlo = 0;
  uint64_t hi = 0, rhi = 0;
  const int kl = k < 13 ? k : 13, kh = k - kl;
  for (int j = kl - 1; j >= 0; --j) lo = lo * 5u + digit_fw(sc[o + j]);
  for (int j = k - 1; j >= kl; --j) hi = hi * 5u + digit_fw(sc[o + j]);
  for (int j = 0; j < kh; ++j) rhi = rhi * 5u + digit_rc(sc[o + j]);
  for (int j = kh; j < k; ++j) rlo = rlo * 5u + digit_rc(sc[o + j]);
  K = (uint64_t)lo + hi * 1220703125ull;         // 5^13
  Kr = (uint64_t)rlo + rhi * 1220703125ull;
}

// K3 tile: record r's windows [stripe*TILE, (stripe+1)*TILE), with the
// record's compacted start and length carried along (one load per block).
struct TileDesc {
  long long rs, rn;
  int r, stripe;
  long long pad;
};

// ---- positional dedup against a reference record (see k_insert).  A window q
// of record g with neither record end in it, whose bytes [q-1, q+k] equal the
// reference's bytes [q'-1, q'+k] at q' = q - delta (q' interior too), has the
// reference window's key and both masks (:1069-1080); the reference inserts
// that window, so g's insert would OR nothing new and is skipped.  The drift
// delta only decides how much is skipped, never what is inserted.
constexpr int DRIFT = 512;                    // searched offsets: [-DRIFT, DRIFT]
constexpr int RSPAN = TILE + 2 * DRIFT + 96;  // staged reference bytes
constexpr int NANCH = 3;                      // anchors per tile
constexpr int ALEN = 32;                      // anchor length (bytes)

// bit j of the result: byte j of a equals byte j of b (ND dwords)
template <int ND>
__device__ __forceinline__ uint64_t byte_eq_bits(const uint32_t (&a)[ND], const uint32_t (&b)[ND]) {
  uint64_t e = 0;
#pragma unroll
  for (int i = 0; i < ND; ++i) {
    const uint32_t x = a[i] ^ b[i];
    const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
    e |= (uint64_t)(((z >> 7) | (z >> 14) | (z >> 21) | (z >> 28)) & 0xFu) << (4 * i);
  }
  return e;
}
// bit i of the result: bits [i, i+w) of e are all set (w <= 63)
__device__ __forceinline__ uint64_t run_and(uint64_t e, int w) {
  uint64_t p[6];
  p[0] = e;
#pragma unroll
  for (int b = 1; b < 6; ++b) p[b] = p[b - 1] & (p[b - 1] >> (1 << (b - 1)));
  uint64_t r = ~0ull;
  int off = 0;
#pragma unroll
  for (int b = 5; b >= 0; --b)
    if ((w >> b) & 1) { r &= p[b] >> off; off += 1 << b; }
  return r;
}

// The IW windows q0 .. q0+IW-1 (clipped at the record's last window) of one
// record staged in s_cls (s_cls[base + q] = class of position q): both
// strands' rolling keys, the canonical key and mask word of each window, and
// the probes / updates in batches of IB (windows with a `covered` bit are
// inserted by the reference record and send nothing).  Interior segments run
// from registers; a segment holding window 0 or the last window takes the
// generic path with the boundary rules.
template <bool RC>
__device__ __forceinline__ void insert_segment(const uint8_t* s_cls, long long base, long long q0, long long last,
                                               int k, uint64_t shift, const TableView& T, unsigned* flags,
                                               uint32_t covered, int dbg, unsigned& created) {
  const long long q1 = q0 + IW <= last + 1 ? q0 + IW : last + 1;
  auto S = [&](long long q) -> uint32_t { return s_cls[base + q]; };
  uint64_t K = 0, Kr = 0;
  init_keys(s_cls, (uint32_t)(base + q0), k, K, Kr);
  auto probe = [&](const uint64_t (&cc)[IB], const uint64_t (&hh)[IB], const uint32_t (&mm)[IB]) {
    if (dbg & 1) {                                 // dev knob: windows only
#pragma unroll
      for (int i = 0; i < IB; ++i) created += (unsigned)(hh[i] ^ mm[i]) & 1u;
      return;
    }
    ulonglong2 v[IB];
#pragma unroll
    for (int i = 0; i < IB; ++i)                   // IB independent probes in flight; a skipped
      v[i] = mm[i] ? *reinterpret_cast<const ulonglong2*>(T.prim + 2 * (hh[i] >> T.qbits))   // window
                   : make_ulonglong2(0ull, 0ull);                                           // sends none
    if (dbg & 2) {                                 // dev knob: loads only
#pragma unroll
      for (int i = 0; i < IB; ++i) created += (unsigned)(v[i].x ^ v[i].y) & 1u;
      return;
    }
    tab_or_batch(T, cc, hh, mm, v, flags, created, dbg);
  };
  if (q0 > 0 && q0 + IW <= last) {
    // interior segment (no window 0, no last window, all IW live): the context
    // bytes come from LDS once, into registers; P(i) = S(q-1), D(i) = S(q+k-1)
    // for window q = q0 + i, and D(i+1) = S(q+k)
    const uint32_t o = (uint32_t)(base + q0);
    uint32_t P[IW / 4], D[IW / 4 + 1];
    lds_bytes(s_cls, o - 1, P);
    lds_bytes(s_cls, o + (uint32_t)k - 1, D);
#pragma unroll
    for (int h = 0; h < IW / IB; ++h) {
      uint64_t cc[IB], hh[IB];
      uint32_t mm[IB];
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        const int x = h * IB + i;
        const uint32_t p = byte_at(P, x), s = byte_at(D, x + 1);
        if (x) {                                   // Nu // 5 + alpha * 5^(k-1) (:1072)
          const uint32_t din = byte_at(D, x);
          K = (K - digit_fw(p)) * INV5 + (uint64_t)digit_fw(din) * shift;
          Kr = (Kr - (uint64_t)digit_rc(p) * shift) * 5 + digit_rc(din);
        }
        const uint32_t mf = (lam_fw(p) << OFFBIT) | lam_fw(s) | PRES_A;
        if (RC) {
          const uint32_t mr = (lam_rc(s) << OFFBIT) | lam_rc(p) | PRES_A;
          const bool lt = K < Kr, eq = K == Kr;
          cc[i] = lt ? K : Kr;
          mm[i] = eq ? (mf | mr) : lt ? (mf | (mr << B_SHIFT)) : (mr | (mf << B_SHIFT));
        } else {
          const bool le = K <= Kr;
          cc[i] = le ? K : Kr;
          mm[i] = le ? mf : (mf << B_SHIFT);
        }
        if ((covered >> x) & 1u) mm[i] = 0;        // the reference inserts this window
        hh[i] = T.perm(cc[i]);
      }
      probe(cc, hh, mm);
    }
    return;
  }
  for (long long qb = q0; qb < q1; qb += IB) {
    uint64_t cc[IB], hh[IB];
    uint32_t mm[IB];
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const long long q = qb + i;
      cc[i] = 0;
      mm[i] = 0;
      if (q < q1) {
        if (q != q0) {                             // Nu // 5 + alpha * 5^(k-1) (:1072)
          const uint32_t dout = S(q - 1), din = S(q + k - 1);
          K = (K - digit_fw(dout)) * INV5 + (uint64_t)digit_fw(din) * shift;
          Kr = (Kr - (uint64_t)digit_rc(dout) * shift) * 5 + digit_rc(din);
        }
        // forward window q: pred '#' at q==0, s[q-2] at the last window (:1080 quirk), else s[q-1]
        const uint32_t fpred = q == 0 ? LAM_HASH : lam_fw(S(q - (q == last ? 2 : 1)));
        const uint32_t fsucc = q == last ? LAM_DOLLAR : lam_fw(S(q + k));
        const uint32_t mf = (fpred << OFFBIT) | fsucc | PRES_A;
        if (RC) {
          // its twin: reverse-strand window n-k-q, same boundary rules on that strand
          const uint32_t rpred = q == last ? LAM_HASH : lam_rc(S(q + k + (q == 0 ? 1 : 0)));
          const uint32_t rsucc = q == 0 ? LAM_DOLLAR : lam_rc(S(q - 1));
          const uint32_t mr = (rpred << OFFBIT) | rsucc | PRES_A;
          if (K < Kr)      { cc[i] = K;  mm[i] = mf | (mr << B_SHIFT); }
          else if (K > Kr) { cc[i] = Kr; mm[i] = mr | (mf << B_SHIFT); }
          else             { cc[i] = K;  mm[i] = mf | mr; }
        } else {
          if (K <= Kr) { cc[i] = K; mm[i] = mf; } else { cc[i] = Kr; mm[i] = mf << B_SHIFT; }
        }
      }
      hh[i] = T.perm(cc[i]);
    }
    probe(cc, hh, mm);
  }
}

// K3.  One block per tile (record, stripe j): windows [j*TILE, (j+1)*TILE) of
// a record with n >= k+2.  The tile's class codes (plus the k+3 bytes of
// context around it) are staged in LDS with 16-byte loads; thread t takes IW
// consecutive windows, rolls both strands' keys across them, and probes the
// table in batches of IB windows: IB independent bucket loads in flight per
// lane, and only windows whose entry is not already complete take the CAS /
// atomicOr / overflow path.
// A segment left with work after the coverage pass (k_cover).
struct WorkItem {
  long long rs, last, q0;
  uint32_t covered, pad;
};

// The queue is NQ sub-queues, each with its own counter on its own 64-byte
// line; a tile appends to sub-queue (its block) % NQ.  One counter shared by
// all ~120 K tiles of a C3 launch serialises their atomics at the memory side
// (1.48 ms measured, tools/rates.hip) - as long as the whole coverage pass;
// 64 counters take 0.045 ms.  A tile appends at most IBLOCK items.
constexpr int NQ = 64;
constexpr int QSTRIDE = 8;                    // counter spacing (unsigned long long words)

// Drift of the tile's record against a reference record at NANCH anchors:
// s_best[a] = (|delta| << 16) | (delta + DRIFT) of a delta in [-DRIFT, DRIFT]
// whose ALEN bytes match, ~0u if none.  Any match serves: the drift only
// decides how much is skipped, never what is inserted.
//
// The coverage pass is VALU-bound (PMC: ~1200 VALU per wave per tile, at
// 4 cycles per wave64 instruction), so the search is staged:
//  1. around the record's last drift found by any of its tiles (`hint`,
//     +-HWIN): one wave per anchor, <= 34 dword tasks.  Tiles in flight are
//     ~20 stripes apart, over which the drift of the synthetic pangenomes
//     moves by ~25 (indels of 1-10 bp, 2e-4 per base per pair), so this
//     almost always hits;
//  2. the full [-DRIFT, DRIFT] for anchors still without a match.
// A task is one reference dword w (4 candidate starts), whose shifted words
// are compared with the anchor's first 4 bytes (~1 in 256 candidates passes
// on a ~2-bit stream) before the full ALEN-byte check.  Ends with a barrier;
// thread 0 publishes the drift to *hint_out.
constexpr int ASTEP = (TILE - ALEN - 16) / (NANCH - 1);      // anchor spacing
constexpr int HWIN = 120;                                    // stage-1 window: hint +- HWIN
__device__ __forceinline__ void find_drift(const uint8_t* s_cls, long long base, const uint8_t* s_ref,
                                           long long rbase, long long qt, long long rn, long long plo,
                                           long long phi, int hint, unsigned* s_best, int* hint_out,
                                           unsigned* diag = nullptr) {
  static_assert(NANCH * 64 <= IBLOCK && (2 * HWIN) / 4 + 2 <= 64, "one wave per anchor in stage 1");
  constexpr int NW = (2 * DRIFT + 3) / 4 + 2;                 // dword tasks per anchor (full range)
  const uint32_t* rw = reinterpret_cast<const uint32_t*>(s_ref);
  // anchor ai's candidates: reference starts ib in [lo, hi] (s_ref indices);
  // ib = ibhi - d for d = delta + DRIFT
  auto geom = [&](int ai, int& ia, int& ibhi, int& lo, int& hi) {
    const long long a = qt + 8 + (long long)ai * ASTEP;       // anchor: record positions [a, a + ALEN)
    ia = (int)(base + a);
    ibhi = (int)(rbase + a + DRIFT);
    lo = max(ibhi - 2 * DRIFT, (int)(rbase + plo));
    hi = a + ALEN > rn ? -1 : min(ibhi, (int)(rbase + phi) - ALEN);
  };
  // The prefilter compares 8 bytes: with 4, ~63% of waves had a lane whose
  // candidate passed, and the whole wave then ran the full check (SIMT).
  auto task = [&](int ai, int ia, int ibhi, int lo, int hi, int w) {
    uint32_t x[2];
    lds_bytes(s_cls, (uint32_t)ia, x);                        // one address per anchor: broadcast
    const uint32_t W0 = rw[w], W1 = rw[w + 1], W2 = rw[w + 2];
    // the 4 candidates' prefilter as a bit set, without branches: one
    // divergent branch per task (rarely taken) instead of one per candidate
    uint32_t hit = 0;
#pragma unroll
    for (int sb = 0; sb < 4; ++sb) {
      const int ib = 4 * w + sb;
      const bool h = (ib >= lo) & (ib <= hi) & (__builtin_amdgcn_alignbyte(W1, W0, sb) == x[0]) &
                     (__builtin_amdgcn_alignbyte(W2, W1, sb) == x[1]);
      hit |= (uint32_t)h << sb;
    }
    if (hit) {
      uint32_t A[ALEN / 4];
      lds_bytes(s_cls, (uint32_t)ia, A);
      do {
        const int ib = 4 * w + __builtin_ctz(hit);
        hit &= hit - 1u;
        uint32_t B[ALEN / 4];
        lds_bytes(s_ref, (uint32_t)ib, B);
        bool eq = true;
#pragma unroll
        for (int i = 0; i < ALEN / 4; ++i) eq &= B[i] == A[i];
        const int d = ibhi - ib;                              // delta + DRIFT
        const unsigned ad = (unsigned)(d > DRIFT ? d - DRIFT : DRIFT - d);
        if (eq) atomicMin(&s_best[ai], (ad << 16) | (unsigned)d);
      } while (hit);
    }
  };
  if (hint >= 0) {                                            // block-uniform
    const int ai = (int)threadIdx.x >> 6, m = (int)threadIdx.x & 63;
    if (ai < NANCH) {
      int ia, ibhi, lo, hi;
      geom(ai, ia, ibhi, lo, hi);
      lo = max(lo, ibhi - (hint + HWIN));
      hi = min(hi, ibhi - (hint - HWIN));
      const int w = (lo >> 2) + m;
      if (lo <= hi && 4 * w <= hi) task(ai, ia, ibhi, lo, hi, w);
    }
    __syncthreads();
  }
  // Stage 2 only when stage 1 found no anchor at all: an anchor that misses
  // next to found ones sits on a variant (or an indel), where the full range
  // finds nothing either (PMC: stage 2 ran for ~1.5 anchors per tile when it
  // ran per missing anchor); segment_covered tries the drifts that were found.
  const bool any = (s_best[0] & s_best[1] & s_best[2]) != ~0u;   // block-uniform
  static_assert(NANCH == 3, "any-anchor test");
  if (diag && threadIdx.x == 0) {                             // dev counters: hint stage ran / missed
    atomicAdd(diag, hint >= 0 ? 1u : 0u);
    atomicAdd(diag + 1, any ? 0u : 1u);
  }
#pragma unroll 1
  for (int ai = 0; ai < NANCH; ++ai) {
    if (any || s_best[ai] != ~0u) continue;                   // block-uniform
    int ia, ibhi, lo, hi;
    geom(ai, ia, ibhi, lo, hi);
    for (int w = (lo >> 2) + (int)threadIdx.x; 4 * w <= hi && w < (lo >> 2) + NW; w += IBLOCK)
      task(ai, ia, ibhi, lo, hi, w);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int h = -1;
    for (int ai = NANCH - 1; ai >= 0; --ai)
      if (s_best[ai] != ~0u) h = (int)(s_best[ai] & 0xFFFFu);
    if (h >= 0) *hint_out = h;
  }
}

// find_drift for k_cover's two references at once: stage 1 of all 2 x NANCH
// (reference, anchor) pairs runs in one round, two pairs per wave (32 lanes
// each: hint +- HWIN2), then stage 2 for a reference whose stage 1 found
// nothing.  One barrier instead of four; the hints and drift sets are
// published by the caller.
constexpr int HWIN2 = 56;
struct DriftRef {
  const uint8_t* s;
  long long rbase, plo, phi;
  int hint;
  unsigned* best;
};
__device__ __forceinline__ void find_drift_pair(const uint8_t* s_cls, long long base, long long qt, long long rn,
                                                const DriftRef& A, const DriftRef& B, bool two,
                                                unsigned* diag = nullptr) {
  static_assert(2 * NANCH * 32 <= IBLOCK && (2 * HWIN2) / 4 + 2 <= 32, "two pairs per wave in stage 1");
  constexpr int NW = (2 * DRIFT + 3) / 4 + 2;
  auto task = [&](const uint8_t* s_ref, int ia, int ibhi, int lo, int hi, int w, unsigned* best) {
    const uint32_t* rw = reinterpret_cast<const uint32_t*>(s_ref);
    uint32_t x[2];
    lds_bytes(s_cls, (uint32_t)ia, x);
    const uint32_t W0 = rw[w], W1 = rw[w + 1], W2 = rw[w + 2];
    uint32_t hit = 0;
#pragma unroll
    for (int sb = 0; sb < 4; ++sb) {
      const int ib = 4 * w + sb;
      const bool h = (ib >= lo) & (ib <= hi) & (__builtin_amdgcn_alignbyte(W1, W0, sb) == x[0]) &
                     (__builtin_amdgcn_alignbyte(W2, W1, sb) == x[1]);
      hit |= (uint32_t)h << sb;
    }
    if (hit) {
      uint32_t Aw[ALEN / 4];
      lds_bytes(s_cls, (uint32_t)ia, Aw);
      do {
        const int ib = 4 * w + __builtin_ctz(hit);
        hit &= hit - 1u;
        uint32_t Bw[ALEN / 4];
        lds_bytes(s_ref, (uint32_t)ib, Bw);
        bool eq = true;
#pragma unroll
        for (int i = 0; i < ALEN / 4; ++i) eq &= Bw[i] == Aw[i];
        const int d = ibhi - ib;
        const unsigned ad = (unsigned)(d > DRIFT ? d - DRIFT : DRIFT - d);
        if (eq) atomicMin(best, (ad << 16) | (unsigned)d);
      } while (hit);
    }
  };
  auto geom = [&](const DriftRef& R, int ai, int& ia, int& ibhi, int& lo, int& hi) {
    const long long a = qt + 8 + (long long)ai * ASTEP;
    ia = (int)(base + a);
    ibhi = (int)(R.rbase + a + DRIFT);
    lo = max(ibhi - 2 * DRIFT, (int)(R.rbase + R.plo));
    hi = a + ALEN > rn ? -1 : min(ibhi, (int)(R.rbase + R.phi) - ALEN);
  };
  {
    const int pr = (int)threadIdx.x >> 5, m = (int)threadIdx.x & 31;
    const bool second = pr >= NANCH;
    if (pr < 2 * NANCH && (!second || two)) {
      const DriftRef& R = second ? B : A;
      const int ai = second ? pr - NANCH : pr;
      if (R.hint >= 0) {
        int ia, ibhi, lo, hi;
        geom(R, ai, ia, ibhi, lo, hi);
        lo = max(lo, ibhi - (R.hint + HWIN2));
        hi = min(hi, ibhi - (R.hint - HWIN2));
        const int w = (lo >> 2) + m;
        if (lo <= hi && 4 * w <= hi) task(R.s, ia, ibhi, lo, hi, w, R.best + ai);
      }
    }
  }
  __syncthreads();
  static_assert(NANCH == 3, "any-anchor test");
  const bool anyA = (A.best[0] & A.best[1] & A.best[2]) != ~0u;            // block-uniform
  const bool anyB = !two || (B.best[0] & B.best[1] & B.best[2]) != ~0u;
  if (diag && threadIdx.x == 0) {                             // dev counters: hint stage ran / missed
    atomicAdd(diag, A.hint >= 0 ? 1u : 0u);
    atomicAdd(diag + 1, anyA ? 0u : 1u);
    if (two) {
      atomicAdd(diag + 2, B.hint >= 0 ? 1u : 0u);
      atomicAdd(diag + 3, anyB ? 0u : 1u);
    }
  }
  if (anyA && anyB) return;                                   // (the caller's barrier follows)
#pragma unroll 1
  for (int ri = 0; ri < 2; ++ri) {
    const DriftRef& R = ri ? B : A;
    if (ri ? anyB : anyA) continue;                           // block-uniform
#pragma unroll 1
    for (int ai = 0; ai < NANCH; ++ai) {
      int ia, ibhi, lo, hi;
      geom(R, ai, ia, ibhi, lo, hi);
      for (int w = (lo >> 2) + (int)threadIdx.x; 4 * w <= hi && w < (lo >> 2) + NW; w += IBLOCK)
        task(R.s, ia, ibhi, lo, hi, w, R.best + ai);
    }
  }
  __syncthreads();
}

// the hint a tile publishes: the drift of its first anchor that matched
__device__ __forceinline__ void publish_hint(const unsigned* best, int* hint_out) {
  int h = -1;
  for (int ai = NANCH - 1; ai >= 0; --ai)
    if (best[ai] != ~0u) h = (int)(best[ai] & 0xFFFFu);
  if (h >= 0) *hint_out = h;
}

// Covered windows of the interior segment q0 .. q0+IW-1 (bit i: window q0+i):
// its bytes [q-1, q+k] equal the reference's at q - delta for one of the
// anchors' drifts (reference window interior and staged too).
__device__ __forceinline__ uint32_t segment_covered(const uint8_t* s_cls, long long base, const uint8_t* s_ref,
                                                    long long rbase, long long q0, int k, long long rfn,
                                                    long long plo, long long phi, const unsigned* s_best) {
  const uint32_t o = (uint32_t)(base + q0);
  constexpr int NB = (IW + 27 + 1 + 3) / 4;                  // bytes q0-1 .. q0+IW+k-1, k <= 27
  uint32_t G[NB];
  lds_bytes(s_cls, o - 1, G);
  uint32_t covered = 0;
  unsigned prev = ~0u;
  for (int ai = 0; ai < NANCH; ++ai) {
    const unsigned b = s_best[ai];
    if (b == ~0u || (b & 0xFFFFu) == prev) continue;
    prev = b & 0xFFFFu;
    const long long p0 = q0 - ((long long)(b & 0xFFFFu) - DRIFT);   // reference window of q0
    if (p0 < 1 || p0 + IW > rfn - k || p0 - 1 < plo || p0 + IW + k > phi) continue;
    uint32_t Rw[NB];
    lds_bytes(s_ref, (uint32_t)(rbase + p0 - 1), Rw);
    uint32_t diff = 0;
#pragma unroll
    for (int i = 0; i < NB; ++i) diff |= G[i] ^ Rw[i];
    if (diff == 0) return (1u << IW) - 1u;                    // the common case: all context bytes equal
    covered |= (uint32_t)(run_and(byte_eq_bits(G, Rw), k + 2) & ((1u << IW) - 1u));
  }
  return covered;
}

// 4*ND bytes of LDS from byte index idx through 16-byte reads (ds_read_b128:
// lanes 16 B apart hit distinct banks, where the dword reads of lds_bytes are
// 4-way conflicted), realigned in registers.  idx & 15 must be the same for
// every lane of the wave (it selects the shift by a uniform branch).
template <int ND>
__device__ __forceinline__ void lds_bytes16(const uint8_t* s, uint32_t idx, uint32_t (&out)[ND]) {
  constexpr int NW = ((ND + 3) / 4 + 1) * 4;       // dwords read: ceil(ND/4)+1 chunks of 16 B
  uint32_t raw[NW];
  const uint32_t a = idx & ~15u;
#pragma unroll
  for (int q = 0; q < NW / 4; ++q) {
    const uint4 v = *reinterpret_cast<const uint4*>(s + a + 16u * q);
    raw[4 * q] = v.x; raw[4 * q + 1] = v.y; raw[4 * q + 2] = v.z; raw[4 * q + 3] = v.w;
  }
  const uint32_t sb = idx & 3u;
  auto take = [&](auto W) {
    constexpr int w = decltype(W)::value;
#pragma unroll
    for (int i = 0; i < ND; ++i) out[i] = __builtin_amdgcn_alignbyte(raw[w + i + 1], raw[w + i], sb);
  };
  switch ((idx >> 2) & 3u) {
    case 0: take(std::integral_constant<int, 0>{}); break;
    case 1: take(std::integral_constant<int, 1>{}); break;
    case 2: take(std::integral_constant<int, 2>{}); break;
    default: take(std::integral_constant<int, 3>{}); break;
  }
}

// The distinct drifts the anchors found, with everything segment_cover
// needs precomputed once per tile in 32-bit tile-relative form (block-uniform,
// so scalar): segment q0 = qt + rel may use drift j iff lo[j] <= rel <= hi[j]
// (its reference window p0 = q0 - delta interior and staged), and then reads
// the reference bytes at LDS index o + off[j], o = the segment's s_cls index.
struct Drifts {
  int n;
  int off[NANCH], lo[NANCH], hi[NANCH];
};
__device__ __forceinline__ Drifts drifts_of(const unsigned* s_best, long long qt, long long base, long long rbase,
                                            long long rfn, long long plo, long long phi, int k) {
  Drifts D;
  D.n = 0;
#pragma unroll
  for (int j = 0; j < NANCH; ++j) D.off[j] = D.lo[j] = D.hi[j] = 0;
  const long long pl = plo + 1 > 1 ? plo + 1 : 1;                       // p0 - 1 >= plo, p0 >= 1
  const long long ph = rfn - k - IW < phi - IW - k ? rfn - k - IW : phi - IW - k;   // p0 + IW <= rfn - k, .. <= phi
#pragma unroll
  for (int ai = 0; ai < NANCH; ++ai) {
    const unsigned b = s_best[ai];
    if (b == ~0u) continue;
    const int d = (int)(b & 0xFFFFu) - DRIFT;                           // delta: q0 - p0
    bool dup = false;
#pragma unroll
    for (int j = 0; j < ai; ++j) dup |= j < D.n && D.off[j] == (int)(rbase - base) - d;
    if (dup) continue;
    const long long lo = pl + d - qt, hi = ph + d - qt;
    const int l32 = (int)(lo < -(1ll << 30) ? -(1ll << 30) : lo), h32 = (int)(hi > (1ll << 30) ? (1ll << 30) : hi);
    const int o32 = (int)(rbase - base) - d;
#pragma unroll
    for (int j = 0; j <= ai; ++j)                             // static indices: registers, not scratch
      if (j == D.n) { D.lo[j] = l32; D.hi[j] = h32; D.off[j] = o32; }
    ++D.n;
  }
  return D;
}

// Covered windows of the interior segment whose context bytes start at s_cls
// index o (rel = q0 - qt), against the reference drifts D: segment_covered's
// rule, on 16-byte LDS reads (lds_bytes16: the segment start q0 - 1 has the
// same alignment in every lane of a tile, and so does its reference window),
// with a partial segment resolved at dword granularity.  Dword granularity is
// conservative (a window next to a mismatch may be left to the work pass,
// which only costs a probe) and costs ~30 VALU where the byte-exact run test
// cost ~150 — and a wave pays it whenever any of its 64 segments is partial
// (C3: ~13 % are, so nearly every wave), which made the compare the largest
// part of this pass (PMC: 327 of 659 VALU per wave).
__device__ __forceinline__ uint32_t segment_cover(const uint8_t* s_cls, const uint8_t* s_ref, uint32_t o, int rel,
                                                  const uint32_t (&G)[(IW + 27 + 1 + 3) / 4], const Drifts& D,
                                                  int k) {
  static_assert(IW == 16, "uniform 16-byte alignment of segment starts");
  constexpr int NB = (IW + 27 + 1 + 3) / 4;
  constexpr uint32_t ALL = (1u << IW) - 1u;
  uint32_t covered = 0;
  // branch-free per lane: a segment outside drift j's valid range reads its
  // (staged, in-bounds) bytes anyway and discards the result
#pragma unroll
  for (int j = 0; j < NANCH; ++j) {
    if (j >= D.n) break;                                      // block-uniform
    const bool ok = (rel >= D.lo[j]) & (rel <= D.hi[j]);
    uint32_t Rw[NB];
    lds_bytes16(s_ref, o + (uint32_t)(ok ? D.off[j] : 0), Rw);
    uint32_t nz = 0;
#pragma unroll
    for (int i = 0; i < NB; ++i) nz |= (G[i] != Rw[i] ? 1u : 0u) << i;
    nz &= (2u << ((k + IW) >> 2)) - 1u;                       // bytes past k+IW do not matter
    const int first = 4 * __builtin_ctz(nz | 0x80000000u), last = 4 * (31 - __builtin_clz(nz | 1u)) + 3;
    const int ulo = max(0, first - k - 1), uhi = min(IW - 1, last);
    const uint32_t c = nz == 0 ? ALL : ALL & ~(((2u << uhi) - 1u) & ~((1u << ulo) - 1u));
    covered |= ok ? c : 0u;
  }
  return covered;
}

// Staging geometry of tile (record [rs, rs+rn), stripe): class positions
// [lo, hi) from the 16-byte aligned a0 (windows qt .. qt+TILE-1 read from q-2,
// the last-window pred, to q+k+1, the twin pred of window 0), and the
// reference positions [plo, phi) = this stripe +- DRIFT from ra0.
struct Stage {
  long long qt, a0, hi, plo, phi, ra0, rend;
};
// the reference span of stripe qt (record [rfs, rfs + rfn))
__device__ __forceinline__ void ref_span(Stage& g, int k, long long rfs, long long rfn) {
  g.plo = g.qt - 1 - DRIFT > 0 ? g.qt - 1 - DRIFT : 0;
  g.phi = g.qt + TILE + k + 1 + DRIFT < rfn ? g.qt + TILE + k + 1 + DRIFT : rfn;
  g.ra0 = (rfs + g.plo) & ~15ll;
  g.rend = rfs + g.phi;
}
__device__ __forceinline__ Stage stage_of(const TileDesc& td, int k, bool dedup, long long rfs, long long rfn) {
  Stage g;
  g.qt = (long long)td.stripe * TILE;
  const long long lo = td.rs + (g.qt >= 2 ? g.qt - 2 : 0);
  g.hi = td.rs + (g.qt + TILE + k + 2 < td.rn ? g.qt + TILE + k + 2 : td.rn);
  g.a0 = lo & ~15ll;
  g.plo = g.phi = g.ra0 = g.rend = 0;
  if (dedup) ref_span(g, k, rfs, rfn);
  return g;
}

// K3 (fused form: PG_K3_DBG=256 or no reference).  One block per tile
// (record, stripe j): windows [j*TILE, (j+1)*TILE) of a record with n >= k+2.
// The tile's class codes (plus the k+3 bytes of context around it) are
// staged in LDS with 16-byte loads; thread t takes IW consecutive windows,
// rolls both strands' keys across them, and probes the table in batches of
// IB windows: IB independent bucket loads in flight per lane, and only
// windows whose entry is not already complete take the CAS / atomicOr /
// overflow path.  Segments fully covered by the reference record send
// nothing; the rest are compacted so that only they run insert_segment.
template <bool RC>
__global__ void __launch_bounds__(IBLOCK)
k_insert(const uint8_t* __restrict__ cls, const TileDesc* __restrict__ descs, int k, uint64_t shift, TableView T,
         unsigned* __restrict__ flags, int ref, long long rfs, long long rfn, int dbg) {
  __shared__ __attribute__((aligned(16))) uint8_t s_cls[SPAN + 16];
  __shared__ __attribute__((aligned(16))) uint8_t s_ref[RSPAN];
  __shared__ unsigned s_best[NANCH];
  __shared__ uint32_t s_work[IBLOCK];
  __shared__ uint32_t s_scan[IBLOCK / 64];
  const TileDesc td = descs[xcd_swizzle(blockIdx.x, gridDim.x)];   // one dependent load per block
  const int r = td.r;
  const long long rs = td.rs, rn = td.rn;
  const long long last = rn - k;                              // last window index
  const bool dedup = ref >= 0 && ref != r && !(dbg & 32);    // block-uniform
  const Stage g = stage_of(td, k, dedup, rfs, rfn);
  for (long long off = (long long)threadIdx.x * 16; g.a0 + off < g.hi; off += IBLOCK * 16)
    *reinterpret_cast<uint4*>(s_cls + off) = *reinterpret_cast<const uint4*>(cls + g.a0 + off);
  if (dedup) {
    for (long long off = (long long)threadIdx.x * 16; g.ra0 + off < g.rend; off += IBLOCK * 16)
      *reinterpret_cast<uint4*>(s_ref + off) = *reinterpret_cast<const uint4*>(cls + g.ra0 + off);
    if (threadIdx.x < NANCH) s_best[threadIdx.x] = ~0u;
  }
  __syncthreads();
  const long long base = rs - g.a0, rbase = rfs - g.ra0;      // LDS index of record position 0
  int dummy = -1;
  if (dedup) find_drift(s_cls, base, s_ref, rbase, g.qt, rn, g.plo, g.phi, -1, s_best, &dummy);
  uint32_t covered = 0;
  unsigned created_acc = 0;
  const long long q0 = g.qt + (long long)threadIdx.x * IW;
  if (dedup && q0 > 0 && q0 + IW <= last)
    covered = segment_covered(s_cls, base, s_ref, rbase, q0, k, rfn, g.plo, g.phi, s_best);
  const bool work = q0 <= last && covered != (1u << IW) - 1u;
  uint32_t nwork;
  const uint32_t pos = block_excl_scan<IBLOCK>(work ? 1u : 0u, s_scan, nwork);
  if (work) s_work[pos] = threadIdx.x | (covered << 16);
  if ((dbg & 64) && threadIdx.x == 0) {           // dev knob: segments with work / with windows
    atomicAdd(flags + 16 * (2 + N_CNT) + 8, nwork);
    atomicAdd(flags + 16 * (2 + N_CNT) + 9, (unsigned)(dedup ? 1 : 0));
  }
  if ((dbg & 64) && q0 <= last) {
    atomicAdd(flags + 16 * (2 + N_CNT) + 10, 1u);
    atomicAdd(flags + 16 * (2 + N_CNT) + 11, (unsigned)__builtin_popcount(covered));
  }
  __syncthreads();
  if (threadIdx.x < nwork) {
    covered = s_work[threadIdx.x] >> 16;
    insert_segment<RC>(s_cls, base, g.qt + (long long)(s_work[threadIdx.x] & 0xFFFFu) * IW, last, k, shift, T,
                       flags, covered, dbg, created_acc);
  }
  block_count(created_acc, flags);                 // every thread: one barrier per wave
}

// tiles [t, te) of XCD x in chunk c of nch (host and device)
// (a chunk is the fraction [b0, b1) / bt of every XCD's eighth)
__host__ __device__ __forceinline__ void xcd_chunk(uint64_t ntiles, uint32_t b0, uint32_t b1, uint32_t bt, uint64_t x,
                                                   uint64_t& t, uint64_t& te) {
  const uint64_t xs = ntiles * x / 8, xl = ntiles * (x + 1) / 8 - xs;
  t = xs + xl * b0 / bt;
  te = xs + xl * b1 / bt;
}

// K3 coverage pass (two-pass form, the default with a lead record).  One
// block per tile, like k_insert: the drift against the lead (find_drift),
// each segment's covered windows (segment_cover), and the segments left
// with work appended to the queue for k_insert_work.
// Second reference.  Every follower also differs from the lead at the lead's
// own variant sites, where all followers share the other allele: with the
// lead alone those windows were probed once per follower (C3: ~14 M of 51 M
// probes found their key already there).  So a second record (ref2) is
// searched too, and a window covered by either reference is skipped.  ref2's
// own windows are deduped against the lead only; a window it leaves to the
// lead has the lead's context, key and masks, so "covered by ref2" still
// means "inserted".
// Chunks and XCDs: each XCD owns a contiguous eighth of the tile list
// (stripe-major, so its blocks share reference spans in its own L2), and
// chunk c of nch launches takes the c-th part of every XCD's eighth, so an
// XCD's drift hints carry over from the end of its previous chunk to the
// start of the next (a contiguous chunk jumped each XCD a quarter genome
// ahead, and the stage-2 search then ran on ~9 % of tiles).  A persistent, software-pipelined form of
// this kernel (register prefetch of the next tile) measured slower: 1.02 vs
// 0.76 ms at 64 VGPRs with spills, against one-tile blocks at 8 waves/SIMD.
__global__ void __launch_bounds__(IBLOCK)
k_cover(const uint8_t* __restrict__ cls, const TileDesc* __restrict__ descs, WorkItem* __restrict__ queue,
        unsigned long long* __restrict__ qcount, unsigned long long qcap, int k, int ref, long long rfs,
        long long rfn, int ref2, long long r2s, long long r2n, int* __restrict__ hints, int nrec,
        uint64_t ntiles, uint32_t b0, uint32_t b1, uint32_t bt, int dbg) {
  __shared__ __attribute__((aligned(16))) uint8_t s_cls[SPAN + 16];
  __shared__ __attribute__((aligned(16))) uint8_t s_ref[RSPAN];
  __shared__ __attribute__((aligned(16))) uint8_t s_ref2[RSPAN];
  __shared__ unsigned s_best[NANCH], s_best2[NANCH];
  __shared__ uint32_t s_scan[IBLOCK / 64];
  __shared__ unsigned long long s_qbase;
  uint64_t t, te;
  xcd_chunk(ntiles, b0, b1, bt, blockIdx.x & 7, t, te);
  t += blockIdx.x >> 3;
  if (t >= te) return;                             // (block-uniform, before any barrier)
  const TileDesc td = descs[t];
  const long long rs = td.rs, rn = td.rn, last = rn - k;
  const bool dedup = ref >= 0 && ref != td.r && !(dbg & 32);  // block-uniform
  const bool dedup2 = dedup && ref2 >= 0 && ref2 != td.r && !(dbg & 16384);
  // hints per (XCD, reference, record): the XCD swizzle gives each XCD its
  // own contiguous eighth of the tile list, so one shared hint per record
  // alternated between stripes ~150 apart and the hint window missed on
  // 15-24 % of the tiles
  int* hx = hints + (size_t)(blockIdx.x & 7) * 2 * nrec;
  // (no drift known yet: try delta 0 first, the drift at a record's start)
  // (plain loads may return a stale line from this CU's L1: device-scope
  // loads cut the stage-2 searches 14 k -> 0.9 k per build and k_cover alone
  // 1.56 -> 1.49 ms, yet the whole K3 span measured ~0.5 % slower with them)
  int h1 = dedup ? hx[td.r] : -1, h2 = dedup2 ? hx[nrec + td.r] : -1;   // in flight with staging
  if (!(dbg & 65536)) { h1 = h1 < 0 ? DRIFT : h1; h2 = h2 < 0 ? DRIFT : h2; }
  const Stage g = stage_of(td, k, dedup, rfs, rfn);
  Stage g2 = g;
  if (dedup2) ref_span(g2, k, r2s, r2n);
  // staging: at most two 16-byte chunks per thread and span, predicated
  // (the spans are < 2 * IBLOCK * 16 bytes: SPAN, RSPAN)
  static_assert(SPAN + 16 <= 2 * IBLOCK * 16 && RSPAN <= 2 * IBLOCK * 16, "two chunks per thread");
  auto stage2 = [&](uint8_t* dst, long long from, long long to) {
    const long long o0 = (long long)threadIdx.x * 16, o1 = o0 + IBLOCK * 16;
    const bool l0 = from + o0 < to, l1 = from + o1 < to;
    uint4 v0 = make_uint4(0u, 0u, 0u, 0u), v1 = v0;
    if (l0) v0 = *reinterpret_cast<const uint4*>(cls + from + o0);
    if (l1) v1 = *reinterpret_cast<const uint4*>(cls + from + o1);
    if (l0) *reinterpret_cast<uint4*>(dst + o0) = v0;
    if (l1) *reinterpret_cast<uint4*>(dst + o1) = v1;
  };
  stage2(s_cls, g.a0, g.hi);
  // dev knobs (PG_K3_DBG, timing only): 512 no drift search (delta 0), 1024
  // no segment compare, 2048 no reference staging, 4096 no queue atomic /
  // writes, 16384 no second reference, 65536 no delta-0 first guess
  if (dedup) {
    if (!(dbg & 2048)) stage2(s_ref, g.ra0, g.rend);
    if (threadIdx.x < NANCH) s_best[threadIdx.x] = (dbg & 512) ? (unsigned)DRIFT : ~0u;
  }
  if (dedup2) {
    stage2(s_ref2, g2.ra0, g2.rend);
    if (threadIdx.x < NANCH) s_best2[threadIdx.x] = (dbg & 512) ? (unsigned)DRIFT : ~0u;
  }
  __syncthreads();
  const long long base = rs - g.a0, rbase = rfs - g.ra0, rbase2 = r2s - g2.ra0;   // LDS index of position 0
  unsigned* diag = (dbg & 64) ? reinterpret_cast<unsigned*>(hints + 16 * nrec + 2) : nullptr;   // dev counters
  if (dedup && !(dbg & 512))
    find_drift_pair(s_cls, base, g.qt, rn, DriftRef{s_ref, rbase, g.plo, g.phi, h1, s_best},
                    DriftRef{s_ref2, rbase2, g2.plo, g2.phi, h2, s_best2}, dedup2, diag);
  const long long q0 = g.qt + (long long)threadIdx.x * IW;
  constexpr uint32_t ALL = (1u << IW) - 1u;
  uint32_t covered = 0;
  // hints and the drift sets once per block (one lane's scalar work, read
  // back from LDS) instead of once per wave
  __shared__ Drifts s_dr[2];
  if (dedup) {                                       // block-uniform
    if (threadIdx.x == 0) {
      if (!(dbg & 512)) {
        publish_hint(s_best, hx + td.r);
        if (dedup2) publish_hint(s_best2, hx + nrec + td.r);
      }
      s_dr[0] = drifts_of(s_best, g.qt, base, rbase, rfn, g.plo, g.phi, k);
      if (dedup2) s_dr[1] = drifts_of(s_best2, g.qt, base, rbase2, r2n, g2.plo, g2.phi, k);
    }
    __syncthreads();
  }
  if (dedup && q0 > 0 && q0 + IW <= last && !(dbg & 1024)) {
    constexpr int NB = (IW + 27 + 1 + 3) / 4;                // bytes q0-1 .. q0+IW+k-1, k <= 27
    const uint32_t o = (uint32_t)(base + q0 - 1);
    const int rel = (int)threadIdx.x * IW;
    uint32_t G[NB];
    lds_bytes16(s_cls, o, G);
    covered = segment_cover(s_cls, s_ref, o, rel, G, s_dr[0], k);
    if (dedup2 && covered != ALL) covered |= segment_cover(s_cls, s_ref2, o, rel, G, s_dr[1], k);
  }
  if (dbg & 128) covered = ALL;                    // dev knob: prologue + coverage only
  const bool work = q0 <= last && covered != ALL;
  uint32_t nwork;
  const uint32_t pos = block_excl_scan<IBLOCK>(work ? 1u : 0u, s_scan, nwork);
  const unsigned sub = blockIdx.x % NQ;
  if (!(dbg & 4096)) {
    if (threadIdx.x == 0) s_qbase = nwork ? atomicAdd(qcount + QSTRIDE * sub, (unsigned long long)nwork) : 0ull;
    __syncthreads();
    if (work) queue[sub * qcap + s_qbase + pos] = WorkItem{rs, last, q0, covered, 0u};
  }
}

// K3 work pass: one queued segment per thread, every lane busy.  The NQ
// sub-queues are read as one concatenated list (their counts scanned in LDS).
// The segment's 64 context bytes (from position q0-2, 16-byte aligned) are
// staged in the thread's own LDS slot and insert_segment runs on them.
template <bool RC>
__global__ void __launch_bounds__(IBLOCK)
k_insert_work(const uint8_t* __restrict__ cls, const WorkItem* __restrict__ queue,
              const unsigned long long* __restrict__ qcount, unsigned long long qcap, int k, uint64_t shift,
              TableView T, unsigned* __restrict__ flags, int dbg) {
  static_assert(NQ == 64, "one wave scans the sub-queue counts");
  // 16-byte front pad + 64 staged bytes per thread (the realigning dword reads
  // past them land in the next row, or read 0 past the allocation); 20 KiB so
  // that a work block fits beside the coverage blocks of the next chunk
  __shared__ __attribute__((aligned(16))) uint8_t scratch[IBLOCK][80];
  __shared__ unsigned long long s_pre[NQ + 1];
  if (threadIdx.x < 64) {
    const unsigned long long c = qcount[QSTRIDE * threadIdx.x];
    unsigned long long x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned long long y = __shfl_up(x, o, 64);
      if ((int)threadIdx.x >= o) x += y;
    }
    s_pre[threadIdx.x + 1] = x;                    // inclusive -> s_pre[j+1]
    if (threadIdx.x == 0) s_pre[0] = 0ull;
  }
  __syncthreads();
  uint8_t* slot = scratch[threadIdx.x] + 16;
  const unsigned long long n = s_pre[NQ];
  unsigned created = 0;
  for (unsigned long long i = blockIdx.x * (unsigned long long)IBLOCK + threadIdx.x; i < n;
       i += (unsigned long long)gridDim.x * IBLOCK) {
    int lo = 0;                                    // largest j with s_pre[j] <= i
#pragma unroll
    for (int step = NQ / 2; step > 0; step >>= 1)
      if (s_pre[lo + step] <= i) lo += step;
    const WorkItem w = queue[(unsigned long long)lo * qcap + (i - s_pre[lo])];
    const long long from = w.rs + w.q0 - 2, aligned = from > 0 ? from & ~15ll : 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *reinterpret_cast<uint4*>(slot + 16 * j) = *reinterpret_cast<const uint4*>(cls + aligned + 16 * j);
    insert_segment<RC>(slot, w.rs - aligned, w.q0, w.last, k, shift, T, flags, w.covered, dbg, created);
  }
  block_count(created, flags);
}

// K3, group form (pangenome inputs).  One block takes stripe j (GW windows) of
// GG records at once.  Every genome of a pangenome repeats most k-mers of its
// neighbours at nearly the same offset, so the block first merges its
// windows' (canonical key, mask) pairs in an LDS hash table (OR is idempotent
// and commutative: the table ends the same), then probes / updates the HBM
// table once per distinct key instead of once per window (C3: ~18% of the
// windows of 8 genomes' stripe are distinct).  A window that finds no LDS slot
// within a few probes goes straight to the HBM table.
constexpr int GG = 8;                         // records per group
constexpr int GNW = 16;                       // consecutive windows per thread
constexpr int GTPR = IBLOCK / GG;             // threads per record (32)
constexpr int GW = GTPR * GNW;                // stripe length (512 windows)
constexpr int GPAD = 16;                      // staging front pad (window q0-2 of q0 < 2)
constexpr int GSPAN = GPAD + GW + 64;         // staged bytes per record (+ k + 3 context)
constexpr int HBITS = 11;
constexpr int HCAP = 1 << HBITS;              // LDS hash slots
constexpr int LB = 8;                         // LDS lookups in flight per thread
static_assert(HCAP * 2 <= GG * GSPAN, "slot list reuses the staging bytes");

__device__ __forceinline__ uint32_t lds_hash(uint64_t c) {
  return (uint32_t)((c * 0x9E3779B97F4A7C15ull) >> (64 - HBITS));
}

template <bool RC>
__global__ void __launch_bounds__(IBLOCK)
k_insert_grp(const uint8_t* __restrict__ cls, const unsigned long long* __restrict__ tiles,
             const int* __restrict__ groups, const long long* __restrict__ rec_start,
             const long long* __restrict__ rec_len, int k, uint64_t shift, TableView T, unsigned* __restrict__ flags,
             int dbg) {
  __shared__ __attribute__((aligned(16))) uint8_t s_cls[GG][GSPAN];
  __shared__ unsigned long long hkey[HCAP];
  __shared__ uint32_t hmask[HCAP];
  __shared__ uint32_t s_scan[IBLOCK / 64];
  const unsigned long long tile = tiles[xcd_swizzle(blockIdx.x, gridDim.x)];
  const int* grp = groups + (size_t)(tile >> 32) * GG;
  const long long qt = (long long)(tile & 0xFFFFFFFFull) * GW;
  for (int s = threadIdx.x; s < HCAP; s += IBLOCK) { hkey[s] = 0ull; hmask[s] = 0u; }
  // stage record positions [qt-2, qt+GW+k+2) of each record at s_cls[g][GPAD-2 ..]
  constexpr int CPR = (GSPAN - GPAD + 15) / 16;  // 16-byte chunks per record
  for (int i = threadIdx.x; i < GG * CPR; i += IBLOCK) {
    const int g = i / CPR, ch = i % CPR;
    const int r = grp[g];
    if (r < 0) continue;
    const long long rs = rec_start[r], rn = rec_len[r];
    if (qt > rn - k) continue;
    const long long lo = rs + (qt >= 2 ? qt - 2 : 0);
    const long long hi = rs + (qt + GW + k + 2 < rn ? qt + GW + k + 2 : rn);
    const long long a0 = lo & ~15ll;
    if (a0 + 16 * ch < hi)
      *reinterpret_cast<uint4*>(&s_cls[g][GPAD + 16 * ch]) = *reinterpret_cast<const uint4*>(cls + a0 + 16 * ch);
  }
  __syncthreads();
  unsigned created = 0;
  {
    const int g = threadIdx.x / GTPR;
    const int r = grp[g];
    const long long rs = r >= 0 ? rec_start[r] : 0, rn = r >= 0 ? rec_len[r] : 0;
    const long long last = rn - k;
    const long long q0 = qt + (long long)(threadIdx.x % GTPR) * GNW;
    const long long q1 = q0 + GNW <= last + 1 ? q0 + GNW : last + 1;
    if (r >= 0 && q0 < q1) {
      const uint8_t* sc = s_cls[g];
      // s_cls index of record position q: GPAD + q - a0 + rs
      const long long base = GPAD + rs - ((rs + (qt >= 2 ? qt - 2 : 0)) & ~15ll);
      uint32_t A[(GNW + 1 + 3) / 4], B[(GNW + 2 + 3) / 4];
      lds_bytes(sc, (uint32_t)(base + q0 - 2), A);           // A(j) = S(q0 - 2 + j)
      lds_bytes(sc, (uint32_t)(base + q0 + k - 1), B);       // B(j) = S(q0 + k - 1 + j)
      uint64_t K = 0, Kr = 0;
      init_keys(sc, (uint32_t)(base + q0), k, K, Kr);
      uint64_t cb[LB];
      uint32_t mb[LB];
      int nb = 0;
#pragma unroll
      for (int i = 0; i < GNW; ++i) {
        const long long q = q0 + i;
        const bool live = q < q1;
        if (i) {                                              // Nu // 5 + alpha * 5^(k-1) (:1072)
          const uint32_t dout = byte_at(A, i + 1), din = byte_at(B, i);
          K = (K - digit_fw(dout)) * INV5 + (uint64_t)digit_fw(din) * shift;
          Kr = (Kr - (uint64_t)digit_rc(dout) * shift) * 5 + digit_rc(din);
        }
        // forward window q: pred '#' at q==0, s[q-2] at the last window (:1080 quirk), else s[q-1]
        const uint32_t fpred = q == 0 ? LAM_HASH : lam_fw(q == last ? byte_at(A, i) : byte_at(A, i + 1));
        const uint32_t fsucc = q == last ? LAM_DOLLAR : lam_fw(byte_at(B, i + 1));
        const uint32_t mf = (fpred << OFFBIT) | fsucc | PRES_A;
        uint64_t c;
        uint32_t m;
        if (RC) {
          // its twin: reverse-strand window n-k-q, same boundary rules on that strand
          const uint32_t rpred = q == last ? LAM_HASH : lam_rc(q == 0 ? byte_at(B, i + 2) : byte_at(B, i + 1));
          const uint32_t rsucc = q == 0 ? LAM_DOLLAR : lam_rc(byte_at(A, i + 1));
          const uint32_t mr = (rpred << OFFBIT) | rsucc | PRES_A;
          if (K < Kr)      { c = K;  m = mf | (mr << B_SHIFT); }
          else if (K > Kr) { c = Kr; m = mr | (mf << B_SHIFT); }
          else             { c = K;  m = mf | mr; }
        } else {
          if (K <= Kr) { c = K; m = mf; } else { c = Kr; m = mf << B_SHIFT; }
        }
        cb[i % LB] = c;
        mb[i % LB] = live ? m : 0u;
        if (i % LB == LB - 1) {                              // merge a batch: LB lookups in flight
          if (dbg & 1) {
#pragma unroll
            for (int x = 0; x < LB; ++x) created += (unsigned)(cb[x] ^ mb[x]) & 1u;
          } else {
            // all LB entries advance together: a round issues every pending
            // entry's CAS (empty slot) or next-slot read, then resolves them
            uint32_t hb[LB];
            unsigned long long cur[LB];
            uint32_t pend = 0;
#pragma unroll
            for (int x = 0; x < LB; ++x) {
              hb[x] = lds_hash(cb[x]);
              cur[x] = hkey[hb[x]];
              pend |= (mb[x] != 0u) << x;
            }
            for (int round = 0; pend && round < 16; ++round) {
              bool empty[LB];
#pragma unroll
              for (int x = 0; x < LB; ++x) {
                empty[x] = false;
                if (((pend >> x) & 1u) && cur[x] == 0ull) {
                  empty[x] = true;
                  cur[x] = atomicCAS(&hkey[hb[x]], 0ull, (unsigned long long)cb[x] + 1ull);
                }
              }
#pragma unroll
              for (int x = 0; x < LB; ++x) {
                if (!((pend >> x) & 1u)) continue;
                const unsigned long long k1 = (unsigned long long)cb[x] + 1ull;
                if ((empty[x] && cur[x] == 0ull) || cur[x] == k1) {
                  atomicOr(&hmask[hb[x]], mb[x]);
                  pend &= ~(1u << x);
                } else {                                      // another key: next slot
                  hb[x] = (hb[x] + 1u) & (HCAP - 1);
                  cur[x] = hkey[hb[x]];
                }
              }
            }
#pragma unroll
            for (int x = 0; x < LB; ++x)                      // no LDS slot: straight to HBM
              if ((pend >> x) & 1u) created += (unsigned)tab_or(T, cb[x], mb[x], flags);
          }
        }
        (void)nb;
      }
    }
  }
  __syncthreads();
  // compact the occupied slots (their indices reuse the staging bytes)
  constexpr int HPT = HCAP / IBLOCK;
  uint16_t* list = reinterpret_cast<uint16_t*>(&s_cls[0][0]);
  uint32_t cnt = 0;
#pragma unroll
  for (int i = 0; i < HPT; ++i) cnt += hkey[threadIdx.x * HPT + i] != 0ull;
  uint32_t U;
  uint32_t o = block_excl_scan<IBLOCK>(cnt, s_scan, U);
#pragma unroll
  for (int i = 0; i < HPT; ++i)
    if (hkey[threadIdx.x * HPT + i] != 0ull) list[o++] = (uint16_t)(threadIdx.x * HPT + i);
  __syncthreads();
  for (uint32_t b0 = 0; b0 < ((dbg & 4) ? 0u : U); b0 += IBLOCK * IB) {   // dev knob 4: no HBM phase
    uint64_t cc[IB], hh[IB];
    uint32_t mm[IB];
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const uint32_t idx = b0 + (uint32_t)i * IBLOCK + threadIdx.x;
      mm[i] = 0;
      cc[i] = 0;
      if (idx < U) {
        const uint32_t s = list[idx];
        cc[i] = hkey[s] - 1ull;
        mm[i] = hmask[s];
      }
      hh[i] = T.perm(cc[i]);
    }
    ulonglong2 v[IB];
#pragma unroll
    for (int i = 0; i < IB; ++i) v[i] = *reinterpret_cast<const ulonglong2*>(T.prim + 2 * (hh[i] >> T.qbits));
    if (dbg & 2) {                                 // dev knob: loads only
#pragma unroll
      for (int i = 0; i < IB; ++i) created += (unsigned)(v[i].x ^ v[i].y) & 1u;
      continue;
    }
    tab_or_batch(T, cc, hh, mm, v, flags, created);
  }
  block_count(created, flags);
}

// one reference window of an explicit strand (used for records with n <= k+1)
__device__ __forceinline__ void oriented_or(const TableView& T, int k, uint64_t x, uint32_t m12,
                                            unsigned* flags, unsigned& created) {
  const uint64_t xr = T.rc(x);
  const uint32_t m = m12 | PRES_A;
  if (x <= xr) created += (unsigned)tab_or(T, x, m, flags);
  else created += (unsigned)tab_or(T, xr, m << B_SHIFT, flags);
}

__global__ void __launch_bounds__(IBLOCK)
k_short(const uint8_t* __restrict__ cls, const long long* __restrict__ rec_start,
        const long long* __restrict__ rec_len, const uint8_t* __restrict__ rec_flag, uint64_t R, int k,
        uint64_t shift, int rc, TableView T, unsigned* flags) {
  unsigned created = 0;
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < R;
       r += (uint64_t)gridDim.x * blockDim.x) {
    if (!rec_flag[r]) continue;
    const long long n = rec_len[r];
    if (n > k + 1) continue;
    if (n < k) { atomicOr(flags, 1u); continue; }          // key -1, mask '$' (:1087-1088)
    auto emit = [&](uint64_t x, uint32_t m12) { oriented_or(T, k, x, m12, flags, created); };
    short_strand(cls, rec_start[r], n, 0, k, shift, emit);
    if (rc) short_strand(cls, rec_start[r], n, 1, k, shift, emit);
  }
  block_count(created, flags);
}

// Extra empty records that the reference's checkpoint/resume yields (see
// pangenome_amd/host.py): each adds the n<k sentinel.
__global__ void k_set_flag(unsigned* flags) { atomicOr(flags, 1u); }

// Staged slots of a loaded npz (pg_dbg_load): OR each oriented (key, mask)
// into the table as add_kmer would (the sentinel sets the flag).
__global__ void __launch_bounds__(IBLOCK)
k_preload_merge(const PreEnt* __restrict__ e, uint64_t n, TableView T, unsigned* __restrict__ flags) {
  unsigned created = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t x = e[i].key;
    if (x == SENTINEL) { atomicOr(flags, 1u); continue; }
    oriented_or(T, 0, x, e[i].mask & MASK12, flags, created);
  }
  block_count(created, flags);
}

void merge_preload(Ctx& c, unsigned* flags) {
  if (!c.n_preload) return;
  hipLaunchKernelGGL(k_preload_merge, dim3(grid_for(c.n_preload, IBLOCK, 4096)), dim3(IBLOCK), 0, c.stream,
                     c.preload.as<PreEnt>(), c.n_preload, c.tv, flags);
  PG_HIP(hipGetLastError());
}

// ---- table scans.  Entry index space: [0, 2*buckets) primary words, then
// [2*buckets, 2*buckets + ovf) overflow slots.


// K5: degree scan.  The table is swept as 16-byte elements (a primary bucket
// = two words, or one overflow slot), RU per thread per 16 KiB unit, with
// 16-byte loads and the next unit in flight.  A unit's members (at most 4 per
// element) are block-scanned into an LDS stage of RCAP keys; the stage goes
// out with ONE global atomic per flush — a single device counter takes ~80
// returning atomics per us (tools/rates.hip), so per-unit atomics would cost
// more than the sweep itself, and the grid is kept to RGRID persistent blocks
// (their final flushes all meet that counter at the end).
constexpr int RT = 256, RU_DEF = 2;
constexpr unsigned RGRID = 4096;                   // RU = 4 on 1024 blocks measured slower (0.29 vs 0.26 ms)
template <int RU> constexpr uint64_t runit() { return (uint64_t)RT * RU; }
template <int RU> constexpr int rcap() { return 4 * (int)runit<RU>(); }   // a whole unit fits an empty stage

// Stage entries are the bucket-hash value h = perm(c) with bit 63 = "B
// orientation"; keys are rebuilt here, one entry per lane (dense), rather than
// by the few member lanes of every wave during the sweep.
__device__ __forceinline__ void reduce_flush(const TableView& T, unsigned long long* stage, uint32_t n,
                                             unsigned long long* s_base, unsigned long long* __restrict__ out,
                                             uint64_t cap, unsigned long long* __restrict__ counter) {
  if (threadIdx.x == 0) *s_base = atomicAdd(counter, (unsigned long long)n);
  __syncthreads();
  const unsigned long long b = *s_base;
  for (uint32_t x = threadIdx.x; x < n; x += RT) {
    const unsigned long long v = stage[x];
    const uint64_t c = T.unperm(v & ~(1ull << 63));
    if (b + x < cap) out[b + x] = (v >> 63) ? T.rc(c) : c;   // the host rejects a count above cap
  }
  __syncthreads();
}

template <int RU>
__device__ __forceinline__ void reduce_load(const TableView& T, uint64_t nb, uint64_t nel, uint64_t u,
                                            uint4 (&e)[RU]) {
#pragma unroll
  for (int j = 0; j < RU; ++j) {
    const uint64_t i = u * runit<RU>() + (uint64_t)j * RT + threadIdx.x;
    e[j] = i >= nel ? make_uint4(0, 0, 0, 0)
                    : i < nb ? *reinterpret_cast<const uint4*>(T.prim + 2 * i)
                             : *reinterpret_cast<const uint4*>(T.ovf + (i - nb));
  }
}

template <int RU>
__global__ void __launch_bounds__(RT)
k_reduce(TableView T, uint64_t nb, uint64_t nel, int k, unsigned long long* __restrict__ out, uint64_t cap,
         unsigned long long* __restrict__ counters) {
  __shared__ unsigned long long stage[rcap<RU>()];
  __shared__ uint32_t lds[RT / 64];
  __shared__ unsigned long long s_base;
  __shared__ unsigned long long red[RT / 64];
  uint32_t staged = 0;                             // block-uniform
  uint32_t ndbg = 0;                               // per thread: <= 4 per element it visits
  const uint64_t nunit = (nel + runit<RU>() - 1) / runit<RU>();
  uint4 e[RU];
  if (blockIdx.x < nunit) reduce_load<RU>(T, nb, nel, blockIdx.x, e);
  for (uint64_t u = blockIdx.x; u < nunit; u += gridDim.x) {
    uint4 nx[RU];                                  // next unit in flight while this one is reduced
    if (u + gridDim.x < nunit) reduce_load<RU>(T, nb, nel, u + gridDim.x, nx);
    // membership bits, computed once: bit 4j + 2h + o = word h of element j
    // (an overflow slot has one key, in "word 0"), orientation o (B = 1)
    const uint64_t ubase = u * runit<RU>();
    const bool prim = ubase + runit<RU>() <= nb;      // block-uniform: no overflow slot in this unit
    uint32_t mem = 0;
#pragma unroll
    for (int j = 0; j < RU; ++j) {
      const bool isp = prim || ubase + (uint64_t)j * RT + threadIdx.x < nb;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t lo = h ? e[j].z : e[j].x, hi = h ? e[j].w : e[j].y;
        const uint32_t mm = isp ? ((lo | hi) ? (lo & (uint32_t)MW_MASK) : 0u)
                                : (h == 0 && (e[j].x | e[j].y) ? e[j].z : 0u);   // Slot {key1, mask, aux}
        const uint32_t pa = (mm >> 12) & 1u, pb = (mm >> 25) & 1u;     // PRES_A, PRES_B
        ndbg += pa + pb;
        mem |= (uint32_t)(pa && rdbg_member(mm & MASK12)) << (4 * j + 2 * h);
        mem |= (uint32_t)(pb && rdbg_member((mm >> B_SHIFT) & MASK12)) << (4 * j + 2 * h + 1);
      }
    }
    const uint32_t cnt = (uint32_t)__builtin_popcount(mem);
    uint32_t tot;
    const uint32_t pre = block_excl_scan<RT>(cnt, lds, tot);
    if (staged + tot > (uint32_t)rcap<RU>()) {           // block-uniform
      reduce_flush(T, stage, staged, &s_base, out, cap, counters);
      staged = 0;
    }
    if (mem) {
      uint32_t o = staged + pre;
#pragma unroll
      for (int j = 0; j < RU; ++j) {
        const uint64_t i = ubase + (uint64_t)j * RT + threadIdx.x;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t b = (mem >> (4 * j + 2 * h)) & 3u;
          if (b) {
            const unsigned long long w = h ? ((unsigned long long)e[j].z | (unsigned long long)e[j].w << 32)
                                           : ((unsigned long long)e[j].x | (unsigned long long)e[j].y << 32);
            // perm(c): the bucket / quotient split of a primary word; overflow
            // slots hold c + 1 (rare: hash it here)
            const uint64_t hv = i < nb ? ((i << T.qbits) | (uint64_t)(w >> MW_BITS)) : T.perm(w - 1ull);
            if (b & 1u) stage[o++] = hv;
            if (b & 2u) stage[o++] = hv | (1ull << 63);
          }
        }
      }
    }
    __syncthreads();
    staged += tot;
#pragma unroll
    for (int j = 0; j < RU; ++j) e[j] = nx[j];
  }
  if (staged) reduce_flush(T, stage, staged, &s_base, out, cap, counters);
  unsigned long long nd = ndbg;
  for (int o = 32; o > 0; o >>= 1) nd += __shfl_down(nd, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = nd;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < RT / 64; ++w) t += red[w];
    if (t) atomicAdd(counters + 8 * (1 + blockIdx.x % 64), t);   // 64 spread lines
  }
}

// dBG export: (key, 12-bit mask) of both orientations of every entry
__global__ void k_export_dbg(TableView T, uint64_t nw, uint64_t ntot, int k,
                             unsigned long long* __restrict__ keys, unsigned short* __restrict__ masks,
                             uint64_t cap, unsigned long long* __restrict__ counter) {
  const int lane = threadIdx.x & 63;
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < ntot;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t m = entry_mask(T, nw, i);
    const bool pa = m & PRES_A, pb = m & PRES_B;
    const unsigned long long ba = __ballot(pa), bb = __ballot(pb);
    const unsigned na = __builtin_popcountll(ba), nbb = __builtin_popcountll(bb);
    if (na + nbb == 0) continue;
    const int leader = __builtin_ctzll(ba | bb);
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(counter, (unsigned long long)(na + nbb));
    base = __shfl(base, leader, 64);
    if (!(pa || pb)) continue;
    const uint64_t c = entry_key(T, nw, i);
    // writes past cap are dropped; the host rejects a count above cap
    const uint64_t oa = base + __builtin_popcountll(ba & lt), ob = base + na + __builtin_popcountll(bb & lt);
    if (pa && oa < cap) { keys[oa] = c; masks[oa] = m & MASK12; }
    if (pb && ob < cap) { keys[ob] = T.rc(c); masks[ob] = (m >> B_SHIFT) & MASK12; }
  }
}

// ---- multi-GPU exchange: owner = high bits of a key hash mod nparts
__device__ __forceinline__ int owner_of(uint64_t c, int nparts) {
  return (int)((fmix64(c) >> 40) % (uint64_t)nparts);
}

__global__ void k_part_count(TableView T, uint64_t nw, uint64_t ntot, int nparts,
                             unsigned long long* __restrict__ counts) {
  __shared__ unsigned long long hist[64];
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < ntot;
       i += (uint64_t)gridDim.x * blockDim.x)
    if (entry_mask(T, nw, i)) atomicAdd(&hist[owner_of(entry_key(T, nw, i), nparts)], 1ull);
  __syncthreads();
  for (int i = threadIdx.x; i < nparts; i += blockDim.x)
    if (hist[i]) atomicAdd(&counts[i], hist[i]);
}

// Owner-partitioned copy of the table's entries.  Per chunk of PCH entries a
// block counts its entries per owner in LDS, reserves each owner's run with
// ONE global atomic, then writes.  (One atomic per wave and owner on the
// shared owner cursors serialised ~8 M same-address atomics at the memory
// side for a C3 table, tens of ms; see NQ above.)  Record order inside an
// owner's run is arbitrary: the owner OR-merges them.
constexpr int PT = 256, PE = 8, PCH = PT * PE;
__global__ void __launch_bounds__(PT)
k_part_scatter(TableView T, uint64_t nw, uint64_t ntot, int nparts, unsigned long long* __restrict__ cursor,
               Slot* __restrict__ out) {
  __shared__ unsigned s_cnt[64];
  __shared__ unsigned long long s_base[64];
  for (uint64_t c0 = blockIdx.x * (uint64_t)PCH; c0 < ntot; c0 += (uint64_t)gridDim.x * PCH) {
    if (threadIdx.x < 64) s_cnt[threadIdx.x] = 0u;
    __syncthreads();
    uint32_t m[PE], rank[PE];
    uint64_t key[PE];
    int own[PE];
#pragma unroll
    for (int j = 0; j < PE; ++j) {
      const uint64_t i = c0 + (uint64_t)j * PT + threadIdx.x;
      m[j] = i < ntot ? entry_mask(T, nw, i) : 0u;
      key[j] = m[j] ? entry_key(T, nw, i) : 0ull;
      own[j] = m[j] ? owner_of(key[j], nparts) : 0;
      rank[j] = m[j] ? atomicAdd(&s_cnt[own[j]], 1u) : 0u;
    }
    __syncthreads();
    if ((int)threadIdx.x < nparts && s_cnt[threadIdx.x])
      s_base[threadIdx.x] = atomicAdd(&cursor[threadIdx.x], (unsigned long long)s_cnt[threadIdx.x]);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PE; ++j)
      if (m[j]) out[s_base[own[j]] + rank[j]] = Slot{key[j] + 1ull, m[j], 0u};
    __syncthreads();
  }
}

__global__ void __launch_bounds__(IBLOCK)
k_merge(const Slot* __restrict__ pairs, uint64_t n, TableView T, unsigned* __restrict__ flags) {
  unsigned created = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const Slot s = pairs[i];
    if (!s.key1) continue;
    created += (unsigned)tab_or(T, s.key1 - 1ull, s.mask & (uint32_t)MW_MASK, flags);
  }
  block_count(created, flags);
}

// ------------------------------------------------------------------ host
constexpr int N_FLAGS = 16 * (N_CNT + 2) + 16;       // + diagnostic counters

static void alloc_table(Ctx& c, uint64_t keys) {
  uint64_t buckets = 0, ovf = 0;
  TableView t = make_geometry(c.k, keys, buckets, ovf);
  if (c.pre_ptr && 16 * buckets > c.table.cap) PG_HIP(hipStreamSynchronize(c.stream2));   // its buffer is freed
  c.table.reserve(16 * buckets);
  c.ovf.reserve(sizeof(Slot) * ovf);
  t.prim = c.table.as<unsigned long long>();
  t.ovf = c.ovf.as<Slot>();
  c.tv = t;
  c.cap = buckets;
  c.ovf_cap = ovf;
  c.flags.reserve(4 * N_FLAGS);
}

// 16-byte streaming stores: 5.1 TB/s measured (tools/fetch_calib.hip) where
// hipMemsetAsync's fill kernel ran the 1 GiB table at 3.3 TB/s.
__global__ void __launch_bounds__(256) k_zero16(uint4* __restrict__ p, uint64_t n16) {
  const uint4 z = make_uint4(0u, 0u, 0u, 0u);
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256ull) p[i] = z;
}

// Small per-build fills (overflow slots, flags, K3 queue counters, drift
// hints) in ONE launch, one grid row per region, instead of a
// hipMemsetAsync each (~5 us of dispatch apiece on the critical stream).
struct Fill { uint4* p; uint64_t n16; unsigned v; };
struct Fills { Fill r[4]; };
__global__ void __launch_bounds__(256) k_fills(Fills f) {
  const Fill r = f.r[blockIdx.y];
  const uint4 v = make_uint4(r.v, r.v, r.v, r.v);
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < r.n16; i += (uint64_t)gridDim.x * 256ull) r.p[i] = v;
}
static void launch_fills(const Fills& f, int n, uint64_t max_n16, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_fills, dim3(grid_for(max_n16, 256, 1024), (unsigned)n), dim3(256), 0, s, f);
  PG_HIP(hipGetLastError());
}

// The next build's table clear, queued on stream2 by pg_parse so that it runs
// beside the parse instead of beside the first coverage pass (parse
// invalidates the dBG anyway; a build whose table keeps its place and size
// skips its own clear).  A narrow grid (PRECLEAR_GRID blocks) trickles the
// stores out without taking the parse's CUs: C3, per step, K3 1.92 -> 1.73
// ms for parse 0.45 -> 0.57 ms (8192 blocks: parse 0.66 ms).
constexpr unsigned PRECLEAR_GRID = 128, K3_ZGRID = 256;
void preclear_table(Ctx& c) {
  const char* ge = getenv("PG_PRECLEAR_GRID");            // dev knob (0: no pre-clear)
  if (!c.table.p || !c.cap || (ge && atoi(ge) == 0)) return;
  PG_HIP(hipEventRecord(c.ev[14], c.stream));            // after everything queued on the table
  PG_HIP(hipStreamWaitEvent(c.stream2, c.ev[14], 0));
  hipLaunchKernelGGL(k_zero16, dim3(grid_for(c.cap, 256, ge ? (unsigned)atoi(ge) : PRECLEAR_GRID)), dim3(256), 0,
                     c.stream2,
                     reinterpret_cast<uint4*>(c.table.p), (uint64_t)c.cap);
  PG_HIP(hipGetLastError());
  c.pre_ptr = c.table.p;
  c.pre_n16 = c.cap;
}

// primary = false: the two-pass K3 clears the primary buckets on stream2
// (launch_insert), unless pg_parse's clear there already covers them
static void clear_table(Ctx& c, bool primary) {
  const bool pre = c.pre_ptr && c.pre_ptr == c.table.p && c.pre_n16 >= c.cap;
  if (c.pre_ptr && primary) {                            // the table is written on stream: wait for it
    PG_HIP(hipEventRecord(c.ev[14], c.stream2));
    PG_HIP(hipStreamWaitEvent(c.stream, c.ev[14], 0));
  }
  c.pre_ptr = nullptr;
  c.k3_skip_clear = pre && !primary;                     // (stream2 runs it before the work passes)
  if (primary && !pre) {
    hipLaunchKernelGGL(k_zero16, dim3(grid_for(c.cap, 256, 8192)), dim3(256), 0, c.stream,
                       reinterpret_cast<uint4*>(c.table.p), (uint64_t)c.cap);
    PG_HIP(hipGetLastError());
  }
  static_assert(sizeof(Slot) == 16 && (4 * N_FLAGS) % 16 == 0, "k_fills works in 16-byte units");
  c.k3_defer_fill = !primary;                            // the two-pass K3 folds them into its own fill
  if (!primary) return;
  Fills f{};
  f.r[0] = Fill{reinterpret_cast<uint4*>(c.ovf.p), c.ovf_cap, 0u};
  f.r[1] = Fill{reinterpret_cast<uint4*>(c.flags.p), (uint64_t)(4 * N_FLAGS / 16), 0u};
  launch_fills(f, 2, std::max<uint64_t>(c.ovf_cap, 4 * N_FLAGS / 16), c.stream);
}

static uint64_t n_entries(const Ctx& c) { return 2 * c.cap + c.ovf_cap; }

// read back [sentinel, overflow, sum of spread counters]
static void read_flags(Ctx& c, unsigned& sentinel, unsigned& overflow, uint64_t& created) {
  c.h_pin.reserve(4 * N_FLAGS);
  PG_HIP(hipMemcpyAsync(c.h_pin.p, c.flags.p, 4 * N_FLAGS, hipMemcpyDeviceToHost, c.stream));
  c.sync();
  const unsigned* f = c.h_pin.as<unsigned>();
  sentinel = f[0];
  overflow = f[1];
  created = 0;
  for (int i = 0; i < N_CNT; ++i) created += f[16 * (1 + i)];
#ifdef PG_DIAG
  fprintf(stderr, "PG_DIAG calls=%u casA=%u okA=%u orA=%u casB=%u okB=%u orB=%u ovf=%u created=%llu\n",
          f[16 * (2 + N_CNT)], f[16 * (2 + N_CNT) + 1], f[16 * (2 + N_CNT) + 2], f[16 * (2 + N_CNT) + 3],
          f[16 * (2 + N_CNT) + 4], f[16 * (2 + N_CNT) + 5], f[16 * (2 + N_CNT) + 6], f[16 * (2 + N_CNT) + 7],
          (unsigned long long)created);
#endif
}

// Tiles of records with n >= k+2, stripe-major: stripe 0 of every record, then
// stripe 1, ...  (records with more stripes first within a stripe).  One lead
// record runs LEAD stripes ahead of the others: it creates the k-mers the
// genomes share before its followers probe them, instead of every genome
// reading the same empty bucket at once and racing to CAS it (a stale empty
// costs a failed memory-side CAS).  Packed as record << 32 | stripe.  Cached
// while the record table and flags repeat.
constexpr uint64_t LEAD = 4;

static uint64_t make_tiles(Ctx& c, const std::vector<uint8_t>& flag) {
  const uint64_t R = c.n_records;
  if (c.tile_sig_len == c.h_rec_len && c.tile_sig_flag == flag && c.tile_k == c.k && c.tile_mode == 0)
    return c.n_tiles;
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
  c.k3_ref = nt.size() >= 2 ? nt[0].second : -1;      // the lead is every follower's dedup reference
  c.k3_ref2 = nt.size() >= 3 ? nt[1].second : -1;     // the second reference (k_cover)
  c.k3_hint.reserve(64 * (R + 1) + 64);                 // drift hints per XCD, reference, record (+ dev counters)
  std::vector<unsigned long long> tiles;
  tiles.reserve(total);
  size_t live = nt.size();
  for (uint64_t j = 0; j < maxs + LEAD; ++j) {
    if (!nt.empty() && j < nt[0].first)                        // the lead, LEAD stripes ahead
      tiles.push_back(((unsigned long long)nt[0].second << 32) | j);
    if (j < LEAD) continue;
    const uint64_t jf = j - LEAD;                              // the followers' stripe
    while (live && nt[live - 1].first <= jf) --live;
    for (size_t i = 1; i < live; ++i) tiles.push_back(((unsigned long long)nt[i].second << 32) | jf);
  }
  std::vector<TileDesc> descs(total);
  for (uint64_t i = 0; i < total; ++i) {
    const int r = (int)(tiles[i] >> 32);
    descs[i] = TileDesc{c.h_rec_start[r], c.h_rec_len[r], r, (int)(tiles[i] & 0xFFFFFFFFull), 0};
  }
  c.tiles.reserve(8 * (total + 1));
  c.tile_desc.reserve(sizeof(TileDesc) * (total + 1));
  if (total) {
    PG_HIP(hipMemcpyAsync(c.tiles.p, tiles.data(), 8 * total, hipMemcpyHostToDevice, c.stream));
    PG_HIP(hipMemcpyAsync(c.tile_desc.p, descs.data(), sizeof(TileDesc) * total, hipMemcpyHostToDevice, c.stream));
  }
  c.sync();
  c.tile_sig_len = c.h_rec_len;
  c.tile_sig_flag = flag;
  c.tile_k = c.k;
  c.tile_mode = 0;
  c.n_tiles = total;
  return total;
}

// Group tiles for k_insert_grp: records (n >= k+2) sorted by length, in groups
// of GG; tile = group << 32 | stripe (GW windows), stripe-major, the first
// group LEAD stripes ahead of the rest (see make_tiles).
static uint64_t make_group_tiles(Ctx& c, const std::vector<uint8_t>& flag) {
  const uint64_t R = c.n_records;
  if (c.tile_sig_len == c.h_rec_len && c.tile_sig_flag == flag && c.tile_k == c.k && c.tile_mode == 1)
    return c.n_tiles;
  std::vector<std::pair<uint64_t, int>> nt;           // (stripes, record)
  for (uint64_t r = 0; r < R; ++r) {
    const int64_t n = c.h_rec_len[r];
    if (!flag[r] || n < c.k + 2) continue;
    nt.push_back({(uint64_t)((n - c.k + 1 + GW - 1) / GW), (int)r});
  }
  std::stable_sort(nt.begin(), nt.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
  const size_t ng = (nt.size() + GG - 1) / GG;
  std::vector<int> grp(ng * GG, -1);
  std::vector<uint64_t> gs(ng, 0);
  for (size_t i = 0; i < nt.size(); ++i) {
    grp[i] = nt[i].second;
    gs[i / GG] = std::max(gs[i / GG], nt[i].first);
  }
  std::vector<unsigned long long> tiles;
  const uint64_t maxs = ng ? gs[0] : 0;
  for (uint64_t j = 0; j < maxs + LEAD; ++j) {
    if (ng && j < gs[0]) tiles.push_back(j);                   // group 0 leads
    if (j < LEAD) continue;
    const uint64_t jf = j - LEAD;
    for (size_t g = 1; g < ng; ++g)
      if (jf < gs[g]) tiles.push_back(((unsigned long long)g << 32) | jf);
  }
  const uint64_t total = tiles.size();
  c.tiles.reserve(8 * (total + 1));
  c.groups.reserve(4 * (grp.size() + 1));
  if (total) PG_HIP(hipMemcpyAsync(c.tiles.p, tiles.data(), 8 * total, hipMemcpyHostToDevice, c.stream));
  if (!grp.empty()) PG_HIP(hipMemcpyAsync(c.groups.p, grp.data(), 4 * grp.size(), hipMemcpyHostToDevice, c.stream));
  c.sync();
  c.tile_sig_len = c.h_rec_len;
  c.tile_sig_flag = flag;
  c.tile_k = c.k;
  c.tile_mode = 1;
  c.n_tiles = total;
  return total;
}

// K3 form: per-record tiles (k_insert) by default; PG_K3=group selects the
// group kernel (needs at least GG long records to pay off).  On C3 the tile
// form is ahead today (6.3 vs 7.8 ms: the group form's LDS merge is
// latency-bound at its occupancy); both are parity-tested.
static int k3_mode(const Ctx& c, const std::vector<uint8_t>& flag) {
  const char* e = getenv("PG_K3");
  if (!e || strcmp(e, "group")) return 0;
  uint64_t n = 0;
  for (uint64_t r = 0; r < c.n_records; ++r) n += flag[r] && c.h_rec_len[r] >= c.k + 2;
  return n >= (uint64_t)GG ? 1 : 0;
}

// chunks of the tile list whose work pass overlaps the next coverage pass
constexpr int K3_CHUNKS = 4;
constexpr int K3_COVPAD = 8 * 1024;           // dynamic LDS pad per coverage block (chunked form)
constexpr int K3_WBLK = 2;                    // work blocks per CU (chunked form)
// the coverage pass + work pass form of k_insert (needs the lead record)
static bool two_pass(const Ctx& c, uint64_t ntiles, int dbg) { return ntiles && c.k3_ref >= 0 && !(dbg & 256); }

static void launch_short(Ctx& c, hipStream_t s, int rc0, uint64_t shift, unsigned* flags) {
  if (!c.n_records) return;
  hipLaunchKernelGGL(k_short, dim3(grid_for(c.n_records, IBLOCK, 1024)), dim3(IBLOCK), 0, s, c.cls.as<uint8_t>(),
                     c.rec_start.as<long long>(), c.rec_len.as<long long>(), c.rec_flag.as<uint8_t>(), c.n_records,
                     c.k, shift, rc0, c.tv, flags);
  PG_HIP(hipGetLastError());
}

// Returns true when it has also queued k_short (records with n <= k+1).
static bool launch_insert(Ctx& c, int mode, int rc0, uint64_t ntiles, uint64_t shift, unsigned* flags, int dbg) {
  bool short_done = false;
  const dim3 g((unsigned)ntiles), b(IBLOCK);
  const uint8_t* cls = c.cls.as<uint8_t>();
  const auto* tiles = c.tiles.as<unsigned long long>();
  const auto* rs = c.rec_start.as<long long>();
  const auto* rl = c.rec_len.as<long long>();
  if (mode && rc0)
    hipLaunchKernelGGL(k_insert_grp<true>, g, b, 0, c.stream, cls, tiles, c.groups.as<int>(), rs, rl, c.k, shift, c.tv,
                       flags, dbg);
  else if (mode)
    hipLaunchKernelGGL(k_insert_grp<false>, g, b, 0, c.stream, cls, tiles, c.groups.as<int>(), rs, rl, c.k, shift, c.tv,
                       flags, dbg);
  else {
    const long long rfs = c.k3_ref >= 0 ? c.h_rec_start[c.k3_ref] : 0, rfn = c.k3_ref >= 0 ? c.h_rec_len[c.k3_ref] : 0;
    const TileDesc* td = c.tile_desc.as<TileDesc>();
    if (two_pass(c, ntiles, dbg)) {
      // Coverage pass, then the dense work pass over the queued segments, in
      // NCH chunks of the tile list on two streams: the work pass of chunk i
      // (memory-side-atomic-bound) runs beside the coverage pass of chunk
      // i+1 (issue-bound), and the table clear beside the first coverage
      // pass.  Coverage never touches the table, so only the clear must
      // precede the first work pass.
      const char* ce = getenv("PG_K3_CHUNKS");                  // dev knob
      int nch = ce ? std::max(1, std::min(6, atoi(ce))) : K3_CHUNKS;
      const char* me = getenv("PG_K3_CHUNK_MIN");              // dev knob (tests): tiles per chunk
      if (ntiles < (uint64_t)nch * (uint64_t)(me ? atoi(me) : 4096)) nch = 1;
      // chunk sizes (weights; cb = cumulative): the work stream is the
      // critical path (K3 ~ first coverage pass + all work passes), so the
      // first chunk is small and the work stream starts early
      uint32_t cb[8] = {0};
      {
        const char* se = getenv("PG_K3_SPLIT");                  // dev knob: "w0,w1,..."
        int n = 0;
        if (se && nch > 1) {
          for (const char* x = se; *x && n < 6; ++n) {
            cb[n + 1] = cb[n] + (uint32_t)std::max(1, atoi(x));
            while (*x && *x != ',') ++x;
            if (*x == ',') ++x;
          }
          nch = n;
        } else {
          for (int i = 0; i < nch; ++i) cb[i + 1] = cb[i] + 1;
        }
      }
      // Overlap needs room on every CU: the coverage blocks are held to ~6 per
      // CU by padding their LDS (covpad bytes of dynamic LDS), which leaves a
      // work block (20 KiB) per CU; the work pass then runs as a persistent
      // grid of wgrid blocks beside the next chunk's coverage pass.
      const char* pe = getenv("PG_K3_COVPAD");                   // dev knobs
      const char* we = getenv("PG_K3_WGRID");
      const size_t covpad = nch > 1 ? (size_t)(pe ? atoi(pe) : K3_COVPAD) : 0;
      const unsigned wgrid = we ? (unsigned)atoi(we) : (unsigned)c.n_cu * K3_WBLK;
      // the last work pass has no coverage pass beside it: more blocks per CU
      const char* le = getenv("PG_K3_WLAST");                    // dev knob (blocks per CU)
      const unsigned wlast = le && atoi(le) > 0 ? (unsigned)c.n_cu * (unsigned)atoi(le) : wgrid;
      uint64_t gc[8], qoff[8], qcapc[8];               // per chunk: blocks (8 x the longest XCD part)
      uint64_t items = 0;
      for (int i = 0; i < nch; ++i) {
        gc[i] = 0;
        for (int x = 0; x < 8; ++x) {
          uint64_t t, te;
          xcd_chunk(ntiles, cb[i], cb[i + 1], cb[nch], (uint64_t)x, t, te);
          gc[i] = std::max<uint64_t>(gc[i], 8 * (te - t));
        }
        qcapc[i] = (gc[i] + NQ - 1) / NQ * IBLOCK;      // per sub-queue
        qoff[i] = items;
        items += NQ * qcapc[i];
      }
      const size_t qbytes = sizeof(WorkItem) * items;
      const size_t cbytes = 8 * QSTRIDE * NQ;                    // counters per chunk
      c.k3_queue.reserve(qbytes + cbytes * nch);
      auto* q = c.k3_queue.as<WorkItem>();
      auto* qn = reinterpret_cast<unsigned long long*>(c.k3_queue.as<uint8_t>() + qbytes);
      {                                                          // counters 0, hints "no drift known yet"
        static_assert(sizeof(WorkItem) % 16 == 0 && (8 * QSTRIDE * NQ) % 16 == 0, "16-byte fill units");
        Fills f{};
        int nf = 0;
        f.r[nf++] = Fill{reinterpret_cast<uint4*>(qn), cbytes * nch / 16, 0u};
        f.r[nf++] = Fill{c.k3_hint.as<uint4>(), 4 * (c.n_records + 1), 0xFFFFFFFFu};
        if (c.k3_defer_fill) {
          f.r[nf++] = Fill{reinterpret_cast<uint4*>(c.ovf.p), c.ovf_cap, 0u};
          f.r[nf++] = Fill{reinterpret_cast<uint4*>(c.flags.p), (uint64_t)(4 * N_FLAGS / 16), 0u};
        }
        uint64_t mx = 0;
        for (int j = 0; j < nf; ++j) mx = std::max(mx, f.r[j].n16);
        launch_fills(f, nf, mx, c.stream);
        c.k3_defer_fill = false;
      }
      if (dbg & 64) PG_HIP(hipMemsetAsync(c.k3_hint.as<int>() + 16 * c.n_records + 2, 0, 16, c.stream));
      const long long r2s = c.k3_ref2 >= 0 ? c.h_rec_start[c.k3_ref2] : 0;
      const long long r2n = c.k3_ref2 >= 0 ? c.h_rec_len[c.k3_ref2] : 0;
      hipStream_t s0 = c.stream, s1 = c.stream2;
      // the clear on s1, after everything already queued on s0
      PG_HIP(hipEventRecord(c.ev[0], s0));
      PG_HIP(hipStreamWaitEvent(s1, c.ev[0], 0));
      if (!c.k3_skip_clear) {
        const char* ze = getenv("PG_K3_ZGRID");                  // dev knob
        hipLaunchKernelGGL(k_zero16, dim3(grid_for(c.cap, 256, ze ? (unsigned)atoi(ze) : K3_ZGRID)), dim3(256), 0, s1,
                           reinterpret_cast<uint4*>(c.table.p), (uint64_t)c.cap);
        PG_HIP(hipGetLastError());
      }
      c.k3_skip_clear = false;
      PG_HIP(hipEventRecord(c.ev[13], s1));                     // the table is clear from here on
      // the last work pass on s0, right behind the last coverage pass and
      // beside the previous work pass (chunks' inserts commute: atomics), so
      // that the cross-stream join before K5 waits on s1's shorter tail
      const char* l0 = getenv("PG_K3_LAST_S0");                  // dev knob
      const bool last_s0 = nch > 1 && !(l0 && atoi(l0) == 0);
      for (int i = 0; i < nch; ++i) {
        auto* qi = q + qoff[i];
        auto* qni = qn + (cbytes / 8) * i;
        if (gc[i])
          hipLaunchKernelGGL(k_cover, dim3((unsigned)gc[i]), b, covpad, s0, cls, td, qi, qni,
                             (unsigned long long)qcapc[i], c.k, c.k3_ref, rfs, rfn, c.k3_ref2, r2s, r2n,
                             c.k3_hint.as<int>(), (int)c.n_records, ntiles, cb[i], cb[i + 1], cb[nch], dbg);
        PG_HIP(hipGetLastError());
        hipStream_t ws = s1;
        if (last_s0 && i + 1 == nch) {
          ws = s0;
          PG_HIP(hipStreamWaitEvent(s0, c.ev[13], 0));
          launch_short(c, s1, rc0, shift, flags);                // k_short on s1 beside it
          short_done = true;
        } else {
          PG_HIP(hipEventRecord(c.ev[1 + i], s0));
          PG_HIP(hipStreamWaitEvent(s1, c.ev[1 + i], 0));      // s1: clear, work 0 .. i-1, then this
        }
        const uint64_t mi = std::min<uint64_t>(NQ * qcapc[i], c.windows_fw / IW + c.n_records + 1);
        const unsigned gw = nch > 1 ? (i + 1 == nch ? wlast : wgrid) : grid_for(mi, IBLOCK, 16384);
        if (rc0)
          hipLaunchKernelGGL(k_insert_work<true>, dim3(gw), b, 0, ws, cls, qi, qni, (unsigned long long)qcapc[i],
                             c.k, shift, c.tv, flags, dbg);
        else
          hipLaunchKernelGGL(k_insert_work<false>, dim3(gw), b, 0, ws, cls, qi, qni, (unsigned long long)qcapc[i],
                             c.k, shift, c.tv, flags, dbg);
        PG_HIP(hipGetLastError());
      }
      // k_short beside the last work pass (on whichever stream it is not on), not after the join
      if (!short_done) {
        PG_HIP(hipStreamWaitEvent(s0, c.ev[13], 0));
        launch_short(c, s0, rc0, shift, flags);
        short_done = true;
      }
      PG_HIP(hipEventRecord(c.ev[15], s1));                     // join: s0 continues after the last work pass
      PG_HIP(hipStreamWaitEvent(s0, c.ev[15], 0));
    } else if (rc0) {
      hipLaunchKernelGGL(k_insert<true>, g, b, 0, c.stream, cls, td, c.k, shift, c.tv, flags, c.k3_ref, rfs, rfn,
                         dbg);
    } else {
      hipLaunchKernelGGL(k_insert<false>, g, b, 0, c.stream, cls, td, c.k, shift, c.tv, flags, c.k3_ref, rfs, rfn,
                         dbg);
    }
  }
  PG_HIP(hipGetLastError());
  return short_done;
}

static void reduce_enqueue(Ctx& c, uint64_t cap_keys);
static bool reduce_finish(Ctx& c);

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
  c.last_flag = flag;
  c.last_extra = extra_empty;
  c.dump_ready = false;
  const int mode = k3_mode(c, flag);
  const uint64_t ntiles = mode ? make_group_tiles(c, flag) : make_tiles(c, flag);
  // expected canonical keys: learned from the previous build, else the
  // forward windows (every one distinct) divided by the number of long
  // records up to 4 (a pangenome of G genomes repeats most k-mers G times;
  // C3's first build would otherwise size a 17 GB table for 19.5 M keys),
  // plus the staged npz slots; an overflow rebuilds larger
  uint64_t nlong = 0;
  for (uint64_t r = 0; r < R; ++r) nlong += flag[r] && c.h_rec_len[r] >= c.k + 2;
  const uint64_t redund = std::max<uint64_t>(1, std::min<uint64_t>(4, nlong));
  uint64_t keys = c.cap_hint ? c.cap_hint : std::max<uint64_t>(1024, c.windows_fw / redund + c.n_preload);
  const uint64_t shift = pow5(c.k - 1);
  // PG_K3_DBG (development only): 1 = windows only, 2 = HBM loads without
  // updates, 4 = group form without its HBM phase; PG_K3_KEYS fixes the table
  // size for such runs.  The product path never sets them.
  const int dbg = getenv("PG_K3_DBG") ? atoi(getenv("PG_K3_DBG")) : 0;
  if (dbg && getenv("PG_K3_KEYS")) keys = strtoull(getenv("PG_K3_KEYS"), nullptr, 10);
  c.t0.init(); c.t1.init();
  for (int attempt = 0; attempt < 8; ++attempt) {
    alloc_table(c, keys);
    c.t0.start(c.stream);
    clear_table(c, mode != 0 || !two_pass(c, ntiles, dbg));
    c.t0.stop(c.stream);
    unsigned* flags = c.flags.as<unsigned>();
    c.t1.start(c.stream);
    const bool short_done = ntiles && launch_insert(c, mode, rc0, ntiles, shift, flags, dbg);
    c.t1.stop(c.stream);
    if (!short_done) launch_short(c, c.stream, rc0, shift, flags);
    if (extra_empty) hipLaunchKernelGGL(k_set_flag, dim3(1), dim3(1), 0, c.stream, flags);
    merge_preload(c, flags);
    const bool spec = c.spec_k5 && c.rdbg_hint && !dbg;
    if (spec) reduce_enqueue(c, c.rdbg_hint);
    unsigned sentinel = 0, overflow = 0;
    uint64_t created = 0;
    read_flags(c, sentinel, overflow, created);
    c.ms_clear = c.t0.ms();
    c.ms_insert = c.t1.ms();
    if (dbg & 64) {                  // dev counters of k_cover's drift search
      unsigned d[4];
      PG_HIP(hipMemcpy(d, c.k3_hint.as<int>() + 16 * c.n_records + 2, 16, hipMemcpyDeviceToHost));
      fprintf(stderr, "PG_K3_DBG drift search: ref1 hinted %u full %u, ref2 hinted %u full %u, tiles %llu\n", d[0],
              d[1], d[2], d[3], (unsigned long long)ntiles);
    }
    if (dbg) {                       // dev knob run: timings only, the table is not a dBG
      std::vector<unsigned> f(N_FLAGS);
      PG_HIP(hipMemcpy(f.data(), c.flags.p, 4 * N_FLAGS, hipMemcpyDeviceToHost));
      const unsigned* d = f.data() + 16 * (2 + N_CNT);
      fprintf(stderr, "PG_K3_DBG=%d mode=%d insert=%.3f ms work_segments=%u dedup_blocks=%u segments=%u "
              "covered_windows=%u\n", dbg, mode, c.ms_insert, d[8], d[9], d[10], d[11]);
      return;
    }
    if (!overflow) {
      c.n_canon = created;
      c.sentinel = sentinel ? 1 : 0;
      c.cap_hint = std::max<uint64_t>(1024, created + created / 4);
      c.built = true;
      ++c.build_gen;
      if (spec && !reduce_finish(c)) c.rdbg_hint = 0;   // outgrown: build_rdbg runs K5 again
      return;
    }
    keys = std::max<uint64_t>(keys * 4, created * 2);
  }
  throw Error(-12, "build_dbg: hash table overflow after resizing");
}

// K5 in two halves, so that pg_build can enqueue it right behind K3 (before
// build_dbg's flag read-back, with a capacity learned from the last build)
// and read both back with one synchronisation.
constexpr size_t K5_CNT_BYTES = 8 * 8 * 65;             // [0] member count, [8 * (1 + i)] dBG size partials
static void reduce_enqueue(Ctx& c, uint64_t cap_keys) {
  c.rdbg_keys.reserve(8 * (cap_keys + 1));
  DevBuf& cnt = c.n_sel;
  cnt.reserve(K5_CNT_BYTES);
  PG_HIP(hipMemsetAsync(cnt.p, 0, K5_CNT_BYTES, c.stream));
  c.t5.init();
  c.t5.start(c.stream);
  const uint64_t nel = c.cap + c.ovf_cap;               // 16-byte elements: buckets, then overflow slots
  const int ru = getenv("PG_K5_RU") ? atoi(getenv("PG_K5_RU")) : RU_DEF;            // dev knobs
  const unsigned rg = getenv("PG_K5_GRID") ? (unsigned)atoi(getenv("PG_K5_GRID")) : RGRID;
  auto* rk = c.rdbg_keys.as<unsigned long long>();
  auto* rc = cnt.as<unsigned long long>();
  if (ru == 1)
    hipLaunchKernelGGL(k_reduce<1>, dim3(grid_for(nel / runit<1>(), 1, rg)), dim3(RT), 0, c.stream, c.tv, c.cap, nel,
                       c.k, rk, 2 * c.n_canon + 1, rc);
  else if (ru == 4)
    hipLaunchKernelGGL(k_reduce<4>, dim3(grid_for(nel / runit<4>(), 1, rg)), dim3(RT), 0, c.stream, c.tv, c.cap, nel,
                       c.k, rk, 2 * c.n_canon + 1, rc);
  else
    hipLaunchKernelGGL(k_reduce<2>, dim3(grid_for(nel / runit<2>(), 1, rg)), dim3(RT), 0, c.stream, c.tv, c.cap, nel,
                       c.k, rk, cap_keys, rc);
  PG_HIP(hipGetLastError());
  c.t5.stop(c.stream);
  c.k5_pin.reserve(K5_CNT_BYTES);
  PG_HIP(hipMemcpyAsync(c.k5_pin.p, cnt.p, K5_CNT_BYTES, hipMemcpyDeviceToHost, c.stream));
  c.k5_cap = cap_keys;
}

// after the stream has synchronised; false if the rdBG outgrew k5_cap
static bool reduce_finish(Ctx& c) {
  const unsigned long long* res = c.k5_pin.as<unsigned long long>();
  if (res[0] > c.k5_cap) return false;
  c.ms_scan = c.t5.ms();
  c.n_rdbg = res[0];
  c.n_dbg = 0;
  for (int i = 0; i < 64; ++i) c.n_dbg += res[8 * (1 + i)];
  if (c.sentinel) {         // key 2^64-1, mask 32: always an rdBG member
    unsigned long long s = SENTINEL;
    PG_HIP(hipMemcpyAsync(c.rdbg_keys.as<unsigned long long>() + c.n_rdbg, &s, 8, hipMemcpyHostToDevice,
                          c.stream));
    c.sync();
    c.n_rdbg += 1;
    c.n_dbg += 1;
  }
  c.reduced = true;
  c.rdbg_hint = c.n_rdbg + c.n_rdbg / 4 + 4096;
  return true;
}

void build_rdbg(Ctx& c) {
  if (!c.built) throw Error(-22, "build_rdbg: no dBG (call pg_build_dbg first)");
  if (c.reduced) return;                                // K5 already ran behind K3 (pg_build)
  reduce_enqueue(c, 2 * c.n_canon + 1);
  c.sync();
  if (!reduce_finish(c)) throw Error(-5, "build_rdbg: member count exceeds the table's key count");
}

uint64_t export_dbg(Ctx& c, uint64_t* h_keys, uint16_t* h_masks, uint64_t cap) {
  if (!c.built) throw Error(-22, "export_dbg: no dBG");
  const uint64_t nmax = 2 * c.n_canon + 1;
  DevBuf keys, masks, cnt;
  keys.reserve(8 * nmax);
  masks.reserve(2 * nmax);
  cnt.reserve(8);
  PG_HIP(hipMemsetAsync(cnt.p, 0, 8, c.stream));
  hipLaunchKernelGGL(k_export_dbg, dim3(grid_for(n_entries(c), 256, 8192)), dim3(256), 0, c.stream, c.tv,
                     2 * c.cap, n_entries(c), c.k, keys.as<unsigned long long>(), masks.as<unsigned short>(), nmax,
                     cnt.as<unsigned long long>());
  PG_HIP(hipGetLastError());
  unsigned long long n = 0;
  PG_HIP(hipMemcpyAsync(&n, cnt.p, 8, hipMemcpyDeviceToHost, c.stream));
  c.sync();
  if (n > nmax) {
    keys.release(); masks.release(); cnt.release();
    throw Error(-5, "export_dbg: entry count exceeds the table's key count");
  }
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
  DevBuf& cnt = c.part_cnt;                             // [0, 64) counts, [64, 128) cursors
  cnt.reserve(16 * 64);
  auto* counts = cnt.as<unsigned long long>();
  c.h_pin.reserve(16 * 64);
  auto* h = c.h_pin.as<unsigned long long>();
  if (!d_out) {                                         // count pass
    PG_HIP(hipMemsetAsync(cnt.p, 0, 8 * 64, c.stream));
    hipLaunchKernelGGL(k_part_count, dim3(grid_for(n_entries(c), 256, 4096)), dim3(256), 0, c.stream, c.tv,
                       2 * c.cap, n_entries(c), nparts, counts);
    PG_HIP(hipGetLastError());
    PG_HIP(hipMemcpyAsync(h, counts, 8 * nparts, hipMemcpyDeviceToHost, c.stream));
    c.sync();
    uint64_t total = 0;
    for (int i = 0; i < nparts; ++i) { h_counts[i] = h[i]; total += h[i]; }
    c.part_total = total;
    c.part_nparts = nparts;
    c.part_gen = c.build_gen;
    for (int i = 0; i < nparts; ++i) c.part_counts[i] = h[i];
    return total;
  }
  // scatter pass: the counts of the last count pass give every owner's run
  uint64_t total = 0;
  for (int i = 0; i < nparts; ++i) { h[64 + i] = total; total += c.part_counts[i]; h_counts[i] = c.part_counts[i]; }
  if (c.part_gen != c.build_gen || c.part_nparts != nparts)
    throw Error(-22, "partition_dbg: call with d_out = NULL (count pass) first");
  if (out_cap < total) throw Error(-22, "partition_dbg: output buffer too small");
  if (total) {
    PG_HIP(hipMemcpyAsync(counts + 64, h + 64, 8 * nparts, hipMemcpyHostToDevice, c.stream));
    hipLaunchKernelGGL(k_part_scatter, dim3(grid_for(n_entries(c), PCH, 4096)), dim3(PT), 0, c.stream, c.tv,
                       2 * c.cap, n_entries(c), nparts, counts + 64, reinterpret_cast<Slot*>(d_out));
    PG_HIP(hipGetLastError());
    c.sync();
  }
  return total;
}

void merge_dbg(Ctx& c, const void* d_pairs, uint64_t n, uint64_t cap_hint, int sentinel) {
  uint64_t keys = cap_hint ? cap_hint : std::max<uint64_t>(1024, n);
  c.t1.init();
  for (int attempt = 0; attempt < 8; ++attempt) {
    alloc_table(c, keys);
    clear_table(c, true);
    if (sentinel) hipLaunchKernelGGL(k_set_flag, dim3(1), dim3(1), 0, c.stream, c.flags.as<unsigned>());
    c.t1.start(c.stream);
    if (n)
      hipLaunchKernelGGL(k_merge, dim3(grid_for(n, IBLOCK, 8192)), dim3(IBLOCK), 0, c.stream,
                         reinterpret_cast<const Slot*>(d_pairs), n, c.tv, c.flags.as<unsigned>());
    PG_HIP(hipGetLastError());
    c.t1.stop(c.stream);
    unsigned s = 0, overflow = 0;
    uint64_t created = 0;
    read_flags(c, s, overflow, created);
    c.ms_insert = c.t1.ms();
    if (!overflow) {
      c.n_canon = created;
      c.sentinel = s ? 1 : 0;
      c.built = true;
      c.reduced = false;
      ++c.build_gen;
      return;
    }
    keys *= 4;
  }
  throw Error(-12, "merge_dbg: hash table overflow after resizing");
}

}  // namespace pg
