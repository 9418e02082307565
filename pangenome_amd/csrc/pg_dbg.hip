// pg_dbg.hip — K3: k-mer windows -> the dBG hash table, built by partition,
// with K5 (degree scan + rdBG compaction) fused into the partition merge;
// exports and the owner-partitioned exchange of the multi-GPU build.
//
// Reference path: seq2rdbg (kmer_numba.py:1234-1268) -> seq2dbg_jit_
// (:1202-1230) -> build_dbg (:1052-1090) -> add_kmer (:1036-1047), then
// dbg2rdbg (:1313-1321) -> build_rdbg_jit_ (:1292-1309).
//
// Every forward-strand window q of a record carries its reverse-strand twin
// (window n-k-q of tab_rev(reversed(s)), :1215-1221), so one visit per
// position covers both: the canonical key c = min(K, K') gets the forward
// mask in one 12-bit field and the reverse mask in the other (pg_common.h),
// and the exported dBG is exactly the reference's non-canonical dBG.
//
// The table is never updated with global atomics.  The build runs in three
// stages, all streaming through HBM:
//   A  k_cover + k_emit_work.  The coverage pass drops the windows a
//      reference record provably inserts (a pangenome repeats each k-mer
//      once per genome); every other window becomes a 12-byte record
//      (h = perm(c), 26-bit mask word) appended, in block-aggregated runs, to
//      one of 64 coarse bins (the top bits of h = of the bucket index) with a
//      region per XCD.
//   B  k_split (zero or more passes): a bin's records are split by the next
//      bucket-index bits into fine partitions of at most 4096 buckets.
//   C  k_build_range: one block per fine partition OR-merges its records into
//      an LDS copy of its bucket range, streams the range out whole (the
//      table needs no clear), and applies the rdBG rule (build_rdbg_jit_
//      :1300-1305) to each key of the range, whose masks are final there.
// The table is sized from stage A's exact record count, so nothing is
// learned from earlier builds except the stage A region size (re-run if
// outgrown).
#include <algorithm>
#include <type_traits>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "pg_internal.h"

// Development experiments (tools/exp_build.sh builds variants with
// -DPG_EXP_BITS=n into separate libraries; the product build has none)
#ifndef PG_EXP_BITS
#define PG_EXP_BITS 0
#endif

namespace pg {

// Development (PG_DEBUG_BOUNDS builds only, tools/exp_build.sh -D...): index
// checks in the coverage / work passes that record the first violation in
// g_dbg (code, values) and skip the access instead of faulting.
#ifdef PG_DEBUG_BOUNDS
// per code slot (code % 16): count g_dbg[slot], then up to 4 entries of 5 words (code, a, b, block, thread)
__device__ unsigned long long g_dbg[16 + 16 * 4 * 5];
__device__ __forceinline__ bool pg_bok(bool ok, unsigned code, long long a, long long b) {
  if (!ok) {
    const unsigned slot = code % 16;
    const unsigned long long i = atomicAdd(&g_dbg[slot], 1ull);
    if (i < 4) {
      unsigned long long* e = g_dbg + 16 + (slot * 4 + i) * 5;
      e[0] = code; e[1] = (unsigned long long)a; e[2] = (unsigned long long)b; e[3] = blockIdx.x; e[4] = threadIdx.x;
    }
  }
  return ok;
}
#define PG_BOK(ok, code, a, b) pg_bok((ok), (code), (long long)(a), (long long)(b))
#else
#define PG_BOK(ok, code, a, b) true
#endif

constexpr int IBLOCK = 256;
constexpr int IW = 16;                        // windows per thread (one segment)
constexpr int CBLOCK = 256;                   // coverage block (one tile)
constexpr int TILE = CBLOCK * IW;             // windows per tile (one coverage block)
constexpr int SPAN = TILE + 64;               // staged bytes (k <= 27: TILE + k + 3 <= SPAN - 16)
constexpr int CSTRIDE = 8;                    // counter spacing: one 64-byte line (uint64 words)

// flags (uint32 words): [0] the n<k sentinel was seen, [1] stage A bits,
// [4] stage B/C bits (a separate 16-byte unit: stage C re-runs clear it alone)
enum : unsigned { F_OVF_FULL = 1u, F_A_OVER = 2u, F_LDS_SPILL = 4u, F_SPLIT_OVER = 8u, F_RSEG_OVER = 16u };
constexpr int N_FLAGS = 16;
// a 64-bit counter at this flag index (cleared with the flags when stage A
// starts): the work pass's items (one atomic per launch)
constexpr int F_WORK_ITEMS = 12;

// overflow table: linear probing on 16-byte slots (CAS on key1, then OR);
// a full table sets F_OVF_FULL in *fl (C3: ~2 % of the keys land here, in
// buckets that drew a third key)
__device__ int ovf_or(const TableView& T, uint64_t c, uint32_t mw, unsigned* fl) {
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
  atomicOr(fl, F_OVF_FULL);
  return 0;
}

// 4*ND bytes of LDS starting at byte index idx, realigned into dwords
template <int ND>
__device__ __forceinline__ void lds_bytes(const uint8_t* s, uint32_t idx, uint32_t (&out)[ND]) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(s + (idx & ~3u));
  const uint32_t sb = idx & 3u;
  uint32_t raw[ND + 1];
#pragma unroll
  for (int i = 0; i <= ND; ++i) raw[i] = w[i];
#pragma unroll
  for (int i = 0; i < ND; ++i) out[i] = __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], sb);   // one v_alignbyte each
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
  auto S = [&](int j) { return (uint32_t)sc[o + j]; };
  for (int j = kl - 1; j >= 0; --j) lo = lo * 5u + digit_fw(S(j));
  for (int j = k - 1; j >= kl; --j) hi = hi * 5u + digit_fw(S(j));
  for (int j = 0; j < kh; ++j) rhi = rhi * 5u + digit_rc(S(j));
  for (int j = kh; j < k; ++j) rlo = rlo * 5u + digit_rc(S(j));
  K = (uint64_t)lo + hi * 1220703125ull;         // 5^13
  Kr = (uint64_t)rlo + rhi * 1220703125ull;
}

// init_keys for k = 27 from seven dword reads of the row (realigned by
// v_alignbyte) instead of 2 x 27 byte reads: the digits come out of registers
// at constant positions (the work pass's LDS instructions were half these
// byte reads)
__device__ __forceinline__ void init_keys27(const uint8_t* sc, uint32_t o, uint64_t& K, uint64_t& Kr) {
  uint32_t w[7];
  lds_bytes(sc, o, w);
  uint32_t lo = 0, rlo = 0;
  uint64_t hi = 0, rhi = 0;
#pragma unroll
  for (int j = 12; j >= 0; --j) lo = lo * 5u + digit_fw(byte_at(w, j));
#pragma unroll
  for (int j = 26; j >= 13; --j) hi = hi * 5u + digit_fw(byte_at(w, j));
#pragma unroll
  for (int j = 0; j < 14; ++j) rhi = rhi * 5u + digit_rc(byte_at(w, j));
#pragma unroll
  for (int j = 14; j < 27; ++j) rlo = rlo * 5u + digit_rc(byte_at(w, j));
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

// ---- positional dedup against a reference record (k_cover).  A window q of
// record g with neither record end in it, whose bytes [q-1, q+k] equal the
// reference's bytes [q'-1, q'+k] at q' = q - delta (q' interior too), has the
// reference window's key and both masks (:1069-1080); the reference inserts
// that window, so g's record would OR nothing new and is not emitted.  The
// drift delta only decides how much is skipped, never what is inserted.
constexpr int DRIFT = (PG_EXP_BITS & 128) ? 384 : (PG_EXP_BITS & 256) ? 256 : 512;  // searched offsets: [-DRIFT, DRIFT]
constexpr int RSPAN = TILE + 2 * DRIFT + 96;  // staged reference bytes
constexpr int NANCH = 3;                      // anchors per tile
constexpr int ALEN = 32;                      // anchor length (bytes)
constexpr int ASTEP = (TILE - ALEN - 16) / (NANCH - 1);      // anchor spacing

// The IW windows q0 .. q0+IW-1 (clipped at the record's last window) of one
// record staged in s_cls (s_cls[base + q] = class of position q): both
// strands' rolling keys (k2n_jit :975-985, updated as :1072 does), and per
// window i the bucket hash hh[i] = perm(c) of the canonical key c = min(K, K')
// with its 26-bit mask word mm[i] — the forward window's lastc[pred] << 6 |
// lastc[succ] in c's orientation field, its reverse-strand twin's in the
// other (:1069-1080).  mm[i] == 0: no record (a window with a `covered` bit,
// which a reference record inserts, or past the record's last window).
// Interior segments run from registers; a segment holding window 0 or the
// last window takes the generic path with the boundary rules.
template <bool RC, int X0 = 0, int NX = IW>
__device__ __forceinline__ void segment_records(const uint8_t* s_cls, long long base, long long q0, long long last,
                                                int k, uint64_t shift, const TableView& T, uint32_t covered,
                                                uint64_t& K, uint64_t& Kr, uint64_t (&hh)[NX], uint32_t (&mm)[NX]) {
  static_assert(X0 % 4 == 0 && NX % 4 == 0 && X0 + NX <= IW, "whole dwords of the segment");
  if (X0 == 0) {
    if (k == 27) init_keys27(s_cls, (uint32_t)(base + q0), K, Kr);
    else init_keys(s_cls, (uint32_t)(base + q0), k, K, Kr);
  }
  if (q0 > 0 && q0 + IW <= last) {
    // interior segment (no window 0, no last window, all IW live): the context
    // bytes come from LDS once, into registers; P(i) = S(q-1), D(i) = S(q+k-1)
    // for window q = q0 + X0 + i, and D(i+1) = S(q+k)
    const uint32_t o = (uint32_t)(base + q0) + X0;
    uint32_t P[NX / 4], D[NX / 4 + 1];
    lds_bytes(s_cls, o - 1, P);
    lds_bytes(s_cls, o + (uint32_t)k - 1, D);
#pragma unroll
    for (int x = 0; x < NX; ++x) {
      const uint32_t p = byte_at(P, x), s = byte_at(D, x + 1);
      if (X0 + x) {                              // Nu // 5 + alpha * 5^(k-1) (:1072)
        const uint32_t din = byte_at(D, x);
        K = (K - digit_fw(p)) * INV5 + (uint64_t)digit_fw(din) * shift;
        Kr = (Kr - (uint64_t)digit_rc(p) * shift) * 5 + digit_rc(din);
      }
      const uint32_t mf = (lam_fw(p) << OFFBIT) | lam_fw(s) | PRES_A;
      uint64_t c;
      uint32_t m;
      if (RC) {
        const uint32_t mr = (lam_rc(s) << OFFBIT) | lam_rc(p) | PRES_A;
        const bool lt = K < Kr, eq = K == Kr;
        c = lt ? K : Kr;
        m = eq ? (mf | mr) : lt ? (mf | (mr << B_SHIFT)) : (mr | (mf << B_SHIFT));
      } else {
        const bool le = K <= Kr;
        c = le ? K : Kr;
        m = le ? mf : (mf << B_SHIFT);
      }
      mm[x] = ((covered >> (X0 + x)) & 1u) ? 0u : m;
      hh[x] = T.perm(c);
    }
    return;
  }
  auto S = [&](long long q) -> uint32_t { return s_cls[base + q]; };
#pragma unroll
  for (int x = 0; x < NX; ++x) {
    const long long q = q0 + X0 + x;
    hh[x] = 0;
    mm[x] = 0;
    if (q <= last) {
      if (X0 + x) {                              // Nu // 5 + alpha * 5^(k-1) (:1072)
        const uint32_t dout = S(q - 1), din = S(q + k - 1);
        K = (K - digit_fw(dout)) * INV5 + (uint64_t)digit_fw(din) * shift;
        Kr = (Kr - (uint64_t)digit_rc(dout) * shift) * 5 + digit_rc(din);
      }
      // forward window q: pred '#' at q==0, s[q-2] at the last window (:1080 quirk), else s[q-1]
      const uint32_t fpred = q == 0 ? LAM_HASH : lam_fw(S(q - (q == last ? 2 : 1)));
      const uint32_t fsucc = q == last ? LAM_DOLLAR : lam_fw(S(q + k));
      const uint32_t mf = (fpred << OFFBIT) | fsucc | PRES_A;
      uint64_t c;
      uint32_t m;
      if (RC) {
        // its twin: reverse-strand window n-k-q, same boundary rules on that strand
        const uint32_t rpred = q == last ? LAM_HASH : lam_rc(S(q + k + (q == 0 ? 1 : 0)));
        const uint32_t rsucc = q == 0 ? LAM_DOLLAR : lam_rc(S(q - 1));
        const uint32_t mr = (rpred << OFFBIT) | rsucc | PRES_A;
        if (K < Kr)      { c = K;  m = mf | (mr << B_SHIFT); }
        else if (K > Kr) { c = Kr; m = mr | (mf << B_SHIFT); }
        else             { c = K;  m = mf | mr; }
      } else {
        if (K <= Kr) { c = K; m = mf; } else { c = Kr; m = mf << B_SHIFT; }
      }
      mm[x] = ((covered >> (X0 + x)) & 1u) ? 0u : m;
      hh[x] = T.perm(c);
    }
  }
}

// The work pass's packed form of an interior k = 27 segment whose 64 staged
// bases are all ACGT (no exception chunk): the bases are read as 2-bit codes
// (= their classes) from four packed words in registers, shifted so that code
// 0 is position q0 - 1 - no LDS row, no byte reads.  init_keys27 from the
// codes: 7 bytes of 4 codes, each looked up in K5 (the base-5 value of its 4
// digits forward, low 16 bits, and reversed, high 16), combined in 32-bit
// pieces of 12 digits; the reverse strand's key from the reversed digits R
// as Kr = sum (3 - d_j) 5^(26-j) = 3 (5^27 - 1) / 4 - R, and R from 5 R
// (28 digits, the last one 0) by the exact division K / 5 = K * INV5.
constexpr uint64_t KR27 = 5587935447692871093ull;   // 3 (5^27 - 1) / 4
__device__ __forceinline__ uint32_t k5_entry(uint32_t b) {
  uint32_t t = 0, tr = 0;
  for (int i = 0; i < 4; ++i) {
    const uint32_t d = digit_fw((b >> (2 * i)) & 3u);
    t = t * 5u + digit_fw((b >> (2 * (3 - i))) & 3u);
    tr = tr * 5u + d;
  }
  return t | tr << 16;
}
__device__ __forceinline__ void init_keys27_pk(const uint32_t (&cw)[4], const uint32_t* k5, uint64_t& K,
                                               uint64_t& Kr) {
  const uint32_t v0 = __builtin_amdgcn_alignbit(cw[1], cw[0], 2), v1 = __builtin_amdgcn_alignbit(cw[2], cw[1], 2);
  uint32_t t[7];
#pragma unroll
  for (int c = 0; c < 4; ++c) t[c] = k5[(v0 >> (8 * c)) & 0xFFu];
  t[4] = k5[v1 & 0xFFu];
  t[5] = k5[(v1 >> 8) & 0xFFu];
  t[6] = k5[(v1 >> 16) & 0x3Fu];                  // digits 24 .. 26 (27: 0)
  auto lo16 = [&](int c) { return t[c] & 0xFFFFu; };
  auto hi16 = [&](int c) { return t[c] >> 16; };
  const uint32_t lo = __umul24(__umul24(lo16(2), 625u) + lo16(1), 625u) + lo16(0);
  const uint32_t mid = __umul24(__umul24(lo16(5), 625u) + lo16(4), 625u) + lo16(3);
  K = ((uint64_t)lo16(6) * 244140625ull + mid) * 244140625ull + lo;        // 5^12
  const uint32_t hr = __umul24(__umul24(hi16(0), 625u) + hi16(1), 625u) + hi16(2);
  const uint32_t mr = __umul24(__umul24(hi16(3), 625u) + hi16(4), 625u) + hi16(5);
  const uint64_t r5 = (uint64_t)hr * 152587890625ull + (uint64_t)mr * 625ull + hi16(6);   // 5^16, 5^4
  Kr = KR27 - r5 * INV5;
}
// segment_records' interior path with code i = base q0 - 1 + i of the record
template <bool RC, int X0, int NX>
__device__ __forceinline__ void segment_records_pk(const uint32_t (&cw)[4], const uint32_t* k5, uint64_t shift,
                                                   const TableView& T, uint32_t covered, uint64_t& K, uint64_t& Kr,
                                                   uint64_t (&hh)[NX], uint32_t (&mm)[NX]) {
  static_assert(X0 + NX + 28 <= 48, "codes of the shifted 128 bits");
  auto code = [&](int i) -> uint32_t { return (cw[i >> 4] >> (2 * (i & 15))) & 3u; };
  if (X0 == 0) init_keys27_pk(cw, k5, K, Kr);
#pragma unroll
  for (int x = 0; x < NX; ++x) {
    const int xi = X0 + x;
    const uint32_t p = code(xi), s = code(xi + 28);
    if (xi) {                                      // Nu // 5 + alpha * 5^(k-1) (:1072)
      const uint32_t din = code(xi + 27);
      K = (K - digit_fw(p)) * INV5 + (uint64_t)digit_fw(din) * shift;
      Kr = (Kr - (uint64_t)digit_rc(p) * shift) * 5 + digit_rc(din);
    }
    const uint32_t mf = (lam_fw(p) << OFFBIT) | lam_fw(s) | PRES_A;
    uint64_t c;
    uint32_t m;
    if (RC) {
      const uint32_t mr = (lam_rc(s) << OFFBIT) | lam_rc(p) | PRES_A;
      const bool lt = K < Kr, eq = K == Kr;
      c = lt ? K : Kr;
      m = eq ? (mf | mr) : lt ? (mf | (mr << B_SHIFT)) : (mr | (mf << B_SHIFT));
    } else {
      const bool le = K <= Kr;
      c = le ? K : Kr;
      m = le ? mf : (mf << B_SHIFT);
    }
    mm[x] = ((covered >> xi) & 1u) ? 0u : m;
    hh[x] = T.perm(c);
  }
}

// A segment left with work after the coverage pass (k_cover).
struct WorkItem {
  long long rs, last, q0;
  uint32_t covered, pad;
};

// The queue is NQ sub-queues, each with its own counter on its own 64-byte
// line; a tile appends to sub-queue (its block) % NQ.  One counter shared by
// all ~120 K tiles of a C3 launch serialises their atomics at the memory side
// (1.48 ms measured, tools/rates.hip) - as long as the whole coverage pass;
// 64 counters take 0.045 ms.  A tile appends at most CBLOCK items.
constexpr int NQ = 64;
constexpr int QSTRIDE = 8;                    // counter spacing (unsigned long long words)

// Drift search of a coverage block: QM member tiles (one stripe) x 2
// references x NANCH anchors.  Stage 1: every (member, reference, anchor)
// triple searches hint +- HWIN2 with 32 lanes, 8 triples per round of the
// block; stage 2, for a (member, reference) whose anchors all missed, searches
// the full +-DRIFT with the whole block (rare: ~1 % of tiles).  best[] gets
// (|delta| << 16 | drift) of every matching candidate (atomicMin: the
// smallest drift wins).  The hints and drift sets are published by the caller.
constexpr int HWIN2 = (PG_EXP_BITS & 32768) ? 40 : 56;
constexpr int QM = 4;                         // member tiles per coverage block (one stripe; 8 measured slower)
struct MemGeo {                               // a member tile: record, staging window, hints
  long long rs, rn, a0, hi;
  int r, h[2];                                // h: the XCD's last drift per reference (DRIFT: none)
};
struct RefGeo {                               // a reference record's staged span (same for all members)
  long long rbase, plo, phi, rfn;             // rbase: LDS index of the record's position 0
};
__device__ __forceinline__ void drift_task(const uint8_t* s_cls, const uint8_t* s_ref, int ia, int ibhi, int lo,
                                           int hi, int w, unsigned* best) {
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
}
// anchor ai of a member (LDS base `base`, record length rn) against reference R
__device__ __forceinline__ void drift_geom(const RefGeo& R, long long qt, long long base, long long rn, int ai,
                                           int& ia, int& ibhi, int& lo, int& hi) {
  const long long a = qt + 8 + (long long)ai * ASTEP;
  ia = (int)(base + a);
  ibhi = (int)(R.rbase + a + DRIFT);
  lo = max(ibhi - 2 * DRIFT, (int)(R.rbase + R.plo));
  hi = a + ALEN > rn ? -1 : min(ibhi, (int)(R.rbase + R.phi) - ALEN);
}
__device__ __forceinline__ void cover_search(uint8_t (*s_cls)[SPAN + 16], uint8_t (*s_ref)[RSPAN],
                                             const MemGeo* geo, const RefGeo& R0, const RefGeo& R1,
                                             unsigned (*best)[2][NANCH], long long qt, uint32_t dm0, uint32_t dm1) {
  static_assert((2 * HWIN2) / 4 + 2 <= 32, "32 lanes per triple in stage 1");
  constexpr int NT = QM * 2 * NANCH, PER = CBLOCK / 32;
  constexpr int NW = (2 * DRIFT + 3) / 4 + 2;
#pragma unroll 1
  for (int t0 = 0; t0 < NT; t0 += PER) {
    const int t = t0 + ((int)threadIdx.x >> 5), l = (int)threadIdx.x & 31;
    const int m = t / (2 * NANCH), ri = (t / NANCH) & 1, ai = t % NANCH;
    if (t < NT && (((ri ? dm1 : dm0) >> m) & 1u)) {
      const MemGeo& G = geo[m];
      int ia, ibhi, lo, hi;
      drift_geom(ri ? R1 : R0, qt, G.rs - G.a0, G.rn, ai, ia, ibhi, lo, hi);
      lo = max(lo, ibhi - (G.h[ri] + HWIN2));
      hi = min(hi, ibhi - (G.h[ri] - HWIN2));
      const int w = (lo >> 2) + l;
      if (lo <= hi && 4 * w <= hi) drift_task(s_cls[m], s_ref[ri], ia, ibhi, lo, hi, w, &best[m][ri][ai]);
    }
  }
  __syncthreads();
  static_assert(NANCH == 3, "any-anchor test");
  uint32_t need = 0;                                          // (as cover_search_q: decided before any search)
#pragma unroll
  for (int p = 0; p < 2 * QM; ++p) {
    const int m = p >> 1, ri = p & 1;
    unsigned all = ~0u;
#pragma unroll
    for (int ai = 0; ai < NANCH; ++ai) all &= best[m][ri][ai];
    if ((((ri ? dm1 : dm0) >> m) & 1u) && all == ~0u) need |= 1u << p;
  }
  if (!need) return;                                          // (block-uniform)
  __syncthreads();
#pragma unroll 1
  for (int p = 0; p < 2 * QM; ++p) {
    const int m = p >> 1, ri = p & 1;
    if (!((need >> p) & 1u)) continue;
    const MemGeo& G = geo[m];
#pragma unroll 1
    for (int ai = 0; ai < NANCH; ++ai) {
      int ia, ibhi, lo, hi;
      drift_geom(ri ? R1 : R0, qt, G.rs - G.a0, G.rn, ai, ia, ibhi, lo, hi);
      for (int w = (lo >> 2) + (int)threadIdx.x; 4 * w <= hi && w < (lo >> 2) + NW; w += CBLOCK)
        drift_task(s_cls[m], s_ref[ri], ia, ibhi, lo, hi, w, &best[m][ri][ai]);
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

// 4*ND bytes of LDS from byte index idx through 16-byte reads (ds_read_b128:
// lanes 16 B apart hit distinct banks, where the dword reads of lds_bytes are
// 4-way conflicted), realigned in registers.  idx & 15 must be the same for
// every lane of the wave (it selects the shift by a uniform branch).
template <int ND>
__device__ __forceinline__ void lds_bytes16(const uint8_t* s, uint32_t idx, uint32_t (&out)[ND]) {
  constexpr int NW = ((ND + 3) / 4 + 1) * 4;       // dwords read: ceil(ND/4)+1 chunks of 16 B
  uint32_t raw[NW];
  // Whole 16-byte reads, pinned as such: left alone, the compiler sinks them
  // into the switch below and narrows each to the dwords its case uses,
  // ds_read2_b32 pairs whose 32-lane banking makes the 16-byte-strided lanes
  // 4-way conflicted (822 conflict cycles per k_cover wave, PMC)
  const uint4* s16 = reinterpret_cast<const uint4*>(__builtin_assume_aligned(s, 16));
#pragma unroll
  for (int q = 0; q < NW / 4; ++q) {
    uint4 v = s16[(idx >> 4) + (uint32_t)q];
    asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
    raw[4 * q] = v.x; raw[4 * q + 1] = v.y; raw[4 * q + 2] = v.z; raw[4 * q + 3] = v.w;
  }
  // (uniform by contract: a scalar branch and an SGPR shift, not four
  // exec-masked cases; stage A -1.5 %)
  const uint32_t sb = __builtin_amdgcn_readfirstlane(idx & 3u);
  auto take = [&](auto W) {
    constexpr int w = decltype(W)::value;
#pragma unroll
    for (int i = 0; i < ND; ++i) out[i] = __builtin_amdgcn_alignbyte(raw[w + i + 1], raw[w + i], sb);
  };
  switch (__builtin_amdgcn_readfirstlane((idx >> 2) & 3u)) {
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
    // (a lane outside the range reads in-bounds bytes at the same alignment)
    lds_bytes16(s_ref, o + (uint32_t)(ok ? D.off[j] : (D.off[j] & 15)), Rw);
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

// tiles [t, te) of XCD x in chunk c of nch (host and device)
// (a chunk is the fraction [b0, b1) / bt of every XCD's eighth)
__host__ __device__ __forceinline__ void xcd_chunk(uint64_t ntiles, uint32_t b0, uint32_t b1, uint32_t bt, uint64_t x,
                                                   uint64_t& t, uint64_t& te) {
  const uint64_t xs = ntiles * x / 8, xl = ntiles * (x + 1) / 8 - xs;
  t = xs + xl * b0 / bt;
  te = xs + xl * b1 / bt;
}

// K3 coverage pass.  One block per coverage group: QM tiles of one stripe of
// QM follower records (the lead's own tiles form groups of one).  The
// members share one staging of the two references' spans, so a CU keeps ~4x
// the windows in flight of a one-tile block at the same LDS (the pass is
// latency-bound: SQ_WAIT_ANY was 58 % of wave cycles with one tile per block,
// ~9 us per block for three dependent memory round trips and six barriers).
// Per member: the drift against the lead record and a second reference
// (cover_search), each segment's covered windows (segment_cover), and the
// segments left with work appended to the queue for k_emit_work.  A member
// with no reference (a single long record, or the lead's own tiles) queues
// every segment with nothing covered.
// Second reference.  Every follower also differs from the lead at the lead's
// own variant sites, where all followers share the other allele: with the
// lead alone those windows were emitted once per follower (C3: ~14 M of 51 M
// probes found their key already there).  So a second record (ref2) is
// searched too, and a window covered by either reference is skipped.  ref2's
// own windows are deduped against the lead only; a window it leaves to the
// lead has the lead's context, key and masks, so "covered by ref2" still
// means "inserted".
// Chunks and XCDs: each XCD owns a contiguous eighth of the group list
// (stripe-major, so its blocks share reference spans in its own L2), and
// chunk c of nch launches takes the c-th part of every XCD's eighth, so an
// XCD's drift hints carry over from the end of its previous chunk to the
// start of the next.  (A persistent, software-pipelined one-tile form of this
// kernel measured slower: 909 vs 845 us for all of C3's tiles.)
#ifdef PG_COVER_LEGACY   // (rounds 2-3's class-byte forms: test-only builds, PG_TUNE_K3_COVER 1 / 2)
__global__ void __launch_bounds__(CBLOCK)
k_cover(const uint8_t* __restrict__ cls, const TileDesc* __restrict__ descs, WorkItem* __restrict__ queue,
        unsigned long long* __restrict__ qcount, unsigned long long qcap, int k, int ref, long long rfs,
        long long rfn, int ref2, long long r2s, long long r2n, int* __restrict__ hints, int nrec,
        uint64_t ngroups, uint32_t b0, uint32_t b1, uint32_t bt) {
  __shared__ __attribute__((aligned(16))) uint8_t s_cls[QM][SPAN + 16];
  __shared__ __attribute__((aligned(16))) uint8_t s_ref[2][RSPAN];
  __shared__ unsigned s_best[QM][2][NANCH];
  __shared__ uint32_t s_scan[CBLOCK / 64];
  __shared__ unsigned long long s_qbase;
  __shared__ MemGeo s_geo[QM];
  __shared__ Drifts s_dr[QM][2];
  uint64_t g, ge;
  xcd_chunk(ngroups, b0, b1, bt, blockIdx.x & 7, g, ge);
  g += blockIdx.x >> 3;
  if (g >= ge) return;                             // (block-uniform, before any barrier)
  // the members' descriptors (uniform loads) -> which members dedup
  const long long qt = (long long)descs[QM * g].stripe * TILE;
  uint32_t dm0 = 0, dm1 = 0;
#pragma unroll
  for (int m = 0; m < QM; ++m) {
    const int r = descs[QM * g + m].r;
    const bool d0 = r >= 0 && ref >= 0 && ref != r;
    dm0 |= (uint32_t)d0 << m;
    dm1 |= (uint32_t)(d0 && ref2 >= 0 && ref2 != r) << m;
  }
  // per member: staging window and hints (hints per XCD, reference and
  // record: the XCD swizzle gives each XCD its own eighth of the group list,
  // so one shared hint per record alternated between stripes ~150 apart)
  int* hx = hints + (size_t)(blockIdx.x & 7) * 2 * nrec;
  if (threadIdx.x < QM) {
    const TileDesc td = descs[QM * g + threadIdx.x];
    MemGeo G;
    G.r = td.r;
    G.rs = td.rs;
    G.rn = td.rn;
    const long long lo = td.rs + (qt >= 2 ? qt - 2 : 0);
    G.hi = td.rs + (qt + TILE + k + 2 < td.rn ? qt + TILE + k + 2 : td.rn);
    G.a0 = lo & ~15ll;
    if (td.r < 0) G.a0 = G.hi = 0;                 // an empty slot stages nothing
    // (no drift known yet: try delta 0 first, the drift at a record's start)
    const int h0 = ((dm0 >> threadIdx.x) & 1u) ? hx[td.r] : -1;
    const int h1 = ((dm1 >> threadIdx.x) & 1u) ? hx[nrec + td.r] : -1;
    G.h[0] = h0 < 0 ? DRIFT : h0;
    G.h[1] = h1 < 0 ? DRIFT : h1;
    s_geo[threadIdx.x] = G;
  }
  if (threadIdx.x < QM * 2 * NANCH) (&s_best[0][0][0])[threadIdx.x] = ~0u;
  // the references' spans of this stripe: [qt-1-DRIFT, qt+TILE+k+1+DRIFT) clipped
  RefGeo rg[2];
  long long ra0[2], rend[2];
#pragma unroll
  for (int ri = 0; ri < 2; ++ri) {
    const long long s = ri ? r2s : rfs, n = ri ? r2n : rfn;
    rg[ri].plo = qt - 1 - DRIFT > 0 ? qt - 1 - DRIFT : 0;
    rg[ri].phi = qt + TILE + k + 1 + DRIFT < n ? qt + TILE + k + 1 + DRIFT : n;
    rg[ri].rfn = n;
    ra0[ri] = (s + rg[ri].plo) & ~15ll;
    rend[ri] = s + rg[ri].phi;
    rg[ri].rbase = s - ra0[ri];
  }
  __syncthreads();
  // staging: every span's loads in flight before the first LDS store (at most
  // two 16-byte chunks per thread and span: SPAN, RSPAN < 2 * CBLOCK * 16)
  static_assert(SPAN + 16 <= 2 * CBLOCK * 16 && RSPAN <= 2 * CBLOCK * 16, "two chunks per thread");
  {
    constexpr int NS = QM + 2;
    uint4 v[NS][2];
    bool lv[NS][2];
    const long long o0 = (long long)threadIdx.x * 16, o1 = o0 + CBLOCK * 16;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      long long from, to;
      if (s < QM) { from = s_geo[s].a0; to = s_geo[s].hi; }
      else {
        const int ri = s - QM;
        const bool use = ri ? dm1 != 0 : dm0 != 0;
        from = ra0[ri];
        to = use ? rend[ri] : from;
      }
      lv[s][0] = from + o0 < to;
      lv[s][1] = from + o1 < to;
      v[s][0] = lv[s][0] ? *reinterpret_cast<const uint4*>(cls + from + o0) : make_uint4(0u, 0u, 0u, 0u);
      v[s][1] = lv[s][1] ? *reinterpret_cast<const uint4*>(cls + from + o1) : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      uint8_t* dst = s < QM ? s_cls[s] : s_ref[s - QM];
      if (lv[s][0]) *reinterpret_cast<uint4*>(dst + o0) = v[s][0];
      if (lv[s][1]) *reinterpret_cast<uint4*>(dst + o1) = v[s][1];
    }
  }
  __syncthreads();
  if (dm0 && !(PG_EXP_BITS & 32)) cover_search(s_cls, s_ref, s_geo, rg[0], rg[1], s_best, qt, dm0, dm1);
  // hints and drift sets: one lane per (member, reference)
  if (threadIdx.x < 2 * QM) {
    const int m = threadIdx.x >> 1, ri = threadIdx.x & 1;
    if ((((ri ? dm1 : dm0) >> m) & 1u)) {
      const MemGeo& G = s_geo[m];
      publish_hint(s_best[m][ri], hx + (ri ? nrec : 0) + G.r);
      const RefGeo R = ri ? rg[1] : rg[0];
      s_dr[m][ri] = drifts_of(s_best[m][ri], qt, G.rs - G.a0, R.rbase, R.rfn, R.plo, R.phi, k);
    }
  }
  __syncthreads();
  constexpr uint32_t ALL = (1u << IW) - 1u;
  constexpr int NB = (IW + 27 + 1 + 3) / 4;                  // bytes q0-1 .. q0+IW+k-1, k <= 27
  const long long q0 = qt + (long long)threadIdx.x * IW;
  const int rel = (int)threadIdx.x * IW;
  uint32_t cov[QM], nwk = 0, wmask = 0;
#pragma unroll
  for (int m = 0; m < QM; ++m) {
    const MemGeo& G = s_geo[m];
    const long long last = G.rn - k;
    uint32_t covered = 0;
    if (!(PG_EXP_BITS & 64) && ((dm0 >> m) & 1u) && q0 > 0 && q0 + IW <= last) {
      const uint32_t o = (uint32_t)(G.rs - G.a0 + q0 - 1);
      uint32_t Gb[NB];
      lds_bytes16(s_cls[m], o, Gb);
      covered = segment_cover(s_cls[m], s_ref[0], o, rel, Gb, s_dr[m][0], k);
      if (((dm1 >> m) & 1u) && covered != ALL) covered |= segment_cover(s_cls[m], s_ref[1], o, rel, Gb, s_dr[m][1], k);
    }
    cov[m] = covered;
    const bool work = G.r >= 0 && q0 <= last && covered != ALL;
    wmask |= (uint32_t)work << m;
    nwk += work ? 1u : 0u;
  }
  uint32_t nwork;
  uint32_t pos = block_excl_scan<CBLOCK>(nwk, s_scan, nwork);
  const unsigned sub = blockIdx.x % NQ;
  if (threadIdx.x == 0) s_qbase = nwork ? atomicAdd(qcount + QSTRIDE * sub, (unsigned long long)nwork) : 0ull;
  __syncthreads();
#pragma unroll
  for (int m = 0; m < QM; ++m)
    if ((wmask >> m) & 1u) {
      const MemGeo& G = s_geo[m];
      queue[sub * qcap + s_qbase + pos++] = WorkItem{G.rs, G.rn - k, q0, cov[m], 0u};
    }
}

// ---- K3 coverage pass, quad form (the default).  Same groups, drift search
// and coverage rule as k_cover, with the members never staged in LDS: thread
// t compares ONE 16-byte quad of each member (dwords D0+4t .. D0+4t+3 of the
// class stream, D0 = the dword holding the tile's first context byte
// rs+qt-1) against every drift of both references, a 4-bit mismatch nibble
// per (reference, drift), and segment t then reads the nibbles of quads t,
// t+1, t+2 (the 12 dwords that hold its IW+k+1 context bytes) from LDS.
// Each context byte is compared once instead of ~2.75 times, the member
// bytes go straight from HBM into registers (one coalesced 16-byte load per
// thread and member, issued beside the reference staging), and the block
// holds 16 KB of LDS instead of 27.8 KB.  The anchors of the drift search (3
// x 32 bytes per member) are staged on their own.
constexpr int RPAD = 32;                      // s_ref front pad: quads reaching below the span stay in bounds
constexpr int RSZ = RPAD + RSPAN + 32;        // + tail slack: a quad holding a staged byte never reads past it
constexpr int NQD = CBLOCK + 2;               // quads per member: segment t reads quads t .. t+2
typedef unsigned int u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

// the 16 bytes of class stream at byte address a (4-byte aligned), 0 outside [0, ncls)
__device__ __forceinline__ uint4 quad_at(const uint8_t* cls, long long a, uint64_t ncls, bool live) {
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (live && a >= 0 && (uint64_t)a + 16 <= ncls) {
    const u32x4a4 x = *reinterpret_cast<const u32x4a4*>(cls + a);
    v = make_uint4(x.x, x.y, x.z, x.w);
  }
  return v;
}
// mismatch nibble of a member quad against the reference quad at s_ref index
// e (e & 15 uniform over the wave); an index whose two 16-byte reads would
// leave s_ref reads at e & 15 instead (no covered segment uses such a quad)
__device__ __forceinline__ uint32_t quad_nib(const uint8_t* s_ref, int e, const uint4& M) {
  if (e < 0 || e > RSZ - 32) e &= 15;
  uint32_t R[4];
  lds_bytes16(s_ref, (uint32_t)e, R);
  return (uint32_t)(M.x != R[0]) | (uint32_t)(M.y != R[1]) << 1 | (uint32_t)(M.z != R[2]) << 2 |
         (uint32_t)(M.w != R[3]) << 3;
}
// covered windows of a segment from the 12-bit dword mismatch map of its
// quads (bit i: dword i from the dword holding byte q0-1, which sits sh
// bytes into it): segment_cover's rule on that grid
__device__ __forceinline__ uint32_t map_cover(uint32_t nz, int sh, int k) {
  constexpr uint32_t ALL = (1u << IW) - 1u;
  nz &= (2u << ((IW + k + sh) >> 2)) - 1u;                 // dwords holding bytes q0-1 .. q0+IW+k-1
  if (!nz) return ALL;
  const int first = 4 * __builtin_ctz(nz) - sh, last = 4 * (31 - __builtin_clz(nz)) + 3 - sh;
  const int ulo = max(0, first - k - 1), uhi = min(IW - 1, last);
  return ALL & ~(((2u << uhi) - 1u) & ~((1u << ulo) - 1u));
}
// drift_task for an anchor staged dword-aligned (A: its 32 bytes)
__device__ __forceinline__ void drift_task_anc(const uint32_t* A, const uint8_t* s_ref, int ibhi, int lo, int hi, int w,
                                               unsigned* best) {
  const uint32_t* rw = reinterpret_cast<const uint32_t*>(s_ref);
  const uint32_t x0 = A[0], x1 = A[1];
  const uint32_t W0 = rw[w], W1 = rw[w + 1], W2 = rw[w + 2];
  uint32_t hit = 0;
#pragma unroll
  for (int sb = 0; sb < 4; ++sb) {
    const int ib = 4 * w + sb;
    const bool h = (ib >= lo) & (ib <= hi) & (__builtin_amdgcn_alignbyte(W1, W0, sb) == x0) &
                   (__builtin_amdgcn_alignbyte(W2, W1, sb) == x1);
    hit |= (uint32_t)h << sb;
  }
  while (hit) {
    const int ib = 4 * w + __builtin_ctz(hit);
    hit &= hit - 1u;
    uint32_t Bw[ALEN / 4];
    lds_bytes(s_ref, (uint32_t)ib, Bw);
    bool eq = true;
#pragma unroll
    for (int i = 2; i < ALEN / 4; ++i) eq &= Bw[i] == A[i];
    const int d = ibhi - ib;
    const unsigned ad = (unsigned)(d > DRIFT ? d - DRIFT : DRIFT - d);
    if (eq) atomicMin(best, (ad << 16) | (unsigned)d);
  }
}
// cover_search on the staged anchors: member m's anchor ai is s_anc[m][ai]
// (its 32 bytes, realigned to dwords when staged)
// (Checking each triple's hint drift exactly first and searching only the
// misses measured neutral: stage A 0.599 ms either way.)
__device__ __forceinline__ void cover_search_q(uint32_t (*s_anc)[NANCH][ALEN / 4], uint8_t (*s_ref)[RSZ],
                                               const TriGeo* tri, unsigned (*best)[2][NANCH], uint32_t dm0,
                                               uint32_t dm1) {
  constexpr int NT = QM * 2 * NANCH, PER = CBLOCK / 32;
  constexpr int NW = (2 * DRIFT + 3) / 4 + 2;
#pragma unroll 1
  for (int t0 = 0; t0 < NT; t0 += PER) {
    const int t = t0 + ((int)threadIdx.x >> 5), l = (int)threadIdx.x & 31;
    if (t < NT) {
      const int m = t / (2 * NANCH), ri = (t / NANCH) & 1, ai = t % NANCH;
      const TriGeo g = tri[t];
      const int w = (g.lo1 >> 2) + l;
      if (g.lo1 <= g.hi1 && 4 * w <= g.hi1)
        drift_task_anc(s_anc[m][ai], s_ref[ri], g.ibhi, g.lo1, g.hi1, w, &best[m][ri][ai]);
    }
  }
  __syncthreads();
  // pairs whose three anchors all missed: decided by every wave from the
  // state the barrier above published, and the barrier below keeps any
  // wave's search from changing best[] before every wave has decided (a
  // wave deciding late would otherwise skip the pair and the barriers)
  uint32_t need = 0;
#pragma unroll
  for (int p = 0; p < 2 * QM; ++p) {
    const int m = p >> 1, ri = p & 1;
    unsigned all = ~0u;
#pragma unroll
    for (int ai = 0; ai < NANCH; ++ai) all &= best[m][ri][ai];
    if ((((ri ? dm1 : dm0) >> m) & 1u) && all == ~0u) need |= 1u << p;
  }
  if (!need) return;                                          // (block-uniform)
  __syncthreads();
#pragma unroll 1
  for (int p = 0; p < 2 * QM; ++p) {
    const int m = p >> 1, ri = p & 1;
    if (!((need >> p) & 1u)) continue;
#pragma unroll 1
    for (int ai = 0; ai < NANCH; ++ai) {
      const TriGeo g = tri[(m * 2 + ri) * NANCH + ai];
      for (int w = (g.lo >> 2) + (int)threadIdx.x; 4 * w <= g.hi && w < (g.lo >> 2) + NW; w += CBLOCK)
        drift_task_anc(s_anc[m][ai], s_ref[ri], g.ibhi, g.lo, g.hi, w, &best[m][ri][ai]);
    }
  }
  __syncthreads();
}

// (8 waves per SIMD: 78 SGPRs with 24 spilled to VGPR lanes, against 106 and
// 7 waves unbounded: stage A 0.599 vs 0.637 ms)
__global__ void __launch_bounds__(CBLOCK, 8)
k_cover_q(const uint8_t* __restrict__ cls, uint64_t ncls, const TileDesc* __restrict__ descs,
          WorkItem* __restrict__ queue, unsigned long long* __restrict__ qcount, unsigned long long qcap, int k,
          int ref, long long rfs, long long rfn, int ref2, long long r2s, long long r2n, int* __restrict__ hints,
          int nrec, uint64_t ngroups, uint32_t b0, uint32_t b1, uint32_t bt) {
  __shared__ __attribute__((aligned(16))) uint8_t s_ref[2][RSZ];
  __shared__ __attribute__((aligned(16))) uint32_t s_anc[QM][NANCH][ALEN / 4];
  __shared__ __attribute__((aligned(16))) uint4 s_xq[QM][2];       // member quads CBLOCK, CBLOCK+1
  __shared__ uint32_t s_nib[QM][NQD];                              // bit 4*(3*ri+j)+i: dword i, reference ri, drift j
  __shared__ unsigned s_best[QM][2][NANCH];
  __shared__ uint32_t s_scan[CBLOCK / 64];
  __shared__ unsigned long long s_qbase;
  __shared__ MemGeo s_geo[QM];
  __shared__ Drifts s_dr[QM][2];
  __shared__ TriGeo s_tri[QM * 2 * NANCH];
  uint64_t g, ge;
  xcd_chunk(ngroups, b0, b1, bt, blockIdx.x & 7, g, ge);
  g += blockIdx.x >> 3;
  if (g >= ge) return;                             // (block-uniform, before any barrier)
  const int t = (int)threadIdx.x;
  const long long qt = (long long)descs[QM * g].stripe * TILE;
  // the references' spans of this stripe: [qt-1-DRIFT, qt+TILE+k+1+DRIFT) clipped
  RefGeo rg[2];
  long long ra0[2], rend[2];
#pragma unroll
  for (int ri = 0; ri < 2; ++ri) {
    const long long s = ri ? r2s : rfs, n = ri ? r2n : rfn;
    rg[ri].plo = qt - 1 - DRIFT > 0 ? qt - 1 - DRIFT : 0;
    rg[ri].phi = qt + TILE + k + 1 + DRIFT < n ? qt + TILE + k + 1 + DRIFT : n;
    rg[ri].rfn = n;
    ra0[ri] = (s + rg[ri].plo) & ~15ll;
    rend[ri] = s + rg[ri].phi;
    rg[ri].rbase = s - ra0[ri] + RPAD;
  }
  // the members (uniform loads): records, which members dedup
  long long mrs[QM], mrn[QM];
  uint32_t dm0 = 0, dm1 = 0, live = 0;
#pragma unroll
  for (int m = 0; m < QM; ++m) {
    const TileDesc td = descs[QM * g + m];
    mrs[m] = td.rs;
    mrn[m] = td.rn;
    const bool d0 = td.r >= 0 && ref >= 0 && ref != td.r;
    live |= (uint32_t)(td.r >= 0) << m;
    dm0 |= (uint32_t)d0 << m;
    dm1 |= (uint32_t)(d0 && ref2 >= 0 && ref2 != td.r) << m;
  }
  // member quads straight into registers: dwords D0+4t .. (D0 = floor((rs+qt-1)/4))
  uint4 Mq[QM];
#pragma unroll
  for (int m = 0; m < QM; ++m) {
    const long long d0 = (mrs[m] + qt - 1) >> 2;
    Mq[m] = quad_at(cls, 4 * d0 + 16ll * t, ncls, (dm0 >> m) & 1u);
  }
  if (t < 2 * QM) {                                // quads CBLOCK, CBLOCK+1 of member t/2
    const int m = t >> 1;
    long long rs = mrs[0];
#pragma unroll
    for (int x = 1; x < QM; ++x) rs = m == x ? mrs[x] : rs;
    s_xq[m][t & 1] = quad_at(cls, 4 * ((rs + qt - 1) >> 2) + 16ll * (CBLOCK + (t & 1)), ncls, (dm0 >> m) & 1u);
  } else if (t >= 64 && t < 64 + QM * NANCH) {     // anchors: 32 bytes each, realigned to dwords
    const int x = t - 64, m = x / NANCH, ai = x % NANCH;
    long long rs = mrs[0];
#pragma unroll
    for (int y = 1; y < QM; ++y) rs = m == y ? mrs[y] : rs;
    const long long a = rs + qt + 8 + (long long)ai * ASTEP, a4 = a & ~3ll;
    const bool lv = (dm0 >> m) & 1u;
    const uint4 q0 = quad_at(cls, a4, ncls, lv), q1 = quad_at(cls, a4 + 16, ncls, lv),
                q2 = quad_at(cls, a4 + 32, ncls, lv);
    const uint32_t r[9] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x};
    const uint32_t sb = (uint32_t)(a & 3);
    uint32_t o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = __builtin_amdgcn_alignbyte(r[i + 1], r[i], sb);
    *reinterpret_cast<uint4*>(&s_anc[m][ai][0]) = make_uint4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<uint4*>(&s_anc[m][ai][4]) = make_uint4(o[4], o[5], o[6], o[7]);
  } else if (t >= 160 && t < 160 + QM) {           // the members' records
    const int m = t - 160;
    const TileDesc td = descs[QM * g + m];
    MemGeo G;
    G.r = td.r;
    G.rs = td.rs;
    G.rn = td.rn;
    G.a0 = G.hi = 0;
    G.h[0] = G.h[1] = 0;
    s_geo[m] = G;
  }
  static_assert(2 * QM <= 64 && 64 + QM * NANCH <= 160 && 160 + QM <= 192 && 192 + QM * 2 * NANCH <= CBLOCK,
                "thread ranges of the staging roles");
  if (t >= 192 && t < 192 + QM * 2 * NANCH) {     // triples: search geometry around the hint (per XCD,
                                                   // reference and record)
    const int x = t - 192, m = x / (2 * NANCH), ri = (x / NANCH) & 1, ai = x % NANCH;
    (&s_best[0][0][0])[x] = ~0u;
    TriGeo G{0, 0, -1, 0, -1};
    if ((((ri ? dm1 : dm0) >> m) & 1u)) {
      const TileDesc td = descs[QM * g + m];
      const int hh = hints[(size_t)(blockIdx.x & 7) * 2 * nrec + (ri ? nrec : 0) + td.r];
      const int h = hh < 0 ? DRIFT : hh;
      const RefGeo& R = ri ? rg[1] : rg[0];
      const long long a = qt + 8 + (long long)ai * ASTEP;
      G.ibhi = (int)(R.rbase + a + DRIFT);
      G.lo = max(G.ibhi - 2 * DRIFT, (int)(R.rbase + R.plo));
      G.hi = a + ALEN > td.rn ? -1 : min(G.ibhi, (int)(R.rbase + R.phi) - ALEN);
      G.lo1 = max(G.lo, G.ibhi - (h + HWIN2));
      G.hi1 = min(G.hi, G.ibhi - (h - HWIN2));
    }
    s_tri[x] = G;
  }
  {
    static_assert(RSPAN <= 2 * CBLOCK * 16, "two chunks per thread");
    uint4 v[2][2];
    bool lv[2][2];
    const long long o0 = (long long)t * 16, o1 = o0 + CBLOCK * 16;
#pragma unroll
    for (int ri = 0; ri < 2; ++ri) {
      const long long from = ra0[ri], to = (ri ? dm1 != 0 : dm0 != 0) ? rend[ri] : from;
      lv[ri][0] = from + o0 < to;
      lv[ri][1] = from + o1 < to;
      v[ri][0] = lv[ri][0] ? *reinterpret_cast<const uint4*>(cls + from + o0) : make_uint4(0u, 0u, 0u, 0u);
      v[ri][1] = lv[ri][1] ? *reinterpret_cast<const uint4*>(cls + from + o1) : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int ri = 0; ri < 2; ++ri) {
      if (lv[ri][0]) *reinterpret_cast<uint4*>(s_ref[ri] + RPAD + o0) = v[ri][0];
      if (lv[ri][1]) *reinterpret_cast<uint4*>(s_ref[ri] + RPAD + o1) = v[ri][1];
    }
  }
  __syncthreads();
  if (dm0) cover_search_q(s_anc, s_ref, s_tri, s_best, dm0, dm1);
  // hints and drift sets: one lane per (member, reference); a drift set's
  // offsets index s_ref from thread 0's quad (add 16 t)
  if (t < 2 * QM) {
    const int m = t >> 1, ri = t & 1;
    if ((((ri ? dm1 : dm0) >> m) & 1u)) {
      const MemGeo& G = s_geo[m];
      publish_hint(s_best[m][ri], hints + (size_t)(blockIdx.x & 7) * 2 * nrec + (ri ? nrec : 0) + G.r);
      const RefGeo R = ri ? rg[1] : rg[0];
      const long long qs = qt - 1 - ((G.rs + qt - 1) & 3);   // record position of thread 0's quad
      s_dr[m][ri] = drifts_of(s_best[m][ri], qt, -qs, R.rbase, R.rfn, R.plo, R.phi, k);
    }
  }
  __syncthreads();
  // mismatch nibbles of every quad against every drift of both references
#pragma unroll
  for (int m = 0; m < QM; ++m) {
    uint32_t w = 0, wx = 0;
    if ((dm0 >> m) & 1u) {
#pragma unroll
      for (int ri = 0; ri < 2; ++ri) {
        if (ri && !((dm1 >> m) & 1u)) break;
        const int nd = __builtin_amdgcn_readfirstlane(s_dr[m][ri].n);
#pragma unroll
        for (int j = 0; j < NANCH; ++j) {
          if (j >= nd) break;
          const int off = __builtin_amdgcn_readfirstlane(s_dr[m][ri].off[j]);
          w |= quad_nib(s_ref[ri], off + 16 * t, Mq[m]) << (4 * (3 * ri + j));
          if (t >= CBLOCK - 2)                     // (the last wave: wave 0 computes the drift sets)
            wx |= quad_nib(s_ref[ri], off + 16 * (t + 2), s_xq[m][t - (CBLOCK - 2)]) << (4 * (3 * ri + j));
        }
      }
    }
    s_nib[m][t] = w;
    if (t >= CBLOCK - 2) s_nib[m][t + 2] = wx;
  }
  __syncthreads();
  const long long q0 = qt + (long long)t * IW;
  const int rel = t * IW;
  uint32_t cov[QM], nwk = 0, wmask = 0;
#pragma unroll
  for (int m = 0; m < QM; ++m) {
    const long long last = mrn[m] - k;
    uint32_t covered = 0;
    if (((dm0 >> m) & 1u) && q0 > 0 && q0 + IW <= last) {
      const int sh = (int)((mrs[m] + qt - 1) & 3);
      const uint32_t w0 = s_nib[m][t], w1 = s_nib[m][t + 1], w2 = s_nib[m][t + 2];
#pragma unroll
      for (int ri = 0; ri < 2; ++ri) {
        if (ri && !((dm1 >> m) & 1u)) break;
        const int nd = __builtin_amdgcn_readfirstlane(s_dr[m][ri].n);
#pragma unroll
        for (int j = 0; j < NANCH; ++j) {
          if (j >= nd) break;
          const int lo = __builtin_amdgcn_readfirstlane(s_dr[m][ri].lo[j]);
          const int hi = __builtin_amdgcn_readfirstlane(s_dr[m][ri].hi[j]);
          const int s = 4 * (3 * ri + j);
          const uint32_t nz = ((w0 >> s) & 15u) | ((w1 >> s) & 15u) << 4 | ((w2 >> s) & 15u) << 8;
          covered |= ((rel >= lo) & (rel <= hi)) ? map_cover(nz, sh, k) : 0u;
        }
      }
    }
    cov[m] = covered;
    const bool work = ((live >> m) & 1u) && q0 <= last && covered != (1u << IW) - 1u;
    wmask |= (uint32_t)work << m;
    nwk += work ? 1u : 0u;
  }
  uint32_t nwork;
  uint32_t pos = block_excl_scan<CBLOCK>(nwk, s_scan, nwork);
  const unsigned sub = blockIdx.x % NQ;
  if (t == 0) s_qbase = nwork ? atomicAdd(qcount + QSTRIDE * sub, (unsigned long long)nwork) : 0ull;
  __syncthreads();
#pragma unroll
  for (int m = 0; m < QM; ++m)
    if ((wmask >> m) & 1u) queue[sub * qcap + s_qbase + pos++] = WorkItem{mrs[m], mrn[m] - k, q0, cov[m], 0u};
}

#endif  // PG_COVER_LEGACY

// Search geometry of one (member, reference, anchor) triple, computed once
// per block in the staging phase: ibhi = the reference index of drift 0's
// candidate + DRIFT; [lo, hi] the full search range, [lo1, hi1] its part
// within the hint window (empty if the triple does not dedup).
struct TriGeo {
  int ibhi, lo, hi, lo1, hi1;
};

// ---- K3 coverage pass, packed form (the default; north_star's "2-bit
// encode ... packed base stream").  Same groups, drift search and coverage
// rule as k_cover_q, on K1's packed stream (16 bases per 32-bit word, 2 bits
// each) instead of the class bytes:
//  * wave m of the block is member m; lane l owns the member's windows
//    64 l .. 64 l + 63 (4 segments) and loads the 7 words that hold their
//    context bases straight from HBM (0.44 B per base where the class stream
//    costs 1 B), with the exception bytes of those words;
//  * the two references' spans are staged in LDS as words (1.4 KB each);
//  * per (reference, drift) the lane XORs its words with the reference words
//    at that drift (three ds_read_b128 and one v_alignbit per word), turns
//    the 2-bit differences into one mismatch bit per base, and smears it over
//    each window's k+2 context bases (log2 steps of v_alignbit + OR): a window
//    is covered iff its smear bit is clear.  That is the coverage rule at base
//    granularity, exact where the quad form resolves it per dword (4 bases),
//    so no more windows go to the work pass than there;
//  * exceptions: a 2-bit code equals the class only for ACGT, so a lane whose
//    context words hold any base that is not ACGT (K1's exception bytes) is
//    not covered, and a reference whose staged span holds one is not used for
//    the stripe (the work pass then emits those windows exactly, as it does
//    every uncovered window);
//  * the drift search compares each anchor's 32 bases as two words, 16
//    candidate offsets per lane and reference word, 8 lanes per triple.
constexpr int RPADW = 4;                          // s_ref words in front of the staged span
constexpr int RSTAGEW = (RSPAN + 15) / 16 + 2;    // staged words per reference (<=)
constexpr int RDW = (RPADW + RSTAGEW + 16 + 3) / 4 * 4;   // + tail: a lane's 12-word read stays inside
constexpr int LW = 7;                             // packed words per lane: 64 windows + k+1 bases, any alignment
static_assert(IW * 4 == 64 && CBLOCK == 64 * QM, "a lane owns 4 segments; a wave owns a member");
// Anchors per (member, reference) in the packed pass, astep_p bases apart.  A
// window is covered under any drift its tile's anchors found, so a run of
// windows between two drift changes (the member's own indels, shared by both
// references) that no anchor falls in is lost to the work pass: with 3
// anchors per 4096-window tile that cost C3 ~25 % more stage A records than
// the ideal coverage of the two references (tools/cover_loss.py).
#ifndef PG_HWIN2P
#define PG_HWIN2P 56
#endif
constexpr int HWIN2P = PG_HWIN2P;                 // the first search: the XCD's hint +- HWIN2P
constexpr int NAP_DEFAULT = 4;                    // pg_tune PG_TUNE_K3_ANCHORS: 3, 4, 5, 6 or 8
template <int NAP>
constexpr int astep_p() { return (TILE - ALEN - 16) / (NAP - 1); }

template <int NAP>
struct Drifts2 {
  int n;
  int U[NAP], lo[NAP], hi[NAP];                   // U: s_ref base index of the member's word-grid base
  int d[NAP];                                     // the drift (q - p) itself
};
__device__ __forceinline__ uint32_t p2_word(const uint32_t* p2, long long i, uint64_t n_p2) {
  return (i >= 0 && (uint64_t)i < n_p2) ? p2[i] : 0u;
}

// candidates ib = 16 w .. 16 w + 15 (s_ref base indices) of the anchor (A0, A1)
// within [lo, hi]: its 32 bases against the reference's 32 from ib
__device__ __forceinline__ void drift_task_p(uint32_t A0, uint32_t A1, const uint32_t* R, int ibhi, int lo, int hi,
                                             int w, unsigned* best) {
  if (!PG_BOK(w >= 0 && w + 2 < RDW, 16, w, hi)) return;
  const uint32_t W0 = R[w], W1 = R[w + 1], W2 = R[w + 2];
  uint32_t hit = 0;
#pragma unroll
  for (int sb = 0; sb < 16; ++sb) hit |= (uint32_t)(__builtin_amdgcn_alignbit(W1, W0, 2 * sb) == A0) << sb;
  const int l = lo - 16 * w, h = hi - 16 * w;
  const uint32_t top = h >= 15 ? 0xFFFFu : h < 0 ? 0u : (2u << h) - 1u;
  const uint32_t bot = l <= 0 ? 0u : l > 15 ? 0xFFFFu : (1u << l) - 1u;
  hit &= top & ~bot;
  while (hit) {
    const int sb = __builtin_ctz(hit);
    hit &= hit - 1u;
    if (__builtin_amdgcn_alignbit(W2, W1, 2 * sb) == A1) {
      const int d = ibhi - (16 * w + sb);
      const unsigned ad = (unsigned)(d > DRIFT ? d - DRIFT : DRIFT - d);
      atomicMin(best, (ad << 16) | (unsigned)d);
    }
  }
}
// A block barrier that orders LDS only (s_waitcnt lgkmcnt(0); s_barrier):
// the packed coverage pass exchanges nothing through global memory inside a
// block, so its global loads stay in flight across its barriers (a
// __syncthreads also waits for every outstanding load, vmcnt(0)).
__device__ __forceinline__ void cover_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
template <int NAP>
__device__ __forceinline__ void cover_search_p(const uint32_t (*s_anc)[NAP][2], const uint32_t (*s_ref)[RDW],
                                               const TriGeo* tri, unsigned (*best)[2][NAP], uint32_t dm0,
                                               uint32_t dm1) {
  constexpr int NT = QM * 2 * NAP;
  constexpr int SLN = (2 * HWIN2P + 16 + 15) / 16;              // lanes per triple: 16 candidates each
  const int t = (int)threadIdx.x;
#pragma unroll
  for (int tr = t / SLN; tr < NT; tr += CBLOCK / SLN) {          // (NT * SLN / CBLOCK rounds)
    const int sub = t % SLN;
    const int m = tr / (2 * NAP), ri = (tr / NAP) & 1, ai = tr % NAP;
    const TriGeo g = tri[tr];
    const int w = (g.lo1 >> 4) + sub;
    if (g.lo1 <= g.hi1 && 16 * w <= g.hi1)
      drift_task_p(s_anc[m][ai][0], s_anc[m][ai][1], s_ref[ri], g.ibhi, g.lo1, g.hi1, w, &best[m][ri][ai]);
  }
  cover_barrier();
  // pairs whose three anchors all missed: decided by every wave from the
  // state the barrier above published, and the barrier below keeps any
  // wave's search from changing best[] before every wave has decided (a
  // wave deciding late would otherwise skip the pair and the barriers)
  uint32_t need = 0;
#pragma unroll
  for (int p = 0; p < 2 * QM; ++p) {
    const int m = p >> 1, ri = p & 1;
    unsigned all = ~0u;
#pragma unroll
    for (int ai = 0; ai < NAP; ++ai) all &= best[m][ri][ai];
    if ((((ri ? dm1 : dm0) >> m) & 1u) && all == ~0u) need |= 1u << p;
  }
  if (!need) return;                                          // (block-uniform)
  cover_barrier();
#pragma unroll 1
  for (int p = 0; p < 2 * QM; ++p) {
    const int m = p >> 1, ri = p & 1;
    if (!((need >> p) & 1u)) continue;
#pragma unroll 1
    for (int ai = 0; ai < NAP; ++ai) {
      const TriGeo g = tri[(m * 2 + ri) * NAP + ai];
      for (int w = (g.lo >> 4) + t; 16 * w <= g.hi; w += CBLOCK)
        drift_task_p(s_anc[m][ai][0], s_anc[m][ai][1], s_ref[ri], g.ibhi, g.lo, g.hi, w, &best[m][ri][ai]);
    }
  }
  cover_barrier();
}

// 8 words of s_ref from word index idx (idx & 3 the same on every lane: a
// scalar branch picks them out of three aligned 16-byte reads)
__device__ __forceinline__ void lds_words8(const uint32_t* R, int idx, uint32_t (&out)[8]) {
  const uint4* r16 = reinterpret_cast<const uint4*>(R);
  uint32_t raw[12];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    uint4 v = r16[(idx >> 2) + q];
    asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
    raw[4 * q] = v.x; raw[4 * q + 1] = v.y; raw[4 * q + 2] = v.z; raw[4 * q + 3] = v.w;
  }
  auto take = [&](auto W) {
    constexpr int w = decltype(W)::value;
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = raw[w + i];
  };
  switch (__builtin_amdgcn_readfirstlane(idx & 3)) {
    case 0: take(std::integral_constant<int, 0>{}); break;
    case 1: take(std::integral_constant<int, 1>{}); break;
    case 2: take(std::integral_constant<int, 2>{}); break;
    default: take(std::integral_constant<int, 3>{}); break;
  }
}
// the even bits of x (one per 2-bit base) compressed into 16 bits
__device__ __forceinline__ uint32_t even_bits(uint32_t x) {
  x = (x | (x >> 1)) & 0x33333333u;
  x = (x | (x >> 2)) & 0x0F0F0F0Fu;
  x = (x | (x >> 4)) & 0x00FF00FFu;
  return (x | (x >> 8)) & 0x0000FFFFu;
}

template <int NAP>
__global__ void __launch_bounds__(CBLOCK, 8)
k_cover_p(const uint32_t* __restrict__ p2, const uint8_t* __restrict__ e16, uint64_t n_p2,
          const uint8_t* __restrict__ cls_dbg, const TileDesc* __restrict__ descs, WorkItem* __restrict__ queue, unsigned long long* __restrict__ qcount,
          unsigned long long qcap, int k, int ref, long long rfs, long long rfn, int ref2, long long r2s,
          long long r2n, int* __restrict__ hints, int nrec, uint64_t ngroups, uint32_t b0, uint32_t b1, uint32_t bt) {
  static_assert(NAP >= 2 && QM * NAP + QM * 2 * NAP <= CBLOCK, "anchor loads and triple geometry: one thread each");
  constexpr int ASTEPP = astep_p<NAP>();
  __shared__ __attribute__((aligned(16))) uint32_t s_ref[2][RDW];
  __shared__ uint32_t s_anc[QM][NAP][2];
  __shared__ unsigned s_best[QM][2][NAP];
  __shared__ uint32_t s_scan[CBLOCK / 64];
  __shared__ unsigned long long s_qbase;
  __shared__ Drifts2<NAP> s_dr[QM][2];
  __shared__ TriGeo s_tri[QM * 2 * NAP];
  __shared__ uint32_t s_rexc;
  uint64_t g, ge;
  xcd_chunk(ngroups, b0, b1, bt, blockIdx.x & 7, g, ge);
  g += blockIdx.x >> 3;
  if (g >= ge) return;                             // (block-uniform, before any barrier)
  const int t = (int)threadIdx.x;
  const long long qt = (long long)descs[QM * g].stripe * TILE;
  // the references' spans of this stripe: [qt-1-DRIFT, qt+TILE+k+1+DRIFT) clipped, staged as the words
  // from rd0 (s_ref word RPADW); rbase = the s_ref base index of record position 0
  RefGeo rg[2];
  long long rd0[2];
  int rnw[2];
#pragma unroll
  for (int ri = 0; ri < 2; ++ri) {
    const long long s = ri ? r2s : rfs, n = ri ? r2n : rfn;
    rg[ri].plo = qt - 1 - DRIFT > 0 ? qt - 1 - DRIFT : 0;
    rg[ri].phi = qt + TILE + k + 1 + DRIFT < n ? qt + TILE + k + 1 + DRIFT : n;
    rg[ri].rfn = n;
    rd0[ri] = (s + rg[ri].plo) >> 4;
    rnw[ri] = (int)(((s + rg[ri].phi + 15) >> 4) - rd0[ri]);
    rg[ri].rbase = 16 * RPADW + s - 16 * rd0[ri];
  }
  long long mrs[QM], mrn[QM];
  uint32_t dm0 = 0, dm1 = 0, live = 0;
#pragma unroll
  for (int m = 0; m < QM; ++m) {
    const TileDesc td = descs[QM * g + m];
    mrs[m] = td.rs;
    mrn[m] = td.rn;
    const bool d0 = td.r >= 0 && ref >= 0 && ref != td.r;
    live |= (uint32_t)(td.r >= 0) << m;
    dm0 |= (uint32_t)d0 << m;
    dm1 |= (uint32_t)(d0 && ref2 >= 0 && ref2 != td.r) << m;
  }
  // the coverage phase's member words and exception bytes, loaded now: they
  // depend on nothing the block computes, and the barriers up to that phase
  // wait for LDS only (cover_barrier), so the loads land under the search
  const int mw = __builtin_amdgcn_readfirstlane(t >> 6), lw = t & 63;
  uint32_t M[LW], eex = 0;
  {
    long long rsm = mrs[0];
#pragma unroll
    for (int y = 1; y < QM; ++y) if (mw == y) rsm = mrs[y];
    const long long wb = ((rsm + qt - 1) >> 4) + 4 * lw, a = wb & ~3ll;
    const bool on = (dm0 >> mw) & 1u;
#pragma unroll
    for (int i = 0; i < LW; ++i) M[i] = on ? p2_word(p2, wb + i, n_p2) : 0u;
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (on && a + 4 * i >= 0 && (uint64_t)(a + 4 * i + 4) <= n_p2 + 16)
        eex |= *reinterpret_cast<const uint32_t*>(e16 + a + 4 * i);
  }
  if (t == 0) s_rexc = 0u;
  if (t < QM * NAP) {                              // anchors: 32 bases = 2 words each
    const int m = t / NAP, ai = t % NAP;
    long long rs = mrs[0];
#pragma unroll
    for (int y = 1; y < QM; ++y) rs = m == y ? mrs[y] : rs;
    const long long ga = rs + qt + 8 + (long long)ai * ASTEPP, x = ga >> 4;
    const uint32_t sb = 2u * (uint32_t)(ga & 15);
    uint32_t P0 = 0, P1 = 0, P2 = 0;
    if ((dm0 >> m) & 1u) { P0 = p2_word(p2, x, n_p2); P1 = p2_word(p2, x + 1, n_p2); P2 = p2_word(p2, x + 2, n_p2); }
    s_anc[m][ai][0] = __builtin_amdgcn_alignbit(P1, P0, sb);
    s_anc[m][ai][1] = __builtin_amdgcn_alignbit(P2, P1, sb);
  } else if (t >= CBLOCK - QM * 2 * NAP) {         // triples: search geometry around the XCD's hint
    const int x = t - (CBLOCK - QM * 2 * NAP), m = x / (2 * NAP), ri = (x / NAP) & 1, ai = x % NAP;
    (&s_best[0][0][0])[x] = ~0u;
    TriGeo G{0, 0, -1, 0, -1};
    if ((((ri ? dm1 : dm0) >> m) & 1u)) {
      const TileDesc td = descs[QM * g + m];
      const int hh = hints[(size_t)(blockIdx.x & 7) * 2 * nrec + (ri ? nrec : 0) + td.r];
      const int h = hh < 0 ? DRIFT : hh;
      const RefGeo& R = ri ? rg[1] : rg[0];
      const long long a = qt + 8 + (long long)ai * ASTEPP;
      G.ibhi = (int)(R.rbase + a + DRIFT);
      G.lo = max(G.ibhi - 2 * DRIFT, (int)(R.rbase + R.plo));
      G.hi = a + ALEN > td.rn ? -1 : min(G.ibhi, (int)(R.rbase + R.phi) - ALEN);
      G.lo1 = max(G.lo, G.ibhi - (h + HWIN2P));
      G.hi1 = min(G.hi, G.ibhi - (h - HWIN2P));
    }
    s_tri[x] = G;
  }
  cover_barrier();                                 // (s_rexc cleared)
  {
    static_assert(RSTAGEW <= 2 * CBLOCK, "two words per thread and reference");
    uint32_t v[2][2], ex = 0;
#pragma unroll
    for (int ri = 0; ri < 2; ++ri) {
      const int nw = (ri ? dm1 != 0 : dm0 != 0) ? rnw[ri] : 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int i = t + h * CBLOCK;
        v[ri][h] = i < nw ? p2_word(p2, rd0[ri] + i, n_p2) : 0u;
        if (i < nw && PG_BOK(rd0[ri] + i >= 0 && (uint64_t)(rd0[ri] + i) < n_p2, 12, rd0[ri] + i, n_p2) &&
            e16[rd0[ri] + i])
          ex |= 1u << ri;
      }
    }
#pragma unroll
    for (int ri = 0; ri < 2; ++ri)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (t + h * CBLOCK < rnw[ri] && PG_BOK(RPADW + t + h * CBLOCK < RDW, 13, rnw[ri], t))
          s_ref[ri][RPADW + t + h * CBLOCK] = v[ri][h];
    if (ex) atomicOr(&s_rexc, ex);
  }
  cover_barrier();
  {
    // a reference whose staged span holds a base that is not ACGT covers nothing here
    const uint32_t rexc = s_rexc;
    if (rexc & 1u) dm0 = dm1 = 0u;
    if (rexc & 2u) dm1 = 0u;
  }
  if (dm0) cover_search_p(s_anc, s_ref, s_tri, s_best, dm0, dm1);
  if (t < QM * 2 * NAP) {                          // hints and drift sets: one lane per (member, reference, anchor)
    const int m = t / (2 * NAP), ri = (t / NAP) & 1, ai = t % NAP;
    if ((((ri ? dm1 : dm0) >> m) & 1u)) {
      const unsigned* B = s_best[m][ri];
      const unsigned b = B[ai];
      // the set holds each distinct drift once, in anchor order: this anchor's
      // slot is the number of distinct drifts the anchors before it found
      auto first = [&](int j) {                     // anchor j found a drift no anchor before it found
        if (B[j] == ~0u) return false;
        for (int i = 0; i < j; ++i)
          if ((B[i] & 0xFFFFu) == (B[j] & 0xFFFFu)) return false;
        return true;
      };
      int slot = 0;
      for (int j = 0; j < ai; ++j) slot += first(j) ? 1 : 0;
      const bool keep = first(ai);
      bool last = b != ~0u;                         // the last anchor that found one
      for (int j = ai + 1; j < NAP; ++j) last &= B[j] == ~0u;
      long long rs = mrs[0];
#pragma unroll
      for (int y = 1; y < QM; ++y) rs = m == y ? mrs[y] : rs;
      const int r = descs[QM * g + m].r;
      (void)PG_BOK(r >= 0 && r < nrec, 52, (long long)r, (long long)nrec);
      // the hint: the drift nearest the record's next stripe
      if (last) hints[(size_t)(blockIdx.x & 7) * 2 * nrec + (ri ? nrec : 0) + r] = (int)(b & 0xFFFFu);
      Drifts2<NAP>& D = s_dr[m][ri];
      if (keep) {
        const RefGeo R = ri ? rg[1] : rg[0];
        const long long pos16 = 16 * ((rs + qt - 1) >> 4) - rs;   // record position of the member's word grid
        const int d = (int)(b & 0xFFFFu) - DRIFT;
        const long long pl = R.plo + 1 > 1 ? R.plo + 1 : 1;
        const long long ph = R.rfn - k - IW < R.phi - IW - k ? R.rfn - k - IW : R.phi - IW - k;
        const long long lo = pl + d - qt, hi = ph + d - qt;
        D.U[slot] = (int)(R.rbase + pos16 - d);
        D.lo[slot] = (int)(lo < -(1ll << 30) ? -(1ll << 30) : lo);
        D.hi[slot] = (int)(hi > (1ll << 30) ? (1ll << 30) : hi);
        D.d[slot] = d;
      }
      if (ai == NAP - 1) D.n = slot + (keep ? 1 : 0);
    }
  }
  cover_barrier();
  // ---- coverage: wave m = member m, lane l = windows 64 l .. 64 l + 63
  const int m = __builtin_amdgcn_readfirstlane(t >> 6), l = t & 63;
  long long rs = mrs[0], rn = mrn[0];
#pragma unroll
  for (int y = 1; y < QM; ++y) if (m == y) { rs = mrs[y]; rn = mrn[y]; }
  const long long last = rn - k;
  uint32_t covS[4] = {0u, 0u, 0u, 0u};            // per segment: bit 2 i = window i covered
  bool mex = false;
  if ((dm0 >> m) & 1u) {
    const long long p0 = rs + qt - 1, wb = (p0 >> 4) + 4 * l;
    const int sh2 = 2 * (int)(p0 & 15);
    // (M: the lane's words wb .. wb + 6, eex: the exception bytes of the three
    // aligned dwords around them, both loaded at the start)
    (void)PG_BOK(wb + LW <= (long long)n_p2 + 4 || wb > (long long)n_p2, 11, wb, n_p2);
    (void)wb;
    mex = eex != 0u;
    const int L = k + 2;                           // context bases of a window
    const int P = L >= 16 ? 16 : L >= 8 ? 8 : L >= 4 ? 4 : 2;
    const uint32_t rsh = 2u * (uint32_t)(L - P);
#pragma unroll
    for (int ri = 0; ri < 2; ++ri) {
      if (ri && !((dm1 >> m) & 1u)) break;
      const int nd = __builtin_amdgcn_readfirstlane(s_dr[m][ri].n);
#pragma unroll 1
      for (int j = 0; j < nd; ++j) {
        const int U = __builtin_amdgcn_readfirstlane(s_dr[m][ri].U[j]);
        const int lo = __builtin_amdgcn_readfirstlane(s_dr[m][ri].lo[j]);
        const int hi = __builtin_amdgcn_readfirstlane(s_dr[m][ri].hi[j]);
        int iw = (U >> 4) + 4 * l;
        if (iw < 0 || iw + 12 > RDW) iw &= 3;      // (an invalid lane: in-bounds words, same alignment)
        if (!PG_BOK(iw >= 0 && iw + 12 <= RDW, 14, iw, U)) iw = 0;
        // the reference words iw .. iw + 7 out of three aligned 16-byte reads;
        // iw & 3 is the same on every lane, and the compare runs inside the
        // uniform branch that knows it, so the words are used where they were
        // loaded (selecting them first cost 32 register moves per drift)
        uint32_t raw[12];
        {
          const uint4* r16 = reinterpret_cast<const uint4*>(s_ref[ri]);
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            uint4 v = r16[(iw >> 2) + q];
            asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
            raw[4 * q] = v.x; raw[4 * q + 1] = v.y; raw[4 * q + 2] = v.z; raw[4 * q + 3] = v.w;
          }
        }
        const uint32_t bs = 2u * (uint32_t)(U & 15);
        uint32_t Z[LW];
        auto zrun = [&](auto W) {
          constexpr int w = decltype(W)::value;
#pragma unroll
          for (int i = 0; i < LW; ++i) {
            // both bits of each base, differing where it mismatches: the smear
            // below moves bits by even counts only, so a base's two bits stay
            // apart until S folds them onto its even bit
            Z[i] = M[i] ^ __builtin_amdgcn_alignbit(raw[w + i + 1], raw[w + i], bs);
          }
        };
        switch (__builtin_amdgcn_readfirstlane(iw & 3)) {
          case 0: zrun(std::integral_constant<int, 0>{}); break;
          case 1: zrun(std::integral_constant<int, 1>{}); break;
          case 2: zrun(std::integral_constant<int, 2>{}); break;
          default: zrun(std::integral_constant<int, 3>{}); break;
        }
        uint32_t T[LW - 1];                         // from the lane's first context base (sh bases in)
#pragma unroll
        for (int i = 0; i < LW - 1; ++i) T[i] = __builtin_amdgcn_alignbit(Z[i + 1], Z[i], (uint32_t)sh2);
        // smear: T[b] = any mismatch in bases b .. b + P - 1, then S = T | T >> (L - P)
#pragma unroll
        for (int e = 1; e <= 4; ++e) {
          if ((1 << e) > P) break;                 // (uniform)
#pragma unroll
          for (int i = 0; i < LW - 1; ++i)         // length 2^(e-1) -> 2^e bases: shift by 2^(e-1) bases
            T[i] |= __builtin_amdgcn_alignbit(i + 1 < LW - 1 ? T[i + 1] : 0u, T[i], (uint32_t)(1 << e));
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int rel = 64 * l + 16 * s;
          const uint32_t S2 = T[s] | __builtin_amdgcn_alignbit(T[s + 1], T[s], rsh);
          const uint32_t S = S2 | (S2 >> 1);         // even bit of each window: any mismatch in it
          covS[s] |= (rel >= lo && rel <= hi) ? ~S & 0x55555555u : 0u;
#ifdef PG_DEBUG_BOUNDS
          {                                        // every window this drift covers, against the class bytes
            const long long q0 = qt + rel;
            const int dd = __builtin_amdgcn_readfirstlane(s_dr[m][ri].d[j]);
            const long long fs = ri ? r2s : rfs;
            const uint32_t cvd = (rel >= lo && rel <= hi && q0 > 0 && q0 + IW <= last) ? (~S & 0x55555555u) : 0u;
            for (int i = 0; i < 16; ++i)
              if ((cvd >> (2 * i)) & 1u) {
                const long long q = q0 + i;
                bool eq = true;
                for (int x = -1; x <= k; ++x) eq &= cls_dbg[rs + q + x] == cls_dbg[fs + q - dd + x];
                (void)pg_bok(eq, 31, (long long)q, (long long)dd);
              }
          }
#endif
        }
      }
    }
  }
  uint32_t nwk = 0, wmask = 0, cov[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const long long q0 = qt + 64 * l + 16 * s;
    const bool interior = q0 > 0 && q0 + IW <= last;
    cov[s] = interior && !mex ? even_bits(covS[s]) : 0u;
    const bool work = ((live >> m) & 1u) && q0 <= last && cov[s] != (1u << IW) - 1u;
    wmask |= (uint32_t)work << s;
    nwk += work ? 1u : 0u;
  }
  uint32_t nwork;
  uint32_t pos = block_excl_scan<CBLOCK>(nwk, s_scan, nwork);
  const unsigned sub = blockIdx.x % NQ;
  if (t == 0) {
    s_qbase = nwork ? atomicAdd(qcount + QSTRIDE * sub, (unsigned long long)nwork) : 0ull;
    (void)PG_BOK(nwork <= QM * CBLOCK && s_qbase + nwork <= qcap, 42, (long long)nwork, (long long)s_qbase);
  }
  cover_barrier();
#pragma unroll
  for (int s = 0; s < 4; ++s)
    if ((wmask >> s) & 1u) {
      if (PG_BOK(s_qbase + pos < qcap && rs >= 0 && qt + 64 * l + 16 * s <= rn, 15, s_qbase + pos, rs))
        queue[sub * qcap + s_qbase + pos] = WorkItem{rs, rn - k, qt + 64 * l + 16 * s, cov[s], 0u};
      ++pos;
    }
}

// the packed coverage pass with na anchors per (member, reference)
template <typename... A>
static void launch_cover_p(int na, dim3 grid, hipStream_t s, A... a) {
  switch (na) {
    case 3: hipLaunchKernelGGL(k_cover_p<3>, grid, dim3(CBLOCK), 0, s, a...); break;
    case 4: hipLaunchKernelGGL(k_cover_p<4>, grid, dim3(CBLOCK), 0, s, a...); break;
    case 5: hipLaunchKernelGGL(k_cover_p<5>, grid, dim3(CBLOCK), 0, s, a...); break;
    case 6: hipLaunchKernelGGL(k_cover_p<6>, grid, dim3(CBLOCK), 0, s, a...); break;
    default: hipLaunchKernelGGL(k_cover_p<8>, grid, dim3(CBLOCK), 0, s, a...); break;
  }
}

#ifdef PG_DEBUG_BOUNDS
// every sub-queue counter of a chunk at most `lim` (code: which check point)
__global__ void k_dbg_counters(const unsigned long long* __restrict__ qcount, unsigned long long lim, unsigned code,
                               unsigned chunk) {
  const unsigned sub = threadIdx.x;
  if (sub < NQ) {
    const unsigned long long v = qcount[QSTRIDE * sub];
    (void)pg_bok(v <= lim, code, (long long)v, (long long)(chunk * 1000 + sub));
  }
}
#endif

// ---------------------------------------------------------------- stage A
// Records go to NBIN coarse bins (h >> shift: the top bits of the bucket
// index), each with one region per XCD (region = bin * 8 + XCD), so that a
// bin's records land as contiguous runs.  A block bins the records of one
// round in LDS (rank by LDS atomic per bin), reserves each bin's run with ONE
// returning global atomic on that region's cursor (512 cursors on lines of
// their own: per cursor ~1.3 K reservations per C3 build), then writes.
constexpr int NBIN = 64;                      // coarse bins (CB <= 6 bits)
constexpr int NREG = NBIN * 8;                // stage A regions
struct BinOut {
  unsigned long long* key;                    // h per record: region r at [r * cap, (r+1) * cap)
  uint32_t* mw;                               // 26-bit mask word per record
  unsigned long long* cursor;                 // per region, CSTRIDE apart
  uint64_t cap;                               // records per region (more: F_A_OVER, dropped)
  uint32_t shift;                             // coarse bin = h >> shift
  unsigned* flags;                            // [0] sentinel, [1] stage A bits
};

// Block emission.  The records of a round (NR per thread, some empty) are
// ranked per (sub-round of ESUB records per thread, bin) by LDS atomics; one
// returning atomic per bin reserves the round's run in the bin's region for
// this XCD; then, sub-round by sub-round, the records are placed in an LDS
// stage in bin order and written out by consecutive threads, so a store
// instruction covers a few contiguous runs instead of one record in each of
// up to 64 bins (the scattered form spent the work pass issuing stores: SQ
// WAIT_INST_ANY 10.7 K quad-cycles per wave, ~100 us per C3 chunk).
// Every thread of the block calls this (2 + 2 * NR / ESUB barriers, the last
// one after the stage's reads); L.cnt must be zero on entry and is left zero.
constexpr int ESUB = 4;                       // records per thread and sub-round
constexpr int EST = IBLOCK * ESUB;            // staged records per sub-round: 12 KB
template <int NS>
struct EmitLds {
  uint32_t cnt[NS][NBIN];                     // per sub-round and bin: records
  uint32_t off[NS][NBIN + 1];                 // their exclusive scan over bins (stage offsets), total last
  unsigned long long base[NS][NBIN];          // region position of the bin's first record of the sub-round
  __device__ __forceinline__ void zero() {    // (threads 0 .. NBIN-1; a barrier before use)
    if (threadIdx.x < NBIN)
      for (int q = 0; q < NS; ++q) cnt[q][threadIdx.x] = 0u;
  }
};
template <int NR, int SUB = ESUB>
__device__ __forceinline__ void block_emit(const BinOut& O, const uint64_t (&h)[NR], const uint32_t (&m)[NR],
                                           EmitLds<NR / SUB>& L, unsigned long long* st_key, uint32_t* st_mw) {
  constexpr int NS = NR / SUB;
  static_assert(NR % SUB == 0 && NBIN == 64, "whole sub-rounds; one wave scans the bins");
  const int t = (int)threadIdx.x;
  uint32_t rk[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) rk[j] = m[j] ? atomicAdd(&L.cnt[j / SUB][(uint32_t)(h[j] >> O.shift)], 1u) : 0u;
  __syncthreads();
  const uint32_t x = blockIdx.x & 7;
  if (t < NBIN) {
    uint32_t n[NS], tot = 0;
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      n[q] = L.cnt[q][t];
      L.cnt[q][t] = 0u;
      tot += n[q];
    }
    unsigned long long b = tot ? atomicAdd(O.cursor + CSTRIDE * (t * 8 + x), (unsigned long long)tot) : 0ull;
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      L.base[q][t] = b;
      b += n[q];
      uint32_t v = n[q];
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(v, o, 64);
        if (t >= o) v += y;
      }
      L.off[q][t] = v - n[q];
      if (t == NBIN - 1) L.off[q][NBIN] = v;
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NS; ++q) {
#pragma unroll
    for (int j = q * SUB; j < (q + 1) * SUB; ++j)
      if (m[j]) {
        const uint32_t at = L.off[q][(uint32_t)(h[j] >> O.shift)] + rk[j];
        st_key[at] = h[j];
        st_mw[at] = m[j];
      }
    __syncthreads();
    const uint32_t tot = L.off[q][NBIN];
    for (uint32_t e = (uint32_t)t; e < tot; e += IBLOCK) {
      const unsigned long long hv = st_key[e];
      const uint32_t p = (uint32_t)(hv >> O.shift);
      const unsigned long long pos = L.base[q][p] + (e - L.off[q][p]);
      if (PG_EXP_BITS & (1 << 17)) {
        if (hv == 42ull) O.flags[3] = (unsigned)pos;   // (experiment: no record stores)
      } else if (pos < O.cap) {
        const uint64_t at = (uint64_t)(p * 8 + x) * O.cap + pos;
        O.key[at] = hv;
        O.mw[at] = st_mw[e];
      } else {
        (void)PG_BOK(false, 51, (long long)pos, (long long)O.cap);
        atomicOr(O.flags + 1, F_A_OVER);
      }
    }
    __syncthreads();
  }
}

// (A wave-level multi-split - the lanes of a bin found by 6 ballots, ranks
// by popcount, per-wave counters scanned across the block - in place of the
// LDS rank atomics measured slower: C3 stage A 0.477 ms at 4 waves per SIMD,
// 0.498 capped to 5 with spills, against 0.438 for the atomics.)

// K3 work pass: one queued segment per thread, every lane busy; the records
// of a round of IBLOCK segments leave through block_emit.  The NQ sub-queues
// are read as one concatenated list (their counts scanned in LDS); the
// segment's 64 context bytes (from position q0-2, 16-byte aligned) are
// staged in the thread's own LDS slot.  NP = 2: the segment's windows are
// computed and emitted in two halves (half the records in registers, so
// ~2x the waves per CU; the emission stage is then an LDS array of its own,
// the rows being still in use); NP = 1: all 16 at once, the stage reusing
// the rows.
#ifndef PG_WSUB
#define PG_WSUB 4
#endif
// the work pass's emission sub-round (records per thread): 8 (one 24 KiB
// stage per half segment, 3 blocks per CU) measured slower than 4 (stage A
// 0.432 vs 0.413 ms)
constexpr int WSUB = PG_WSUB;
constexpr bool PK_ON = !(PG_EXP_BITS & (1 << 20));   // (experiment build: the byte form for every segment)
template <bool RC, int NP>
__global__ void __launch_bounds__(IBLOCK)
k_emit_work(PackedCls pc, const WorkItem* __restrict__ queue,
            const unsigned long long* __restrict__ qcount, unsigned long long qcap, int k, uint64_t shift,
            TableView T, BinOut O) {
  static_assert(NQ == 64, "one wave scans the sub-queue counts");
  static_assert(NP == 1 || NP == 2, "one or two parts");
  if (PG_EXP_BITS & (1 << 19)) return;             // (experiment: no work pass)
  constexpr int NX = IW / NP;
  // 64 staged bytes + 4 per thread: rows of 17 dwords, an odd stride, so the
  // rows' dword reads are bank-conflict free (80-byte rows were 4-way
  // conflicted: 1847 conflict cycles per wave, PMC); the realigning dword
  // reads past a row land in the next one, or read 0 past the allocation.
  constexpr int SROW = 68;
  static_assert(SROW % 8 == 4 && SROW >= 64, "odd dword stride, 64 staged bytes");
  __shared__ __attribute__((aligned(16))) uint8_t scratch[IBLOCK][SROW];
  __shared__ __attribute__((aligned(16))) uint8_t stage2[NP == 2 ? 12 * IBLOCK * WSUB : 16];
  __shared__ unsigned long long s_pre[NQ + 1];
  __shared__ EmitLds<NX / WSUB> s_emit;
  __shared__ uint32_t s_k5[256];
  static_assert(NP == 2 || sizeof(scratch) >= 12 * IBLOCK * WSUB, "the emission stage reuses the segment rows");
  static_assert(IBLOCK == 256, "one K5 entry per thread");
  uint8_t* const st = NP == 2 ? &stage2[0] : &scratch[0][0];
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
  s_emit.zero();
  s_k5[threadIdx.x] = k5_entry(threadIdx.x);
  __syncthreads();
  uint8_t* slot = scratch[threadIdx.x];
  const unsigned long long n = s_pre[NQ];
  if (blockIdx.x == 0 && threadIdx.x == 0 && n)                 // the build's work items (pg_stats)
    atomicAdd(reinterpret_cast<unsigned long long*>(O.flags + F_WORK_ITEMS), n);
  for (unsigned long long i0 = (unsigned long long)blockIdx.x * IBLOCK; i0 < n;
       i0 += (unsigned long long)gridDim.x * IBLOCK) {          // block-uniform trip count
    const unsigned long long i = i0 + threadIdx.x;
    uint64_t hh[NX], K = 0, Kr = 0;
    uint32_t mm[NX];
    WorkItem w{0, -1, 0, 0u, 0u};
    long long aligned = 0;
    bool pk = false;                               // the packed form (segment_records_pk)
    uint32_t cw[4] = {0u, 0u, 0u, 0u};
    if (i < n) {
      int lo = 0;                                  // largest j with s_pre[j] <= i
#pragma unroll
      for (int step = NQ / 2; step > 0; step >>= 1)
        if (s_pre[lo + step] <= i) lo += step;
      w = queue[(unsigned long long)lo * qcap + (i - s_pre[lo])];
      if (!PG_BOK(i - s_pre[lo] < qcap && w.rs >= 0 && w.q0 >= 0 && w.q0 <= w.last + 1, 21, w.rs, w.q0))
        w = WorkItem{0, -1, 0, 0u, 0u};
      const long long from = w.rs + w.q0 - 2;
      aligned = from > 0 ? from & ~15ll : 0;
      uint32_t* s32 = reinterpret_cast<uint32_t*>(slot);          // (4-byte aligned rows)
      // the 4 chunks' packed words, unpacked; a chunk with an exception
      // (not all ACGT) from its class bytes
      const uint64_t c0 = (uint64_t)aligned >> 4;
      uint32_t pw[4], ex[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) { pw[j] = pc.p2[c0 + j]; ex[j] = pc.e16[c0 + j]; }
      pk = PK_ON && k == 27 && !(ex[0] | ex[1] | ex[2] | ex[3]) && w.q0 > 0 && w.q0 + IW <= w.last;
      if (pk) {
        // code 0 = position q0 - 1: the 128 bits shifted right by 2 (from + 1 - aligned) in [0, 32]
        const uint32_t sh = 2u * (uint32_t)(from + 1 - aligned);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t nx = j < 3 ? pw[j + 1] : 0u;
          cw[j] = sh >= 32u ? nx : sh ? __builtin_amdgcn_alignbit(nx, pw[j], sh) : pw[j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uint4 v;
          if (ex[j]) v = *reinterpret_cast<const uint4*>(pc.cls + aligned + 16 * j);
          else v = make_uint4(unpack4(pw[j], 0), unpack4(pw[j], 1), unpack4(pw[j], 2), unpack4(pw[j], 3));
          s32[4 * j] = v.x; s32[4 * j + 1] = v.y; s32[4 * j + 2] = v.z; s32[4 * j + 3] = v.w;
        }
      }
    }
    auto part = [&](auto P) {
      constexpr int X0 = decltype(P)::value * NX;
      if (i < n && pk) {
        segment_records_pk<RC, X0, NX>(cw, s_k5, shift, T, w.covered, K, Kr, hh, mm);
      } else if (i < n) {
        segment_records<RC, X0, NX>(slot, w.rs - aligned, w.q0, w.last, k, shift, T, w.covered, K, Kr, hh, mm);
      } else {
#pragma unroll
        for (int x = 0; x < NX; ++x) { hh[x] = 0; mm[x] = 0; }
      }
      if (PG_EXP_BITS & (1 << 18)) {                  // (experiment: no emission)
        uint64_t acc = 0;
#pragma unroll
        for (int x = 0; x < NX; ++x) acc ^= hh[x] + mm[x];
        if (acc == 42ull) O.flags[3] = 1u;
      } else {
        block_emit<NX, WSUB>(O, hh, mm, s_emit, reinterpret_cast<unsigned long long*>(st),
                             reinterpret_cast<uint32_t*>(st + 8 * IBLOCK * WSUB));
      }
    };
    part(std::integral_constant<int, 0>{});
    if constexpr (NP == 2) part(std::integral_constant<int, 1>{});
  }
}

// one oriented key x with its 12-bit mask as the canonical record add_kmer's
// OR would update (:1036-1047)
__device__ __forceinline__ void canon_record(const TableView& T, uint64_t x, uint32_t m12, uint64_t& h, uint32_t& m) {
  const uint64_t xr = T.rc(x);
  const uint32_t mw = m12 | PRES_A;
  if (x <= xr) { h = T.perm(x); m = mw; }
  else { h = T.perm(xr); m = mw << B_SHIFT; }
}

// Records with n <= k+1 (build_dbg's short paths, :1061-1088): the windows of
// both strands as canonical records; n < k sets the n<k sentinel (:1087-1088).
__global__ void __launch_bounds__(IBLOCK)
k_short_emit(PackedCls cls, const long long* __restrict__ rec_start,
             const long long* __restrict__ rec_len, const uint8_t* __restrict__ rec_flag, uint64_t R, int k,
             uint64_t shift, int rc, TableView T, BinOut O) {
  __shared__ EmitLds<1> s_emit;
  __shared__ unsigned long long st_key[EST];
  __shared__ uint32_t st_mw[EST];
  s_emit.zero();
  __syncthreads();
  for (uint64_t r0 = blockIdx.x * (uint64_t)IBLOCK; r0 < R; r0 += (uint64_t)gridDim.x * IBLOCK) {
    const uint64_t r = r0 + threadIdx.x;
    uint64_t hh[4] = {0, 0, 0, 0};
    uint32_t mm[4] = {0, 0, 0, 0};
    if (r < R && rec_flag[r]) {
      const long long n = rec_len[r];
      if (n < k) {
        atomicOr(O.flags, 1u);                                 // key -1, mask '$'
      } else if (n <= k + 1) {
        int j = 0;
        auto emit = [&](uint64_t x, uint32_t m12) {
          uint64_t h;
          uint32_t m;
          canon_record(T, x, m12, h, m);
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (t == j) { hh[t] = h; mm[t] = m; }
          ++j;
        };
        short_strand(cls, rec_start[r], n, 0, k, shift, emit);
        if (rc) short_strand(cls, rec_start[r], n, 1, k, shift, emit);
      }
    }
    block_emit<4>(O, hh, mm, s_emit, st_key, st_mw);
  }
}

// Extra empty records that the reference's checkpoint/resume yields (see
// pangenome_amd/host.py): each adds the n<k sentinel.
__global__ void k_set_flag(unsigned* flags) { atomicOr(flags, 1u); }

// Staged slots of a loaded npz (pg_dbg_load): each oriented (key, mask) as
// add_kmer would OR it (the sentinel sets the flag).
__global__ void __launch_bounds__(IBLOCK)
k_preload_emit(const PreEnt* __restrict__ e, uint64_t n, TableView T, BinOut O) {
  __shared__ EmitLds<1> s_emit;
  __shared__ unsigned long long st_key[EST];
  __shared__ uint32_t st_mw[EST];
  s_emit.zero();
  __syncthreads();
  for (uint64_t b = blockIdx.x * (uint64_t)(4 * IBLOCK); b < n; b += (uint64_t)gridDim.x * 4 * IBLOCK) {
    uint64_t hh[4];
    uint32_t mm[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint64_t i = b + (uint64_t)t * IBLOCK + threadIdx.x;
      hh[t] = 0;
      mm[t] = 0;
      if (i < n) {
        const uint64_t x = e[i].key;
        if (x == SENTINEL) atomicOr(O.flags, 1u);
        else canon_record(T, x, e[i].mask & MASK12, hh[t], mm[t]);
      }
    }
    block_emit<4>(O, hh, mm, s_emit, st_key, st_mw);
  }
}

// Exchange records a multi-GPU owner received (pg_dbg_merge): canonical key
// + 1 and the 26-bit mask word of both orientations.  The sum of the
// records' row_check and the count of non-empty records go to `chk`
// (pg_dbg_merge_check: what the merge read, against what the senders'
// partition sums say was sent).
// (the sums: one per block, spread over MCHK slot pairs of `chk` so that no
// address takes more than a few hundred atomics - thousands on one line
// serialise at the memory side: 0.65 ms on C3's world-1 merge)
constexpr int MCHK = 64;
__global__ void __launch_bounds__(IBLOCK)
k_slots_emit(const Slot* __restrict__ e, uint64_t n, TableView T, BinOut O, unsigned long long* __restrict__ chk) {
  __shared__ EmitLds<1> s_emit;
  __shared__ unsigned long long st_key[EST];
  __shared__ uint32_t st_mw[EST];
  __shared__ unsigned long long s_chk[2][IBLOCK / 64];
  s_emit.zero();
  __syncthreads();
  unsigned long long acc = 0ull, live = 0ull;
  for (uint64_t b = blockIdx.x * (uint64_t)(4 * IBLOCK); b < n; b += (uint64_t)gridDim.x * 4 * IBLOCK) {
    uint64_t hh[4];
    uint32_t mm[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint64_t i = b + (uint64_t)t * IBLOCK + threadIdx.x;
      hh[t] = 0;
      mm[t] = 0;
      if (i < n) {
        const Slot s = e[i];
        acc += row_check(s.key1, (uint64_t)s.mask | ((uint64_t)s.aux << 32));
        if (s.key1) { hh[t] = T.perm(s.key1 - 1ull); mm[t] = s.mask & (uint32_t)MW_MASK; ++live; }
      }
    }
    block_emit<4>(O, hh, mm, s_emit, st_key, st_mw);
  }
  for (int o = 32; o > 0; o >>= 1) {
    acc += __shfl_down(acc, o, 64);
    live += __shfl_down(live, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    s_chk[0][threadIdx.x >> 6] = acc;
    s_chk[1][threadIdx.x >> 6] = live;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long a = 0ull, l = 0ull;
    for (int w = 0; w < IBLOCK / 64; ++w) { a += s_chk[0][w]; l += s_chk[1][w]; }
    if (a || l) {
      unsigned long long* slot = chk + 2 * (blockIdx.x % MCHK);
      atomicAdd(slot, a);
      atomicAdd(slot + 1, l);
    }
  }
}

// Routed stage A records (12-byte rows, pg_route_merge) into this owner's
// regions: h rotated into the owner domain (T.rot), with the same checksum
// slots as k_slots_emit.
__global__ void __launch_bounds__(IBLOCK)
k_route_emit(const Row12* __restrict__ e, uint64_t n, TableView T, BinOut O, unsigned long long* __restrict__ chk) {
  __shared__ EmitLds<1> s_emit;
  __shared__ unsigned long long st_key[EST];
  __shared__ uint32_t st_mw[EST];
  __shared__ unsigned long long s_chk[2][IBLOCK / 64];
  s_emit.zero();
  __syncthreads();
  unsigned long long acc = 0ull, live = 0ull;
  for (uint64_t b = blockIdx.x * (uint64_t)(4 * IBLOCK); b < n; b += (uint64_t)gridDim.x * 4 * IBLOCK) {
    uint64_t hh[4];
    uint32_t mm[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint64_t i = b + (uint64_t)t * IBLOCK + threadIdx.x;
      hh[t] = 0;
      mm[t] = 0;
      if (i < n) {
        const Row12 r = e[i];
        const uint64_t h = (uint64_t)r.w[0] | ((uint64_t)r.w[1] << 32);
        acc += row_check(h, (uint64_t)r.w[2]);
        if (r.w[2]) { hh[t] = T.rot ? T.rotk(h, T.rot) : h; mm[t] = r.w[2] & (uint32_t)MW_MASK; ++live; }
      }
    }
    block_emit<4>(O, hh, mm, s_emit, st_key, st_mw);
  }
  for (int o = 32; o > 0; o >>= 1) {
    acc += __shfl_down(acc, o, 64);
    live += __shfl_down(live, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    s_chk[0][threadIdx.x >> 6] = acc;
    s_chk[1][threadIdx.x >> 6] = live;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long a = 0ull, l = 0ull;
    for (int w = 0; w < IBLOCK / 64; ++w) { a += s_chk[0][w]; l += s_chk[1][w]; }
    if (a || l) {
      unsigned long long* slot = chk + 2 * (blockIdx.x % MCHK);
      atomicAdd(slot, a);
      atomicAdd(slot + 1, l);
    }
  }
}

// ---------------------------------------------------------------- stage B
// Record regions: partition p = sub-regions p * nsub .. p * nsub + nsub - 1
// (stage A: nsub = 8, one per XCD; after a split: nsub = 1).
struct Recs {
  unsigned long long* key;
  uint32_t* mw;
  unsigned long long* cursor;                 // per sub-region, CSTRIDE apart
  uint64_t cap;                               // records per sub-region
  uint32_t nsub;
};

// s_off[0 .. nsub]: prefix of partition p's sub-region counts (clipped at cap:
// a region that overflowed has set its flag)
__device__ __forceinline__ void part_offsets(const Recs& I, uint32_t p, unsigned long long* s_off) {
  if (threadIdx.x == 0) {
    unsigned long long o = 0;
    s_off[0] = 0;
    for (uint32_t s = 0; s < I.nsub; ++s) {
      const unsigned long long n = I.cursor[CSTRIDE * ((uint64_t)p * I.nsub + s)];
      o += n < I.cap ? n : I.cap;
      s_off[s + 1] = o;
    }
  }
}
// array index of record r of partition p
__device__ __forceinline__ uint64_t part_at(const Recs& I, uint32_t p, const unsigned long long* s_off, uint64_t r) {
  uint32_t s = 0;
  while (s + 1 < I.nsub && r >= s_off[s + 1]) ++s;
  return ((uint64_t)p * I.nsub + s) * I.cap + (r - s_off[s]);
}

// Split pass: the records of input region g (partition p = g / nsub) by the
// next S bits of the bucket index ((h >> shift) & (nb - 1)) into output
// partitions p * nb + b.  A block takes SCH consecutive records of one region
// (bpr blocks per region), ranks them per bin in LDS, reserves each bin's run
// with one global atomic, sorts them by bin in LDS and writes the runs
// coalesced.  2 blocks (16 waves) per CU: 6144 records per round (72 KiB of
// LDS) write longer runs per bin than 4096 at 3 blocks per CU (C3 split 0.151-
// 0.153 vs 0.161-0.162 ms; 2048 or 8192 per round: 0.173-0.196 ms), and at
// 4 waves per SIMD (the occupancy the LDS allows) the 12 records per thread
// stay in registers: 0.138-0.139 ms (profiles/r05_ab_split_geometry.log).
// NT: the records are read with non-temporal loads (SPLIT_NT_MAX below;
// non-temporal stores measured slower: C3 0.210 ms, both 0.190).
#ifndef PG_SPLIT_SR
#define PG_SPLIT_SR 12
#endif
#ifndef PG_SPLIT_SB
#define PG_SPLIT_SB 512
#endif
constexpr int SB = PG_SPLIT_SB, SR = PG_SPLIT_SR, SCH = SB * SR;
constexpr int SPLIT_BITS = 7;                 // bits per split pass
constexpr int SMAXB = 1 << SPLIT_BITS;
// start (NULL: 0): per input region, the records below it are already split
// (pg_build_host's early split); a block loops over its region's records in
// steps of bpr * SCH.
// Non-temporal record loads measured faster for C3 (24 M records, one pass:
// 0.148 -> 0.127 ms) and slower for the C5 shard's sub-logs (0.94 G records,
// two passes: 38.8 -> 42.4 ms per pass; profiles/r06_ab_range_split.log), so
// a build's split and range passes use them below SPLIT_NT_MAX records.
constexpr uint64_t SPLIT_NT_MAX = 1ull << 28;
template <bool NT>
__global__ void __launch_bounds__(SB, 4)
k_split(Recs I, Recs O, const unsigned long long* __restrict__ start, uint32_t shift, uint32_t nb, uint32_t bpr,
        unsigned* __restrict__ flags) {
  __shared__ uint32_t s_cnt[SMAXB], s_pos[SMAXB];
  __shared__ unsigned long long s_base[SMAXB];
  __shared__ unsigned long long s_key[SCH];
  __shared__ uint32_t s_mw[SCH];
  const uint32_t g = blockIdx.x / bpr, j = blockIdx.x % bpr, p = g / I.nsub;
  const unsigned long long nr = I.cursor[CSTRIDE * (uint64_t)g];
  const uint64_t n = nr < I.cap ? nr : I.cap;
  uint64_t s0 = start ? start[g] : 0ull;
  s0 = s0 < n ? s0 : n;
  for (uint64_t b0 = s0 + (uint64_t)j * SCH; b0 < n; b0 += (uint64_t)bpr * SCH) {   // block-uniform
    __syncthreads();                                           // (the last round's LDS reads are done)
    if (threadIdx.x < SMAXB) s_cnt[threadIdx.x] = 0u;
    const uint32_t cnt = (uint32_t)(n - b0 < (uint64_t)SCH ? n - b0 : (uint64_t)SCH);
    const uint64_t in0 = (uint64_t)g * I.cap + b0;
    unsigned long long key[SR];
    uint32_t mw[SR], rk[SR];
#pragma unroll
    for (int e = 0; e < SR; ++e) {
      const uint32_t i = (uint32_t)e * SB + threadIdx.x;
      if (NT) {
        key[e] = i < cnt ? __builtin_nontemporal_load(I.key + in0 + i) : 0ull;
        mw[e] = i < cnt ? __builtin_nontemporal_load(I.mw + in0 + i) : 0u;
      } else {
        key[e] = i < cnt ? I.key[in0 + i] : 0ull;
        mw[e] = i < cnt ? I.mw[in0 + i] : 0u;
      }
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < SR; ++e) {
      const uint32_t i = (uint32_t)e * SB + threadIdx.x;
      rk[e] = i < cnt ? atomicAdd(&s_cnt[(uint32_t)(key[e] >> shift) & (nb - 1)], 1u) : 0u;
    }
    __syncthreads();
    if (threadIdx.x < 64) {                   // exclusive scan of the bin counts, SMAXB / 64 bins per lane
      constexpr int BPL = SMAXB / 64;
      const uint32_t l = threadIdx.x;
      uint32_t v[BPL], x = 0;
#pragma unroll
      for (int q = 0; q < BPL; ++q) {
        v[q] = BPL * l + q < nb ? s_cnt[BPL * l + q] : 0u;
        x += v[q];
      }
      const uint32_t own = x;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if ((int)l >= o) x += y;
      }
      uint32_t ex = x - own;
#pragma unroll
      for (int q = 0; q < BPL; ++q) {
        if (BPL * l + q < nb) s_pos[BPL * l + q] = ex;
        ex += v[q];
      }
    }
    if (threadIdx.x < nb) {
      const uint32_t c = s_cnt[threadIdx.x];
      s_base[threadIdx.x] = c ? atomicAdd(O.cursor + CSTRIDE * ((uint64_t)p * nb + threadIdx.x), (unsigned long long)c)
                              : 0ull;
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < SR; ++e) {
      const uint32_t i = (uint32_t)e * SB + threadIdx.x;
      if (i < cnt) {
        const uint32_t b = (uint32_t)(key[e] >> shift) & (nb - 1);
        const uint32_t d = s_pos[b] + rk[e];
        s_key[d] = key[e];
        s_mw[d] = mw[e];
      }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < cnt; i += SB) {
      const unsigned long long kk = s_key[i];
      const uint32_t b = (uint32_t)(kk >> shift) & (nb - 1);
      const unsigned long long pos = s_base[b] + (i - s_pos[b]);
      if (pos < O.cap) {
        const uint64_t at = ((uint64_t)p * nb + b) * O.cap + pos;
        O.key[at] = kk;
        O.mw[at] = s_mw[i];
      } else {
        atomicOr(flags + 4, F_SPLIT_OVER);
      }
    }
  }
}
// the stage A cursors as the early split's next start
__global__ void k_snap(const unsigned long long* __restrict__ cursor, unsigned long long* __restrict__ snap, uint32_t n) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < n) snap[g] = cursor[CSTRIDE * (uint64_t)g];
}

// ---------------------------------------------------------------- stage C
// Fine partition f = buckets [f << rbits, (f + 1) << rbits).  Its records are
// OR-merged into an LDS copy of the range (one 64-bit LDS CAS creates a key
// with its masks, as the HBM table's layout has it: a bucket's second word
// fills after its first; a key whose bucket is full goes to an LDS overflow
// set and, once final, to the HBM overflow table).  One pass over the range
// then writes it out whole with 16-byte stores (every bucket of the table is
// written by exactly one block: no clear), applies the rdBG rule
// (build_rdbg_jit_ :1300-1305) to every key, whose masks are final there, and
// zeroes the LDS copy for the block's next partition.
// Persistent: block b takes partitions b, b + G, ...; the records of the next
// partition are loaded into registers before the current one is merged, so
// their latency hides behind the merge and the pass.  Each block appends its
// rdBG members to its own output segment (no global atomics at all) and
// leaves its key / dBG / member counts in its own counter slot.
constexpr int RB_T = 512;                     // 2 blocks (16 waves) per CU: 70 KiB of LDS each
constexpr int RB_R = 8;                       // records per thread and partition held in registers
// <= 4096 buckets (64 KiB of LDS) per partition (2048-bucket partitions at 3
// blocks per CU behind 8-bit split passes: range 0.42 vs 0.31 ms on C3)
constexpr int RANGE_BITS = 12;
constexpr int RB_PER_CU = 2;                  // persistent range blocks per CU
constexpr int OVL = 512;                      // LDS overflow slots per partition
constexpr int RB_CTR = 4;                     // per-block counters: keys, dBG entries, members
constexpr uint32_t MQ = 64;                   // queued rdBG members per wave
struct RdbgOut {
  unsigned long long* keys;                   // block b's members at [b * cap, (b+1) * cap)
  unsigned long long* ctr;                    // per block: RB_CTR words
  uint64_t cap;
};

__device__ __forceinline__ uint32_t member_bits(uint32_t m) {   // bit0: A member, bit1: B member
  const uint32_t pa = (m >> 12) & 1u, pb = (m >> 25) & 1u;
  return (uint32_t)(pa && rdbg_member(m & MASK12)) | ((uint32_t)(pb && rdbg_member((m >> B_SHIFT) & MASK12)) << 1);
}

// a key whose bucket is full: the LDS overflow set (rare: out of line)
__device__ __forceinline__ void range_or_ovl(unsigned long long* OK, uint32_t* OM, const TableView& T, uint64_t h,
                                          uint32_t m, unsigned* flags) {
  // (h is a permuted key: its low bits, below the bucket bits, are as good a
  // start as a hash of it - C3 range 0.313 vs 0.318 ms with fmix64)
  uint32_t s = (uint32_t)(h >> 7) & (OVL - 1);
  for (int pr = 0; pr < OVL; ++pr) {
    const unsigned long long o2 = atomicCAS(&OK[s], 0ull, h + 1ull);
    if (o2 == 0ull || o2 == h + 1ull) {
      atomicOr(&OM[s], m);
      return;
    }
    s = (s + 1) & (OVL - 1);
  }
  // LDS overflow set full: straight to HBM, membership incomplete (the host re-runs with more buckets)
  ovf_or(T, T.unperm(h), m, flags + 4);
  atomicOr(flags + 4, F_LDS_SPILL);
}

// OR one record (h, m) into the LDS range W (bucket lb) or the LDS overflow set
__device__ __forceinline__ void range_or(unsigned long long* W, unsigned long long* OK, uint32_t* OM,
                                         const TableView& T, uint64_t h, uint32_t m, uint32_t lb, uint64_t qmask,
                                         unsigned* flags) {
  const unsigned long long q = h & qmask, mine = (q << MW_BITS) | m;
  unsigned long long* w = W + 2 * lb;
  unsigned long long old = atomicCAS(w, 0ull, mine);
  if (old == 0ull) return;
  if ((old >> MW_BITS) == q) {
    if ((old & m) != m) atomicOr(w, (unsigned long long)m);
    return;
  }
  old = atomicCAS(w + 1, 0ull, mine);
  if (old == 0ull) return;
  if ((old >> MW_BITS) == q) {
    if ((old & m) != m) atomicOr(w + 1, (unsigned long long)m);
    return;
  }
  range_or_ovl(OK, OM, T, h, m, flags);
}

// records of partition f (one region of the last split level)
__device__ __forceinline__ uint64_t part_count(const Recs& I, uint32_t f, uint32_t z) {
  // z is a zero the compiler cannot see through: a vector load, counted by
  // vmcnt, so that waiting on the LDS atomics does not wait on it
  const unsigned long long n = I.cursor[CSTRIDE * (uint64_t)f + z];
  return n < I.cap ? n : I.cap;
}
// s_waitcnt vmcnt(0), leaving the LDS / scalar counter alone (gfx9 encoding:
// vmcnt 0, expcnt 7, lgkmcnt 15)
__device__ __forceinline__ void wait_vm() { __builtin_amdgcn_s_waitcnt(0x0F70); }

template <bool NT>
__global__ void __launch_bounds__(RB_T, 4)
k_build_range(Recs I, TableView T, uint32_t rbits, uint32_t nparts, RdbgOut R, unsigned* __restrict__ flags) {
  __shared__ unsigned long long W[2 << RANGE_BITS];
  __shared__ unsigned long long OK[OVL];      // h + 1, 0 = empty
  __shared__ uint32_t OM[OVL];
  __shared__ unsigned long long s_mcur;       // this block's members so far
  __shared__ unsigned long long s_mq[RB_T / 64][MQ];   // per-wave member queue
  __shared__ unsigned long long s_red[2][RB_T / 64];
  const uint32_t rng = 1u << rbits, G = gridDim.x;
  const uint64_t qmask = (1ull << T.qbits) - 1ull;
  uint32_t z = 0;
  asm volatile("" : "+v"(z));
  for (uint32_t i = threadIdx.x; i < 2 * rng; i += RB_T) W[i] = 0ull;
  for (uint32_t i = threadIdx.x; i < OVL; i += RB_T) { OK[i] = 0ull; OM[i] = 0u; }
  if (threadIdx.x == 0) s_mcur = 0ull;
  uint32_t f = blockIdx.x;
  unsigned long long ch[RB_R], nh[RB_R];
  uint32_t cm[RB_R], nm[RB_R];
  // (uniform base pointers per e, a 32-bit lane offset: one VGPR of address)
  auto load = [&](uint32_t p, uint64_t n, unsigned long long (&h)[RB_R], uint32_t (&m)[RB_R]) {
    const uint64_t pb = (uint64_t)(p < nparts ? p : 0) * I.cap;
    const uint32_t nn = (uint32_t)(p < nparts ? (n < (uint64_t)RB_T * RB_R ? n : (uint64_t)RB_T * RB_R) : 0);
#pragma unroll
    for (int e = 0; e < RB_R; ++e) {
      const unsigned long long* kp = I.key + pb + e * RB_T;
      const uint32_t* mp = I.mw + pb + e * RB_T;
      const bool ok = (uint32_t)(e * RB_T) + threadIdx.x < nn;
      // (non-temporal below SPLIT_NT_MAX records, as the split: C3 range 0.300
      // vs 0.319 ms with plain loads, C5's sub-logs 42-44 vs 40 ms per shard)
      if (NT) {
        h[e] = ok ? __builtin_nontemporal_load(kp + threadIdx.x) : 0ull;
        m[e] = ok ? __builtin_nontemporal_load(mp + threadIdx.x) : 0u;
      } else {
        h[e] = ok ? kp[threadIdx.x] : 0ull;
        m[e] = ok ? mp[threadIdx.x] : 0u;
      }
    }
  };
  uint64_t n_cur = f < nparts ? part_count(I, f, z) : 0;
  uint64_t n_nxt = f + G < nparts ? part_count(I, f + G, z) : 0;
  load(f, n_cur, ch, cm);
  // Vector memory counts (vmcnt) are in order and count stores too: a wait for
  // a load issued before stores of unknown number is a wait for those stores.
  // So the loads are waited for explicitly at points where nothing else is in
  // flight - here, and in the loop before the range goes out - and never where
  // the compiler would put the wait itself: at the loop head, where the first
  // partition's loads from here meet the back edge (which made every
  // iteration wait for its own prefetch right after issuing it), and at the
  // end, behind the range's stores.
  wait_vm();
  uint32_t created = 0, ndbg = 0;
  const uint64_t mseg = (uint64_t)blockIdx.x * R.cap;
  // rdBG members: each wave queues h (| 1 << 63 for the rc orientation) in its
  // own LDS buffer and turns a full buffer into keys with all 64 lanes busy
  // (unperm + rc cost ~250 VALU per wave: run per bucket, nearly every wave
  // paid them for a handful of member lanes)
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t mp = 0;                                             // queued in this wave's buffer (wave-uniform)
  auto flush = [&]() {
    if (!mp) return;
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(&s_mcur, (unsigned long long)mp);
    base = __shfl(base, 0, 64);
    if (lane < mp) {
      const unsigned long long e = s_mq[wv][lane];
      const uint64_t c = T.unperm(e & ~(1ull << 63));
      const uint64_t o = base + lane;
      if (o < R.cap) R.keys[mseg + o] = (e >> 63) ? T.rc(c) : c;
      else { (void)PG_BOK(false, 53, (long long)o, (long long)R.cap); atomicOr(flags + 4, F_RSEG_OVER); }
    }
    mp = 0;
  };
  auto push1 = [&](unsigned long long e, bool on) {
    const unsigned long long bal = __ballot(on);
    const uint32_t n = (uint32_t)__builtin_popcountll(bal);
    if (!n) return;
    if (mp + n > MQ) flush();
    // (the lanes below this one with the bit set: v_mbcnt, not a masked popcount)
    if (on) s_mq[wv][mp + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))] = e;
    mp += n;
  };
  auto push = [&](uint64_t h, uint32_t mb) {                   // every lane of the wave calls it
    push1(h, mb & 1u);
    push1(h | (1ull << 63), mb & 2u);
  };
  __syncthreads();
  for (; f < nparts; f += G) {                                 // block-uniform
    if (!(PG_EXP_BITS & 4)) load(f + G, n_nxt, nh, nm);       // in flight during this partition
    unsigned long long n_nn = f + 2 * G < nparts ? I.cursor[CSTRIDE * (uint64_t)(f + 2 * G) + z] : 0ull;  // (raw)
#pragma unroll
    for (int e = 0; e < RB_R; ++e)
      if (cm[e] && !(PG_EXP_BITS & 2))
        range_or(W, OK, OM, T, ch[e], cm[e], (uint32_t)(ch[e] >> T.qbits) & (rng - 1), qmask, flags);
    // (Measured and dropped, profiles/r06_ab_range_split.log: batches of
    // records with every first-word CAS of a batch in flight at once, then the
    // second-word CASes - 0.331 ms with 4 per batch (a spill), 0.318 with 2,
    // 0.409 with 8 (spills), against 0.317 record by record; and rounds in
    // which each lane takes its next record still to do, selected out of its
    // registers, so that a path runs as often as the busiest lane needs it
    // rather than once per record - 0.364-0.372 (spills: the kernel is at its
    // 128-VGPR budget).)
    for (uint64_t r = (uint64_t)RB_T * RB_R + threadIdx.x; r < n_cur; r += RB_T) {   // rare: a large partition
      const unsigned long long h = I.key[(uint64_t)f * I.cap + r];
      range_or(W, OK, OM, T, h, I.mw[(uint64_t)f * I.cap + r], (uint32_t)(h >> T.qbits) & (rng - 1), qmask, flags);
    }
    __syncthreads();
    wait_vm();                                                   // the prefetch landed under the merge
    asm volatile("" : "+v"(n_nn));
    n_nn = n_nn < I.cap ? n_nn : I.cap;
    // the LDS overflow set first (its HBM probes wait on vmcnt: before the
    // range's stores, not behind them), then the range out whole; counts;
    // members queued; LDS zeroed
    static_assert(OVL % 64 == 0, "whole waves");
    for (uint32_t i = threadIdx.x; i < OVL; i += RB_T) {
      const unsigned long long kk = OK[i];
      const uint32_t m = OM[i];
      if (kk) {
        ovf_or(T, T.unperm(kk - 1ull), m, flags + 4);
        ++created;
        ndbg += ((m >> 12) & 1u) + ((m >> 25) & 1u);
        OK[i] = 0ull;
        OM[i] = 0u;
      }
      push(kk - 1ull, kk ? member_bits(m) : 0u);
    }
    const uint64_t b0 = (uint64_t)f << rbits;
    for (uint32_t i0 = 0; i0 < rng; i0 += RB_T) {              // every lane runs every trip (wave scans)
      const uint32_t i = i0 + threadIdx.x;
      const bool live = i < rng;
      const unsigned long long x = live ? W[2 * i] : 0ull, y = live ? W[2 * i + 1] : 0ull;
      if (live) {
        if (!(PG_EXP_BITS & 1)) *reinterpret_cast<ulonglong2*>(T.prim + 2 * (b0 + i)) = make_ulonglong2(x, y);
        W[2 * i] = 0ull;
        W[2 * i + 1] = 0ull;
      }
      const uint32_t mx = (uint32_t)(x & MW_MASK), my = (uint32_t)(y & MW_MASK);
      created += (x ? 1u : 0u) + (y ? 1u : 0u);
      ndbg += ((mx >> 12) & 1u) + ((mx >> 25) & 1u) + ((my >> 12) & 1u) + ((my >> 25) & 1u);
      const uint32_t bx = x ? member_bits(mx) : 0u, by = y ? member_bits(my) : 0u;
      if (!(PG_EXP_BITS & 8)) {
        push(((b0 + i) << T.qbits) | (x >> MW_BITS), bx);
        push(((b0 + i) << T.qbits) | (y >> MW_BITS), by);
      }
    }
    __syncthreads();
    if (PG_EXP_BITS & 4) load(f + G, n_nxt, nh, nm);
#pragma unroll
    for (int e = 0; e < RB_R; ++e) { ch[e] = nh[e]; cm[e] = nm[e]; }
    n_cur = n_nxt;
    n_nxt = n_nn;
  }
  flush();
  // the block's counters
  unsigned long long a = created, b = ndbg;
  for (int o = 32; o > 0; o >>= 1) { a += __shfl_down(a, o, 64); b += __shfl_down(b, o, 64); }
  if ((threadIdx.x & 63) == 0) { s_red[0][threadIdx.x >> 6] = a; s_red[1][threadIdx.x >> 6] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long sa = 0, sb = 0;
    for (int w = 0; w < RB_T / 64; ++w) { sa += s_red[0][w]; sb += s_red[1][w]; }
    unsigned long long* o = R.ctr + (uint64_t)blockIdx.x * RB_CTR;
    o[0] = sa;
    o[1] = sb;
    o[2] = s_mcur;
  }
}

// ---------------------------------------------------------------- tiles
// The K3 coverage groups, expanded on the device from the host's compact
// schedule (sched = off[0 .. nj], nf[0 .. nj), ord[0 .. nord)): stripe group
// j holds coverage groups [off[j], off[j+1]); while j < lead_stripes its first
// group is the lead's tile (record ord[0], stripe j) alone, the others hold QM
// followers each, ord[1 + f] for f < nf[j], at stripe j - LEAD (the lead runs
// LEAD stripes ahead).  Group g's members are descs[QM*g .. QM*g + QM); an
// empty slot has r = -1 and the group's stripe.
constexpr uint32_t LEAD = 4;
__global__ void k_tiles(const uint32_t* __restrict__ sched, uint32_t nj, uint32_t lead_stripes, uint32_t lead_off,
                        const long long* __restrict__ rec_start, const long long* __restrict__ rec_len,
                        TileDesc* __restrict__ out, uint64_t ngroups) {
  const uint32_t* off = sched;
  const uint32_t* nf = sched + nj + 1;
  const uint32_t* ord = nf + nj;
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < ngroups * QM;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t g = t / QM;
    const uint32_t m = (uint32_t)(t % QM);
    uint32_t lo = 0, hi = nj;                                  // off[lo] <= g < off[hi]
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (off[mid] <= g) lo = mid; else hi = mid;
    }
    uint32_t i = (uint32_t)(g - off[lo]);
    const bool lead = lo < lead_stripes;
    int r = -1, stripe;
    if (lead && i == 0) {
      stripe = (int)lo;
      if (m == 0) r = (int)ord[0];
    } else {
      if (lead) --i;
      stripe = (int)(lo - lead_off);
      const uint32_t f = i * QM + m;
      if (f < nf[lo]) r = (int)ord[1 + f];
    }
    out[t] = r >= 0 ? TileDesc{rec_start[r], rec_len[r], r, stripe, 0} : TileDesc{0, 0, -1, stripe, 0};
  }
}

// dBG export: (key, 12-bit mask) of both orientations of every entry.  A
// block takes EXE entries per thread in a contiguous chunk and reserves its
// output run with one atomic (one per wave on the single counter serialised
// ~1 M same-address atomics: 13 ms for a C3 table).
constexpr int EXE = 8;
__global__ void __launch_bounds__(256) k_export_dbg(TableView T, uint64_t nw, uint64_t ntot, int k,
                                                   unsigned long long* __restrict__ keys,
                                                   unsigned short* __restrict__ masks, uint64_t cap,
                                                   unsigned long long* __restrict__ counter) {
  __shared__ uint32_t s_scan[4];
  __shared__ unsigned long long s_base;
  for (uint64_t c0 = blockIdx.x * (uint64_t)(256 * EXE); c0 < ntot; c0 += (uint64_t)gridDim.x * 256 * EXE) {
    uint32_t m[EXE];
    uint32_t cnt = 0;
#pragma unroll
    for (int e = 0; e < EXE; ++e) {
      const uint64_t i = c0 + (uint64_t)threadIdx.x * EXE + e;
      m[e] = i < ntot ? entry_mask(T, nw, i) : 0u;
      cnt += ((m[e] & PRES_A) ? 1u : 0u) + ((m[e] & PRES_B) ? 1u : 0u);
    }
    uint32_t tot;
    const uint32_t pre = block_excl_scan<256>(cnt, s_scan, tot);
    if (threadIdx.x == 0) s_base = tot ? atomicAdd(counter, (unsigned long long)tot) : 0ull;
    __syncthreads();
    // writes past cap are dropped; the host rejects a count above cap
    uint64_t o = s_base + pre;
#pragma unroll
    for (int e = 0; e < EXE; ++e) {
      if (!(m[e] & (PRES_A | PRES_B))) continue;
      const uint64_t i = c0 + (uint64_t)threadIdx.x * EXE + e;
      const uint64_t c = entry_key(T, nw, i);
      if (m[e] & PRES_A) {
        if (o < cap) { keys[o] = c; masks[o] = m[e] & MASK12; }
        ++o;
      }
      if (m[e] & PRES_B) {
        if (o < cap) { keys[o] = T.rc(c); masks[o] = (m[e] >> B_SHIFT) & MASK12; }
        ++o;
      }
    }
    __syncthreads();
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
// Each owner's run also gets the sum of its records' row_check (one LDS sum
// per block; at the end one global atomic per block and owner, into one of
// CSPR words per owner, sums[owner * CSPR + block % CSPR], which the host adds).
constexpr int PT = 256, PE = 8, PCH = PT * PE;
constexpr int CSPR = 16;
__global__ void __launch_bounds__(PT)
k_part_scatter(TableView T, uint64_t nw, uint64_t ntot, int nparts, unsigned long long* __restrict__ cursor,
               Slot* __restrict__ out, unsigned long long* __restrict__ sums) {
  __shared__ unsigned s_cnt[64];
  __shared__ unsigned long long s_base[64];
  __shared__ unsigned long long s_sum[64];
  if (threadIdx.x < 64) s_sum[threadIdx.x] = 0ull;
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
      if (m[j]) {
        out[s_base[own[j]] + rank[j]] = Slot{key[j] + 1ull, m[j], 0u};
        atomicAdd(&s_sum[own[j]], (unsigned long long)row_check(key[j] + 1ull, m[j]));
      }
    __syncthreads();
  }
  __syncthreads();
  if ((int)threadIdx.x < nparts && s_sum[threadIdx.x])
    atomicAdd(&sums[threadIdx.x * CSPR + (blockIdx.x % CSPR)], s_sum[threadIdx.x]);
}

// Sums of row_check over segments of 16-byte records: segment s = records
// [off[s], off[s+1]) (grid row s), one atomic per block into
// sums[s * CSPR + block % CSPR].
constexpr int RS_SEG = 32;
struct SegOff { unsigned long long o[RS_SEG + 1]; };
__device__ __forceinline__ unsigned long long row_hash(const Slot& r) {
  return row_check(r.key1, (uint64_t)r.mask | ((uint64_t)r.aux << 32));
}
__device__ __forceinline__ unsigned long long row_hash(const Row12& r) {
  return row_check((uint64_t)r.w[0] | ((uint64_t)r.w[1] << 32), (uint64_t)r.w[2]);
}
template <class Row>
__global__ void __launch_bounds__(256) k_rows_sum(const Row* __restrict__ rows, SegOff so,
                                                  unsigned long long* __restrict__ sums) {
  __shared__ unsigned long long s_red[4];
  const uint32_t s = blockIdx.y;
  const uint64_t lo = so.o[s], hi = so.o[s + 1];
  unsigned long long acc = 0ull;
  for (uint64_t i = lo + blockIdx.x * 256ull + threadIdx.x; i < hi; i += (uint64_t)gridDim.x * 256ull) {
    acc += row_hash(rows[i]);
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t = s_red[0] + s_red[1] + s_red[2] + s_red[3];
    if (t) atomicAdd(&sums[s * CSPR + (blockIdx.x % CSPR)], t);
  }
}

// rdBG export: segment s (off[s+1] - off[s] keys at s * cap) to out + off[s]
__global__ void k_gather_segs(const unsigned long long* __restrict__ seg, uint64_t cap,
                              const unsigned long long* __restrict__ off, unsigned long long* __restrict__ out) {
  const uint64_t s = blockIdx.x, o = off[s], n = off[s + 1] - o;
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) out[o + i] = seg[s * cap + i];
}

// ------------------------------------------------------------------ host
// Small fills (counters, flags, drift hints, the overflow table) in ONE
// launch, one grid row per region, instead of a hipMemsetAsync each (~5 us of
// dispatch apiece on the critical stream).
// The build's last readback in one launch: the stage C counters per block,
// the flags and (spec) stage A's region cursors, copied into pinned host
// memory by plain vector stores (three DMA copies cost ~20 us of copy-engine
// starts on the critical path).
struct Gather { const unsigned long long* src[4]; uint32_t n[4], stride[4]; };
__global__ void __launch_bounds__(256) k_gather_out(Gather g, unsigned long long* __restrict__ dst) {
  uint32_t o = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < g.n[j]; i += gridDim.x * 256u)
      dst[o + i] = g.src[j][(uint64_t)i * g.stride[j]];
    o += g.n[j];
  }
}

struct Fill { uint4* p; uint64_t n16; unsigned v; };
constexpr int NFILL = 8;
struct Fills { Fill r[NFILL]; };
__global__ void __launch_bounds__(256) k_fills(Fills f) {
  const Fill r = f.r[blockIdx.y];
  const uint4 v = make_uint4(r.v, r.v, r.v, r.v);
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < r.n16; i += (uint64_t)gridDim.x * 256ull) r.p[i] = v;
}
struct FillList {
  Fills f{};
  int n = 0;
  uint64_t mx = 0;
  void add(void* p, uint64_t bytes, unsigned v = 0u) {
    if (!bytes) return;
    if (n == NFILL) throw Error(-22, "k_fills: too many regions");
    f.r[n++] = Fill{reinterpret_cast<uint4*>(p), (bytes + 15) / 16, v};
    mx = std::max(mx, (bytes + 15) / 16);
  }
  void launch(hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_fills, dim3(grid_for(mx, 256, 1024), (unsigned)n), dim3(256), 0, s, f);
    PG_HIP(hipGetLastError());
    n = 0;
    mx = 0;
  }
};

// (rot: the owner domain of a routed merge, pg_route_merge; 0 otherwise)
static void init_hash(Ctx& c, uint32_t rot = 0) {
  if (!(c.hash_k == c.k && c.kb)) {
    c.tv = make_hash(c.k, c.kb);
    c.cbits = std::min(6, c.kb);
    c.hash_k = c.k;
  }
  c.tv.rot = rot;
}

// The coverage groups (records with n >= k+2), stripe-major: stripe 0 of
// every record, then stripe 1, ... (records with more stripes first within a
// stripe), QM followers of a stripe per group.  One lead record runs LEAD
// stripes ahead of the others, so that the coverage pass finds the lead's
// windows staged before its followers compare against them in the same L2.
// The host sorts the records and sends the per-stripe group offsets and
// follower counts; k_tiles expands the descriptors on the device.  Cached
// while the record table and flags repeat.  Returns the number of groups.
// follow: the flagged records are all followers of the references already
// chosen (c.k3_ref, c.k3_ref2, left as they are; both skipped if flagged), no
// lead groups (pg_build_host's later chunks); never cached.
// st: the stream the upload and k_tiles go on (NULL: the context's stream)
static uint64_t make_tiles(Ctx& c, const std::vector<uint8_t>& flag, bool follow = false, hipStream_t st = nullptr) {
  if (!st) st = c.stream;
  const uint64_t R = c.n_records;
  if (!follow && c.tile_sig_len == c.h_rec_len && c.tile_sig_flag == flag && c.tile_k == c.k) return c.n_tiles;
  std::vector<std::pair<uint64_t, int>> nt;           // (stripes, record)
  for (uint64_t r = 0; r < R; ++r) {
    const int64_t n = c.h_rec_len[r];
    if (!flag[r] || n < c.k + 2) continue;
    if (follow && ((int)r == c.k3_ref || (int)r == c.k3_ref2)) continue;
    nt.push_back({(uint64_t)((n - c.k + 1 + TILE - 1) / TILE), (int)r});
  }
  std::stable_sort(nt.begin(), nt.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
  if (!follow) {
    c.k3_ref = nt.size() >= 2 ? nt[0].second : -1;    // the lead is every follower's dedup reference
    c.k3_ref2 = nt.size() >= 3 ? nt[1].second : -1;   // the second reference (k_cover)
  }
  c.k3_hint.reserve(64 * (R + 1) + 64);               // drift hints per XCD, reference, record
  // normal: ord[0] = the lead, its tiles one group per stripe, the followers
  // (ord[1..]) LEAD stripes behind; follow: followers only (ord[0] unused)
  const uint64_t lead_s = follow || nt.empty() ? 0 : nt[0].first;
  const uint32_t lead_off = follow ? 0u : LEAD;
  const uint32_t nj = nt.empty() ? 0u : (uint32_t)(follow ? nt[0].first : lead_s + LEAD);
  const size_t skip = follow ? 0 : 1;                 // followers: nt[skip ..]
  std::vector<uint32_t> sched(2 * nj + 2 + nt.size());
  uint64_t total = 0;
  size_t live = nt.size();
  for (uint32_t j = 0; j < nj; ++j) {
    sched[j] = (uint32_t)total;
    uint64_t cnt = j < lead_s ? 1 : 0, nfol = 0;
    if (j >= lead_off) {
      const uint64_t jf = j - lead_off;               // the followers' stripe
      while (live && nt[live - 1].first <= jf) --live;
      nfol = live > skip ? live - skip : 0;
      cnt += (nfol + QM - 1) / QM;
    }
    sched[nj + 1 + j] = (uint32_t)nfol;
    total += cnt;
  }
  sched[nj] = (uint32_t)total;
  if (follow) sched[2 * nj + 1] = 0u;                 // ord[0] (unused)
  for (size_t i = 0; i < nt.size(); ++i) sched[2 * nj + 1 + (follow ? 1 : 0) + i] = (uint32_t)nt[i].second;
  if (total * QM >= (1ull << 32)) throw Error(-22, "make_tiles: too many tiles");
  c.tile_desc.reserve(sizeof(TileDesc) * (QM * total + 1));
  if (total) {
    c.tile_pin.reserve(4 * sched.size());
    c.tile_sched.reserve(4 * sched.size());
    std::memcpy(c.tile_pin.p, sched.data(), 4 * sched.size());
    PG_HIP(hipMemcpyAsync(c.tile_sched.p, c.tile_pin.p, 4 * sched.size(), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_tiles, dim3(grid_for(QM * total, 256, 2048)), dim3(256), 0, st,
                       c.tile_sched.as<uint32_t>(), nj, (uint32_t)lead_s, lead_off, c.rec_start.as<long long>(),
                       c.rec_len.as<long long>(), c.tile_desc.as<TileDesc>(), total);
    PG_HIP(hipGetLastError());
  }
  if (follow) {
    c.tile_sig_len.clear();                           // the cached list is gone
  } else {
    c.tile_sig_len = c.h_rec_len;
    c.tile_sig_flag = flag;
    c.tile_k = c.k;
  }
  c.n_tiles = total;
  return total;
}

// ---- stage A: buffers for `cap` records per region; the regions' cursors and
// the flags are zeroed by the caller's fill list
// (reset = false: the regions of the stage A in progress take more records)
static BinOut stageA_begin(Ctx& c, uint64_t cap, FillList& fl, bool reset = true) {
  if (reset) {
    c.capA = cap;
    c.recA_key.reserve(8 * NREG * cap);
    c.recA_mw.reserve(4 * NREG * cap);
    c.ctrA.reserve(8 * CSTRIDE * NREG);
    c.flags.reserve(4 * N_FLAGS + 16 * MCHK);      // the flags, then the merge's checksum slots
    fl.add(c.ctrA.p, 8 * CSTRIDE * NREG);
    fl.add(c.flags.p, 4 * N_FLAGS + 16 * MCHK);
  }
  cap = c.capA;
  return BinOut{c.recA_key.as<unsigned long long>(), c.recA_mw.as<uint32_t>(), c.ctrA.as<unsigned long long>(),
                cap, (uint32_t)(c.kb - c.cbits), c.flags.as<unsigned>()};
}

struct ACount {
  uint64_t total = 0, maxreg = 0, maxbin = 0;
  unsigned sentinel = 0, bits = 0, bits_bc = 0;     // bits: flags[1] (stage A), bits_bc: flags[4] (stages B/C)
};
// stage A's counts and flags from a pinned copy of ctrA and the flags
static ACount stageA_counts(const unsigned long long* h, const unsigned* fl, int stride = CSTRIDE) {
  ACount a;
  for (int p = 0; p < NBIN; ++p) {
    uint64_t bin = 0;
    for (int x = 0; x < 8; ++x) {
      const uint64_t n = h[stride * (p * 8 + x)];
      a.total += n;
      bin += n;
      a.maxreg = std::max(a.maxreg, n);
    }
    a.maxbin = std::max(a.maxbin, bin);
  }
  a.sentinel = fl[0];
  a.bits = fl[1];
  a.bits_bc = fl[4];
  return a;
}

// sync #1: the stage A region counts and flags
static ACount stageA_read(Ctx& c) {
  const size_t cb = 8 * CSTRIDE * NREG;
  c.h_pin.reserve(cb + 4 * N_FLAGS);
  PG_HIP(hipMemcpyAsync(c.h_pin.p, c.ctrA.p, cb, hipMemcpyDeviceToHost, c.stream));
  PG_HIP(hipMemcpyAsync(c.h_pin.as<uint8_t>() + cb, c.flags.p, 4 * N_FLAGS, hipMemcpyDeviceToHost, c.stream));
  c.sync();
  return stageA_counts(c.h_pin.as<unsigned long long>(),
                       reinterpret_cast<const unsigned*>(c.h_pin.as<uint8_t>() + cb));
}

// stage A region size for about `est` records (10 % + 512 per region of slack)
static uint64_t region_cap(uint64_t est) { return est / NREG + est / (NREG * 10) + 512; }

// ---- stages B and C over stage A's records, and the build's last sync.  The
// table gets 2^bb buckets with 2^bb >= the record count (>= the key count: at
// most one key per 2-word bucket on average), kb - 38 <= bb <= kb.
// spec: stage A is still in flight on the stream and `a` is a plan (region
// capacity as the largest region, 8 regions' worth as the largest bin, the
// last build's records-per-window ratio as the total), so stages B and C
// are queued right behind it with no host round trip in between; stage A's
// counts and flags come back with the same sync.  Returns false (with the
// exact counts in `a`) if stage A overflowed a region; a B/C flag re-runs B/C
// with the exact counts.
// The table geometry finish_build picks for `total` stage A records: bucket
// bits bb, fine partition bits fp.
static void table_bits(const Ctx& c, uint64_t total, int& bb, int& fp) {
  bb = std::max(1, log2u(std::max<uint64_t>(total, 1)));
  bb = std::min(std::max({bb - c.bb_shift, c.cbits, c.kb - 38}), c.kb);
  fp = std::max(c.cbits, bb - RANGE_BITS);
}
// pg_build_host's early split (stage B under the upload): made for bucket
// bits bb, one split level of S bits into partitions of `cap` records, in
// c.recS_*[0] with cursors at c.ctrS
struct Presplit {
  int bb;
  uint32_t S;
  uint64_t cap;
};

#ifdef PG_DEBUG_BOUNDS
static void debug_report(const char* where) {
  static unsigned long long h[16 + 16 * 4 * 5];
  PG_HIP(hipDeviceSynchronize());
  PG_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_dbg), sizeof(h)));
  bool any = false;
  for (int sl = 0; sl < 16; ++sl) {
    if (!h[sl]) continue;
    any = true;
    std::fprintf(stderr, "PG_DEBUG_BOUNDS %s: slot %d: %llu violations\n", where, sl, h[sl]);
    for (unsigned long long i = 0; i < h[sl] && i < 4; ++i) {
      const unsigned long long* e = h + 16 + (sl * 4 + i) * 5;
      std::fprintf(stderr, "  check %llu a=%lld b=%lld block=%llu thread=%llu\n", e[0], (long long)e[1], (long long)e[2],
                   e[3], e[4]);
    }
  }
  if (any) {
    static unsigned long long z[16 + 16 * 4 * 5] = {};
    PG_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_dbg), z, sizeof(z)));
  }
}
#else
static void debug_report(const char*) {}
#endif

static bool finish_build(Ctx& c, ACount& a, bool spec, const Presplit* pre = nullptr) {
  const int kb = c.kb, cb = c.cbits;
  int bb, fp0;
  table_bits(c, a.total, bb, fp0);
  (void)fp0;
  double capx = 1.15;
  uint64_t ovf_mult = 1;
  double rseg_frac = c.r_ratio > 0 ? std::min(2.0, 1.5 * c.r_ratio + 0.002) : 2.0;
  // a split level that overflowed: its partitions' exact counts (the cursors
  // count every record, kept or not) size it on the next attempt, so skewed
  // keys cost one re-run per level instead of a geometric capacity search
  // (a key repeated in many records lands all of them in one partition: C4's
  // largest level-2 partition holds ~1.9x the mean, so the plan's capacities
  // overflowed on every build until they started from the last re-run's)
  std::vector<uint64_t> lv_exact = c.lv_keep;
  int lv_exact_bb = c.lv_keep_bb;
  c.t6.init();
  debug_report("stage A");
  for (int attempt = 0; attempt < 8; ++attempt) {
    c.bc_attempts = attempt + 1;
    const int fp = std::max(cb, bb - RANGE_BITS);
    const uint32_t rbits = (uint32_t)(bb - fp);
    const uint64_t buckets = 1ull << bb;
    const uint64_t ovf = next_pow2(std::max<uint64_t>(4096, a.total / 8)) * ovf_mult;
    c.table.reserve(16 * buckets);
    c.ovf.reserve(sizeof(Slot) * ovf);
    set_geometry(c.tv, kb, bb, ovf);
    c.tv.prim = c.table.as<unsigned long long>();
    c.tv.ovf = c.ovf.as<Slot>();
    c.cap = buckets;
    c.ovf_cap = ovf;
    c.bb = bb;
    // split levels: partition bits cb -> ... -> fp, <= 7 bits a pass
    // (input regions: stage A's 8 per coarse bin, then one per partition)
    struct Lv { int L, S; uint64_t pin, cap, nreg, bpr, ctr_off; };
    std::vector<Lv> lv;
    uint64_t maxin = a.maxbin, maxreg = a.maxreg, nsub = 8, ctr_words = 0;
    // (no split needed: one S = 0 pass still gathers each bin's 8 regions into one)
    // the early split's partitions, when they are this attempt's only level
    const bool use_pre = pre && attempt == 0 && pre->bb == bb && fp - cb == (int)pre->S && fp > cb &&
                         fp - cb <= SPLIT_BITS;
    for (int L = cb; L < fp || lv.empty();) {
      const int S = std::min(SPLIT_BITS, fp - L);
      const uint64_t pin = 1ull << L, nb = 1ull << S;
      uint64_t capo = (uint64_t)((double)maxin / (double)nb * capx) + 64;
      if (lv_exact_bb == bb && lv.size() < lv_exact.size())
        capo = std::max(capo, lv_exact[lv.size()] + lv_exact[lv.size()] / 16 + 64);
      if (use_pre) capo = pre->cap;
      lv.push_back(Lv{L, S, pin, capo, pin * nsub, std::max<uint64_t>(1, (maxreg + SCH - 1) / SCH), ctr_words});
      ctr_words += CSTRIDE * pin * nb;
      maxin = maxreg = capo;
      nsub = 1;
      L += S;
    }
    uint64_t rec_max = 0;
    for (const Lv& l : lv) rec_max = std::max<uint64_t>(rec_max, l.pin * (1ull << l.S) * l.cap);
    for (int i = 0; i < 2 && !lv.empty(); ++i) {
      c.recS_key[i].reserve(8 * rec_max);
      c.recS_mw[i].reserve(4 * rec_max);
    }
    c.ctrS.reserve(8 * std::max<uint64_t>(ctr_words, 1));
    const uint64_t nparts = 1ull << fp;
    const uint32_t grid = (uint32_t)std::min<uint64_t>(nparts, (uint64_t)RB_PER_CU * (uint64_t)c.n_cu);   // persistent
    const uint64_t rcap = (uint64_t)(rseg_frac * (double)a.total / grid) + 4096;
    c.rseg.reserve(8 * grid * rcap);
    c.rseg_cap = rcap;
    c.rseg_nseg = grid;
    c.k5_ctr.reserve(8 * RB_CTR * grid);
    FillList fl;
    fl.add(c.ovf.p, sizeof(Slot) * ovf);
    if (!use_pre) {                                           // (the early split's counts are in ctrS)
      fl.add(c.ctrS.p, 8 * ctr_words);
      fl.add(c.flags.as<unsigned>() + 4, 16);                 // stage B/C bits (not the sentinel)
    }
    // the fills (C3: the 64 MB overflow table, 12 us) go on the side stream,
    // behind its share of stage A (which touches none of them), so that they
    // run beside stage A's last work pass; stage B waits for them
    // (this is also where the main stream joins stage A's side stream, and
    // where stage A's timer stops when the build queued it unjoined: one
    // wait and one event between stage A's last work pass and k_split)
    fl.launch(c.stream2);
    PG_HIP(hipEventRecord(c.ev[15], c.stream2));
    PG_HIP(hipStreamWaitEvent(c.stream, c.ev[15], 0));
    if (c.t1_open) {
      c.t1.stop(c.stream);
      c.t1_open = false;
    }
    Recs in{c.recA_key.as<unsigned long long>(), c.recA_mw.as<uint32_t>(), c.ctrA.as<unsigned long long>(), c.capA,
            8};
    for (size_t i = 0; i < lv.size(); ++i) {
      const Lv& l = lv[i];
      const uint32_t nb = 1u << l.S;
      Recs out{c.recS_key[i & 1].as<unsigned long long>(), c.recS_mw[i & 1].as<uint32_t>(),
               c.ctrS.as<unsigned long long>() + l.ctr_off, l.cap, 1};
      if (use_pre) {                                          // split already, chunk by chunk
        in = out;
        continue;
      }
      if (l.nreg * l.bpr >= (1ull << 31)) throw Error(-22, "build: split grid too large");
      hipLaunchKernelGGL(a.total < SPLIT_NT_MAX ? k_split<true> : k_split<false>,
                         dim3((unsigned)(l.nreg * l.bpr)), dim3(SB), 0, c.stream, in, out,
                         (const unsigned long long*)nullptr, (uint32_t)(kb - l.L - l.S), nb, (uint32_t)l.bpr,
                         c.flags.as<unsigned>());
      PG_HIP(hipGetLastError());
      in = out;
    }
    c.split_passes = use_pre ? 0 : (int)lv.size();
    unsigned long long* k5 = c.k5_ctr.as<unsigned long long>();
    const RdbgOut ro{c.rseg.as<unsigned long long>(), k5, rcap};
    c.t6.start(c.stream);
    hipLaunchKernelGGL(a.total < SPLIT_NT_MAX ? k_build_range<true> : k_build_range<false>, dim3(grid), dim3(RB_T), 0,
                       c.stream, in, c.tv, rbits, (uint32_t)nparts, ro, c.flags.as<unsigned>());
    PG_HIP(hipGetLastError());
    c.t6.stop(c.stream);
    // one readback: stage C's counters, the flags, (spec) stage A's cursors
    // (one word per region: stride CSTRIDE on the device, 1 in the copy)
    const size_t kbytes = 8 * RB_CTR * grid, abytes = spec ? 8 * NREG : 0;
    c.h_out.reserve(kbytes + 4 * N_FLAGS + abytes + 16 * MCHK);
    Gather gth{{c.k5_ctr.as<unsigned long long>(), c.flags.as<unsigned long long>(), c.ctrA.as<unsigned long long>(),
                c.flags.as<unsigned long long>() + N_FLAGS / 2},
               {(uint32_t)(RB_CTR * grid), (uint32_t)(N_FLAGS / 2), spec ? (uint32_t)NREG : 0u, 2u * MCHK},
               {1u, 1u, (uint32_t)CSTRIDE, 1u}};
    hipLaunchKernelGGL(k_gather_out, dim3(4), dim3(256), 0, c.stream, gth,
                       reinterpret_cast<unsigned long long*>(c.h_out.dp));
    PG_HIP(hipGetLastError());
    c.sync();
    c.ms_range = c.t6.ms();
    float tsplit = 0.f;                        // stage A's end (t1) to stage C's start
    if (!c.t1.off && !c.t6.off) PG_HIP(hipEventElapsedTime(&tsplit, c.t1.b, c.t6.a));   // (else 0)
    c.ms_split = (double)tsplit;
    c.ms_scan = c.ms_split + c.ms_range;
    const unsigned long long* h = c.h_out.as<unsigned long long>();
    const unsigned* hf = reinterpret_cast<const unsigned*>(c.h_out.as<uint8_t>() + kbytes);
    if (spec) {                                // stage A's exact counts, and whether it fit
      a = stageA_counts(reinterpret_cast<const unsigned long long*>(c.h_out.as<uint8_t>() + kbytes + 4 * N_FLAGS), hf,
                        1);
      c.sentinel = a.sentinel ? 1 : 0;
      spec = false;
      if (a.bits & F_A_OVER) return false;
    }
    const unsigned bits = hf[4];
    {                                          // the merge's checksum slots (zero for a build)
      const unsigned long long* mk =
          reinterpret_cast<const unsigned long long*>(c.h_out.as<uint8_t>() + kbytes + 4 * N_FLAGS + abytes);
      uint64_t s = 0, r = 0;
      for (int j = 0; j < MCHK; ++j) s += mk[2 * j], r += mk[2 * j + 1];
      c.merge_sum = s;
      c.merge_rows = r;
    }
    c.work_items = (uint64_t)hf[F_WORK_ITEMS] | ((uint64_t)hf[F_WORK_ITEMS + 1] << 32);
    static const bool dbg_build = std::getenv("PG_DEBUG_BUILD") != nullptr;
    if (dbg_build)
      std::fprintf(stderr, "finish_build attempt %d: total %llu maxreg %llu maxbin %llu bb %d levels %zu rec_max %llu "
                   "capx %.2f ovf %llu rcap %llu bits %u\n", attempt, (unsigned long long)a.total,
                   (unsigned long long)a.maxreg, (unsigned long long)a.maxbin, bb, lv.size(),
                   (unsigned long long)rec_max, capx, (unsigned long long)ovf, (unsigned long long)rcap, bits);
    if (bits & F_SPLIT_OVER) {
      std::vector<unsigned long long> ctr(std::max<uint64_t>(ctr_words, 1));
      PG_HIP(hipMemcpy(ctr.data(), c.ctrS.p, 8 * ctr_words, hipMemcpyDeviceToHost));
      std::vector<uint64_t> ex(lv.size(), 0);
      bool over = false;                          // some level's exact count exceeds its capacity
      for (size_t i = 0; i < lv.size(); ++i) {
        const uint64_t np = lv[i].pin << lv[i].S;
        for (uint64_t q = 0; q < np; ++q) ex[i] = std::max<uint64_t>(ex[i], ctr[lv[i].ctr_off + CSTRIDE * q]);
        over |= ex[i] > lv[i].cap;
      }
      if (lv_exact_bb == bb)
        for (size_t i = 0; i < ex.size() && i < lv_exact.size(); ++i) ex[i] = std::max(ex[i], lv_exact[i]);
      lv_exact = ex;
      lv_exact_bb = bb;
      c.lv_keep = ex;
      c.lv_keep_bb = bb;
      if (!over) capx *= 1.5;                     // (not expected: the flag without a visible overflow)
      continue;
    }
    if (bits & F_LDS_SPILL) {
      if (bb < kb) { ++bb; continue; }
      throw Error(-12, "build: LDS overflow set full at the largest table");
    }
    if (bits & F_OVF_FULL) { ovf_mult *= 4; continue; }
    if (bits & F_RSEG_OVER) { rseg_frac = 2.0; continue; }
    uint64_t created = 0, ndbg = 0, nr = 0;
    c.rseg_cnt.resize(grid);
    for (uint32_t b = 0; b < grid; ++b) {
      created += h[RB_CTR * b];
      ndbg += h[RB_CTR * b + 1];
      c.rseg_cnt[b] = h[RB_CTR * b + 2];
      nr += c.rseg_cnt[b];
    }
    c.n_canon = created;
    c.n_dbg = ndbg + c.sentinel;
    c.n_rdbg = nr + c.sentinel;               // key 2^64-1, mask 32: always an rdBG member
    c.r_ratio = a.total ? (double)nr / (double)a.total : 0.0;
    c.built = c.reduced = true;
    c.early_split_used = use_pre;
    ++c.build_gen;
    return true;
  }
  throw Error(-12, "build: table overflow after resizing");
}

// chunks of the tile list whose work pass overlaps the next coverage pass
constexpr int K3_CHUNKS = (PG_EXP_BITS & 4096) ? 2 : (PG_EXP_BITS & 512) ? 4 : (PG_EXP_BITS & 1024) ? 5 : (PG_EXP_BITS & 2048) ? 6 : 3;
constexpr int K3_WBLK = 4;                    // work blocks per CU (chunked form; pg_tune PG_TUNE_K3_WBLK)
constexpr uint64_t K3_CHUNK_MIN = 1024;       // coverage groups per chunk below which one chunk runs

static void launch_short(Ctx& c, hipStream_t s, int rc0, uint64_t shift, const BinOut& O) {
  if (!c.n_records) return;
  hipLaunchKernelGGL(k_short_emit, dim3(grid_for(c.n_records, IBLOCK, 1024)), dim3(IBLOCK), 0, s, packed_cls(c),
                     c.rec_start.as<long long>(), c.rec_len.as<long long>(), c.rec_flag.as<uint8_t>(), c.n_records,
                     c.k, shift, rc0, c.tv, O);
  PG_HIP(hipGetLastError());
}

// Stage A of one build: the coverage pass and the work pass in NCH chunks of
// the tile list on two streams (the work pass of chunk i runs beside the
// coverage pass of chunk i+1; the last work pass runs on s0 right behind the
// last coverage pass, beside the previous one — chunks' records commute),
// the short records beside it, then the staged npz slots; s1 joins s0.
// part: 0 = a whole stage A; pg_build_host's parts: SA_FIRST starts it (the
// regions reset, no short records yet), SA_MORE adds tiles, SA_TAIL adds the
// short records, the n<k flag and the staged slots (no tiles).
// SA_FIRST_TAIL / SA_MORE_TAIL: SA_FIRST / SA_MORE and SA_TAIL in one call
// (the last batch of records, once the record table is final).
enum { SA_WHOLE = 0, SA_FIRST = 1, SA_MORE = 2, SA_TAIL = 3, SA_FIRST_TAIL = 4, SA_MORE_TAIL = 5 };
// join = false: the side stream is joined (and t1 stopped) by finish_build,
// behind the stage B/C fills it queues on the side stream.
static void enqueue_stageA(Ctx& c, uint64_t cap, uint64_t ntiles, int rc0, int extra_empty, int part = SA_WHOLE,
                           bool join = true) {
  const uint64_t shift = pow5(c.k - 1);
  hipStream_t s0 = c.stream, s1 = c.stream2;
  FillList fl;
  const bool begin = part == SA_WHOLE || part == SA_FIRST || part == SA_FIRST_TAIL;
  const bool tail = part == SA_WHOLE || part == SA_TAIL || part == SA_FIRST_TAIL || part == SA_MORE_TAIL;
  const BinOut O = stageA_begin(c, cap, fl, begin);
  if (part == SA_TAIL) ntiles = 0;
#ifdef PG_COVER_LEGACY
  if (c.k3_cover == 1 || c.k3_cover == 2) ensure_cls(c);   // (the class-byte coverage forms)
#endif
#ifdef PG_DEBUG_BOUNDS
  ensure_cls(c);                                            // (k_cover_p's debug check reads class bytes)
#endif
  const uint8_t* cls = c.cls.as<uint8_t>();
  const PackedCls pc = packed_cls(c);
  const dim3 b(IBLOCK);
  int nch = ntiles >= (uint64_t)K3_CHUNKS * K3_CHUNK_MIN ? K3_CHUNKS : 1;
  if (c.k3_chunks > 0) nch = std::min(6, c.k3_chunks);
  if (!ntiles) nch = 0;
  // chunk i covers the fraction [cb[i], cb[i+1]) / cbt of every XCD's share:
  // 16 parts each, the last chunk 10 (c.k3_tail: a smaller last chunk
  // leaves a smaller work pass behind the last coverage pass: C3 stage A
  // 0.566 / 0.568 / 0.581 ms at 10 / 12 / 8 against 0.586 at 16)
  const uint32_t tailw = c.k3_tail ? (uint32_t)c.k3_tail : 10u;
  const uint32_t headw = c.k3_head ? (uint32_t)c.k3_head : 16u;
  uint32_t cb[8] = {};
  for (int i = 1; i <= nch; ++i) cb[i] = cb[i - 1] + (i == nch ? tailw : i == 1 ? headw : 16u);
  const uint32_t cbt = nch ? cb[nch] : 1u;
  uint64_t gc[8] = {}, qoff[8] = {}, qcapc[8] = {}, items = 0;
  for (int i = 0; i < nch; ++i) {
    for (int x = 0; x < 8; ++x) {
      uint64_t t, te;
      xcd_chunk(ntiles, cb[i], cb[i + 1], cbt, (uint64_t)x, t, te);
      gc[i] = std::max<uint64_t>(gc[i], 8 * (te - t));
    }
    qcapc[i] = (gc[i] + NQ - 1) / NQ * (QM * CBLOCK);   // per sub-queue: a block queues <= QM * CBLOCK
    qoff[i] = items;
    items += NQ * qcapc[i];
  }
  const size_t qbytes = sizeof(WorkItem) * items, cbytes = 8 * QSTRIDE * NQ;
  if (nch) {
    c.k3_queue.reserve(qbytes + cbytes * nch);
    fl.add(c.k3_queue.as<uint8_t>() + qbytes, cbytes * nch);              // queue counters
    fl.add(c.k3_hint.p, 16 * 4 * (c.n_records + 1), 0xFFFFFFFFu);         // "no drift known yet"
  }
  // A whole stage A (pg_build_dbg / the held routed form) puts its fills -
  // like the tile schedule's upload and k_tiles before them (make_tiles) - on
  // the side stream, idle since the last build: they depend on the record
  // table, not on K1's emission, and run beside it; the main stream only
  // waits for them (one event) when K1 is done.  On the main stream those
  // three dispatches followed K1 one by one (~35 us K1-to-stage-A under
  // rocprofv3, profiles/r05_trace_c3_build.txt).  The incremental parts of
  // pg_build_host keep them in order on the main stream (its side stream is
  // busy with the last chunk's work pass).
  const bool side = part == SA_WHOLE;
  if (side) {
    fl.launch(s1);
    PG_HIP(hipEventRecord(c.ev[0], s1));
    PG_HIP(hipStreamWaitEvent(s0, c.ev[0], 0));
  }
  c.t1.init();
  c.t1.start(s0);
  if (!side) fl.launch(s0);
#ifdef PG_DEBUG_BOUNDS
  for (int i = 0; i < nch; ++i)
    hipLaunchKernelGGL(k_dbg_counters, dim3(1), dim3(64), 0, s0,
                       reinterpret_cast<const unsigned long long*>(c.k3_queue.as<uint8_t>() + qbytes) + (cbytes / 8) * i,
                       0ull, 41u, (unsigned)i);
#endif
  const unsigned wgrid = (unsigned)c.n_cu * (c.k3_wblk & 15 ? c.k3_wblk & 15 : K3_WBLK);
  const unsigned wgrid_last = c.k3_wblk >> 4 ? (unsigned)c.n_cu * (c.k3_wblk >> 4) : wgrid;
  auto* q = c.k3_queue.as<WorkItem>();
  auto* qn = reinterpret_cast<unsigned long long*>(c.k3_queue.as<uint8_t>() + qbytes);
  const long long rfs = c.k3_ref >= 0 ? c.h_rec_start[c.k3_ref] : 0, rfn = c.k3_ref >= 0 ? c.h_rec_len[c.k3_ref] : 0;
  const long long r2s = c.k3_ref2 >= 0 ? c.h_rec_start[c.k3_ref2] : 0;
  const long long r2n = c.k3_ref2 >= 0 ? c.h_rec_len[c.k3_ref2] : 0;
  const TileDesc* td = c.tile_desc.as<TileDesc>();
  bool short_done = false;
  if (!side) {
    PG_HIP(hipEventRecord(c.ev[0], s0));                       // s1 starts after the fills
    PG_HIP(hipStreamWaitEvent(s1, c.ev[0], 0));
  }
  for (int i = 0; i < nch; ++i) {
    auto* qi = q + qoff[i];
    auto* qni = qn + (cbytes / 8) * i;
#ifdef PG_COVER_LEGACY
    if (gc[i] && c.k3_cover == 1)
      hipLaunchKernelGGL(k_cover, dim3((unsigned)gc[i]), dim3(CBLOCK), 0, s0, cls, td, qi, qni, (unsigned long long)qcapc[i],
                         c.k, c.k3_ref, rfs, rfn, c.k3_ref2, r2s, r2n, c.k3_hint.as<int>(), (int)c.n_records, ntiles,
                         cb[i], cb[i + 1], cbt);
    else if (gc[i] && c.k3_cover == 2)
      hipLaunchKernelGGL(k_cover_q, dim3((unsigned)gc[i]), dim3(CBLOCK), 0, s0, cls, (uint64_t)c.cls.cap, td, qi, qni,
                         (unsigned long long)qcapc[i], c.k, c.k3_ref, rfs, rfn, c.k3_ref2, r2s, r2n,
                         c.k3_hint.as<int>(), (int)c.n_records, ntiles, cb[i], cb[i + 1], cbt);
    else
#endif
    if (gc[i])
      launch_cover_p(c.k3_anchors ? c.k3_anchors : NAP_DEFAULT, dim3((unsigned)gc[i]), s0, c.p2.as<uint32_t>(),
                     c.e16.as<uint8_t>(), (uint64_t)(c.p2.cap / 4), cls, td, qi, qni, (unsigned long long)qcapc[i], c.k,
                     c.k3_ref, rfs, rfn, c.k3_ref2, r2s, r2n, c.k3_hint.as<int>(), (int)c.n_records, ntiles,
                     cb[i], cb[i + 1], cbt);
    PG_HIP(hipGetLastError());
#ifdef PG_DEBUG_BOUNDS
    for (int j = 0; j < nch; ++j)                 // this chunk's counters in range, the later ones still zero
      hipLaunchKernelGGL(k_dbg_counters, dim3(1), dim3(64), 0, s0, qn + (cbytes / 8) * j,
                         j <= i ? (unsigned long long)qcapc[j] : 0ull, j <= i ? 43u : 44u, (unsigned)(i * 10 + j));
#endif
    hipStream_t ws = s1;
    if (nch > 1 && i + 1 == nch) {
      ws = s0;
      if (tail) {
        launch_short(c, s1, rc0, shift, O);                    // k_short beside the last work pass
        short_done = true;
      }
    } else {
      PG_HIP(hipEventRecord(c.ev[1 + i], s0));
      PG_HIP(hipStreamWaitEvent(s1, c.ev[1 + i], 0));        // s1: work 0 .. i-1, then this
    }
    const uint64_t mi = std::min<uint64_t>(NQ * qcapc[i], c.windows_fw / IW + c.n_records + 1);
    const unsigned gw = nch > 1 ? (i + 1 == nch ? wgrid_last : wgrid) : grid_for(mi, IBLOCK, 16384);
    const bool halves = c.k3_emit != 1;
    auto* kw = rc0 ? (halves ? k_emit_work<true, 2> : k_emit_work<true, 1>)
                   : (halves ? k_emit_work<false, 2> : k_emit_work<false, 1>);
    hipLaunchKernelGGL(kw, dim3(gw), b, 0, ws, pc, qi, qni, (unsigned long long)qcapc[i], c.k, shift, c.tv, O);
    PG_HIP(hipGetLastError());
  }
  if (!short_done && tail) launch_short(c, s0, rc0, shift, O);
  if (extra_empty && tail) hipLaunchKernelGGL(k_set_flag, dim3(1), dim3(1), 0, s0, c.flags.as<unsigned>());
  if (c.n_preload && tail) {
    hipLaunchKernelGGL(k_preload_emit, dim3(grid_for(c.n_preload, 4 * IBLOCK, 4096)), dim3(IBLOCK), 0, s0,
                       c.preload.as<PreEnt>(), c.n_preload, c.tv, O);
    PG_HIP(hipGetLastError());
  }
  if (!join) {
    c.t1_open = true;
    return;
  }
  PG_HIP(hipEventRecord(c.ev[15], s1));                       // join: s0 continues after s1's work
  PG_HIP(hipStreamWaitEvent(s0, c.ev[15], 0));
  c.t1.stop(s0);
}

void build_dbg(Ctx& c, const uint8_t* h_rec_flag, int extra_empty, int rc0) {
  if (!c.parsed) throw Error(-22, "build_dbg: no parsed FASTA (call pg_parse first)");
  c.early_split_used = false;
  const uint64_t R = c.n_records;
  c.rc0 = rc0;
  c.built = c.reduced = false;
  c.n_dbg = c.n_rdbg = c.n_canon = 0;
  c.windows_fw = 0;
  std::vector<uint8_t> flag(R, 1);
  if (h_rec_flag)
    for (uint64_t r = 0; r < R; ++r) flag[r] = h_rec_flag[r] & 1;
  // (the device copy of the flags is kept while it holds these: a pageable
  // upload costs a staged copy on the critical path)
  if (R && !(c.dev_flag_p == c.rec_flag.p && c.dev_flag == flag)) {
    PG_HIP(hipMemcpyAsync(c.rec_flag.p, flag.data(), R, hipMemcpyHostToDevice, c.stream));
    c.dev_flag = flag;
    c.dev_flag_p = c.rec_flag.p;
  }
  uint64_t nshort = 0, nlong = 0;
  for (uint64_t r = 0; r < R; ++r)
    if (flag[r]) {
      const int64_t n = c.h_rec_len[r];
      c.windows_fw += n > c.k ? (uint64_t)(n - c.k + 1) : 1;
      nshort += n >= c.k && n <= c.k + 1;
      nlong += n >= c.k + 2;
    }
  c.windows_total = c.windows_fw * (rc0 ? 2 : 1);
  c.last_flag = flag;
  c.last_extra = extra_empty;
  c.dump_ready = false;
  init_hash(c);
  const uint64_t ntiles = make_tiles(c, flag, false, c.stream2);   // (beside K1's emission: enqueue_stageA)
  // stage A records: at most one per forward window, 4 per short record, one
  // per staged npz slot.  Expected: the last build's records per window, or
  // (first build) the windows divided by the number of long records up to 4
  // (a pangenome of G genomes repeats most k-mers G times); a region that
  // overflows re-runs stage A with the exact counts.
  const uint64_t extra = 4 * nshort + c.n_preload + 64;
  const uint64_t redund = std::max<uint64_t>(1, std::min<uint64_t>(4, nlong));
  uint64_t est = c.u_ratio > 0 ? (uint64_t)(c.u_ratio * 1.25 * (double)c.windows_fw) : c.windows_fw / redund;
  est = std::min(est, c.windows_fw) + extra;
  uint64_t cap = c.region_cap_force ? c.region_cap_force : region_cap(est);
  c.ms_clear = 0;
  ACount a;
  c.route_ready = false;
  const bool hold = c.route_req;                    // (pg_route_stage_a: stage A only)
  c.route_req = false;
  // after a first build the whole build is queued at once (finish_build's
  // spec form: one host round trip instead of two); the table is then sized
  // from the last build's records per window, 5 % up
  if (c.u_ratio > 0 && !c.region_cap_force && !hold) {
    enqueue_stageA(c, cap, ntiles, rc0, extra_empty, SA_WHOLE, false);
    a.total = (uint64_t)(c.u_ratio * 1.05 * (double)c.windows_fw) + extra;
    a.maxreg = cap;
    a.maxbin = 8 * cap;
    const bool ok = finish_build(c, a, true);
    c.ms_insert = c.t1.ms();
    c.n_records_a = a.total;
    if (ok) {
      if (c.windows_fw) c.u_ratio = (double)a.total / (double)c.windows_fw;
      return;
    }
    cap = a.maxreg + a.maxreg / 8 + 512;           // every region's exact count is known now
  }
  for (int attempt = 0; attempt < 3; ++attempt) {
    enqueue_stageA(c, cap, ntiles, rc0, extra_empty);
    a = stageA_read(c);
    if (!(a.bits & F_A_OVER)) break;
    cap = a.maxreg + a.maxreg / 8 + 512;
  }
  if (a.bits & F_A_OVER) throw Error(-12, "build_dbg: stage A regions overflowed");
  c.ms_insert = c.t1.ms();
  c.sentinel = a.sentinel ? 1 : 0;
  c.n_records_a = a.total;
  if (hold) {                                       // the records stay in their regions for their owners
    const unsigned long long* h = c.h_pin.as<unsigned long long>();   // (stageA_read's copy of the cursors)
    const unsigned* hf = reinterpret_cast<const unsigned*>(c.h_pin.as<uint8_t>() + 8 * CSTRIDE * NREG);   // (flags)
    c.work_items = (uint64_t)hf[F_WORK_ITEMS] | ((uint64_t)hf[F_WORK_ITEMS + 1] << 32);
    c.route_reg.assign(NREG, 0);
    for (int r = 0; r < NREG; ++r) c.route_reg[r] = std::min<uint64_t>(h[CSTRIDE * r], c.capA);
    c.route_total = a.total;
    if (c.windows_fw) c.u_ratio = (double)a.total / (double)c.windows_fw;   // (the next held stage A's regions)
    c.route_maxreg = a.maxreg;
    c.route_maxbin = a.maxbin;
    c.route_sentinel = a.sentinel;
    c.route_ready = true;
    return;
  }
  finish_build(c, a, false);
  if (c.windows_fw) c.u_ratio = (double)a.total / (double)c.windows_fw;
}

// ---- routed exchange.  The owner of a stage A record is the top lg bits of
// its coarse bin (the top bits of h = perm(key)): with 2^lg owners, owner o
// holds bins [o, o + 1) << (cbits - lg), i.e. regions of consecutive indices,
// so routing is a segmented copy of whole regions, not a per-record split.
// An owner builds its table over h rotated left by lg bits (TableView.rot):
// its keys, whose top lg bits of h are all o, then spread over the whole
// bucket space and the table is sized from the owner's own records.
static int route_owner(const Ctx& c, int region, int lg) { return (region / 8) >> (c.cbits - lg); }
static void route_check(const Ctx& c, int lg, const char* what) {
  if (!c.route_ready) throw Error(-22, std::string(what) + ": no held stage A (pg_route_stage_a)");
  if (lg < 0 || lg > c.cbits) throw Error(-22, std::string(what) + ": owners must be a power of two <= 2^cbits");
}
void route_counts(Ctx& c, int lg, uint64_t* counts) {
  route_check(c, lg, "route_counts");
  for (int o = 0; o < (1 << lg); ++o) counts[o] = 0;
  for (int r = 0; r < NREG; ++r) counts[route_owner(c, r, lg)] += c.route_reg[r];
}

// rows of region blockIdx.y (records [0, roff[r+1] - roff[r]) of it) to
// out + roff[r] as 12-byte rows {h, mask word} (Row12), and the block's row_check
// sum as a plain store to part[blockIdx.y * gridDim.x + blockIdx.x] (the
// host adds them per owner: one atomic per block on a few owner words
// serialised ~100 K atomics, 0.68 ms at world 1 on C3)
constexpr int RS_ROWS = 16;                    // rows per thread and block pass
__global__ void __launch_bounds__(256) k_route_scatter(const unsigned long long* __restrict__ key,
                                                       const uint32_t* __restrict__ mw, uint64_t cap,
                                                       const unsigned long long* __restrict__ roff, Row12* __restrict__ out,
                                                       unsigned long long* __restrict__ part) {
  __shared__ unsigned long long s_red[4];
  const uint32_t r = blockIdx.y;
  const uint64_t o0 = roff[r], nr = roff[r + 1] - o0;
  unsigned long long acc = 0ull;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nr; i += (uint64_t)gridDim.x * 256ull) {
    const unsigned long long h = key[(uint64_t)r * cap + i];
    const uint32_t m = mw[(uint64_t)r * cap + i];
    out[o0 + i] = Row12{{(uint32_t)h, (uint32_t)(h >> 32), m}};
    acc += row_check(h, (uint64_t)m);
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[(uint64_t)blockIdx.y * gridDim.x + blockIdx.x] = s_red[0] + s_red[1] + s_red[2] + s_red[3];
}

void route_scatter(Ctx& c, int lg, void* d_out, uint64_t out_cap, uint64_t* sums) {
  route_check(c, lg, "route_scatter");
  const int np = 1 << lg;
  uint64_t tot = 0, mx = 0;
  for (int r = 0; r < NREG; ++r) {
    tot += c.route_reg[r];
    mx = std::max<uint64_t>(mx, c.route_reg[r]);
  }
  if (out_cap < tot) throw Error(-22, "route_scatter: output buffer too small");
  const unsigned gx = grid_for(mx, 256 * RS_ROWS, 64);
  const size_t nw = (NREG + 1) + (size_t)NREG * gx;
  c.route_buf.reserve(8 * nw);
  c.route_pin.reserve(8 * nw);
  auto* h = c.route_pin.as<unsigned long long>();
  tot = 0;
  for (int r = 0; r < NREG; ++r) {
    h[r] = tot;
    tot += c.route_reg[r];
  }
  h[NREG] = tot;
  auto* d = c.route_buf.as<unsigned long long>();
  PG_HIP(hipMemcpyAsync(d, h, 8 * (NREG + 1), hipMemcpyHostToDevice, c.stream));
  for (int o = 0; o < np; ++o) sums[o] = 0;
  if (tot) {
    hipLaunchKernelGGL(k_route_scatter, dim3(gx, NREG), dim3(256), 0, c.stream, c.recA_key.as<unsigned long long>(),
                       c.recA_mw.as<uint32_t>(), c.capA, d, reinterpret_cast<Row12*>(d_out), d + NREG + 1);
    PG_HIP(hipGetLastError());
    PG_HIP(hipMemcpyAsync(h + NREG + 1, d + NREG + 1, 8 * (size_t)NREG * gx, hipMemcpyDeviceToHost, c.stream));
  }
  c.sync();
  if (tot)
    for (int r = 0; r < NREG; ++r) {
      uint64_t t = 0;
      for (unsigned j = 0; j < gx; ++j) t += h[NREG + 1 + (size_t)r * gx + j];
      sums[route_owner(c, r, lg)] += t;
    }
}

// the held records are the owner's (every owner is this rank: world 1):
// stages B and C on them where they lie
void route_finish(Ctx& c) {
  route_check(c, 0, "route_finish");
  c.route_ready = false;
  init_hash(c);
  ACount a;
  a.total = c.route_total;
  a.maxreg = c.route_maxreg;
  a.maxbin = c.route_maxbin;
  a.sentinel = c.route_sentinel;
  c.sentinel = a.sentinel ? 1 : 0;
  finish_build(c, a, false);
  if (c.windows_fw) c.u_ratio = (double)a.total / (double)c.windows_fw;
}

void build_rdbg(Ctx& c) {
  if (!c.built) throw Error(-22, "build_rdbg: no dBG (call pg_build_dbg first)");
  // the degree scan runs inside the build (k_build_range): nothing left to do
}

uint64_t export_dbg(Ctx& c, uint64_t* h_keys, uint16_t* h_masks, uint64_t cap) {
  if (!c.built) throw Error(-22, "export_dbg: no dBG");
  const uint64_t nmax = 2 * c.n_canon + 1;
  const uint64_t ntot = 2 * c.cap + c.ovf_cap;
  DevBuf keys, masks, cnt;
  keys.reserve(8 * nmax);
  masks.reserve(2 * nmax);
  cnt.reserve(8);
  PG_HIP(hipMemsetAsync(cnt.p, 0, 8, c.stream));
  hipLaunchKernelGGL(k_export_dbg, dim3(grid_for(ntot, 256 * EXE, 8192)), dim3(256), 0, c.stream, c.tv, 2 * c.cap, ntot,
                     c.k, keys.as<unsigned long long>(), masks.as<unsigned short>(), nmax, cnt.as<unsigned long long>());
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
    // sorted by key on the device (the sentinel, 2^64 - 1, last)
    DevBuf k2, m2, tmp;
    k2.reserve(8 * (n + 1));
    m2.reserve(2 * (n + 1));
    size_t bytes = 0;
    PG_HIP(rocprim::radix_sort_pairs(nullptr, bytes, keys.as<unsigned long long>(), k2.as<unsigned long long>(),
                                     masks.as<unsigned short>(), m2.as<unsigned short>(), (size_t)n, 0, c.kb,
                                     c.stream));
    tmp.reserve(bytes + 16);
    bytes = tmp.cap;
    PG_HIP(rocprim::radix_sort_pairs(tmp.p, bytes, keys.as<unsigned long long>(), k2.as<unsigned long long>(),
                                     masks.as<unsigned short>(), m2.as<unsigned short>(), (size_t)n, 0, c.kb,
                                     c.stream));
    PG_HIP(hipMemcpyAsync(h_keys, k2.p, 8 * n, hipMemcpyDeviceToHost, c.stream));
    PG_HIP(hipMemcpyAsync(h_masks, m2.p, 2 * n, hipMemcpyDeviceToHost, c.stream));
    c.sync();
    if (c.sentinel) { h_keys[n] = SENTINEL; h_masks[n] = 32; }
  }
  keys.release(); masks.release(); cnt.release();
  return total;
}

uint64_t export_rdbg(Ctx& c, uint64_t* h_keys, uint64_t cap) {
  if (!c.reduced) throw Error(-22, "export_rdbg: no rdBG (call pg_build_rdbg first)");
  if (h_keys && cap >= c.n_rdbg) {
    // the blocks' segments gathered on the device into one run, one copy back
    const uint64_t nseg = c.rseg_nseg, n = c.n_rdbg - c.sentinel;
    std::vector<unsigned long long> off(nseg + 1, 0);
    for (uint64_t s = 0; s < nseg; ++s) off[s + 1] = off[s] + c.rseg_cnt[s];
    DevBuf d_off, out;
    d_off.reserve(8 * (nseg + 1));
    out.reserve(8 * std::max<uint64_t>(n, 1));
    c.h_pin.reserve(8 * (nseg + 1));
    std::memcpy(c.h_pin.p, off.data(), 8 * (nseg + 1));
    PG_HIP(hipMemcpyAsync(d_off.p, c.h_pin.p, 8 * (nseg + 1), hipMemcpyHostToDevice, c.stream));
    if (n) {
      hipLaunchKernelGGL(k_gather_segs, dim3((unsigned)nseg), dim3(256), 0, c.stream, c.rseg.as<unsigned long long>(),
                         c.rseg_cap, d_off.as<unsigned long long>(), out.as<unsigned long long>());
      PG_HIP(hipGetLastError());
      DevBuf k2, tmp;                                   // sorted on the device
      k2.reserve(8 * n);
      size_t bytes = 0;
      PG_HIP(rocprim::radix_sort_keys(nullptr, bytes, out.as<unsigned long long>(), k2.as<unsigned long long>(),
                                      (size_t)n, 0, c.kb, c.stream));
      tmp.reserve(bytes + 16);
      bytes = tmp.cap;
      PG_HIP(rocprim::radix_sort_keys(tmp.p, bytes, out.as<unsigned long long>(), k2.as<unsigned long long>(),
                                      (size_t)n, 0, c.kb, c.stream));
      PG_HIP(hipMemcpyAsync(h_keys, k2.p, 8 * n, hipMemcpyDeviceToHost, c.stream));
      c.sync();
    }
    c.sync();
    d_off.release();
    out.release();
    if (c.sentinel) h_keys[n] = SENTINEL;
  }
  return c.n_rdbg;
}

// part_cnt words: [0, 64) counts, [64, 128) cursors, [PCW_SUMS, +64 * CSPR)
// the partition sums, [PCW_ROWS, +RS_SEG * CSPR) rows_checksum's sums
constexpr size_t PCW_SUMS = 128, PCW_ROWS = PCW_SUMS + 64 * CSPR;
uint64_t partition_dbg(Ctx& c, int nparts, void* d_out, uint64_t out_cap, uint64_t* h_counts) {
  if (!c.built) throw Error(-22, "partition_dbg: no dBG");
  if (nparts < 1 || nparts > 64) throw Error(-22, "partition_dbg: nparts must be in [1, 64]");
  const uint64_t ntot = 2 * c.cap + c.ovf_cap;
  DevBuf& cnt = c.part_cnt;                             // [0, 64) counts, [64, 128) cursors, then the sums
  cnt.reserve(8 * PCW_ROWS);
  auto* counts = cnt.as<unsigned long long>();
  c.h_pin.reserve(8 * PCW_ROWS);
  auto* h = c.h_pin.as<unsigned long long>();
  if (!d_out) {                                         // count pass
    PG_HIP(hipMemsetAsync(cnt.p, 0, 8 * 64, c.stream));
    hipLaunchKernelGGL(k_part_count, dim3(grid_for(ntot, 256, 4096)), dim3(256), 0, c.stream, c.tv, 2 * c.cap, ntot,
                       nparts, counts);
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
  if (c.part_gen != c.build_gen || c.part_nparts != nparts)
    throw Error(-22, "partition_dbg: call with d_out = NULL (count pass) first");
  uint64_t total = 0;
  for (int i = 0; i < nparts; ++i) { h[64 + i] = total; total += c.part_counts[i]; h_counts[i] = c.part_counts[i]; }
  if (out_cap < total) throw Error(-22, "partition_dbg: output buffer too small");
  for (int i = 0; i < 64; ++i) c.part_sums[i] = 0;
  if (total) {
    const size_t sw = (size_t)nparts * CSPR;
    for (size_t i = 0; i < sw; ++i) h[PCW_SUMS + i] = 0;
    PG_HIP(hipMemcpyAsync(counts + 64, h + 64, 8 * (64 + sw), hipMemcpyHostToDevice, c.stream));  // cursors, zeroed sums
    hipLaunchKernelGGL(k_part_scatter, dim3(grid_for(ntot, PCH, 4096)), dim3(PT), 0, c.stream, c.tv, 2 * c.cap, ntot,
                       nparts, counts + 64, reinterpret_cast<Slot*>(d_out), counts + PCW_SUMS);
    PG_HIP(hipGetLastError());
    PG_HIP(hipMemcpyAsync(h + PCW_SUMS, counts + PCW_SUMS, 8 * sw, hipMemcpyDeviceToHost, c.stream));
    c.sync();
    for (int i = 0; i < nparts; ++i)
      for (int j = 0; j < CSPR; ++j) c.part_sums[i] += h[PCW_SUMS + (size_t)i * CSPR + j];
  }
  return total;
}

// Sums of row_check over nseg segments of 16-byte records at d_rows
// (segment s = records [off[s], off[s+1])), on the context's stream.
void rows_checksum(Ctx& c, const void* d_rows, const uint64_t* off, uint64_t nseg, uint64_t* sums, bool row12) {
  DevBuf& out = c.part_cnt;                             // (after the partition words)
  out.reserve(8 * (PCW_ROWS + RS_SEG * CSPR));
  auto* d = out.as<unsigned long long>() + PCW_ROWS;
  c.h_pin.reserve(8 * RS_SEG * CSPR);
  auto* h = c.h_pin.as<unsigned long long>();
  for (uint64_t s0 = 0; s0 < nseg; s0 += RS_SEG) {
    const uint32_t ns = (uint32_t)std::min<uint64_t>(RS_SEG, nseg - s0);
    SegOff so{};
    uint64_t mx = 0;
    for (uint32_t s = 0; s <= ns; ++s) so.o[s] = off[s0 + s];
    for (uint32_t s = 0; s < ns; ++s) {
      if (so.o[s + 1] < so.o[s]) throw Error(-22, "rows_checksum: segment offsets decrease");
      mx = std::max<uint64_t>(mx, so.o[s + 1] - so.o[s]);
    }
    PG_HIP(hipMemsetAsync(d, 0, 8 * RS_SEG * CSPR, c.stream));
    if (mx) {
      if (row12)
        hipLaunchKernelGGL(k_rows_sum<Row12>, dim3(grid_for(mx, 256, 2048), ns), dim3(256), 0, c.stream,
                           reinterpret_cast<const Row12*>(d_rows), so, d);
      else
        hipLaunchKernelGGL(k_rows_sum<Slot>, dim3(grid_for(mx, 256, 2048), ns), dim3(256), 0, c.stream,
                           reinterpret_cast<const Slot*>(d_rows), so, d);
      PG_HIP(hipGetLastError());
    }
    PG_HIP(hipMemcpyAsync(h, d, 8 * (size_t)ns * CSPR, hipMemcpyDeviceToHost, c.stream));
    c.sync();
    for (uint32_t s = 0; s < ns; ++s) {
      uint64_t t = 0;
      for (int j = 0; j < CSPR; ++j) t += h[(size_t)s * CSPR + j];
      sums[s0 + s] = t;
    }
  }
}

// OR-merge received exchange records into a fresh owner table (stage A from
// the records, then stages B and C as a build).
// rot >= 0 (pg_route_merge): the rows are routed stage A records (12-byte
// Row12 {h, mask word}) of this owner, re-binned on h rotated left by rot bits.
void merge_dbg(Ctx& c, const void* d_pairs, uint64_t n, uint64_t /*cap_hint*/, int sentinel, int rot) {
  merge_dbg_segs(c, &d_pairs, &n, 1, sentinel, rot);
}

// The same merge over nseg segments of rows (segment s: ns[s] rows at
// segs[s]), emitted into one stage A: a routed owner's sub-log as the runs it
// received round by round, with no device-side concatenation.
void merge_dbg_segs(Ctx& c, const void* const* segs, const uint64_t* ns, int nseg, int sentinel, int rot) {
  init_hash(c, rot > 0 ? (uint32_t)rot : 0u);
  c.route_ready = false;
  c.early_split_used = false;
  uint64_t n = 0;
  for (int s = 0; s < nseg; ++s) n += ns[s];
  uint64_t cap = region_cap(n + 64);
  ACount a;
  // every record count is known here (n): stages B/C go right behind stage A
  // (finish_build's spec form, one host round trip), unless a region overflows
  auto enqueue = [&](uint64_t rcap) {
    FillList fl;
    const BinOut O = stageA_begin(c, rcap, fl);
    c.t1.init();
    c.t1.start(c.stream);
    fl.launch(c.stream);
    PG_HIP(hipEventRecord(c.ev[0], c.stream));           // the side stream (stage B/C fills) after all of this
    PG_HIP(hipStreamWaitEvent(c.stream2, c.ev[0], 0));
    if (sentinel) hipLaunchKernelGGL(k_set_flag, dim3(1), dim3(1), 0, c.stream, c.flags.as<unsigned>());
    for (int s = 0; s < nseg; ++s) {
      if (!ns[s]) continue;
      if (rot >= 0)
        hipLaunchKernelGGL(k_route_emit, dim3(grid_for(ns[s], 4 * IBLOCK, 4096)), dim3(IBLOCK), 0, c.stream,
                           reinterpret_cast<const Row12*>(segs[s]), ns[s], c.tv, O,
                           c.flags.as<unsigned long long>() + N_FLAGS / 2);
      else
        hipLaunchKernelGGL(k_slots_emit, dim3(grid_for(ns[s], 4 * IBLOCK, 4096)), dim3(IBLOCK), 0, c.stream,
                           reinterpret_cast<const Slot*>(segs[s]), ns[s], c.tv, O,
                           c.flags.as<unsigned long long>() + N_FLAGS / 2);
      PG_HIP(hipGetLastError());
    }
    c.t1.stop(c.stream);
  };
  enqueue(cap);
  a.total = n + (sentinel ? 1 : 0);
  a.maxreg = cap;
  a.maxbin = 8 * cap;
  const bool ok = finish_build(c, a, true);
  c.ms_insert = c.t1.ms();
  c.n_records_a = a.total;
  if (ok) return;
  cap = a.maxreg + a.maxreg / 8 + 512;              // every region's exact count is known now
  for (int attempt = 0; attempt < 3; ++attempt) {
    enqueue(cap);
    a = stageA_read(c);
    if (!(a.bits & F_A_OVER)) break;
    cap = a.maxreg + a.maxreg / 8 + 512;
  }
  if (a.bits & F_A_OVER) throw Error(-12, "merge_dbg: stage A regions overflowed");
  c.ms_insert = c.t1.ms();
  c.sentinel = a.sentinel ? 1 : 0;
  c.n_records_a = a.total;
  finish_build(c, a, false);
}

// pg_build_host: K1 over the chunked upload, and stage A streamed under it.
// After each chunk's K1 the host gets the records completed so far; the
// first time there are three long ones, stage A starts with the usual lead
// and second reference among them (SA_FIRST), and every later batch of
// completed records goes through the coverage / emission pass as followers of
// those two (SA_MORE); the short records, once the record table is final
// (SA_TAIL).  Stages B and C then run from stage A's exact counts.  The
// choice of references only decides how much the coverage pass skips, never
// what is inserted, so the table is the one pg_build makes.  A stage A
// region overflow (the regions are sized from the file before the records
// are known), or more records than the parse could stream, falls back to
// pg_build over the parsed records.
void build_host(Ctx& c, const uint8_t* h_src, uint64_t n, int rc0) {
  c.rc0 = rc0;
  c.built = c.reduced = false;
  c.n_dbg = c.n_rdbg = c.n_canon = 0;
  init_hash(c);
  // regions for ~ the last build's records per base (the file's bytes bound
  // the bases), or a quarter record per byte on a first build
  const uint64_t est = c.u_ratio > 0 ? (uint64_t)(c.u_ratio * 1.25 * (double)n) : n / 4;
  const uint64_t cap = region_cap(std::min<uint64_t>(est, n) + 4096);
  uint64_t done = 0;
  bool started = false, broken = c.n_preload != 0;
  c.t1.init();
  // Stage B under the upload: after each chunk's stage A share, the records
  // it added are split into the table's fine partitions (k_split from the
  // stage A cursors' last snapshot, on the main stream, where no stage A
  // kernel runs beside it), so that after the last chunk only its own records
  // are left to split.  The geometry comes from the last build (records per
  // window, windows per byte); at the end finish_build uses the partitions if
  // the exact count gives the same table and nothing overflowed, and splits
  // everything again from stage A's regions (still intact) otherwise.
  Presplit pre{-1, 0u, 0};
  uint32_t pre_bpr = 1;
  if (c.early_split && c.u_ratio > 0 && c.w_ratio > 0 && !broken) {
    const uint64_t est = (uint64_t)(c.u_ratio * c.w_ratio * (double)n) + 4096;
    int bb, fp;
    table_bits(c, est, bb, fp);
    if (fp > c.cbits && fp - c.cbits <= SPLIT_BITS) {
      pre.bb = bb;
      pre.S = (uint32_t)(fp - c.cbits);
      const uint64_t maxbin = est / NBIN + est / (NBIN * 8) + 1024;      // bins are even: h is a bijective hash
      pre.cap = (uint64_t)((double)maxbin / (double)(1u << pre.S) * 1.3) + 256;
      const uint64_t recs = (1ull << c.cbits) * (1ull << pre.S) * pre.cap;
      c.recS_key[0].reserve(8 * recs);
      c.recS_mw[0].reserve(4 * recs);
      c.ctrS.reserve(8 * CSTRIDE * (1ull << fp));
      c.snapA.reserve(8 * NREG);
      pre_bpr = 2;
    }
  }
  bool pre_started = false;
  auto early_split = [&]() {
    if (pre.bb < 0) return;
    if (!pre_started) {
      PG_HIP(hipMemsetAsync(c.ctrS.p, 0, 8 * CSTRIDE * (1ull << (c.cbits + pre.S)), c.stream));
      PG_HIP(hipMemsetAsync(c.snapA.p, 0, 8 * NREG, c.stream));
      pre_started = true;
    }
    const Recs in{c.recA_key.as<unsigned long long>(), c.recA_mw.as<uint32_t>(), c.ctrA.as<unsigned long long>(),
                  c.capA, 8};
    const Recs out{c.recS_key[0].as<unsigned long long>(), c.recS_mw[0].as<uint32_t>(),
                   c.ctrS.as<unsigned long long>(), pre.cap, 1};
    hipLaunchKernelGGL(k_split<true>, dim3((unsigned)(NREG * pre_bpr)), dim3(SB),   // (chunks of a pg_build_host)
                       0, c.stream, in, out,
                       c.snapA.as<unsigned long long>(), (uint32_t)(c.kb - c.cbits - (int)pre.S), 1u << pre.S, pre_bpr,
                       c.flags.as<unsigned>());
    PG_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_snap, dim3((NREG + 255) / 256), dim3(256), 0, c.stream, c.ctrA.as<unsigned long long>(),
                       c.snapA.as<unsigned long long>(), (uint32_t)NREG);
    PG_HIP(hipGetLastError());
  };
  // the record table is final: every record flagged for the short-record pass
  auto final_records = [&]() {
    const uint64_t R = c.n_records;
    if (R) PG_HIP(hipMemsetAsync(c.rec_flag.p, 1, R, c.stream));
    c.dev_flag.assign(R, 1);
    c.dev_flag_p = c.rec_flag.p;
    c.windows_fw = 0;
    for (uint64_t r = 0; r < R; ++r) {
      const int64_t m = c.h_rec_len[r];
      c.windows_fw += m > c.k ? (uint64_t)(m - c.k + 1) : 1;
    }
    c.windows_total = c.windows_fw * (rc0 ? 2 : 1);
    c.last_flag.assign(R, 1);
    c.last_extra = 0;
    c.dump_ready = false;
  };
  bool tail_done = false;
  std::function<void(uint64_t)> on_chunk = [&](uint64_t rc) {
    if (broken) return;
    if (rc == ~0ull) { broken = true; return; }               // the parse could not stream
    if (rc <= done) return;
    std::vector<uint8_t> flag(c.n_records, 0);
    uint64_t nlong = 0;
    for (uint64_t r = done; r < rc; ++r) {
      flag[r] = 1;
      nlong += c.h_rec_len[r] >= c.k + 2;
    }
    // the last batch (the record table final: every record counted) also
    // takes the short records - one stage A call and one split fewer after
    // the last chunk
    const bool final_call = c.parsed && rc == c.n_records;
    if (final_call) final_records();
    if (!started) {
      if (nlong < 3 && !final_call) return;                   // wait for three long records
      const uint64_t nt = make_tiles(c, flag);
      enqueue_stageA(c, cap, nt, rc0, 0, final_call ? SA_FIRST_TAIL : SA_FIRST);
      started = true;
      tail_done = final_call;
      early_split();
    } else {
      const uint64_t nt = make_tiles(c, flag, true);
      if (nt || final_call) {
        enqueue_stageA(c, cap, nt, rc0, 0, final_call ? SA_MORE_TAIL : SA_MORE);
        tail_done = final_call;
        early_split();
      }
    }
    done = rc;
  };
  parse_fasta(c, h_src, &on_chunk);
  const uint64_t R = c.n_records;
  std::vector<uint8_t> all(R, 1);
  if (!broken && (done != R || !started)) broken = true;
  if (!broken) {
    if (!tail_done) {
      final_records();
      enqueue_stageA(c, cap, 0, rc0, 0, SA_TAIL);
      if (pre_started) early_split();                         // the short records
    }
    if (pre_started) {
      // stage C queued right behind the last split, with no host round trip
      // (finish_build's spec form: the table from the early split's plan;
      // stage A's exact counts and every flag come back with the build's one
      // readback - a split overflow re-runs B/C from stage A's regions, a
      // stage A overflow the whole build)
      ACount a;
      a.total = (uint64_t)(c.u_ratio * c.w_ratio * (double)n) + 4096;          // the early split's plan
      a.total = std::max<uint64_t>(a.total, (uint64_t)(c.u_ratio * 1.02 * (double)c.windows_fw) + 4 * R + 64);
      {
        int bbp, fpp;                          // (never past the plan's table: its partitions are what is split)
        table_bits(c, a.total, bbp, fpp);
        if (bbp != pre.bb) a.total = (uint64_t)(c.u_ratio * c.w_ratio * (double)n) + 4096;
      }
      a.maxreg = cap;
      a.maxbin = 8 * cap;
      if (finish_build(c, a, true, &pre)) {
        c.ms_insert = c.t1.ms();
        c.ms_clear = 0;
        c.n_records_a = a.total;
        if (c.windows_fw) c.u_ratio = (double)a.total / (double)c.windows_fw;
        if (n) c.w_ratio = (double)c.windows_fw / (double)n;
        c.tile_sig_len.clear();
        return;
      }
    } else {
      ACount a = stageA_read(c);
      if (!(a.bits & F_A_OVER)) {
        c.ms_insert = c.t1.ms();
        c.ms_clear = 0;
        c.sentinel = a.sentinel ? 1 : 0;
        c.n_records_a = a.total;
        finish_build(c, a, false);
        if (c.windows_fw) c.u_ratio = (double)a.total / (double)c.windows_fw;
        if (n) c.w_ratio = (double)c.windows_fw / (double)n;
        c.tile_sig_len.clear();                               // (the tile list holds the last batch only)
        return;
      }
    }
  }
  c.tile_sig_len.clear();
  build_dbg(c, all.data(), 0, rc0);
}

}  // namespace pg
