// pg_parse.hip — K1: FASTA bytes in HBM -> record table + one class code per base.
//
// Restates readline_jit_ (kmer_numba.py:122-132) and seqio_jit_ (:135-172).
// The byte stream is read twice, streaming, 16 bytes per lane:
//
//   k_span_sum   one wave per 16 KiB span.  Newline / header counts, the last
//                two newline positions, and the span's content-byte count as a
//                function of its in-state (is the line open at the span start
//                a header line?) with the out-state it leaves behind.
//   scan         rocPRIM inclusive scan composing those 2-state functions:
//                every span's output offset, in-state and first record index.
//   k_emit       one wave per span again: each content byte -> its class code at
//                its compacted offset (staged per step in the wave's own LDS
//                slice, written with aligned 16-byte stores); each header's
//                byte span and record start.  No block-wide barrier.
//   k_records    record lengths and seqio's `ptr` value.
//   k_pack_fix   the packed base stream's words at span boundaries (below).
//
// Besides the class bytes K1 writes the packed base stream K3's coverage
// pass reads (north_star's "2-bit encode"): one 32-bit word per 16 bases,
// base j's class & 3 in bits 2j..2j+1 (A0 C1 G2 T3), and one exception byte
// per 16 bases, nonzero when any of them is not ACGT (N, '$', other: the
// 2-bit code is then not the class).  k_emit packs every 16-byte chunk it
// writes whole; a chunk that two spans share is packed by k_pack_fix from
// the class bytes once both spans are emitted.
//
// Line semantics (kmer_numba.py:126-132): a line starts at 0 and after every
// '\n'; it ends at its '\n', or, for a final unterminated line, at byte n-1
// when `end > start > 0` — its last byte then plays the terminator's role
// (line[:-1], :160/:167).  So byte n-1 is never a base, a line starting at n-1
// without '\n' is no line, and a base is any byte < n-1 that is not '\n' and
// whose line does not start with '>' (:155).  Lines before the first header
// land in front of record 0 in the compacted stream and belong to no record
// (:156-161, qid[0] != 62).  A file without any '\n' has no lines at all.
#include <chrono>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include <mutex>

#include <memory>

#include "pg_internal.h"

namespace pg {

constexpr int PBLOCK = 256;                       // threads per block (4 waves)
constexpr int WAVES = PBLOCK / 64;
constexpr int WSTEP = 64 * 16;                    // 1 KiB per wave step (16 B per lane)
constexpr int WSTEPS = 16;
constexpr uint64_t WSPAN = (uint64_t)WSTEP * WSTEPS;   // 16 KiB per wave
// load the 16 bytes at p (16-byte aligned); bytes at or past n read as 0
// The FASTA is read with non-temporal loads (it is read twice, but 508 MB of
// C3 does not stay cached between the passes): C3 k_span_sum 0.164 -> 0.100
// ms, k_emit 0.194 either way (rocprofv3 medians, profiles/r06_ab_range_split.log)
#ifndef PG_K1_NT
#define PG_K1_NT 3                                     // bit 0: span pass, bit 1: emission (experiment builds)
#endif
template <bool NT = false>
__device__ __forceinline__ uint4 load16(const uint8_t* buf, uint64_t p, uint64_t n) {
  if (NT && p + 16 <= n) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(buf + p));
    return make_uint4(x.x, x.y, x.z, x.w);
  }
  if (p + 16 <= n) return *reinterpret_cast<const uint4*>(buf + p);
  uint32_t w[4] = {0, 0, 0, 0};
  for (int j = 0; j < 16; ++j)
    if (p + j < n) w[j >> 2] |= (uint32_t)buf[p + j] << (8 * (j & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// bit j (0..3) set iff byte j of w equals the replicated byte in pat (exact SWAR)
__device__ __forceinline__ uint32_t eq4(uint32_t w, uint32_t pat) {
  const uint32_t x = w ^ pat;
  const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
  return ((z >> 7) | (z >> 14) | (z >> 21) | (z >> 28)) & 0xFu;
}
__device__ __forceinline__ uint32_t eq16(const uint4& v, uint32_t pat) {
  return eq4(v.x, pat) | eq4(v.y, pat) << 4 | eq4(v.z, pat) << 8 | eq4(v.w, pat) << 12;
}
// bit 7 of every byte of w that equals the replicated byte in pat
__device__ __forceinline__ uint32_t zmatch(uint32_t w, uint32_t pat) {
  const uint32_t x = w ^ pat;
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}
// zmatch's byte bits (7, 15, 23, 31) packed into bits 0..3: the four
// partial products land on distinct bit positions, so nothing carries
__device__ __forceinline__ uint32_t pack4(uint32_t z) { return (z * 0x00204081u) >> 28; }

// Fast-path view of one lane's 16 bytes: the '\n' mask, whether a '>' is
// among them, and the class codes of the bytes when every byte but '\n' is
// one of ACGTacgt (`acgt`).  u = the byte with bit 5 cleared (a -> A ...);
// t = (u >> 1) & 3 maps A C T G to 0 1 2 3, so u is ACGT iff the byte of
// "ACTG" at t equals u, and the class (A0 C1 G2 T3) is t ^ (t >> 1).
// '\n' bytes are checked as 'A' (they are dropped anyway).
struct FastLane {
  uint32_t nlm, cls[4];
  bool gt, acgt;
};
__device__ __forceinline__ FastLane fast_lane(const uint4& v) {
  static_assert(CLS_A == 0 && CLS_C == 1 && CLS_G == 2 && CLS_T == 3, "class codes of ACGT");
  FastLane f;
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t gt = 0, bad = 0;
  f.nlm = 0;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t zn = zmatch(w[d], 0x0A0A0A0Au);
    gt |= zmatch(w[d], 0x3E3E3E3Eu);
    f.nlm |= pack4(zn) << (4 * d);
    const uint32_t bm = zn | (zn - (zn >> 7));                 // 0xFF on the '\n' bytes
    const uint32_t u = ((w[d] & ~bm) | (0x41414141u & bm)) & 0xDFDFDFDFu;
    const uint32_t t = (u >> 1) & 0x03030303u;
    bad |= __builtin_amdgcn_perm(0u, 0x47544341u, t) ^ u;
    f.cls[d] = t ^ ((t >> 1) & 0x01010101u);
  }
  f.gt = gt != 0u;
  f.acgt = bad == 0u;
  return f;
}

// bits of the lane's 16 positions below `lim`
__device__ __forceinline__ uint32_t below_mask(uint64_t p, uint64_t lim) {
  return p + 16 <= lim ? 0xFFFFu : (p < lim ? (1u << (uint32_t)(lim - p)) - 1u : 0u);
}

// Header-line bytes of a lane: from each header start (or bit 0 when the lane
// continues a header line) through the first '\n' at or after it.  Header
// starts always follow a '\n', so the borrow chains of E - hs never overlap.
__device__ __forceinline__ uint32_t header_region(uint32_t nlm, uint32_t hs) {
  const uint32_t E = nlm | 0x10000u;
  return ((E - hs) ^ E) & 0xFFFFu;
}

// DPP inclusive prefix sum over the 64 lanes (all lanes active)
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);   // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);   // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);   // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);   // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);   // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);   // row_bcast:31
  return x;
}
__device__ __forceinline__ int wave_max_i32(int x) {
  for (int o = 32; o > 0; o >>= 1) {
    const int y = __shfl_xor(x, o, 64);
    x = y > x ? y : x;
  }
  return x;
}

// Per-lane view of one 16-byte step; `carry_nl` is the byte before the step
// (or BOF) being '\n', updated for the next step.
struct LaneStep {
  uint32_t nlm, lsm, hs, vn1;
  uint64_t B, H;          // lanes holding a line start / whose last line start is a header
  uint64_t lt;            // lanes below this one
};
__device__ __forceinline__ LaneStep lane_step(const uint4& v, uint64_t p, uint64_t n, int lane,
                                              uint32_t& carry_nl) {
  LaneStep s;
  s.nlm = eq16(v, 0x0A0A0A0Au);
  const uint32_t gtm = eq16(v, 0x3E3E3E3Eu);
  const uint64_t Bnl = __ballot((s.nlm >> 15) & 1u);
  const uint32_t prev = lane ? (uint32_t)(Bnl >> (lane - 1)) & 1u : carry_nl;
  carry_nl = (uint32_t)(Bnl >> 63) & 1u;
  s.vn1 = below_mask(p, n - 1);
  s.lsm = ((s.nlm << 1) | prev) & below_mask(p, n);
  s.hs = s.lsm & gtm & s.vn1;
  const bool has = s.lsm != 0;
  const bool lh = has && ((s.hs >> (31 - __builtin_clz(s.lsm | 1u))) & 1u);
  s.B = __ballot(has);
  s.H = __ballot(lh);
  s.lt = (1ull << lane) - 1ull;
  return s;
}
// in-state of the lane given the step's in-state
__device__ __forceinline__ uint32_t lane_in(const LaneStep& s, uint32_t step_in) {
  const uint64_t below = s.B & s.lt;
  return below ? (uint32_t)(s.H >> (63 - __builtin_clzll(below))) & 1u : step_in;
}
__device__ __forceinline__ uint32_t step_out(const LaneStep& s, uint32_t step_in) {
  return s.B ? (uint32_t)(s.H >> (63 - __builtin_clzll(s.B))) & 1u : step_in;
}
__device__ __forceinline__ uint32_t lane_region(const LaneStep& s, uint32_t in) {
  return header_region(s.nlm, s.hs | ((in && !(s.lsm & 1u)) ? 1u : 0u));
}
__device__ __forceinline__ uint32_t lane_content(const LaneStep& s, uint32_t region) {
  return ~s.nlm & ~region & s.vn1 & 0xFFFFu;
}

// A span sequence as a function of its in-state (is the line open before it
// a header line?): bases emitted and out-state for in-state 0 / 1, plus
// newline / header counts and the last two newline positions.
struct Fn {
  unsigned long long c0, c1, nl, hdr;
  long long last, last2;
  uint32_t o;                                       // bit s: out-state for in-state s
};
constexpr uint32_t FN_TODO = 0xFFFFFFFFu;           // (o: a span k_span_whole left to k_span_fix)
__host__ __device__ __forceinline__ Fn fn_identity() { return Fn{0, 0, 0, 0, -1, -1, 2u}; }
struct FnThen {                                     // a, then b (associative, not commutative)
  __host__ __device__ __forceinline__ Fn operator()(const Fn& a, const Fn& b) const {
    const uint32_t a0 = a.o & 1u, a1 = (a.o >> 1) & 1u;
    Fn r;
    r.c0 = a.c0 + (a0 ? b.c1 : b.c0);
    r.c1 = a.c1 + (a1 ? b.c1 : b.c0);
    r.o = ((b.o >> a0) & 1u) | ((b.o >> a1) & 1u) << 1;
    r.nl = a.nl + b.nl;
    r.hdr = a.hdr + b.hdr;
    if (b.last2 >= 0) { r.last = b.last; r.last2 = b.last2; }
    else if (b.last >= 0) { r.last = b.last; r.last2 = a.last; }
    else { r.last = a.last; r.last2 = a.last2; }
    return r;
  }
};

// all of a wave's span loads are issued before the first step is processed
template <bool NT = false>
__device__ __forceinline__ void load_span(const uint8_t* buf, uint64_t p0, uint64_t n, int lane,
                                          uint4 (&v)[WSTEPS]) {
#pragma unroll
  for (int s = 0; s < WSTEPS; ++s) {
    const uint64_t p = p0 + (uint64_t)s * WSTEP + (uint64_t)lane * 16;
    v[s] = p < n ? load16<NT>(buf, p, n) : make_uint4(0, 0, 0, 0);
  }
}

__device__ __forceinline__ int wave_min_i32(int x) {
  for (int o = 32; o > 0; o >>= 1) {
    const int y = __shfl_xor(x, o, 64);
    x = y < x ? y : x;
  }
  return x;
}

// The per-step form of the span pass: per 1 KiB wave step either the fast
// step (below) or the general step.  vs(s) = the lane's 16 bytes of step s.
// The function of the `nsteps` 1 KiB steps from p0 (nothing at or past n),
// the same on every lane.
template <bool UNROLL, class StepBytes>
__device__ __forceinline__ Fn seg_fn(uint64_t n, uint64_t p0, int nsteps, int lane, uint32_t carry, StepBytes vs) {
  uint32_t c0 = 0, c1 = 0, fo = 2u;                           // identity: out(s) = s
  uint32_t nl = 0, hdr = 0;
  int top = -1, second = -1;
  auto last_two = [&](uint32_t nlm, uint64_t p) {             // the span's last two '\n'
    if (nlm) {
      const int rel = (int)(p - p0);
      const int t = 31 - __builtin_clz(nlm);
      const uint32_t rest = nlm & ~(1u << t);
      second = rest ? rel + 31 - __builtin_clz(rest) : top;
      top = rel + t;
    }
  };
  auto step = [&](int s) {
    const uint64_t p = p0 + (uint64_t)s * WSTEP + (uint64_t)lane * 16;
    const uint4 v = vs(s);
    // Fast step (wave-uniform): every byte below n - 1, no '>' in the step,
    // and the span-so-far sends either in-state to out-state 0 - then no
    // header line is open or starts, and every byte but '\n' is content
    if (fo == 0u && p0 + (uint64_t)(s + 1) * WSTEP < n) {
      uint32_t gt = 0, nlm = 0;
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        gt |= zmatch(w[d], 0x3E3E3E3Eu);
        nlm |= pack4(zmatch(w[d], 0x0A0A0A0Au)) << (4 * d);
      }
      if (!__ballot(gt != 0u)) {
        carry = (uint32_t)(__ballot((nlm >> 15) & 1u) >> 63) & 1u;
        const uint32_t cnt = (uint32_t)__builtin_popcount(nlm);
        c0 += 16u - cnt;
        c1 += 16u - cnt;
        nl += cnt;
        last_two(nlm, p);
        return;
      }
    }
    const LaneStep ls = lane_step(v, p, n, lane, carry);
    // lane-local counts for span in-state 0 / 1: a lane's in-state is fixed by
    // a line start in a lower lane, else it is the step's in-state fo(s)
    const uint32_t m0 = lane_content(ls, lane_region(ls, 0)), m1 = lane_content(ls, lane_region(ls, 1));
    const uint32_t f0 = fo & 1u, f1 = (fo >> 1) & 1u;         // span-so-far out-states
    const bool det = (ls.B & ls.lt) != 0;
    const uint32_t d = lane_in(ls, 0);
    c0 += __builtin_popcount((det ? d : f0) ? m1 : m0);
    c1 += __builtin_popcount((det ? d : f1) ? m1 : m0);
    fo = step_out(ls, f0) | step_out(ls, f1) << 1;
    nl += __builtin_popcount(ls.nlm);
    hdr += __builtin_popcount(ls.hs);
    last_two(ls.nlm, p);
  };
  if constexpr (UNROLL) {
#pragma unroll
    for (int s = 0; s < WSTEPS; ++s) {
      if (s >= nsteps || p0 + (uint64_t)s * WSTEP >= n) break;   // wave-uniform
      step(s);
    }
  } else {
#pragma unroll 1
    for (int s = 0; s < nsteps; ++s) {
      if (p0 + (uint64_t)s * WSTEP >= n) break;
      step(s);
    }
  }
  // per lane: c0, c1 <= 256 and nl, hdr <= 256, so the packed sums stay in 16 bits
  const uint32_t cs = __builtin_amdgcn_readlane(wave_incl_sum(c0 | c1 << 16), 63);
  const uint32_t cnts = __builtin_amdgcn_readlane(wave_incl_sum(nl | hdr << 16), 63);
  const int last = wave_max_i32(top);
  const int last2 = wave_max_i32(top != last ? top : second);
  const long long b = (long long)p0;
  return Fn{cs & 0xFFFFu, cs >> 16, cnts & 0xFFFFu, cnts >> 16, last >= 0 ? b + last : -1,
            last2 >= 0 ? b + last2 : -1, fo};
}

// K1's span pass, whole-span form (PG_TUNE_K1 = 1): one wave per 16 KiB
// span -> its function of the in-state.  A span wholly below byte n - 1 with
// no '>' in it is counted in one pass, 4 KiB per round with the next rounds'
// loads in flight (76 VGPRs, 6 waves per SIMD) - per dword the exact
// zero-byte test of w ^ '\n' summed with v_bcnt (bytes == '\n' = 32 -
// popcount(t | x | 0x7F7F7F7F), t = (x & 0x7F7F7F7F) + 0x7F7F7F7F) and the
// any-zero test of w ^ '>' ORed up, no ballot or branch per step.  Its
// function then follows from the newline count, the first newline (in-state 1
// without a line start at the span start: the header bytes before it are no
// content) and the last two (the record table's line ends), found afterwards
// by re-reading the first / last steps (L2).  Any other span is marked
// (o = FN_TODO) for k_span_fix.
__device__ __forceinline__ void span_whole(const uint8_t* __restrict__ buf, uint64_t n, uint64_t span0, uint64_t nspan,
                                         Fn* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const uint64_t span = span0 + (uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
  if (span >= nspan) return;                                  // wave-uniform
  const uint64_t p0 = span * WSPAN;
  const uint32_t carry = p0 == 0 ? 1u : (buf[p0 - 1] == 10 ? 1u : 0u);
  auto step_at = [&](int s) {
    const uint64_t p = p0 + (uint64_t)s * WSTEP + (uint64_t)lane * 16;
    return p < n ? load16(buf, p, n) : make_uint4(0, 0, 0, 0);
  };
  if (p0 + WSPAN < n) {
    constexpr int R = 4;                                      // steps per round
    uint32_t acc = 0, g = 0;
    uint4 cur[R], nxt[R];
    const uint4* src = reinterpret_cast<const uint4*>(buf + p0) + lane;
#pragma unroll
    for (int j = 0; j < R; ++j) cur[j] = src[j * 64];
#pragma unroll
    for (int r = 0; r < WSTEPS / R; ++r) {
      if (r + 1 < WSTEPS / R) {
#pragma unroll
        for (int j = 0; j < R; ++j) nxt[j] = src[((r + 1) * R + j) * 64];
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const uint32_t w[4] = {cur[j].x, cur[j].y, cur[j].z, cur[j].w};
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const uint32_t x = w[d] ^ 0x0A0A0A0Au;
          const uint32_t t = (x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
          acc += (uint32_t)__builtin_popcount(t | x | 0x7F7F7F7Fu);
          const uint32_t y = w[d] ^ 0x3E3E3E3Eu;
          g |= (y - 0x01010101u) & ~y;
        }
      }
#pragma unroll
      for (int j = 0; j < R; ++j) cur[j] = nxt[j];
    }
    if (!__ballot((g & 0x80808080u) != 0u)) {
      const uint32_t nl_lane = 32u * 4u * WSTEPS - acc;
      const uint32_t nl = __builtin_amdgcn_readlane(wave_incl_sum(nl_lane), 63);
      int first = 0x7FFFFFFF, last = -1, last2 = -1;
      if (nl) {
        if (!carry) {
          for (int s = 0; s < WSTEPS; ++s) {                  // the first '\n' (wave-uniform exit)
            const uint32_t m = eq16(step_at(s), 0x0A0A0A0Au);
            first = wave_min_i32(m ? s * WSTEP + lane * 16 + __builtin_ctz(m) : 0x7FFFFFFF);
            if (first != 0x7FFFFFFF) break;
          }
        }
        int found = 0;
        for (int s = WSTEPS - 1; s >= 0; --s) {               // the last two (wave-uniform exit)
          const uint32_t m = eq16(step_at(s), 0x0A0A0A0Au);
          const int t1 = m ? s * WSTEP + lane * 16 + 31 - __builtin_clz(m) : -1;
          const uint32_t rest = m ? m & ~(1u << (31 - __builtin_clz(m))) : 0u;
          const int t2 = rest ? s * WSTEP + lane * 16 + 31 - __builtin_clz(rest) : -1;
          const int a1 = wave_max_i32(t1);
          const int a2 = wave_max_i32(t1 != a1 ? t1 : t2);
          if (found == 0) { last = a1; last2 = a2; found = (a1 >= 0) + (a2 >= 0); }
          else if (a1 >= 0) { last2 = a1; found = 2; }
          if (found >= 2) break;
        }
      }
      if (lane == 0) {
        const long long b = (long long)p0;
        const unsigned long long c0 = WSPAN - nl;
        unsigned long long c1;
        uint32_t o;
        if (!nl) { c1 = carry ? WSPAN : 0ull; o = carry ? 0u : 2u; }
        else { c1 = carry ? c0 : c0 - (unsigned long long)first; o = 0u; }
        out[span] = Fn{c0, c1, nl, 0ull, last >= 0 ? b + last : -1, last2 >= 0 ? b + last2 : -1, o};
      }
      return;
    }
  }
  if (lane == 0) out[span].o = FN_TODO;                       // (k_span_fix)
}
// The per-step form on all 16 loads in flight (PG_TUNE_K1 = 0).
// The span's function from its 16 steps in registers (k_span_sum's steps).
__device__ __forceinline__ Fn span_fn(const uint4 (&v)[WSTEPS], uint64_t n, uint64_t p0, int lane, uint32_t carry) {
  uint32_t c0 = 0, c1 = 0, fo = 2u;                           // identity: out(s) = s
  uint32_t nl = 0, hdr = 0;
  int top = -1, second = -1;
  auto last_two = [&](uint32_t nlm, uint64_t p) {             // the span's last two '\n'
    if (nlm) {
      const int rel = (int)(p - p0);
      const int t = 31 - __builtin_clz(nlm);
      const uint32_t rest = nlm & ~(1u << t);
      second = rest ? rel + 31 - __builtin_clz(rest) : top;
      top = rel + t;
    }
  };
#pragma unroll
  for (int s = 0; s < WSTEPS; ++s) {
    if (p0 + (uint64_t)s * WSTEP >= n) break;                 // wave-uniform
    const uint64_t p = p0 + (uint64_t)s * WSTEP + (uint64_t)lane * 16;
    // Fast step (wave-uniform): every byte below n - 1, no '>' in the step,
    // and the span-so-far sends either in-state to out-state 0 - then no
    // header line is open or starts, and every byte but '\n' is content
    if (fo == 0u && p0 + (uint64_t)(s + 1) * WSTEP < n) {
      uint32_t gt = 0, nlm = 0;
      const uint32_t w[4] = {v[s].x, v[s].y, v[s].z, v[s].w};
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        gt |= zmatch(w[d], 0x3E3E3E3Eu);
        nlm |= pack4(zmatch(w[d], 0x0A0A0A0Au)) << (4 * d);
      }
      if (!__ballot(gt != 0u)) {
        carry = (uint32_t)(__ballot((nlm >> 15) & 1u) >> 63) & 1u;
        const uint32_t cnt = (uint32_t)__builtin_popcount(nlm);
        c0 += 16u - cnt;
        c1 += 16u - cnt;
        nl += cnt;
        last_two(nlm, p);
        continue;
      }
    }
    const LaneStep ls = lane_step(v[s], p, n, lane, carry);
    // lane-local counts for span in-state 0 / 1: a lane's in-state is fixed by
    // a line start in a lower lane, else it is the step's in-state fo(s)
    const uint32_t m0 = lane_content(ls, lane_region(ls, 0)), m1 = lane_content(ls, lane_region(ls, 1));
    const uint32_t f0 = fo & 1u, f1 = (fo >> 1) & 1u;         // span-so-far out-states
    const bool det = (ls.B & ls.lt) != 0;
    const uint32_t d = lane_in(ls, 0);
    c0 += __builtin_popcount((det ? d : f0) ? m1 : m0);
    c1 += __builtin_popcount((det ? d : f1) ? m1 : m0);
    fo = step_out(ls, f0) | step_out(ls, f1) << 1;
    nl += __builtin_popcount(ls.nlm);
    hdr += __builtin_popcount(ls.hs);
    last_two(ls.nlm, p);
  }
  // per lane: c0, c1 <= 256 and nl, hdr <= 256, so the packed sums stay in 16 bits
  const uint32_t cs = __builtin_amdgcn_readlane(wave_incl_sum(c0 | c1 << 16), 63);
  const uint32_t cnts = __builtin_amdgcn_readlane(wave_incl_sum(nl | hdr << 16), 63);
  const int last = wave_max_i32(top);
  const int last2 = wave_max_i32(top != last ? top : second);
  const long long b = (long long)p0;
  return Fn{cs & 0xFFFFu, cs >> 16, cnts & 0xFFFFu, cnts >> 16, last >= 0 ? b + last : -1,
            last2 >= 0 ? b + last2 : -1, fo};
}
__global__ void __launch_bounds__(PBLOCK) k_span_sum(const uint8_t* __restrict__ buf, uint64_t n, uint64_t span0,
                                                     uint64_t nspan, Fn* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const uint64_t span = span0 + (uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
  if (span >= nspan) return;                                  // wave-uniform
  const uint64_t p0 = span * WSPAN;
  uint4 v[WSTEPS];
  load_span<(PG_K1_NT & 1) != 0>(buf, p0, n, lane, v);
  const Fn f = span_fn(v, n, p0, lane, p0 == 0 ? 1u : (buf[p0 - 1] == 10 ? 1u : 0u));
  if (lane == 0) out[span] = f;
}

__global__ void __launch_bounds__(PBLOCK) k_span_whole(const uint8_t* __restrict__ buf, uint64_t n, uint64_t span0,
                                                       uint64_t nspan, Fn* __restrict__ out) {
  span_whole(buf, n, span0, nspan, out);
}
// The spans k_span_whole left (a '>' in them, or the file's last): a block of
// 16 waves per 64 spans finds them by their marker; per such span wave w
// takes step w (its function by the per-step form), and one thread composes
// the 16 (a span's general steps are a serial chain of ballots one wave would
// walk alone: ~16 us).
constexpr int FBLOCK = 64 * WSTEPS;
__global__ void __launch_bounds__(FBLOCK) k_span_fix(const uint8_t* __restrict__ buf, uint64_t n, uint64_t span0,
                                                     uint64_t nspan, Fn* __restrict__ out) {
  __shared__ Fn s_f[WSTEPS];
  __shared__ unsigned long long s_todo;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t base = span0 + (uint64_t)blockIdx.x * 64;
  if (w == 0) {
    const uint64_t mine = base + lane;
    const unsigned long long t = __ballot(mine < nspan && out[mine].o == FN_TODO);
    if (lane == 0) s_todo = t;
  }
  __syncthreads();
  for (unsigned long long todo = s_todo; todo; todo &= todo - 1) {   // block-uniform
    const uint64_t span = base + (uint64_t)__builtin_ctzll(todo);
    const uint64_t ps = span * WSPAN + (uint64_t)w * WSTEP;
    const uint32_t carry = ps == 0 ? 1u : (ps - 1 < n && buf[ps - 1] == 10 ? 1u : 0u);
    const uint64_t p = ps + (uint64_t)lane * 16;
    const uint4 v = p < n ? load16(buf, p, n) : make_uint4(0, 0, 0, 0);
    const Fn f = seg_fn<true>(n, ps, 1, lane, carry, [&](int) { return v; });
    if (lane == 0) s_f[w] = f;
    __syncthreads();
    if (threadIdx.x == 0) {
      Fn r = s_f[0];
      for (int q = 1; q < WSTEPS; ++q) r = FnThen{}(r, s_f[q]);
      out[span] = r;
    }
    __syncthreads();
  }
}

__constant__ uint8_t c_byte_class[256];

// The packed word and exception byte of 16 class bytes (4 dwords, 4 classes
// each): codes class & 3 gathered two bits per base, exception = any class
// with bit 2 set (N, '$', other).
__device__ __forceinline__ uint32_t pack_word(const uint4& v, uint32_t& exc) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t out = 0, e = 0;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    uint32_t t = w[d] & 0x03030303u;                 // 2 bits in each byte
    t = (t | (t >> 6)) & 0x000F000Fu;                // bytes 0,1 -> bits 0..3; 2,3 -> bits 16..19
    t = (t | (t >> 12)) & 0xFFu;                     // 8 bits: 4 bases
    out |= t << (8 * d);
    e |= w[d] & 0x04040404u;
  }
  exc = e;
  return out;
}

// One span's emission: each content byte -> its class code at its compacted
// offset (staged in the wave's `stage` slice), the packed words and
// exception bytes of the chunks the span owns whole.  `pre` = the function
// of the spans before it.
template <int PF>
__device__ __forceinline__ void emit_span(const uint8_t* __restrict__ buf, uint64_t n, uint64_t span, const Fn& pre,
                                          const uint8_t* lut, uint8_t* stage, uint8_t* __restrict__ out,
                                          uint32_t* __restrict__ p2, uint8_t* __restrict__ e16) {
  // pending bytes (< 32) + one step's (<= WSTEP) + the fast step's fifth dword
  constexpr int STAGE = WSTEP + 48;
  const int lane = threadIdx.x & 63;
  auto wave_sync = []() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  // Invariant at every step start: the stage is zero past its pending bytes
  // (the fast step ORs whole dwords in; the general step stores bytes).
  for (int z = 16 * lane; z < STAGE; z += 16 * 64) *reinterpret_cast<uint4*>(stage + z) = make_uint4(0, 0, 0, 0);
  wave_sync();
  const uint64_t p0 = span * WSPAN;
  // the prefix function evaluated at the file's in-state (0; byte 0 starts a line)
  unsigned long long off = pre.c0;
  // stage[0] holds output position cb (16-aligned); bytes below `own` belong
  // to the previous span
  unsigned long long cb = off & ~15ull;
  const unsigned long long own = off;
  uint32_t state = pre.o & 1u;
  uint32_t carry = p0 == 0 ? 1u : (buf[p0 - 1] == 10 ? 1u : 0u);
  // one step of prefetch: occupancy (LDS round trip per step) beats depth here
  // (PF = 2: two steps in flight ahead, PG_TUNE_K1 bit 1)
  uint64_t p = p0 + (uint64_t)lane * 16;
  constexpr bool NT = (PG_K1_NT & 2) != 0;
  uint4 v = p < n ? load16<NT>(buf, p, n) : make_uint4(0, 0, 0, 0);
  uint4 v2 = make_uint4(0, 0, 0, 0);
  if (PF == 2 && p + WSTEP < n) v2 = load16<NT>(buf, p + WSTEP, n);
  for (int s = 0; s < WSTEPS; ++s) {
    if (p0 + (uint64_t)s * WSTEP >= n) break;                 // wave-uniform
    const uint64_t pn = p + WSTEP;
    uint4 vn;
    if (PF == 2) {
      vn = v2;
      const uint64_t pnn = pn + WSTEP;
      v2 = (s + 2 < WSTEPS && pnn < n) ? load16<NT>(buf, pnn, n) : make_uint4(0, 0, 0, 0);
    } else {
      vn = (s + 1 < WSTEPS && pn < n) ? load16<NT>(buf, pn, n) : make_uint4(0, 0, 0, 0);
    }
    uint32_t ctot;
    // Fast step (wave-uniform): in-state 0, every byte below n - 1, no '>',
    // at most one '\n' per lane and every other byte one of ACGTacgt - the
    // lane's bases are its 16 bytes minus the '\n', classed in registers and
    // ORed into the zeroed stage as 5 dwords (no per-byte LDS traffic)
    const FastLane fl = fast_lane(v);
    const bool fast = state == 0u && p0 + (uint64_t)(s + 1) * WSTEP < n &&
                      !__ballot(fl.gt || !fl.acgt || (fl.nlm & (fl.nlm - 1u)) != 0u);
    if (fast) {
      carry = (uint32_t)(__ballot((fl.nlm >> 15) & 1u) >> 63) & 1u;
      // a lane holds 16 or 15 bases (at most one '\n'): its offset is 16 per
      // lane below it less the lanes below holding a '\n' (one ballot and a
      // mask count instead of a dependent chain of DPP adds)
      const uint64_t nlb = __ballot(fl.nlm != 0u);
      const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(nlb >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)nlb, 0u));
      const uint32_t excl = 16u * (uint32_t)lane - below;
      ctot = 16u * 64u - (uint32_t)__builtin_popcountll(nlb);
      // drop the '\n' at byte j (j = 16: none): bytes past it move down by one
      const uint32_t j = fl.nlm ? (uint32_t)__builtin_ctz(fl.nlm) : 16u;
      uint32_t y[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const uint32_t down = d < 3 ? __builtin_amdgcn_alignbyte(fl.cls[d + 1], fl.cls[d], 1) : fl.cls[3] >> 8;
        const int lo = (int)j - 4 * d;                        // bytes of dword d below j
        const uint32_t keep = lo >= 4 ? 0xFFFFFFFFu : lo <= 0 ? 0u : (1u << (8 * lo)) - 1u;
        y[d] = (fl.cls[d] & keep) | (down & ~keep);
      }
      const uint32_t w = (uint32_t)(off - cb) + excl;
      uint32_t* s32 = reinterpret_cast<uint32_t*>(stage) + (w >> 2);
      const uint32_t sh = 32u - 8u * (w & 3u);
      uint32_t prev = 0;
#pragma unroll
      for (int d = 0; d < 5; ++d) {
        const uint32_t cur = d < 4 ? y[d] : 0u;
        atomicOr(s32 + d, (uint32_t)((((uint64_t)cur << 32) | prev) >> sh));
        prev = cur;
      }
    } else {
      const LaneStep ls = lane_step(v, p, n, lane, carry);
      const uint32_t region = lane_region(ls, lane_in(ls, state));
      const uint32_t cm = lane_content(ls, region);
      const uint32_t mine = (uint32_t)__builtin_popcount(cm);
      const uint32_t incl = wave_incl_sum(mine);
      const uint32_t excl = incl - mine;
      const uint32_t tot = __builtin_amdgcn_readlane(incl, 63);
      // (header entries of the record table: k_headers)
      // stage this step's bases after the pending bytes of chunk `cb`
      uint32_t w = (uint32_t)(off - cb) + excl;
      const uint32_t words[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int jj = 0; jj < 16; ++jj)
        if ((cm >> jj) & 1u) stage[w++] = lut[(words[jj >> 2] >> (8 * (jj & 3))) & 0xFFu];
      ctot = tot;
      state = step_out(ls, state);
    }
    wave_sync();
    // write every completed 16-byte chunk; the partial one stays staged.  Only
    // the span's first chunk can hold bytes of the previous span (< own).
    const unsigned long long full = (off + ctot) & ~15ull;
    if (full > cb) {
      for (unsigned long long g = cb + 16ull * lane; g < full; g += 16ull * 64) {
        const uint8_t* src = stage + (g - cb);
        if (g >= own) {
          const uint4 cv = *reinterpret_cast<const uint4*>(src);
          uint32_t exc;
          p2[g >> 4] = pack_word(cv, exc);              // (a shared chunk: k_pack_fix)
          e16[g >> 4] = exc ? 1 : 0;
          if (exc) *reinterpret_cast<uint4*>(out + g) = cv;   // (the class bytes: exception chunks only)
        } else {
          for (int jj = 0; jj < 16; ++jj)
            if (g + jj >= own) out[g + jj] = src[jj];
        }
      }
      wave_sync();
      // (the bytes past the pending ones in that chunk are zero: invariant)
      if (lane == 0)
        *reinterpret_cast<uint4*>(stage) = *reinterpret_cast<const uint4*>(stage + (full - cb));
      cb = full;
      wave_sync();
      for (int z = 16 + 16 * lane; z < STAGE; z += 16 * 64)
        *reinterpret_cast<uint4*>(stage + z) = make_uint4(0, 0, 0, 0);
      wave_sync();
    }
    off += ctot;
    v = vn;
    p = pn;
  }
  // the span's last, partial chunk: byte stores of the bytes this span owns
  if (lane < 16) {
    const unsigned long long q = cb + lane;
    if (q >= own && q < off) out[q] = stage[lane];
  }
}

template <int PF>
__global__ void __launch_bounds__(PBLOCK) k_emit(const uint8_t* __restrict__ buf, uint64_t n, uint64_t span0,
                                                 uint64_t nspan, const Fn* __restrict__ incl,
                                                 uint8_t* __restrict__ out, uint32_t* __restrict__ p2,
                                                 uint8_t* __restrict__ e16) {
  constexpr int STAGE = WSTEP + 48;
  __shared__ uint8_t lut[256];
  __shared__ __attribute__((aligned(16))) uint8_t stage_all[WAVES][STAGE];
  lut[threadIdx.x] = c_byte_class[threadIdx.x];
  __syncthreads();
  const uint64_t span = span0 + (uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
  if (span >= nspan) return;                                  // wave-uniform, after the only barrier
  emit_span<PF>(buf, n, span, span ? incl[span - 1] : fn_identity(), lut, stage_all[threadIdx.x >> 6], out, p2, e16);
}

// The record table's header entries, beside the emission: each header's byte
// span and its record's start in the compacted stream.  Only the spans a
// header starts in, or whose first line continues one, do any work (C3: ~100
// of 31 K spans).  A block of 4 waves per 64 spans finds them by one ballot
// and deals them out to its waves; a wave steps through its span's 16 KiB
// (all loads in flight) with the general step's line logic and content
// counts.  Small blocks and high wave priority: beside the emission they are
// placed and issued at once (blocks of 16 waves, one per step, found no room
// there: ~180 us; alone they took ~10 us on the critical path).
__device__ __forceinline__ void header_span(const uint8_t* __restrict__ buf, uint64_t n, uint64_t span, int lane,
                                            const Fn& pre, uint64_t rcap, long long* __restrict__ rec_start,
                                            long long* __restrict__ hdr_start, long long* __restrict__ hdr_end) {
  uint32_t state = pre.o & 1u;
  const uint64_t p0 = span * WSPAN;
  unsigned long long off = pre.c0, rec = pre.hdr;
  uint4 v[WSTEPS];                                            // (every load in flight at once)
  load_span(buf, p0, n, lane, v);
  uint32_t carry = p0 == 0 ? 1u : (buf[p0 - 1] == 10 ? 1u : 0u);
#pragma unroll
  for (int s = 0; s < WSTEPS; ++s) {
    if (p0 + (uint64_t)s * WSTEP >= n) break;                 // wave-uniform
    const uint64_t p = p0 + (uint64_t)s * WSTEP + (uint64_t)lane * 16;
    const LaneStep ls = lane_step(v[s], p, n, lane, carry);
    const uint32_t region = lane_region(ls, lane_in(ls, state));
    const uint32_t cm = lane_content(ls, region);
    const uint32_t mine = (uint32_t)__builtin_popcount(cm) | (uint32_t)__builtin_popcount(ls.hs) << 16;
    const uint32_t incl_l = wave_incl_sum(mine);
    const uint32_t excl = incl_l - mine;
    const uint32_t tot = __builtin_amdgcn_readlane(incl_l, 63);
    const unsigned long long lane_off = off + (excl & 0xFFFFu);
    const unsigned long long lane_rec = rec + (excl >> 16);
    // header lines: start (record begins at the next base) and terminator
    const uint32_t term = region & (ls.nlm | (~ls.vn1 & below_mask(p, n) & (ls.vn1 + 1u)));
    for (uint32_t m = ls.hs; m; m &= m - 1) {
      const int jj = __builtin_ctz(m);
      const unsigned long long r = lane_rec + __builtin_popcount(ls.hs & ((1u << jj) - 1u));
      if (r >= rcap) continue;                                // the host re-runs with the exact count
      hdr_start[r] = (long long)(p + jj);
      rec_start[r] = (long long)(lane_off + __builtin_popcount(cm & ((1u << jj) - 1u)));
    }
    for (uint32_t m = term; m; m &= m - 1) {
      const int jj = __builtin_ctz(m);
      const unsigned long long r = lane_rec + __builtin_popcount(ls.hs & ((2u << jj) - 1u)) - 1;
      if (r < rcap) hdr_end[r] = (long long)(p + jj);
    }
    off += tot & 0xFFFFu;
    rec += tot >> 16;
    state = step_out(ls, state);
  }
}
__global__ void __launch_bounds__(PBLOCK) k_headers(const uint8_t* __restrict__ buf, uint64_t n, uint64_t span0,
                                                    uint64_t nspan, const Fn* __restrict__ incl, uint64_t rcap,
                                                    long long* __restrict__ rec_start,
                                                    long long* __restrict__ hdr_start, long long* __restrict__ hdr_end) {
  __builtin_amdgcn_s_setprio(3);
  __shared__ unsigned long long s_todo;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t base = span0 + (uint64_t)blockIdx.x * 64;
  if (w == 0) {
    const uint64_t mine = base + lane;
    bool need = false;
    if (mine < nspan) {                                       // a header starts or ends here
      const Fn pre = mine ? incl[mine - 1] : fn_identity();
      need = incl[mine].hdr != pre.hdr || (pre.o & 1u);
    }
    const unsigned long long t = __ballot(need);
    if (lane == 0) s_todo = t;
  }
  __syncthreads();
  int j = 0;
  for (unsigned long long todo = s_todo; todo; todo &= todo - 1, ++j) {   // wave w: every WAVES-th of them
    if ((j & (WAVES - 1)) != w) continue;
    const uint64_t span = base + (uint64_t)__builtin_ctzll(todo);
    header_span(buf, n, span, lane, span ? incl[span - 1] : fn_identity(), rcap, rec_start, hdr_start, hdr_end);
  }
}

// The packed word of every 16-byte chunk that spans s-1 and s share (the one
// holding output offset own_s = incl[s-1].c0, when own_s is not a chunk
// start, and the stream's last, partial chunk), recomputed from the class
// bytes: k_emit writes only chunks one span owns whole.  Boundaries s0 .. s1
// (s >= 1).  Under the chunked upload, the boundary at s1 is packed again by
// the next chunk's call once the span after it is emitted; until then only
// its bytes below own_s1 are final, and nothing reads the others.
// (grid-stride: the launch's grid is capped)
__global__ void k_pack_fix(const Fn* __restrict__ incl, uint64_t s0, uint64_t s1, const uint8_t* __restrict__ cls,
                           uint32_t* __restrict__ p2, uint8_t* __restrict__ e16) {
  for (uint64_t s = s0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= s1;
       s += (uint64_t)gridDim.x * blockDim.x) {
    if (s == 0) continue;
    const unsigned long long own = incl[s - 1].c0;
    if (!(own & 15ull)) continue;                             // (no shared chunk)
    const unsigned long long g = own & ~15ull;
    const uint4 cv = *reinterpret_cast<const uint4*>(cls + g);
    uint32_t exc;
    p2[g >> 4] = pack_word(cv, exc);
    e16[g >> 4] = exc ? 1 : 0;
  }
}

// The class bytes of the chunks K1 left packed (e16 == 0: all ACGT, class =
// the 2-bit code), 16 bases per thread, grid-stride.
__global__ void k_unpack_cls(const uint32_t* __restrict__ p2, const uint8_t* __restrict__ e16, uint64_t nchunk,
                             uint8_t* __restrict__ cls) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nchunk; i += (uint64_t)gridDim.x * blockDim.x) {
    if (e16[i]) continue;
    const uint32_t w = p2[i];
    *reinterpret_cast<uint4*>(cls + 16 * i) = make_uint4(unpack4(w, 0), unpack4(w, 1), unpack4(w, 2), unpack4(w, 3));
  }
}

void ensure_cls(Ctx& c) {
  if (c.cls_full || !c.parsed) return;
  const uint64_t nchunk = (c.n_cls + 15) / 16;
  if (nchunk) {
    hipLaunchKernelGGL(k_unpack_cls, dim3(grid_for(nchunk, 256, 8192)), dim3(256), 0, c.stream, c.p2.as<uint32_t>(),
                       c.e16.as<uint8_t>(), nchunk, c.cls.as<uint8_t>());
    PG_HIP(hipGetLastError());
  }
  c.cls_full = true;
}

// The record table from the scan's total (read on the device: no host round
// trip between the scan and the emission): record lengths, seqio's `ptr`,
// header lengths, gathered side by side ([5][rcap] int64 after the total) for
// one device-to-host copy.  R = the header count, clipped at rcap (the host
// re-runs the emission when it was larger).
__global__ void k_records(const Fn* __restrict__ tot_p, uint64_t n, uint64_t rcap,
                          const long long* __restrict__ rec_start, const long long* __restrict__ hdr,
                          long long* __restrict__ rec_len, long long* __restrict__ out) {
  const Fn tot = *tot_p;
  if (blockIdx.x == 0 && threadIdx.x == 0) *reinterpret_cast<Fn*>(out) = tot;
  if (tot.nl == 0) return;                                    // no line at all (:126-132)
  const uint64_t R = tot.hdr < rcap ? tot.hdr : rcap;
  // the unterminated last line counts when end > start > 0 (:131)
  const bool has_tail = (long long)n - 1 > tot.last + 1;
  const long long last_line_start = has_tail ? tot.last + 1 : (tot.last2 >= 0 ? tot.last2 + 1 : 0);
  long long* pk = out + 8;                                    // (a Fn fits in 8 words)
  // hdr: [0, rcap) header start, [rcap, 2 rcap) header terminator
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < R;
       r += (uint64_t)gridDim.x * blockDim.x) {
    const long long s = rec_start[r];
    pk[r] = s;
    const long long len = (r + 1 < R ? rec_start[r + 1] : (long long)tot.c0) - s;
    rec_len[r] = len;
    pk[rcap + r] = len;
    // seqio's ptr[0] when this record is yielded: the next header line's
    // start, or the last line's start at EOF (:153, :170-172)
    pk[2 * rcap + r] = r + 1 < R ? hdr[r + 1] : last_line_start;
    pk[3 * rcap + r] = hdr[r];
    pk[4 * rcap + r] = hdr[rcap + r] - hdr[r];                // qid = line[:-1] (:160)
  }
}

// The byte-class table lives in each device's constant memory: upload it once
// per device (hipMemcpyToSymbol writes the current device only).
static void upload_byte_class(int device) {
  static std::mutex mu;
  static uint64_t done = 0;                                 // one bit per device id < 64
  std::lock_guard<std::mutex> lock(mu);
  const uint64_t bit = device < 64 ? 1ull << device : 0ull;
  if (bit && (done & bit)) return;
  uint8_t t[256];
  for (int i = 0; i < 256; ++i) t[i] = CLS_OTHER;
  const char* s = "ACGTN";
  const uint8_t c[5] = {CLS_A, CLS_C, CLS_G, CLS_T, CLS_N};
  for (int i = 0; i < 5; ++i) { t[(uint8_t)s[i]] = c[i]; t[(uint8_t)(s[i] | 0x20)] = c[i]; }
  t[(uint8_t)'$'] = CLS_DOLLAR;
  PG_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_byte_class), t, 256));
  done |= bit;
}

// Host input (h_src != NULL): the FASTA goes up in chunks of whole spans on
// the side stream, and K1 works on each chunk as soon as it has landed -
// span functions, the scan of every span so far, the emission of the chunk's
// spans - so only the last chunk's K1 follows the copy.
void parse_fasta(Ctx& c, const uint8_t* h_src, const std::function<void(uint64_t)>* on_chunk) {
  upload_byte_class(c.device);
  const hipStream_t st = c.stream;
  const uint64_t n = c.n_bytes;
  c.parsed = false;
  c.cls_full = false;
  c.n_lines = c.n_records = c.n_bases = c.n_nl = c.n_cls = 0;
  c.h_rec_start.clear(); c.h_rec_len.clear(); c.h_rec_hdr_start.clear();
  c.h_rec_hdr_len.clear(); c.h_rec_ptr.clear();
  if (n == 0) {
    c.parsed = true;
    if (on_chunk) (*on_chunk)(0);
    return;
  }

  c.t0.init();
  c.t0.start(st);
  const uint64_t nspan = (n + WSPAN - 1) / WSPAN;
  c.span_sum.reserve(sizeof(Fn) * nspan);
  c.span_start.reserve(sizeof(Fn) * nspan);
  auto* fns = c.span_sum.as<Fn>();
  auto* incl = c.span_start.as<Fn>();
  size_t bytes = 0;
  PG_HIP(rocprim::inclusive_scan(nullptr, bytes, fns, incl, (size_t)nspan, FnThen{}, st));
  c.scratch.reserve(bytes + 16);
  auto scan = [&](uint64_t upto) {
    size_t b = c.scratch.cap;
    PG_HIP(rocprim::inclusive_scan(c.scratch.p, b, fns, incl, (size_t)upto, FnThen{}, st));
  };
  // span functions of spans s0 .. s1 (k_span_whole + k_span_fix, or the
  // per-step k_span_sum)
  auto span_pass = [&](uint64_t s0, uint64_t s1) {
    const unsigned g = (unsigned)((s1 - s0 + WAVES - 1) / WAVES);
    if (c.k1_form & 1) {
      hipLaunchKernelGGL(k_span_whole, dim3(g), dim3(PBLOCK), 0, st, c.d_fasta, n, s0, s1, fns);
      PG_HIP(hipGetLastError());
      hipLaunchKernelGGL(k_span_fix, dim3((unsigned)((s1 - s0 + 63) / 64)), dim3(FBLOCK), 0, st, c.d_fasta, n, s0, s1,
                         fns);
    } else {
      hipLaunchKernelGGL(k_span_sum, dim3(g), dim3(PBLOCK), 0, st, c.d_fasta, n, s0, s1, fns);
    }
    PG_HIP(hipGetLastError());
  };
  c.cls.reserve(n + 64);
  c.p2.reserve(4 * (n / 16 + 8));
  c.e16.reserve(n / 16 + 32);
  const uint64_t rcap0 = std::max<uint64_t>(c.rec_cap, on_chunk ? 4096 : 64);
  auto reserve_records = [&](uint64_t rcap) {
    c.rec_start.reserve(8 * (rcap + 1));
    c.rec_len.reserve(8 * (rcap + 1));
    c.rec_hdr.reserve(16 * (rcap + 1));
    c.rec_ptr.reserve(8 * (rcap + 1));
    const size_t fcap = c.rec_flag.cap;
    c.rec_flag.reserve(rcap + 1);
    if (c.rec_flag.cap != fcap) c.dev_flag_p = nullptr;     // new memory (possibly at the old address)
    c.rec_pack.reserve(64 + 40 * rcap);
    c.h_pin.reserve(64 + 40 * rcap);
  };
  auto emit = [&](uint64_t s0, uint64_t s1) {
    hipLaunchKernelGGL((c.k1_form & 2) ? k_emit<2> : k_emit<1>, dim3((unsigned)((s1 - s0 + WAVES - 1) / WAVES)),
                       dim3(PBLOCK), 0, st, c.d_fasta, n, s0,
                       s1, incl, c.cls.as<uint8_t>(), c.p2.as<uint32_t>(), c.e16.as<uint8_t>());
    PG_HIP(hipGetLastError());
    // boundaries s0 .. s1 (s1 = nspan: the stream's end, incl[nspan - 1])
    hipLaunchKernelGGL(k_pack_fix, dim3(grid_for(s1 - s0 + 1, 256, 65535)), dim3(256), 0, st, incl, s0, s1,
                       c.cls.as<uint8_t>(), c.p2.as<uint32_t>(), c.e16.as<uint8_t>());
    PG_HIP(hipGetLastError());
  };
  // the header entries of spans s0 .. s1 (k_headers), then the record table
  // of the spans so far (k_records, total = incl[s1 - 1]) and its copy to the
  // host, marked by rec_ev: queued before the spans' emission, so the host
  // reads the table while the emission runs
  // (on `rs`: the context's stream, or for a whole-file parse the
  // high-priority stream, beside the emission)
  hipStream_t rs = st;
  auto records = [&](uint64_t s0, uint64_t s1, uint64_t rcap) {
    auto* hdr = c.rec_hdr.as<long long>();
    hipLaunchKernelGGL(k_headers, dim3((unsigned)((s1 - s0 + 63) / 64)), dim3(PBLOCK), 0, rs, c.d_fasta, n,
                       s0, s1, incl, rcap, c.rec_start.as<long long>(), hdr, hdr + rcap);
    PG_HIP(hipGetLastError());
  };
  auto table_copy = [&](uint64_t s1, uint64_t rcap) {
    hipLaunchKernelGGL(k_records, dim3(grid_for(rcap, 256, 1024)), dim3(256), 0, rs, incl + s1 - 1, n, rcap,
                       c.rec_start.as<long long>(), c.rec_hdr.as<long long>(), c.rec_len.as<long long>(),
                       c.rec_pack.as<long long>());
    PG_HIP(hipGetLastError());
    PG_HIP(hipMemcpyAsync(c.h_pin.p, c.rec_pack.p, 64 + 40 * rcap, hipMemcpyDeviceToHost, rs));
    PG_HIP(hipEventRecord(c.rec_ev, rs));
  };
  // (a polling wait, as Ctx::sync: a blocking wait's wake-up is on the path)
  auto table_wait = [&]() {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const hipError_t e = hipEventQuery(c.rec_ev);
      if (e == hipSuccess) return;
      if (e != hipErrorNotReady) break;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) break;
    }
    PG_HIP(hipEventSynchronize(c.rec_ev));
  };
  reserve_records(rcap0);
  bool streaming = on_chunk != nullptr;
  std::pair<uint64_t, uint64_t> pending{0, 0};               // spans whose emission follows the table's copy
  // (the stager's last work - waiting for the DMAs and unregistering the
  // chunks' pages - is waited for right after the last chunk's K1 is queued:
  // left to run beside the last record round trip and stage A share, its
  // runtime calls made those steps slower and uneven, 9.81 ms (max 9.92)
  // against 9.77 (max 9.80) on C3 with alternating inputs)
  std::unique_ptr<Upload> upload;
  if (h_src) {
    const uint64_t C = std::max<uint64_t>(WSPAN, c.h2d_chunk / WSPAN * WSPAN);
    // chunks of C bytes (whole spans); pg_build_host's last one small
    // (h2d_tail): what follows the last byte's arrival - that chunk's K1 and
    // its records' stage A share - then covers a few MB instead of up to C
    std::vector<uint64_t> bounds{0};
    const uint64_t tl = on_chunk ? (std::min(c.h2d_tail, C / 2) + WSPAN - 1) / WSPAN * WSPAN : 0;
    const uint64_t body = tl && n > C + tl ? (n - tl) / WSPAN * WSPAN : n;
    for (uint64_t o = 0; o < body; o += C) bounds.push_back(std::min(body, o + C));
    if (bounds.size() > 2 && bounds.back() - bounds[bounds.size() - 2] < C / 4)
      bounds.erase(bounds.end() - 2);                       // no sliver: the body's remainder joins its neighbour
    if (body < n) bounds.push_back(n);
    // pinned source: DMA up to 8 chunks ahead; pageable (an mmap): through
    // the pinned staging ring (pg_stage.hip)
    upload.reset(new Upload(c, c.fasta_own.as<uint8_t>(), h_src, n, bounds));
    Upload& up = *upload;
    const uint64_t nch = up.chunks();
    for (uint64_t i = 0; i < nch; ++i) {
      up.wait_queued(i);
      const uint64_t off = up.off(i), len = up.len(i);
      const uint64_t s0 = off / WSPAN, s1 = std::min(nspan, (off + len + WSPAN - 1) / WSPAN);
      PG_HIP(hipStreamWaitEvent(st, c.cev[i & 15], 0));
      up.consumed(i);
      span_pass(s0, s1);
      PG_HIP(hipGetLastError());
      scan(s1);
      records(s0, s1, rcap0);
      if (i + 1 == nch) {                                     // (after the final table's copy, below)
        pending = {s0, s1};
        continue;
      }
      if (!streaming) {
        emit(s0, s1);
        continue;
      }
      // the records complete so far (every header seen but the last one):
      // the host reads them while this chunk's emission and the copies go on
      table_copy(s1, rcap0);
      emit(s0, s1);
      table_wait();
      const Fn t = *c.h_pin.as<Fn>();
      const uint64_t Rs = t.nl ? t.hdr : 0;
      if (Rs > rcap0) { streaming = false; continue; }        // more records than the arrays hold
      const int64_t* pk = c.h_pin.as<int64_t>() + 8;
      const uint64_t Rc = Rs ? Rs - 1 : 0;
      c.h_rec_start.assign(pk, pk + Rc);
      c.h_rec_len.assign(pk + rcap0, pk + rcap0 + Rc);
      c.n_records = Rc;
      (*on_chunk)(Rc);
    }
    upload->finish();
  } else {
    span_pass(0, nspan);
    PG_HIP(hipGetLastError());
    scan(nspan);
    // the header pass, the record table and its copy to the host on the
    // high-priority stream, beside the emission (they read the FASTA's
    // header spans and the scan, nothing the emission writes); K1 bit 2: on
    // the context's stream ahead of the emission
    if (!(c.k1_form & 4)) {
      PG_HIP(hipEventRecord(c.ev[14], st));
      PG_HIP(hipStreamWaitEvent(c.stream_hi, c.ev[14], 0));
      rs = c.stream_hi;
    }
    records(0, nspan, rcap0);
    pending = {0, nspan};
  }
  // The record table's copy is queued behind the header pass and ahead of the
  // (last) emission, with no host round trip before it: the class stream is
  // sized by the file (bases < n), the record arrays by the last parse's
  // record count (the header pass re-run with the exact count if exceeded).
  static_assert(sizeof(Fn) <= 64, "the total in front of the packed record table");
  uint64_t R = 0;
  Fn tot{};
  for (int attempt = 0; attempt < 2; ++attempt) {
    const uint64_t rcap = attempt ? std::max<uint64_t>(c.rec_cap, 64) : rcap0;
    if (attempt) {                                            // the exact record count: the header pass again
      reserve_records(rcap);
      records(0, nspan, rcap);
    }
    table_copy(nspan, rcap);
    if (pending.second > pending.first) {
      emit(pending.first, pending.second);
      pending = {0, 0};
      c.t0.stop(st);                                          // K1's end on the stream
    }
    table_wait();
    tot = *c.h_pin.as<Fn>();
    R = tot.nl ? tot.hdr : 0;
    if (R <= rcap) {
      const int64_t* pk = c.h_pin.as<int64_t>() + 8;
      c.h_rec_start.assign(pk, pk + R);
      c.h_rec_len.assign(pk + rcap, pk + rcap + R);
      c.h_rec_ptr.assign(pk + 2 * rcap, pk + 2 * rcap + R);
      c.h_rec_hdr_start.assign(pk + 3 * rcap, pk + 3 * rcap + R);
      c.h_rec_hdr_len.assign(pk + 4 * rcap, pk + 4 * rcap + R);
      break;
    }
    c.rec_cap = R;
  }
  c.n_nl = tot.nl;
  c.n_cls = tot.c0;
  if (tot.nl == 0) {                                        // no line at all (:126-132)
    c.parsed = true;
    if (on_chunk) (*on_chunk)(streaming ? 0 : ~0ull);
    if (upload) upload->finish();
    return;
  }
  const bool has_tail = (long long)n - 1 > tot.last + 1;
  c.n_lines = tot.nl + (has_tail ? 1 : 0);
  c.n_records = R;
  c.rec_cap = std::max(c.rec_cap, R);
  uint64_t nb = 0;
  for (uint64_t r = 0; r < R; ++r) nb += (uint64_t)c.h_rec_len[r];
  c.n_bases = nb;
  c.parsed = true;
  if (on_chunk) (*on_chunk)(streaming ? R : ~0ull);          // ~0: the stream broke off
  if (upload) upload->finish();
}

}  // namespace pg
