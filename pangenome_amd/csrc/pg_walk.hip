// pg_walk.hip — the two sequence walks that follow the rdBG build:
//   edges  rdbg_edge_weight_jit_ / rdbg_edge_weight (kmer_numba.py:1446-1518,
//          :1808-1827): consecutive rdBG members of a walk -> weighted edges
//   rows   seqs2path_jit_ / seq2path_jit_ (:1523-1573, :1830-1849): label
//          lookups + greedy region merge -> (start, end, label) rows
//
// A walk is one strand of one record, in the reference's order (record r
// forward, then its reverse strand if the strand bit is set).  Windows are
// enumerated as runs of WW consecutive forward positions; a run's reverse-
// strand twins are the same positions read backwards, so each walk's hits are
// compacted in walk order by a count pass, a device scan and a write pass
// (reverse-strand hits are written mirrored inside their record's segment).
#include <cstring>
#include <algorithm>
#include <rocprim/rocprim.hpp>

#include "pg_internal.h"

namespace pg {

constexpr int WW = 16;        // windows per thread run
constexpr int WBLOCK = 256;

struct Occ { unsigned long long key; unsigned int v; unsigned int walk; };   // edge pass
struct Hit { unsigned long long idx; long long label; };                    // rows pass
struct EdgeSlot { unsigned long long n0p1, n1p1; unsigned int vv, count; unsigned long long first; };
struct LabSlot { long long key, val, id; unsigned long long occ; };

// --------------------------------------------------------------- windows
// One window of each strand at forward position q of record (rs, n):
// forward window q and reverse-strand window p' = n-k-q, with their keys,
// the reverse complement of each key, and the lastc of pred/succ.
struct Win {
  uint64_t xf, xr;        // forward-window key, reverse-strand-window key
  uint64_t xf_rc, xr_rc;  // reverse complements (for the canonical table lookup)
  uint32_t fp, fs, rp, rs;
};

// Explicit strand enumeration for records with n <= k+1 (rare).
__device__ void short_window(const uint8_t* cls, long long rs, long long n, int k, uint64_t shift,
                             int strand, long long j, uint64_t& x, uint32_t& pred, uint32_t& succ) {
  auto S = [&](long long i) -> uint32_t {
    return strand == 0 ? (uint32_t)cls[rs + i] : comp_class(cls[rs + n - 1 - i]);
  };
  if (n < k) { x = SENTINEL; pred = LAM_HASH; succ = LAM_DOLLAR; return; }
  uint64_t K0 = 0, pw = 1;
  for (int t = 0; t < k; ++t) { K0 += (uint64_t)digit_fw(S(t)) * pw; pw *= 5; }
  if (n == k) { x = K0; pred = LAM_HASH; succ = LAM_DOLLAR; return; }
  if (j == 0) { x = K0; pred = LAM_HASH; succ = lam_fw(S(k)); return; }
  x = K0 / 5 + (uint64_t)digit_fw(S(1)) * shift;     // numba's unbound loop variable == 0
  pred = lam_fw(S(1));
  succ = LAM_DOLLAR;
}

// Iterate windows q in [q0, q1) of one record and call f(q, Win).
template <class F>
__device__ __forceinline__ void for_windows(const uint8_t* __restrict__ cls, long long rs, long long n, int k,
                                            uint64_t shift, long long q0, long long q1, F&& f) {
  if (n <= k + 1) {
    for (long long q = q0; q < q1; ++q) {
      Win w;
      const long long nw = n < k ? 1 : n - k + 1;
      short_window(cls, rs, n, k, shift, 0, q, w.xf, w.fp, w.fs);
      short_window(cls, rs, n, k, shift, 1, nw - 1 - q, w.xr, w.rp, w.rs);
      w.xf_rc = w.xf == SENTINEL ? SENTINEL : rc_key(w.xf, k);
      w.xr_rc = w.xr == SENTINEL ? SENTINEL : rc_key(w.xr, k);
      f(q, w);
    }
    return;
  }
  const long long last = n - k;
  uint64_t K = 0, Kr = 0;
  for (long long q = q0; q < q1; ++q) {
    const uint64_t p = (uint64_t)(rs + q);
    if (q == q0) {
      uint64_t pw = 1;
      for (int j = 0; j < k; ++j) {
        const uint32_t cj = cls[p + j];
        K += (uint64_t)digit_fw(cj) * pw;
        Kr = Kr * 5 + digit_rc(cj);
        pw *= 5;
      }
    } else {
      const uint32_t dout = cls[p - 1], din = cls[p + k - 1];
      K = (K - digit_fw(dout)) * INV5 + (uint64_t)digit_fw(din) * shift;
      Kr = (Kr - (uint64_t)digit_rc(dout) * shift) * 5 + digit_rc(din);
    }
    Win w;
    w.xf = K; w.xf_rc = Kr; w.xr = Kr; w.xr_rc = K;
    w.fp = q == 0 ? LAM_HASH : lam_fw(cls[p - (q == last ? 2 : 1)]);
    w.fs = q == last ? LAM_DOLLAR : lam_fw(cls[p + k]);
    w.rp = q == last ? LAM_HASH : lam_rc(cls[p + k + (q == 0 ? 1 : 0)]);
    w.rs = q == 0 ? LAM_DOLLAR : lam_rc(cls[p - 1]);
    f(q, w);
  }
}

// rdbg_dict.has_key (:1465): rdBG member, or key 0 (has_key never checks counts, :599-603)
__device__ __forceinline__ bool edge_member(const TableView& T, uint64_t x, uint64_t xrc) {
  if (x == SENTINEL) return false;             // skipped before the lookup (:1461-1462)
  if (x == 0) return true;
  const uint64_t c = x < xrc ? x : xrc;
  const uint32_t m = tab_get(T, c);
  if (x == c) return (m & PRES_A) && rdbg_member(m & MASK12);
  return (m & PRES_B) && rdbg_member((m >> B_SHIFT) & MASK12);
}

__device__ __forceinline__ uint64_t lab_hash(long long a, long long b) {
  return fmix64((uint64_t)a * 0x9e3779b97f4a7c15ull ^ fmix64((uint64_t)b));
}

__device__ __forceinline__ bool label_get(const LabSlot* __restrict__ lab, uint64_t capmask, long long a,
                                          long long b, long long& id) {
  uint64_t slot = lab_hash(a, b) & capmask;
  for (uint64_t probe = 0; probe <= capmask; ++probe) {
    const LabSlot s = lab[slot];
    if (!s.occ) return false;
    if (s.key == a && s.val == b) { id = s.id; return true; }
    slot = (slot + 1) & capmask;
  }
  return false;
}

struct WalkArgs {
  const uint8_t* cls;
  const long long* rec_start;
  const long long* rec_len;
  const unsigned long long* run_off;   // per walked record: first run index (size nrec+1)
  const int* run_rec;                  // walked record -> record index
  uint64_t nrec;                       // walked records
  int k; uint64_t shift; int rc;
  TableView T;                         // edges: the dBG table
  const LabSlot* lab; uint64_t lab_capmask;   // rows
};

__device__ __forceinline__ void run_locate(const WalkArgs& a, uint64_t u, uint64_t& wr, int& r, long long& rs,
                                           long long& n, long long& q0, long long& q1) {
  uint64_t lo = 0, hi = a.nrec;              // last wr with run_off[wr] <= u
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (a.run_off[mid] <= u) lo = mid + 1; else hi = mid;
  }
  wr = lo - 1;
  r = a.run_rec[wr];
  rs = a.rec_start[r];
  n = a.rec_len[r];
  const long long nw = n < a.k ? 1 : n - a.k + 1;
  q0 = (long long)(u - a.run_off[wr]) * WW;
  q1 = q0 + WW < nw ? q0 + WW : nw;
}

// MODE 0: edge members, MODE 1: label hits.  Pass 1: per-run counts and bit masks.
template <int MODE>
__global__ void __launch_bounds__(WBLOCK) k_walk_count(WalkArgs a, uint64_t nruns, unsigned* __restrict__ cnt_f,
                                                       unsigned* __restrict__ cnt_r, unsigned* __restrict__ bits) {
  for (uint64_t u = blockIdx.x * (uint64_t)WBLOCK + threadIdx.x; u < nruns; u += (uint64_t)gridDim.x * WBLOCK) {
    uint64_t wr; int r; long long rs, n, q0, q1;
    run_locate(a, u, wr, r, rs, n, q0, q1);
    unsigned bf = 0, br = 0;
    for_windows(a.cls, rs, n, a.k, a.shift, q0, q1, [&](long long q, const Win& w) {
      bool hf, hr = false;
      if (MODE == 0) {
        hf = edge_member(a.T, w.xf, w.xf_rc);
        if (a.rc) hr = edge_member(a.T, w.xr, w.xr_rc);
      } else {
        long long id;
        hf = label_get(a.lab, a.lab_capmask, (long long)w.xf, (long long)((w.fp << OFFBIT) | w.fs), id);
        if (a.rc) hr = label_get(a.lab, a.lab_capmask, (long long)w.xr, (long long)((w.rp << OFFBIT) | w.rs), id);
      }
      bf |= (unsigned)hf << (q - q0);
      br |= (unsigned)hr << (q - q0);
    });
    cnt_f[u] = __builtin_popcount(bf);
    cnt_r[u] = __builtin_popcount(br);
    bits[u] = bf | (br << 16);
  }
}

// Pass 2: write hits in walk order.  Segment of walked record wr: forward hits
// [seg, seg+F), reverse-strand hits [seg+F, seg+F+Rv) in descending q.
template <int MODE>
__global__ void __launch_bounds__(WBLOCK) k_walk_write(WalkArgs a, uint64_t nruns,
                                                       const unsigned long long* __restrict__ sf,
                                                       const unsigned long long* __restrict__ sr,
                                                       const unsigned* __restrict__ bits, void* __restrict__ out) {
  for (uint64_t u = blockIdx.x * (uint64_t)WBLOCK + threadIdx.x; u < nruns; u += (uint64_t)gridDim.x * WBLOCK) {
    const unsigned b = bits[u];
    if (!b) continue;
    uint64_t wr; int r; long long rs, n, q0, q1;
    run_locate(a, u, wr, r, rs, n, q0, q1);
    const uint64_t u0 = a.run_off[wr], u1 = a.run_off[wr + 1];
    const unsigned long long gf0 = sf[u0], gr0 = sr[u0];
    const unsigned long long F = sf[u1] - gf0, Rv = sr[u1] - gr0;
    const unsigned long long seg = gf0 + gr0;
    unsigned long long of = sf[u] - gf0, orr = sr[u] - gr0;   // ranks within the record
    const long long nw = n < a.k ? 1 : n - a.k + 1;
    for_windows(a.cls, rs, n, a.k, a.shift, q0, q1, [&](long long q, const Win& w) {
      const int j = (int)(q - q0);
      if (b & (1u << j)) {
        const unsigned long long o = seg + of++;
        if (MODE == 0) {
          reinterpret_cast<Occ*>(out)[o] = Occ{w.xf, (w.fp << EDGE_OFFBIT) | w.fs, (unsigned)(2 * r)};
        } else {
          long long id = 0;
          label_get(a.lab, a.lab_capmask, (long long)w.xf, (long long)((w.fp << OFFBIT) | w.fs), id);
          reinterpret_cast<Hit*>(out)[o] = Hit{(unsigned long long)q, id};
        }
      }
      if (b & (1u << (16 + j))) {
        const unsigned long long o = seg + F + (Rv - 1 - orr++);
        if (MODE == 0) {
          reinterpret_cast<Occ*>(out)[o] = Occ{w.xr, (w.rp << EDGE_OFFBIT) | w.rs, (unsigned)(2 * r + 1)};
        } else {
          long long id = 0;
          label_get(a.lab, a.lab_capmask, (long long)w.xr, (long long)((w.rp << OFFBIT) | w.rs), id);
          reinterpret_cast<Hit*>(out)[o] = Hit{(unsigned long long)(nw - 1 - q), id};
        }
      }
    });
  }
}

// ------------------------------------------------------------ edge table
// Memory-side reads of words other lanes publish with atomics.  Device-scope
// atomics execute beyond the XCD's L2 and do not refresh it, so a plain (or
// relaxed atomic) load can keep returning a stale 0 from L2; an idempotent
// read-modify-write such as atomicAdd(p, 0) may be rewritten into such a load
// by the compiler.  A compare-and-swap of 0 with 0 cannot be, and returns the
// memory-side value (it writes 0 only where 0 already is).
__device__ __forceinline__ unsigned long long atomic_read64(unsigned long long* p) {
  return atomicCAS(p, 0ull, 0ull);
}
__device__ __forceinline__ unsigned atomic_read32(unsigned* p) { return atomicCAS(p, 0u, 0u); }

// Find-or-insert the edge (n0, v0, n1, v1).  Slots are claimed by CAS on
// n0+1 and completed with atomic stores; every field goes from 0 to its final
// value once, so a nonzero read is final.  Nothing ever waits: an occurrence
// that meets a claimed slot whose other fields are not visible yet returns
// EDGE_RETRY and is re-run by the next launch (all claims of a launch are
// published when it ends).  Spinning instead deadlocks: the compiler lays the
// winner's publish out after the loop, behind its waiting wave-mates.
constexpr uint64_t EDGE_RETRY = ~0ull - 1;
constexpr uint64_t EDGE_PROBES = 4096;
__device__ uint64_t edge_find_or_insert(EdgeSlot* __restrict__ tab, uint64_t capmask, uint64_t n0, uint32_t v0,
                                        uint64_t n1, uint32_t v1, unsigned* err) {
  const unsigned long long a = n0 + 1ull, bkey = n1 + 1ull;
  const unsigned vv = v0 | (v1 << 16) | 0x80000000u;
  uint64_t slot = fmix64(n0 * 0x9e3779b97f4a7c15ull ^ fmix64(n1 ^ ((uint64_t)vv << 40))) & capmask;
  // (the table is sized from the rdBG; a long probe sequence means it is too
  // small for this input: the error bit makes the host re-run with more slots)
  const uint64_t limit = capmask < EDGE_PROBES ? capmask : EDGE_PROBES;
  for (uint64_t probe = 0; probe <= limit; ++probe) {
    EdgeSlot* s = tab + slot;
    unsigned long long w0 = s->n0p1;          // a stale plain read can only show 0
    if (w0 == 0ull) {
      w0 = atomicCAS(&s->n0p1, 0ull, a);
      if (w0 == 0ull) {
        atomicExch(&s->vv, vv);
        atomicExch(&s->n1p1, bkey);
        return slot;
      }
    }
    if (w0 == a) {
      unsigned long long w1 = s->n1p1;
      unsigned w2 = s->vv;
      if (w1 == 0ull) w1 = atomic_read64(&s->n1p1);
      if (w2 == 0u) w2 = atomic_read32(&s->vv);
      if (w1 == 0ull || w2 == 0u) return EDGE_RETRY;
      if (w1 == bkey && w2 == vv) return slot;
    }
    slot = (slot + 1) & capmask;
  }
  atomicOr(err, 2u);
  return ~0ull;
}

// set of (edge slot, walk) pairs: returns true for the first insert
__device__ __forceinline__ bool pair_insert(unsigned long long* __restrict__ set, uint64_t capmask,
                                            unsigned long long key, unsigned* err) {
  const unsigned long long k1 = key + 1ull;
  uint64_t slot = fmix64(key) & capmask;
  for (uint64_t probe = 0; probe <= capmask; ++probe) {
    unsigned long long v = set[slot];
    if (v == k1) return false;
    if (v == 0ull) {
      v = atomicCAS(set + slot, 0ull, k1);
      if (v == 0ull) return true;
      if (v == k1) return false;
    }
    slot = (slot + 1) & capmask;
  }
  atomicOr(err, 4u);
  return false;
}

// one launch over occurrence indices (all of them, or a retry list)
__global__ void k_edges(const Occ* __restrict__ occ, uint64_t m, const unsigned long long* __restrict__ list,
                        uint64_t nlist, EdgeSlot* __restrict__ tab, uint64_t capmask,
                        unsigned long long* __restrict__ pairs, uint64_t pair_capmask,
                        unsigned long long* __restrict__ retry, unsigned long long* __restrict__ nretry,
                        unsigned* err) {
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < nlist;
       j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = list ? list[j] : j;
    if (i + 1 >= m) continue;
    const Occ a = occ[i], b = occ[i + 1];
    if (a.walk != b.walk) continue;
    const uint64_t s = edge_find_or_insert(tab, capmask, a.key, a.v, b.key, b.v, err);
    if (s == EDGE_RETRY) { retry[atomicAdd(nretry, 1ull)] = i; continue; }
    if (s == ~0ull) continue;
    atomicMax(&tab[s].first, ~(unsigned long long)i);   // zeroed slots: max of ~i == ~(min i)
    if (pair_insert(pairs, pair_capmask, (s << 32) | a.walk, err)) atomicAdd(&tab[s].count, 1u);
  }
}

struct EdgeOut { unsigned long long n0, n1; unsigned v0, v1; unsigned long long count, first, walk; };

__global__ void k_edges_compact(const EdgeSlot* __restrict__ tab, uint64_t cap, const Occ* __restrict__ occ,
                                EdgeOut* __restrict__ out, unsigned long long* __restrict__ first_key,
                                unsigned* __restrict__ iota, unsigned long long* __restrict__ counter) {
  const int lane = threadIdx.x & 63;
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const EdgeSlot s = tab[i];
    const bool used = s.n0p1 != 0ull;
    const unsigned long long bal = __ballot(used);
    if (!bal) continue;
    const int leader = __builtin_ctzll(bal);
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(counter, (unsigned long long)__builtin_popcountll(bal));
    base = __shfl(base, leader, 64);
    if (used) {
      const unsigned long long o = base + __builtin_popcountll(bal & lt);
      out[o] = EdgeOut{s.n0p1 - 1ull, s.n1p1 - 1ull, s.vv & 0xFFFFu, (s.vv >> 16) & 0x7FFFu, s.count, ~s.first,
                       occ[~s.first].walk};
      first_key[o] = ~s.first;
      iota[o] = (unsigned)o;
    }
  }
}

// The edges in first-occurrence order (typed-Dict insertion order,
// :1479-1484) as the export layout: 4 x uint64 tuple, int64 count, int64 walk.
__global__ void k_edges_order(const EdgeOut* __restrict__ e, const unsigned* __restrict__ order, uint64_t n,
                              unsigned long long* __restrict__ tup, long long* __restrict__ cnt,
                              long long* __restrict__ walk) {
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const EdgeOut x = e[order[j]];
    tup[4 * j] = x.n0; tup[4 * j + 1] = x.v0; tup[4 * j + 2] = x.n1; tup[4 * j + 3] = x.v1;
    cnt[j] = (long long)x.count;
    walk[j] = (long long)x.walk;
  }
}

// ------------------------------------------------------------ labels
__global__ void k_lab_insert(const long long* __restrict__ key, const long long* __restrict__ val,
                             const long long* __restrict__ id, uint64_t n, LabSlot* __restrict__ tab,
                             uint64_t capmask) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t slot = lab_hash(key[i], val[i]) & capmask;
    for (uint64_t probe = 0; probe <= capmask; ++probe) {
      if (atomicCAS(&tab[slot].occ, 0ull, 1ull) == 0ull) {
        tab[slot].key = key[i]; tab[slot].val = val[i]; tab[slot].id = id[i];
        break;
      }
      slot = (slot + 1) & capmask;
    }
  }
}

// ------------------------------------------------------------ regions
// seq2path_jit_'s greedy merge (:1546-1560), in parallel.  Per walk, with
// last = 0 and last_label = -1 at its start, a hit (idx, label) is taken iff
// idx > last (then last = idx + k); a taken hit whose label differs from the
// previous taken one opens a row (start = last before it, end = its idx + k),
// an equal label extends the open row's end.
//
// Taken hits: a hit more than k past its walk predecessor is always taken
// (last <= that predecessor's idx + k), so a walk splits into runs at such
// hits (and at the walk's first hit, entered with last = 0); one thread
// resolves each run sequentially.  Rows: the taken hits compacted in walk
// order; a row starts at a taken hit that is its walk's first or changes the
// label, and ends at the taken hit before the next row's start.

// walk of hit j: the last w with seg_off[w] <= j (seg_off: nseg + 1 bounds)
__device__ __forceinline__ uint32_t walk_of(const unsigned long long* __restrict__ seg_off, uint32_t nseg,
                                            unsigned long long j) {
  uint32_t lo = 0, hi = nseg;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (seg_off[mid] <= j) lo = mid + 1; else hi = mid;
  }
  return lo - 1;
}

__global__ void k_taken(const Hit* __restrict__ hits, uint64_t m, const unsigned long long* __restrict__ seg_off,
                        uint32_t nseg, int k, uint8_t* __restrict__ taken) {
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < m; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t w = walk_of(seg_off, nseg, j);
    const unsigned long long w0 = seg_off[w], w1 = seg_off[w + 1];
    const long long idx = (long long)hits[j].idx;
    const bool first = j == w0;
    if (!first && idx <= (long long)hits[j - 1].idx + k) continue;       // inside a run
    long long last = first ? 0 : idx - 1;
    long long prev = idx;
    for (unsigned long long t = j; t < w1; ++t) {
      const long long x = t == j ? idx : (long long)hits[t].idx;
      if (t > j && x > prev + k) break;                                   // the next run
      const bool tk = last < x;
      taken[t] = tk;
      if (tk) last = x + k;
      prev = x;
    }
  }
}

__global__ void k_row_heads(const Hit* __restrict__ hits, const unsigned long long* __restrict__ acc, uint64_t na,
                            const unsigned long long* __restrict__ seg_off, uint32_t nseg,
                            uint8_t* __restrict__ head) {
  for (uint64_t a = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; a < na; a += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long j = acc[a];
    bool h = a == 0;
    if (!h) {
      const unsigned long long jp = acc[a - 1];
      h = walk_of(seg_off, nseg, jp) != walk_of(seg_off, nseg, j) || hits[jp].label != hits[j].label;
    }
    head[a] = h;
  }
}

// rows in print order (walk order = record, forward then reverse strand,
// :1836-1844): (record, start, end, strand +1/-1, label) as int64, the
// values through int32 (:1533) and reverse-strand rows mirrored (:1843)
__global__ void k_rows(const Hit* __restrict__ hits, const unsigned long long* __restrict__ acc, uint64_t na,
                       const unsigned long long* __restrict__ starts, uint64_t nrows,
                       const unsigned long long* __restrict__ seg_off, uint32_t nseg, const int* __restrict__ walk_rec,
                       const long long* __restrict__ rec_len, int k, long long* __restrict__ rows) {
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nrows;
       r += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long s = starts[r], e = (r + 1 < nrows ? starts[r + 1] : na) - 1;
    const unsigned long long js = acc[s], je = acc[e];
    const uint32_t w = walk_of(seg_off, nseg, js);
    long long start = 0;
    if (s > 0) {
      const unsigned long long jp = acc[s - 1];
      if (walk_of(seg_off, nseg, jp) == w) start = (long long)hits[jp].idx + k;
    }
    const long long end = (long long)hits[je].idx + k;
    const int rec = walk_rec[w >> 1];
    const int st = (int)start, ed = (int)end, lb = (int)hits[js].label;
    long long* o = rows + 5 * r;
    o[0] = rec;
    if (w & 1) {
      const long long lseq = rec_len[rec];
      o[1] = (int)(lseq - ed);
      o[2] = (int)(lseq - st);
      o[3] = -1;
    } else {
      o[1] = st;
      o[2] = ed;
      o[3] = 1;
    }
    o[4] = lb;
  }
}

// ------------------------------------------------------------ text
// decimal digits of v (v >= 0)
__host__ __device__ __forceinline__ uint32_t ndig(unsigned long long v) {
  uint32_t d = 1;
  while (v >= 10ull) { v /= 10ull; ++d; }
  return d;
}
__device__ __forceinline__ uint32_t ndig_i(long long v) {
  return v < 0 ? 1 + ndig((unsigned long long)0 - (unsigned long long)v) : ndig((unsigned long long)v);
}
__device__ __forceinline__ char* put_dec(char* o, unsigned long long v) {
  const uint32_t d = ndig(v);
  for (uint32_t i = d; i-- > 0;) { o[i] = (char)('0' + v % 10ull); v /= 10ull; }
  return o + d;
}
__device__ __forceinline__ char* put_dec_i(char* o, long long v) {
  if (v < 0) { *o++ = '-'; return put_dec(o, (unsigned long long)0 - (unsigned long long)v); }
  return put_dec(o, (unsigned long long)v);
}

// `.xyz` lines "%d_%d\t%d_%d\t%d\n" (:1901), keys printed as unsigned
__global__ void k_xyz_len(const unsigned long long* __restrict__ tup, const long long* __restrict__ cnt, uint64_t n,
                          unsigned long long* __restrict__ len) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    len[i] = ndig(tup[4 * i]) + ndig(tup[4 * i + 1]) + ndig(tup[4 * i + 2]) + ndig(tup[4 * i + 3]) +
             ndig_i(cnt[i]) + 5;
}
__global__ void k_xyz_write(const unsigned long long* __restrict__ tup, const long long* __restrict__ cnt, uint64_t n,
                            const unsigned long long* __restrict__ off, char* __restrict__ out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    char* o = out + off[i];
    o = put_dec(o, tup[4 * i]); *o++ = '_'; o = put_dec(o, tup[4 * i + 1]); *o++ = '\t';
    o = put_dec(o, tup[4 * i + 2]); *o++ = '_'; o = put_dec(o, tup[4 * i + 3]); *o++ = '\t';
    o = put_dec_i(o, cnt[i]); *o = '\n';
  }
}

// region rows "%s\t%d\t%d\t%s\t%d\n" (:1947-1949); qid of record r is
// names[name_off[r] .. name_off[r+1])
__global__ void k_rowtxt_len(const long long* __restrict__ rows, uint64_t n, const long long* __restrict__ name_off,
                             unsigned long long* __restrict__ len) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const long long* w = rows + 5 * i;
    len[i] = (unsigned long long)(name_off[w[0] + 1] - name_off[w[0]]) + ndig_i(w[1]) + ndig_i(w[2]) +
             ndig_i(w[4]) + 6;
  }
}
__global__ void k_rowtxt_write(const long long* __restrict__ rows, uint64_t n, const char* __restrict__ names,
                               const long long* __restrict__ name_off, const unsigned long long* __restrict__ off,
                               char* __restrict__ out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const long long* w = rows + 5 * i;
    char* o = out + off[i];
    for (long long b = name_off[w[0]]; b < name_off[w[0] + 1]; ++b) *o++ = names[b];
    *o++ = '\t'; o = put_dec_i(o, w[1]); *o++ = '\t'; o = put_dec_i(o, w[2]);
    *o++ = '\t'; *o++ = w[3] == 1 ? '+' : '-'; *o++ = '\t'; o = put_dec_i(o, w[4]); *o = '\n';
  }
}

// ------------------------------------------------------------ labels from edges
// seq2graph :1932-1944: every `.xyz` node (n0_v0, then n1_v1 of each edge, in
// file order) that the `.mcl` did not label gets the next label, in order of
// first appearance.  Nodes sorted by (key, value) with their positions
// (stable radix sorts: each group's first element is its first appearance).
__global__ void k_nodes(const unsigned long long* __restrict__ tup, uint64_t nn, unsigned long long* __restrict__ key,
                        unsigned* __restrict__ val, unsigned long long* __restrict__ pos) {
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < nn; t += (uint64_t)gridDim.x * blockDim.x) {
    key[t] = tup[2 * t];                       // (n0, v0, n1, v1): node t is words 2t, 2t+1
    val[t] = (unsigned)tup[2 * t + 1];
    pos[t] = t;
  }
}
__global__ void k_gather_key(const unsigned long long* __restrict__ src, const unsigned long long* __restrict__ pos,
                             uint64_t n, unsigned long long* __restrict__ dst) {
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x)
    dst[t] = src[pos[t]];
}
// first appearances not in the .mcl table: flag the group heads
__global__ void k_node_heads(const unsigned long long* __restrict__ skey, const unsigned long long* __restrict__ pos,
                             const unsigned* __restrict__ val0, uint64_t n, const LabSlot* __restrict__ lab,
                             uint64_t lab_capmask, int have_mcl, uint8_t* __restrict__ head) {
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long kk = skey[t];
    const unsigned v = val0[pos[t]];
    bool h = t == 0 || skey[t - 1] != kk || val0[pos[t - 1]] != v;
    long long id;
    if (h && have_mcl && label_get(lab, lab_capmask, (long long)kk, (long long)v, id)) h = false;
    head[t] = h;
  }
}
__global__ void k_lab_new(const unsigned long long* __restrict__ first, uint64_t nu,
                          const unsigned long long* __restrict__ tup, long long next_id,
                          long long* __restrict__ out_key, long long* __restrict__ out_val,
                          long long* __restrict__ out_id) {
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nu; r += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long t = first[r];
    out_key[r] = (long long)tup[2 * t];
    out_val[r] = (long long)tup[2 * t + 1];
    out_id[r] = next_id + (long long)r;
  }
}

__global__ void k_gather_bounds(const unsigned long long* __restrict__ sf, const unsigned long long* __restrict__ sr,
                                const unsigned long long* __restrict__ run_off, uint64_t n,
                                unsigned long long* __restrict__ out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    out[2 * i] = sf[run_off[i]];
    out[2 * i + 1] = sr[run_off[i]];
  }
}

__global__ void k_iota64(unsigned long long* __restrict__ out, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = i;
}

// ------------------------------------------------------------------ host
template <class F>
static void with_temp(Ctx& c, F&& f) {
  size_t bytes = 0;
  PG_HIP(f((void*)nullptr, bytes));
  c.scratch.reserve(bytes + 16);
  bytes = c.scratch.cap;
  PG_HIP(f(c.scratch.p, bytes));
}

struct WalkPlan {
  std::vector<int> recs;                   // walked records, in order
  std::vector<unsigned long long> run_off; // per walked record
  uint64_t nruns = 0;
  DevBuf d_recs, d_run_off;
};

static void plan_walk(Ctx& c, const uint8_t* h_rec_flag, WalkPlan& P) {
  const uint64_t R = c.n_records;
  P.recs.clear(); P.run_off.clear();
  uint64_t runs = 0;
  for (uint64_t r = 0; r < R; ++r) {
    if (h_rec_flag && !(h_rec_flag[r] & 1)) continue;
    const int64_t n = c.h_rec_len[r];
    const int64_t nw = n < c.k ? 1 : n - c.k + 1;
    P.recs.push_back((int)r);
    P.run_off.push_back(runs);
    runs += (uint64_t)((nw + WW - 1) / WW);
  }
  P.run_off.push_back(runs);
  P.nruns = runs;
  P.d_recs.reserve(4 * (P.recs.size() + 1));
  P.d_run_off.reserve(8 * P.run_off.size());
  if (!P.recs.empty())
    PG_HIP(hipMemcpyAsync(P.d_recs.p, P.recs.data(), 4 * P.recs.size(), hipMemcpyHostToDevice, c.stream));
  PG_HIP(hipMemcpyAsync(P.d_run_off.p, P.run_off.data(), 8 * P.run_off.size(), hipMemcpyHostToDevice, c.stream));
}

static WalkArgs make_args(Ctx& c, WalkPlan& P, int rc) {
  WalkArgs a;
  ensure_cls(c);                              // (the walks read class bytes)
  a.cls = c.cls.as<uint8_t>();
  a.rec_start = c.rec_start.as<long long>();
  a.rec_len = c.rec_len.as<long long>();
  a.run_off = P.d_run_off.as<unsigned long long>();
  a.run_rec = P.d_recs.as<int>();
  a.nrec = P.recs.size();
  a.k = c.k;
  a.shift = pow5(c.k - 1);
  a.rc = rc;
  a.T = c.tv;
  a.lab = c.lab_tab.as<LabSlot>();
  a.lab_capmask = c.lab_cap ? c.lab_cap - 1 : 0;
  return a;
}

// count + scan + write: returns total hits; fills per-walk segment offsets/counts
template <int MODE>
static uint64_t walk_collect(Ctx& c, WalkPlan& P, WalkArgs& a, DevBuf& out, size_t elem,
                             std::vector<unsigned long long>& seg_off, std::vector<unsigned long long>& seg_cnt) {
  const uint64_t nr = P.nruns;
  seg_off.assign(2 * P.recs.size(), 0);
  seg_cnt.assign(2 * P.recs.size(), 0);
  if (nr == 0) return 0;
  c.tile_cnt.reserve(4 * 3 * (nr + 1));
  c.tile_off.reserve(8 * 2 * (nr + 1));
  unsigned* cf = c.tile_cnt.as<unsigned>();
  unsigned* cr = cf + (nr + 1);
  unsigned* bits = cr + (nr + 1);
  unsigned long long* sf = c.tile_off.as<unsigned long long>();
  unsigned long long* sr = sf + (nr + 1);
  PG_HIP(hipMemsetAsync(cf + nr, 0, 4, c.stream));
  PG_HIP(hipMemsetAsync(cr + nr, 0, 4, c.stream));
  hipLaunchKernelGGL((k_walk_count<MODE>), dim3(grid_for(nr, WBLOCK, 8192)), dim3(WBLOCK), 0, c.stream, a, nr, cf,
                     cr, bits);
  PG_HIP(hipGetLastError());
  with_temp(c, [&](void* tmp, size_t& bytes) {
    return rocprim::exclusive_scan(tmp, bytes, cf, sf, 0ull, (size_t)nr + 1, rocprim::plus<unsigned long long>(),
                                   c.stream);
  });
  with_temp(c, [&](void* tmp, size_t& bytes) {
    return rocprim::exclusive_scan(tmp, bytes, cr, sr, 0ull, (size_t)nr + 1, rocprim::plus<unsigned long long>(),
                                   c.stream);
  });
  // per-record segment bounds: scan values at each record's first run
  const size_t nb = P.run_off.size();
  DevBuf g;
  g.reserve(16 * nb);
  hipLaunchKernelGGL(k_gather_bounds, dim3(grid_for(nb, 256, 4096)), dim3(256), 0, c.stream, sf, sr,
                     P.d_run_off.as<unsigned long long>(), (uint64_t)nb, g.as<unsigned long long>());
  PG_HIP(hipGetLastError());
  std::vector<unsigned long long> hb(2 * nb), hf(nb), hr(nb);
  PG_HIP(hipMemcpyAsync(hb.data(), g.p, 16 * nb, hipMemcpyDeviceToHost, c.stream));
  c.sync();
  g.release();
  for (size_t i = 0; i < nb; ++i) { hf[i] = hb[2 * i]; hr[i] = hb[2 * i + 1]; }
  const uint64_t total = hf.back() + hr.back();
  for (size_t i = 0; i < P.recs.size(); ++i) {
    const unsigned long long F = hf[i + 1] - hf[i], Rv = hr[i + 1] - hr[i];
    seg_off[2 * i] = hf[i] + hr[i];
    seg_cnt[2 * i] = F;
    seg_off[2 * i + 1] = hf[i] + hr[i] + F;
    seg_cnt[2 * i + 1] = Rv;
  }
  out.reserve(elem * (total + 1));
  if (total)
    hipLaunchKernelGGL((k_walk_write<MODE>), dim3(grid_for(nr, WBLOCK, 8192)), dim3(WBLOCK), 0, c.stream, a, nr,
                       sf, sr, bits, out.p);
  PG_HIP(hipGetLastError());
  c.sync();
  return total;
}

// rocPRIM helpers on the context's stream and scratch
template <class K, class V>
static void sort_pairs(Ctx& c, const K* kin, K* kout, const V* vin, V* vout, uint64_t n, int end_bit) {
  with_temp(c, [&](void* tmp, size_t& bytes) {
    return rocprim::radix_sort_pairs(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0, end_bit, c.stream);
  });
}
template <class T>
static uint64_t select_flagged(Ctx& c, const T* in, const uint8_t* flags, T* out, uint64_t n, DevBuf& cnt) {
  cnt.reserve(16);
  with_temp(c, [&](void* tmp, size_t& bytes) {
    return rocprim::select(tmp, bytes, in, flags, out, cnt.as<unsigned long long>(), (size_t)n, c.stream);
  });
  unsigned long long h = 0;
  PG_HIP(hipMemcpyAsync(&h, cnt.p, 8, hipMemcpyDeviceToHost, c.stream));
  c.sync();
  return h;
}
static uint64_t excl_scan_total(Ctx& c, const unsigned long long* len, unsigned long long* off, uint64_t n) {
  // off[0..n]: exclusive prefix sums, off[n] = total
  PG_HIP(hipMemsetAsync(const_cast<unsigned long long*>(len) + n, 0, 8, c.stream));
  with_temp(c, [&](void* tmp, size_t& bytes) {
    return rocprim::exclusive_scan(tmp, bytes, len, off, 0ull, (size_t)n + 1, rocprim::plus<unsigned long long>(),
                                   c.stream);
  });
  unsigned long long h = 0;
  PG_HIP(hipMemcpyAsync(&h, off + n, 8, hipMemcpyDeviceToHost, c.stream));
  c.sync();
  return h;
}
static int bits_for(uint64_t maxv) {
  int b = 1;
  while (b < 64 && (maxv >> b)) ++b;
  return b;
}

uint64_t walk_edges(Ctx& c, const uint8_t* h_rec_flag, int rc1) {
  if (!c.reduced) throw Error(-22, "pg_edges: no rdBG (call pg_build_rdbg first)");
  WalkPlan P;
  plan_walk(c, h_rec_flag, P);
  WalkArgs a = make_args(c, P, rc1);
  std::vector<unsigned long long> so, sc;
  const uint64_t m = walk_collect<0>(c, P, a, c.occ, sizeof(Occ), so, sc);
  c.n_edges = 0;
  c.text_xyz = false;
  // Distinct edges join rdBG members: the edge table starts at 4 slots per
  // rdBG key (C3: 1.93 M keys, 2.5 M edges among 1e8 member occurrences) and
  // grows (x4, up to 2 per occurrence) when a probe sequence runs long.  The
  // (edge, walk) set holds one entry per occurrence at most.
  const uint64_t emax = next_pow2(std::max<uint64_t>(1024, 2 * m));
  uint64_t ecap = std::min(emax, next_pow2(std::max<uint64_t>(1024, 4 * (c.n_rdbg + 1))));
  const uint64_t pcap = emax;
  c.pair_cap = pcap;
  c.pair_tab.reserve(8 * pcap);
  DevBuf err;
  err.reserve(16);
  unsigned long long n_out = 0;
  for (;;) {
    c.edge_cap = ecap;
    c.edge_tab.reserve(sizeof(EdgeSlot) * ecap);
    PG_HIP(hipMemsetAsync(c.edge_tab.p, 0, sizeof(EdgeSlot) * ecap, c.stream));
    PG_HIP(hipMemsetAsync(c.pair_tab.p, 0, 8 * pcap, c.stream));
    PG_HIP(hipMemsetAsync(err.p, 0, 16, c.stream));
    if (m > 1) {
      DevBuf rb;
      rb.reserve(8 * 2 * (m + 2));
      unsigned long long* lists[2] = {rb.as<unsigned long long>(), rb.as<unsigned long long>() + (m + 1)};
      DevBuf nr;
      nr.reserve(16);
      const unsigned long long* cur = nullptr;
      uint64_t ncur = m;
      for (int round = 0; ncur && round < 64; ++round) {
        unsigned long long* out = lists[round & 1];
        PG_HIP(hipMemsetAsync(nr.p, 0, 8, c.stream));
        hipLaunchKernelGGL(k_edges, dim3(grid_for(ncur, 256, 16384)), dim3(256), 0, c.stream, c.occ.as<Occ>(), m,
                           cur, ncur, c.edge_tab.as<EdgeSlot>(), ecap - 1, c.pair_tab.as<unsigned long long>(),
                           pcap - 1, out, nr.as<unsigned long long>(), err.as<unsigned>());
        PG_HIP(hipGetLastError());
        unsigned long long nn = 0;
        PG_HIP(hipMemcpyAsync(&nn, nr.p, 8, hipMemcpyDeviceToHost, c.stream));
        c.sync();
        cur = out;
        ncur = nn;
      }
      if (ncur) throw Error(-5, "pg_edges: edge insert did not converge");
    }
    unsigned e = 0;
    // (c.stream is non-blocking: a null-stream hipMemcpy would not wait for the
    // memset above when m <= 1 queued nothing that synced)
    PG_HIP(hipMemcpyAsync(&e, err.p, 4, hipMemcpyDeviceToHost, c.stream));
    c.sync();
    if ((e & 2u) && ecap < emax) {                              // the edge table was too small: again, larger
      ecap = std::min(emax, ecap * 4);
      continue;
    }
    if (e) throw Error(-5, "pg_edges: edge table error " + std::to_string(e));
    break;
  }
  if (m > 1) {
    // compact, then order by first occurrence on the device
    DevBuf cnt;
    cnt.reserve(8);
    PG_HIP(hipMemsetAsync(cnt.p, 0, 8, c.stream));
    c.edge_out.reserve(sizeof(EdgeOut) * std::max<uint64_t>(m, 1));
    DevBuf kv;
    kv.reserve((8 + 8 + 4 + 4) * std::min<uint64_t>(m, ecap) + 64);
    auto* k0 = kv.as<unsigned long long>();
    auto* k1 = k0 + std::min<uint64_t>(m, ecap);
    auto* v0 = reinterpret_cast<unsigned*>(k1 + std::min<uint64_t>(m, ecap));
    auto* v1 = v0 + std::min<uint64_t>(m, ecap);
    hipLaunchKernelGGL(k_edges_compact, dim3(grid_for(ecap, 256, 8192)), dim3(256), 0, c.stream,
                       c.edge_tab.as<EdgeSlot>(), ecap, c.occ.as<Occ>(), c.edge_out.as<EdgeOut>(), k0, v0,
                       cnt.as<unsigned long long>());
    PG_HIP(hipGetLastError());
    PG_HIP(hipMemcpyAsync(&n_out, cnt.p, 8, hipMemcpyDeviceToHost, c.stream));
    c.sync();
    if (n_out) {
      sort_pairs(c, k0, k1, v0, v1, n_out, bits_for(m));
      c.edge_exp.reserve((8 * 4 + 8 + 8) * n_out);
      auto* tup = c.edge_exp.as<unsigned long long>();
      auto* ecnt = reinterpret_cast<long long*>(tup + 4 * n_out);
      auto* ewalk = ecnt + n_out;
      hipLaunchKernelGGL(k_edges_order, dim3(grid_for(n_out, 256, 8192)), dim3(256), 0, c.stream,
                         c.edge_out.as<EdgeOut>(), v1, n_out, tup, ecnt, ewalk);
      PG_HIP(hipGetLastError());
      c.sync();
    }
  }
  c.n_edges = n_out;
  return n_out;
}

void export_edges(Ctx& c, uint64_t* tuples, int64_t* counts, int64_t* first_walk, uint64_t cap) {
  const uint64_t n = std::min<uint64_t>(cap, c.n_edges);
  if (!n) return;
  const auto* tup = c.edge_exp.as<unsigned long long>();
  const auto* ecnt = reinterpret_cast<const long long*>(tup + 4 * c.n_edges);
  const auto* ewalk = ecnt + c.n_edges;
  PG_HIP(hipMemcpyAsync(tuples, tup, 32 * n, hipMemcpyDeviceToHost, c.stream));
  PG_HIP(hipMemcpyAsync(counts, ecnt, 8 * n, hipMemcpyDeviceToHost, c.stream));
  PG_HIP(hipMemcpyAsync(first_walk, ewalk, 8 * n, hipMemcpyDeviceToHost, c.stream));
  c.sync();
}

// the .xyz text of the last edge pass, in first-occurrence order: its size
// (out null, fd < 0), copied into out, or written to descriptor fd
uint64_t format_edges(Ctx& c, char* out, uint64_t cap, int fd) {
  const uint64_t n = c.n_edges;
  if (!c.text_xyz) {
    c.text_len.reserve(8 * (n + 1));
    c.text_off.reserve(8 * (n + 1));
    const auto* tup = c.edge_exp.as<unsigned long long>();
    const auto* ecnt = reinterpret_cast<const long long*>(tup + 4 * n);
    if (n) {
      hipLaunchKernelGGL(k_xyz_len, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c.stream, tup, ecnt, n,
                         c.text_len.as<unsigned long long>());
      PG_HIP(hipGetLastError());
    }
    c.text_total = excl_scan_total(c, c.text_len.as<unsigned long long>(), c.text_off.as<unsigned long long>(), n);
    c.text_xyz = true;
    c.text_rows = false;
  }
  if (!out && fd < 0) return c.text_total;
  if (out && cap < c.text_total) throw Error(-34, "pg_edges_format: buffer too small");
  if (n) {
    c.text_buf.reserve(c.text_total + 16);
    const auto* tup = c.edge_exp.as<unsigned long long>();
    const auto* ecnt = reinterpret_cast<const long long*>(tup + 4 * n);
    hipLaunchKernelGGL(k_xyz_write, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c.stream, tup, ecnt, n,
                       c.text_off.as<unsigned long long>(), c.text_buf.as<char>());
    PG_HIP(hipGetLastError());
    if (out) PG_HIP(hipMemcpyAsync(out, c.text_buf.p, c.text_total, hipMemcpyDeviceToHost, c.stream));
    c.sync();
    if (!out) text_to_fd(c, c.text_buf.as<uint8_t>(), c.text_total, fd, "pg_edges_format_fd");
  }
  return c.text_total;
}

static void lab_build(Ctx& c, const long long* d_key, const long long* d_val, const long long* d_id, uint64_t n) {
  const uint64_t cap = next_pow2(std::max<uint64_t>(1024, 2 * n + 16));
  c.lab_cap = cap;
  c.lab_tab.reserve(sizeof(LabSlot) * cap);
  PG_HIP(hipMemsetAsync(c.lab_tab.p, 0, sizeof(LabSlot) * cap, c.stream));
  if (n) {
    hipLaunchKernelGGL(k_lab_insert, dim3(grid_for(n, 256, 4096)), dim3(256), 0, c.stream, d_key, d_val, d_id, n,
                       c.lab_tab.as<LabSlot>(), cap - 1);
    PG_HIP(hipGetLastError());
  }
}

void set_labels(Ctx& c, const int64_t* key, const int64_t* val, const int64_t* id, uint64_t n) {
  c.lab_list.reserve(24 * (n + 1));
  long long* dk = c.lab_list.as<long long>();
  if (n) {
    PG_HIP(hipMemcpyAsync(dk, key, 8 * n, hipMemcpyHostToDevice, c.stream));
    PG_HIP(hipMemcpyAsync(dk + n, val, 8 * n, hipMemcpyHostToDevice, c.stream));
    PG_HIP(hipMemcpyAsync(dk + 2 * n, id, 8 * n, hipMemcpyHostToDevice, c.stream));
  }
  lab_build(c, dk, dk + n, dk + 2 * n, n);
  c.n_labels = n;
  c.sync();
}

// seq2graph's label dictionary (:1918-1944) built on the device: the `.mcl`
// entries (the host's dict of line indices, a later line winning), then the
// `.xyz` nodes the .mcl did not label, numbered next_id, next_id + 1, ... in
// order of first appearance.  Edges: h_tuples (n x 4, file order) or, when
// NULL, the last edge pass in first-occurrence order.
uint64_t labels_from_edges(Ctx& c, const uint64_t* h_tuples, uint64_t n_edges, const int64_t* mk, const int64_t* mv,
                           const int64_t* mi, uint64_t n_mcl, int64_t next_id) {
  DevBuf up;
  const unsigned long long* tup;
  if (h_tuples) {
    up.reserve(32 * (n_edges + 1));
    if (n_edges) PG_HIP(hipMemcpyAsync(up.p, h_tuples, 32 * n_edges, hipMemcpyHostToDevice, c.stream));
    tup = up.as<unsigned long long>();
  } else {
    n_edges = c.n_edges;
    tup = c.edge_exp.as<unsigned long long>();
  }
  // the .mcl entries first (their table answers "labelled by the .mcl?")
  DevBuf mcl;
  mcl.reserve(24 * (n_mcl + 1));
  long long* dk = mcl.as<long long>();
  if (n_mcl) {
    PG_HIP(hipMemcpyAsync(dk, mk, 8 * n_mcl, hipMemcpyHostToDevice, c.stream));
    PG_HIP(hipMemcpyAsync(dk + n_mcl, mv, 8 * n_mcl, hipMemcpyHostToDevice, c.stream));
    PG_HIP(hipMemcpyAsync(dk + 2 * n_mcl, mi, 8 * n_mcl, hipMemcpyHostToDevice, c.stream));
  }
  lab_build(c, dk, dk + n_mcl, dk + 2 * n_mcl, n_mcl);
  const uint64_t nn = 2 * n_edges;
  uint64_t nu = 0;
  DevBuf firsts;
  if (nn) {
    // nodes -> sorted by value, then stably by key, positions carried
    DevBuf w;
    w.reserve((8 + 8 + 4 + 4 + 8 + 8 + 8) * nn + 64);
    auto* key = w.as<unsigned long long>();
    auto* skey = key + nn;
    auto* pos = skey + nn;
    auto* pos2 = pos + nn;
    auto* tmpk = pos2 + nn;
    auto* val = reinterpret_cast<unsigned*>(tmpk + nn);
    auto* sval = val + nn;
    hipLaunchKernelGGL(k_nodes, dim3(grid_for(nn, 256, 8192)), dim3(256), 0, c.stream, tup, nn, key, val, pos);
    PG_HIP(hipGetLastError());
    uint64_t maxv = 0xFFFFu, maxk = ~0ull;
    if (h_tuples) {
      maxv = 0;
      for (uint64_t i = 0; i < nn; ++i) maxv = std::max<uint64_t>(maxv, h_tuples[2 * i + 1]);
    }
    if (maxv > 0xFFFFFFFFull) throw Error(-22, "pg_labels_from_edges: node value above 2^32");
    sort_pairs(c, val, sval, pos, pos2, nn, bits_for(maxv));          // by value
    hipLaunchKernelGGL(k_gather_key, dim3(grid_for(nn, 256, 8192)), dim3(256), 0, c.stream, key, pos2, nn, tmpk);
    PG_HIP(hipGetLastError());
    sort_pairs(c, tmpk, skey, pos2, pos, nn, bits_for(maxk));           // then stably by key
    DevBuf flag, cnt;
    flag.reserve(nn + 16);
    hipLaunchKernelGGL(k_node_heads, dim3(grid_for(nn, 256, 8192)), dim3(256), 0, c.stream, skey, pos, val, nn,
                       c.lab_tab.as<LabSlot>(), c.lab_cap - 1, (int)(n_mcl != 0), flag.as<uint8_t>());
    PG_HIP(hipGetLastError());
    firsts.reserve(16 * nn + 16);
    auto* f0 = firsts.as<unsigned long long>();
    nu = select_flagged(c, pos, flag.as<uint8_t>(), f0, nn, cnt);
    if (nu) {
      with_temp(c, [&](void* tmp, size_t& bytes) {
        return rocprim::radix_sort_keys(tmp, bytes, f0, f0 + nn, (size_t)nu, 0, bits_for(nn), c.stream);
      });
    }
    // the label list: .mcl entries, then the new ones in order
    c.lab_list.reserve(24 * (n_mcl + nu + 1));
    long long* L = c.lab_list.as<long long>();
    const uint64_t nl = n_mcl + nu;
    if (n_mcl) {
      PG_HIP(hipMemcpyAsync(L, dk, 8 * n_mcl, hipMemcpyDeviceToDevice, c.stream));
      PG_HIP(hipMemcpyAsync(L + nl, dk + n_mcl, 8 * n_mcl, hipMemcpyDeviceToDevice, c.stream));
      PG_HIP(hipMemcpyAsync(L + 2 * nl, dk + 2 * n_mcl, 8 * n_mcl, hipMemcpyDeviceToDevice, c.stream));
    }
    if (nu) {
      hipLaunchKernelGGL(k_lab_new, dim3(grid_for(nu, 256, 8192)), dim3(256), 0, c.stream, f0 + nn, nu, tup,
                         (long long)next_id, L + n_mcl, L + nl + n_mcl, L + 2 * nl + n_mcl);
      PG_HIP(hipGetLastError());
    }
    lab_build(c, L, L + nl, L + 2 * nl, nl);
    c.n_labels = nl;
  } else {
    c.lab_list.reserve(24 * (n_mcl + 1));
    long long* L = c.lab_list.as<long long>();
    if (n_mcl) PG_HIP(hipMemcpyAsync(L, dk, 24 * n_mcl, hipMemcpyDeviceToDevice, c.stream));
    c.n_labels = n_mcl;
  }
  c.sync();
  return c.n_labels;
}

void export_labels(Ctx& c, int64_t* key, int64_t* val, int64_t* id, uint64_t cap) {
  const uint64_t n = c.n_labels;
  if (cap < n) throw Error(-34, "pg_labels_export: buffer too small");
  if (!n) return;
  const long long* L = c.lab_list.as<long long>();
  PG_HIP(hipMemcpyAsync(key, L, 8 * n, hipMemcpyDeviceToHost, c.stream));
  PG_HIP(hipMemcpyAsync(val, L + n, 8 * n, hipMemcpyDeviceToHost, c.stream));
  PG_HIP(hipMemcpyAsync(id, L + 2 * n, 8 * n, hipMemcpyDeviceToHost, c.stream));
  c.sync();
}

uint64_t walk_rows(Ctx& c, const uint8_t* h_rec_flag, int rc1) {
  if (!c.parsed) throw Error(-22, "pg_rows: no parsed FASTA");
  if (!c.lab_cap) set_labels(c, nullptr, nullptr, nullptr, 0);
  WalkPlan P;
  plan_walk(c, h_rec_flag, P);
  WalkArgs a = make_args(c, P, rc1);
  std::vector<unsigned long long> so, sc;
  DevBuf hits;
  const uint64_t m = walk_collect<1>(c, P, a, hits, sizeof(Hit), so, sc);
  const uint64_t nseg = so.size();
  c.n_rows = 0;
  c.text_rows = false;
  if (nseg == 0 || m == 0) return 0;
  // walk bounds (segments are contiguous in walk order)
  DevBuf meta;
  meta.reserve(8 * (nseg + 2));
  std::vector<unsigned long long> bounds(nseg + 1);
  for (size_t w = 0; w < nseg; ++w) bounds[w] = so[w];
  bounds[nseg] = m;
  PG_HIP(hipMemcpyAsync(meta.p, bounds.data(), 8 * (nseg + 1), hipMemcpyHostToDevice, c.stream));
  const auto* d_bounds = meta.as<unsigned long long>();
  DevBuf flag, cnt, acc;
  flag.reserve(m + 16);
  acc.reserve(8 * (m + 1));
  hipLaunchKernelGGL(k_taken, dim3(grid_for(m, 256, 16384)), dim3(256), 0, c.stream, hits.as<Hit>(), m, d_bounds,
                     (uint32_t)nseg, c.k, flag.as<uint8_t>());
  PG_HIP(hipGetLastError());
  // indices of the taken hits (a counting iterator through rocprim::select)
  DevBuf idx;
  idx.reserve(8 * (m + 1));
  hipLaunchKernelGGL(k_iota64, dim3(grid_for(m, 256, 16384)), dim3(256), 0, c.stream, idx.as<unsigned long long>(), m);
  PG_HIP(hipGetLastError());
  const uint64_t na = select_flagged(c, idx.as<unsigned long long>(), flag.as<uint8_t>(),
                                     acc.as<unsigned long long>(), m, cnt);
  if (na == 0) return 0;
  hipLaunchKernelGGL(k_row_heads, dim3(grid_for(na, 256, 16384)), dim3(256), 0, c.stream, hits.as<Hit>(),
                     acc.as<unsigned long long>(), na, d_bounds, (uint32_t)nseg, flag.as<uint8_t>());
  PG_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_iota64, dim3(grid_for(na, 256, 16384)), dim3(256), 0, c.stream, idx.as<unsigned long long>(), na);
  PG_HIP(hipGetLastError());
  DevBuf starts;
  starts.reserve(8 * (na + 1));
  const uint64_t nrows = select_flagged(c, idx.as<unsigned long long>(), flag.as<uint8_t>(),
                                        starts.as<unsigned long long>(), na, cnt);
  c.rows_buf.reserve(40 * (nrows + 1));
  hipLaunchKernelGGL(k_rows, dim3(grid_for(nrows, 256, 16384)), dim3(256), 0, c.stream, hits.as<Hit>(),
                     acc.as<unsigned long long>(), na, starts.as<unsigned long long>(), nrows, d_bounds,
                     (uint32_t)nseg, P.d_recs.as<int>(), c.rec_len.as<long long>(), c.k, c.rows_buf.as<long long>());
  PG_HIP(hipGetLastError());
  c.sync();
  c.n_rows = nrows;
  return nrows;
}

void export_rows(Ctx& c, int64_t* rows5, uint64_t cap) {
  if (cap < c.n_rows) throw Error(-34, "pg_rows_export: buffer too small");
  if (!c.n_rows) return;
  PG_HIP(hipMemcpyAsync(rows5, c.rows_buf.p, 40 * c.n_rows, hipMemcpyDeviceToHost, c.stream));
  c.sync();
}

// the region rows' text of the last row pass; names[name_off[r] ..
// name_off[r+1]) is record r's qid (R + 1 offsets).  Its size (out null,
// fd < 0), copied into out, or written to descriptor fd.
uint64_t format_rows_text(Ctx& c, const char* names, const int64_t* name_off, uint64_t n_names, char* out,
                          uint64_t cap, int fd) {
  const uint64_t n = c.n_rows;
  if (!c.text_rows) {
    c.text_names.reserve(8 * (n_names + 1) + (uint64_t)std::max<int64_t>(name_off[n_names], 0) + 16);
    long long* d_off = c.text_names.as<long long>();
    char* d_names = reinterpret_cast<char*>(d_off + n_names + 1);
    PG_HIP(hipMemcpyAsync(d_off, name_off, 8 * (n_names + 1), hipMemcpyHostToDevice, c.stream));
    if (name_off[n_names])
      PG_HIP(hipMemcpyAsync(d_names, names, (size_t)name_off[n_names], hipMemcpyHostToDevice, c.stream));
    c.text_len.reserve(8 * (n + 1));
    c.text_off.reserve(8 * (n + 1));
    if (n) {
      hipLaunchKernelGGL(k_rowtxt_len, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c.stream,
                         c.rows_buf.as<long long>(), n, d_off, c.text_len.as<unsigned long long>());
      PG_HIP(hipGetLastError());
    }
    c.text_total = excl_scan_total(c, c.text_len.as<unsigned long long>(), c.text_off.as<unsigned long long>(), n);
    c.text_rows = true;
    c.text_xyz = false;
  }
  if (!out && fd < 0) return c.text_total;
  if (out && cap < c.text_total) throw Error(-34, "pg_rows_format: buffer too small");
  if (n) {
    const long long* d_off = c.text_names.as<long long>();
    const char* d_names = reinterpret_cast<const char*>(d_off + n_names + 1);
    c.text_buf.reserve(c.text_total + 16);
    hipLaunchKernelGGL(k_rowtxt_write, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c.stream,
                       c.rows_buf.as<long long>(), n, d_names, d_off, c.text_off.as<unsigned long long>(),
                       c.text_buf.as<char>());
    PG_HIP(hipGetLastError());
    if (out) PG_HIP(hipMemcpyAsync(out, c.text_buf.p, c.text_total, hipMemcpyDeviceToHost, c.stream));
    c.sync();
    if (!out) text_to_fd(c, c.text_buf.as<uint8_t>(), c.text_total, fd, "pg_rows_format_fd");
  }
  return c.text_total;
}

}  // namespace pg
