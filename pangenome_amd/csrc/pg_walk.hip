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
__device__ uint64_t edge_find_or_insert(EdgeSlot* __restrict__ tab, uint64_t capmask, uint64_t n0, uint32_t v0,
                                        uint64_t n1, uint32_t v1, unsigned* err) {
  const unsigned long long a = n0 + 1ull, bkey = n1 + 1ull;
  const unsigned vv = v0 | (v1 << 16) | 0x80000000u;
  uint64_t slot = fmix64(n0 * 0x9e3779b97f4a7c15ull ^ fmix64(n1 ^ ((uint64_t)vv << 40))) & capmask;
  for (uint64_t probe = 0; probe <= capmask; ++probe) {
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
                                EdgeOut* __restrict__ out, unsigned long long* __restrict__ counter) {
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
    if (used)
      out[base + __builtin_popcountll(bal & lt)] =
          EdgeOut{s.n0p1 - 1ull, s.n1p1 - 1ull, s.vv & 0xFFFFu, (s.vv >> 16) & 0x7FFFu, s.count, ~s.first,
                  occ[~s.first].walk};
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

// seq2path_jit_'s greedy merge (:1546-1560) for one walk per thread.  State is
// (starts[-1], labels[-1]); rows (starts[i-1], starts[i], labels[i]) leave as
// int32 (:1533) and reverse-strand rows are mirrored to (n-end, n-start) (:1843).
__global__ void k_regions(const Hit* __restrict__ hits, const unsigned long long* __restrict__ seg_off,
                          const unsigned long long* __restrict__ seg_cnt, const long long* __restrict__ seg_len,
                          uint64_t nseg, int k, long long* __restrict__ rows, unsigned long long* __restrict__ nrows) {
  for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < nseg; w += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long off = seg_off[w], cnt = seg_cnt[w];
    const long long lseq = seg_len[w >> 1];
    const bool rc = w & 1;
    long long last = 0, last_label = -1;
    unsigned long long nr = 0;
    long long* out = rows + 3 * off;
    for (unsigned long long j = 0; j < cnt; ++j) {
      const Hit h = hits[off + j];
      if (last < (long long)h.idx) {
        const long long pos = (long long)h.idx + k;
        if (last_label != h.label) {
          out[3 * nr] = last; out[3 * nr + 1] = pos; out[3 * nr + 2] = h.label;
          ++nr;
          last_label = h.label;
        } else if (nr > 0) {
          out[3 * (nr - 1) + 1] = pos;
        }
        last = pos;
      }
    }
    for (unsigned long long i = 0; i < nr; ++i) {
      const int st = (int)out[3 * i], ed = (int)out[3 * i + 1];
      const int lb = (int)out[3 * i + 2];
      if (rc) { out[3 * i] = (int)(lseq - ed); out[3 * i + 1] = (int)(lseq - st); }
      else { out[3 * i] = st; out[3 * i + 1] = ed; }
      out[3 * i + 2] = lb;
    }
    nrows[w] = nr;
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

uint64_t walk_edges(Ctx& c, const uint8_t* h_rec_flag, int rc1) {
  if (!c.reduced) throw Error(-22, "pg_edges: no rdBG (call pg_build_rdbg first)");
  WalkPlan P;
  plan_walk(c, h_rec_flag, P);
  WalkArgs a = make_args(c, P, rc1);
  std::vector<unsigned long long> so, sc;
  const uint64_t m = walk_collect<0>(c, P, a, c.occ, sizeof(Occ), so, sc);
  c.n_edges = 0;
  const uint64_t ecap = next_pow2(std::max<uint64_t>(1024, 2 * m));
  c.edge_cap = ecap;
  c.pair_cap = ecap;
  c.edge_tab.reserve(sizeof(EdgeSlot) * ecap);
  c.pair_tab.reserve(8 * ecap);
  PG_HIP(hipMemsetAsync(c.edge_tab.p, 0, sizeof(EdgeSlot) * ecap, c.stream));
  PG_HIP(hipMemsetAsync(c.pair_tab.p, 0, 8 * ecap, c.stream));
  DevBuf err;
  err.reserve(16);
  PG_HIP(hipMemsetAsync(err.p, 0, 16, c.stream));
  c.edge_out.reserve(sizeof(EdgeOut) * (m + 1));
  unsigned long long n_out = 0;
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
                         ecap - 1, out, nr.as<unsigned long long>(), err.as<unsigned>());
      PG_HIP(hipGetLastError());
      unsigned long long nn = 0;
      PG_HIP(hipMemcpyAsync(&nn, nr.p, 8, hipMemcpyDeviceToHost, c.stream));
      c.sync();
      cur = out;
      ncur = nn;
    }
    if (ncur) throw Error(-5, "pg_edges: edge insert did not converge");
    rb.release();
    nr.release();
    DevBuf cnt;
    cnt.reserve(8);
    PG_HIP(hipMemsetAsync(cnt.p, 0, 8, c.stream));
    hipLaunchKernelGGL(k_edges_compact, dim3(grid_for(ecap, 256, 8192)), dim3(256), 0, c.stream,
                       c.edge_tab.as<EdgeSlot>(), ecap, c.occ.as<Occ>(), c.edge_out.as<EdgeOut>(),
                       cnt.as<unsigned long long>());
    PG_HIP(hipGetLastError());
    PG_HIP(hipMemcpyAsync(&n_out, cnt.p, 8, hipMemcpyDeviceToHost, c.stream));
    c.sync();
    cnt.release();
  }
  unsigned e = 0;
  // (c.stream is non-blocking: a null-stream hipMemcpy would not wait for the
  // memset above when m <= 1 queued nothing that synced)
  PG_HIP(hipMemcpyAsync(&e, err.p, 4, hipMemcpyDeviceToHost, c.stream));
  c.sync();
  err.release();
  if (e) throw Error(-5, "pg_edges: edge table error " + std::to_string(e));
  c.n_edges = n_out;
  return n_out;
}

void export_edges(Ctx& c, uint64_t* tuples, int64_t* counts, int64_t* first_walk, uint64_t cap) {
  const uint64_t n = std::min<uint64_t>(cap, c.n_edges);
  std::vector<EdgeOut> h(n);
  if (n) {
    PG_HIP(hipMemcpyAsync(h.data(), c.edge_out.p, sizeof(EdgeOut) * n, hipMemcpyDeviceToHost, c.stream));
    c.sync();
  }
  // order by first occurrence (typed-Dict insertion order, :1479-1484)
  std::vector<uint64_t> idx(n);
  for (uint64_t i = 0; i < n; ++i) idx[i] = i;
  std::sort(idx.begin(), idx.end(), [&](uint64_t a, uint64_t b) { return h[a].first < h[b].first; });
  for (uint64_t j = 0; j < n; ++j) {
    const EdgeOut& e = h[idx[j]];
    tuples[4 * j] = e.n0; tuples[4 * j + 1] = e.v0; tuples[4 * j + 2] = e.n1; tuples[4 * j + 3] = e.v1;
    counts[j] = (int64_t)e.count;
    first_walk[j] = (int64_t)e.walk;
  }
}

void set_labels(Ctx& c, const int64_t* key, const int64_t* val, const int64_t* id, uint64_t n) {
  const uint64_t cap = next_pow2(std::max<uint64_t>(1024, 2 * n + 16));
  c.lab_cap = cap;
  c.lab_tab.reserve(sizeof(LabSlot) * cap);
  PG_HIP(hipMemsetAsync(c.lab_tab.p, 0, sizeof(LabSlot) * cap, c.stream));
  if (n) {
    DevBuf tmp;
    tmp.reserve(24 * n);
    long long* dk = tmp.as<long long>();
    PG_HIP(hipMemcpyAsync(dk, key, 8 * n, hipMemcpyHostToDevice, c.stream));
    PG_HIP(hipMemcpyAsync(dk + n, val, 8 * n, hipMemcpyHostToDevice, c.stream));
    PG_HIP(hipMemcpyAsync(dk + 2 * n, id, 8 * n, hipMemcpyHostToDevice, c.stream));
    hipLaunchKernelGGL(k_lab_insert, dim3(grid_for(n, 256, 4096)), dim3(256), 0, c.stream, dk, dk + n, dk + 2 * n,
                       n, c.lab_tab.as<LabSlot>(), cap - 1);
    PG_HIP(hipGetLastError());
    c.sync();
    tmp.release();
  }
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
  c.h_rows.clear();
  c.n_rows = 0;
  if (nseg == 0) return 0;
  DevBuf meta;
  meta.reserve(8 * 4 * nseg);
  auto* d_so = meta.as<unsigned long long>();
  auto* d_sc = d_so + nseg;
  auto* d_len = reinterpret_cast<long long*>(d_sc + nseg);
  auto* d_nr = reinterpret_cast<unsigned long long*>(d_len + nseg);
  std::vector<long long> lens(nseg / 2);
  for (size_t i = 0; i < P.recs.size(); ++i) lens[i] = c.h_rec_len[P.recs[i]];
  PG_HIP(hipMemcpyAsync(d_so, so.data(), 8 * nseg, hipMemcpyHostToDevice, c.stream));
  PG_HIP(hipMemcpyAsync(d_sc, sc.data(), 8 * nseg, hipMemcpyHostToDevice, c.stream));
  PG_HIP(hipMemcpyAsync(d_len, lens.data(), 8 * lens.size(), hipMemcpyHostToDevice, c.stream));
  c.rows_buf.reserve(24 * (m + 1));
  hipLaunchKernelGGL(k_regions, dim3(grid_for(nseg, 64, 4096)), dim3(64), 0, c.stream, hits.as<Hit>(), d_so, d_sc,
                     d_len, nseg, c.k, c.rows_buf.as<long long>(), d_nr);
  PG_HIP(hipGetLastError());
  std::vector<unsigned long long> nr(nseg);
  PG_HIP(hipMemcpyAsync(nr.data(), d_nr, 8 * nseg, hipMemcpyDeviceToHost, c.stream));
  std::vector<long long> rows(3 * (m + 1));
  if (m) PG_HIP(hipMemcpyAsync(rows.data(), c.rows_buf.p, 24 * m, hipMemcpyDeviceToHost, c.stream));
  c.sync();
  // rows in reference order: record, forward rows then reverse rows (:1836-1844)
  for (size_t i = 0; i < P.recs.size(); ++i) {
    for (int s = 0; s < 2; ++s) {
      const size_t w = 2 * i + s;
      for (unsigned long long j = 0; j < nr[w]; ++j) {
        const long long* rw = &rows[3 * (so[w] + j)];
        c.h_rows.push_back(P.recs[i]);
        c.h_rows.push_back(rw[0]);
        c.h_rows.push_back(rw[1]);
        c.h_rows.push_back(s == 0 ? 1 : -1);
        c.h_rows.push_back(rw[2]);
      }
    }
  }
  c.n_rows = c.h_rows.size() / 5;
  meta.release();
  hits.release();
  return c.n_rows;
}

}  // namespace pg
