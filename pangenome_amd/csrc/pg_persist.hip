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
//   k_dump_place     each present oriented key claims the first free slot of
//       oakht.pointer's probe sequence (:521-538): j = FNV-1a(low 4 key bytes)
//       mod capacity, then j, j+1, j+4, j+9, ... .  Any insertion order gives a
//       layout lookups accept: a key's earlier probes were occupied when it
//       was placed and nothing is ever removed.
#include <cstring>

#include "pg_internal.h"

namespace pg {

constexpr int PBLK = 256;
constexpr int CW = 16;                              // windows per thread
constexpr uint64_t CCHUNK = (uint64_t)PBLK * CW;   // windows per block

__device__ __forceinline__ void count_at(const TableView& T, unsigned* cnt, uint64_t c, int orient, unsigned add) {
  const uint64_t e = tab_find(T, c);
  if (e != ~0ull) atomicAdd(cnt + 2 * e + orient, add);
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
    if (RC && K == Kr) { count_at(T, cnt, c, 0, 2u); continue; }   // palindrome: one key, twice
    count_at(T, cnt, c, K <= Kr ? 0 : 1, 1u);
    if (RC) count_at(T, cnt, c, Kr <= K ? 0 : 1, 1u);
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

__global__ void k_dump_place(TableView T, uint64_t nw, uint64_t ntot, const unsigned* __restrict__ cnt, uint64_t M,
                             unsigned* __restrict__ occ, unsigned long long* __restrict__ okeys,
                             unsigned short* __restrict__ ovals, unsigned char* __restrict__ ocnts,
                             unsigned* __restrict__ fail) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < ntot;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t m = entry_mask(T, nw, i);
    if (!(m & (PRES_A | PRES_B))) continue;
    const uint64_t c = entry_key(T, nw, i);
    for (int o = 0; o < 2; ++o) {
      if (!(m & (o ? PRES_B : PRES_A))) continue;
      const uint64_t x = o ? T.rc(c) : c;
      const unsigned short v = (unsigned short)((o ? (m >> B_SHIFT) : m) & MASK12);
      const unsigned n = cnt[2 * i + o];
      const uint64_t j0 = oak_fnv(x) % M;
      bool placed = false;
      for (uint64_t kk = 0; kk < M && !placed; ++kk) {
        const uint64_t s = (j0 + kk * kk) % M;
        if (atomicCAS(occ + s, 0u, 1u) == 0u) {
          okeys[s] = x;
          ovals[s] = v;
          ocnts[s] = (unsigned char)(n > 255u ? 255u : (n ? n : 1u));
          placed = true;
        }
      }
      if (!placed) atomicOr(fail, 1u);
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

uint64_t dbg_dump(Ctx& c, uint64_t& capacity, uint64_t* keys, uint16_t* values, uint8_t* counts) {
  if (!c.built) throw Error(-22, "pg_dbg_dump: no dBG (call pg_build_dbg first)");
  if (!c.dump_ready) dump_counts(c);
  const uint64_t M = capacity ? capacity : oakht_capacity(c.dump_size);
  if (M < c.dump_size) throw Error(-34, "pg_dbg_dump: capacity below the key count");
  capacity = M;
  if (!keys) return c.dump_size;
  if (!values || !counts) throw Error(-22, "pg_dbg_dump: values and counts are required with keys");
  const uint64_t nw = 2 * c.cap, ntot = nw + c.ovf_cap;
  DevBuf occ, ok, ov, oc, fail;
  occ.reserve(4 * M); ok.reserve(8 * M); ov.reserve(2 * M); oc.reserve(M); fail.reserve(4);
  PG_HIP(hipMemsetAsync(occ.p, 0, 4 * M, c.stream));
  PG_HIP(hipMemsetAsync(ok.p, 0, 8 * M, c.stream));
  PG_HIP(hipMemsetAsync(ov.p, 0, 2 * M, c.stream));
  PG_HIP(hipMemsetAsync(oc.p, 0, M, c.stream));
  PG_HIP(hipMemsetAsync(fail.p, 0, 4, c.stream));
  hipLaunchKernelGGL(k_dump_place, dim3(grid_for(ntot, 256, 8192)), dim3(256), 0, c.stream, c.tv, nw, ntot,
                     c.dump_cnt.as<unsigned>(), M, occ.as<unsigned>(), ok.as<unsigned long long>(),
                     ov.as<unsigned short>(), oc.as<unsigned char>(), fail.as<unsigned>());
  PG_HIP(hipGetLastError());
  unsigned failed = 0;
  PG_HIP(hipMemcpyAsync(&failed, fail.p, 4, hipMemcpyDeviceToHost, c.stream));
  PG_HIP(hipMemcpyAsync(keys, ok.p, 8 * M, hipMemcpyDeviceToHost, c.stream));
  PG_HIP(hipMemcpyAsync(values, ov.p, 2 * M, hipMemcpyDeviceToHost, c.stream));
  PG_HIP(hipMemcpyAsync(counts, oc.p, M, hipMemcpyDeviceToHost, c.stream));
  c.sync();
  occ.release(); ok.release(); ov.release(); oc.release(); fail.release();
  if (failed) throw Error(-34, "pg_dbg_dump: a key found no free slot on its probe sequence");
  if (c.sentinel) {                                  // key 2^64-1, mask '$' (:1087-1088)
    const uint64_t j0 = oak_fnv(SENTINEL) % M;
    uint64_t kk = 0, s = j0;
    for (; kk < M; ++kk) {
      s = (j0 + kk * kk) % M;
      if (counts[s] == 0) break;
    }
    if (kk == M) throw Error(-34, "pg_dbg_dump: no free slot for the n<k sentinel");
    keys[s] = SENTINEL;
    values[s] = 32;
    counts[s] = (uint8_t)(c.dump_sentinel > 255 ? 255 : (c.dump_sentinel ? c.dump_sentinel : 1));
  }
  return c.dump_size;
}

}  // namespace pg
