// pg_parse.hip — K1: FASTA bytes in HBM -> record table + one class code per base.
//
// Restates readline_jit_ (kmer_numba.py:122-132) and seqio_jit_ (:135-172)
// as data-parallel passes over the byte stream:
//   k_nl_count  newlines per 64 KiB chunk (16-byte vector loads, SWAR compare)
//   scan        chunk offsets (rocPRIM)
//   k_nl_write  newline positions, in order (block-wide scan per 4 KiB step)
//   k_lines     per line: start, header flag, content length (= len - 1: every
//               line loses its last byte, :160/:167)
//   scan        line -> offset in the compacted base stream
//   select      header lines -> records
//   k_records   per record: offset, length, header span, resume pointer
//   k_copy      every content byte -> its class code at its compacted offset
// A final line without '\n' counts when `end > start > 0` (:131-132); its last
// byte then plays the terminator's role, so it is appended as a virtual
// newline at n-1.  Lines before the first header land in front of record 0
// in the compacted stream and belong to no record (:156-161).
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "pg_internal.h"

namespace pg {

constexpr int PBLOCK = 256;                       // threads per block
constexpr int PVEC = 16;                          // bytes per thread per step
constexpr int PSTEP = PBLOCK * PVEC;              // 4 KiB per block step
constexpr int PSTEPS = 16;
constexpr uint64_t PCHUNK = (uint64_t)PSTEP * PSTEPS;   // 64 KiB per block

__device__ __forceinline__ uint32_t count_nl_word(uint32_t w) {
  uint32_t x = w ^ 0x0A0A0A0Au;
  uint32_t t = ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x;
  return __builtin_popcount(~t & 0x80808080u);
}

// load the 16 bytes at p (16-byte aligned); bytes at or past n read as 0
__device__ __forceinline__ uint4 load16(const uint8_t* buf, uint64_t p, uint64_t n) {
  if (p + 16 <= n) return *reinterpret_cast<const uint4*>(buf + p);
  uint32_t w[4] = {0, 0, 0, 0};
  for (int j = 0; j < 16; ++j)
    if (p + j < n) w[j >> 2] |= (uint32_t)buf[p + j] << (8 * (j & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ uint32_t count_nl16(uint4 v) {
  return count_nl_word(v.x) + count_nl_word(v.y) + count_nl_word(v.z) + count_nl_word(v.w);
}

__device__ __forceinline__ uint32_t byte_of(const uint4& v, int j) {
  uint32_t w = j < 4 ? v.x : j < 8 ? v.y : j < 12 ? v.z : v.w;
  return (w >> (8 * (j & 3))) & 0xFFu;
}

__global__ void __launch_bounds__(PBLOCK) k_nl_count(const uint8_t* __restrict__ buf, uint64_t n,
                                                     unsigned long long* __restrict__ blk_nl) {
  __shared__ uint32_t lds[PBLOCK / 64];
  const uint64_t base = (uint64_t)blockIdx.x * PCHUNK;
  uint32_t cnt = 0;
#pragma unroll 4
  for (int s = 0; s < PSTEPS; ++s) {
    uint64_t p = base + (uint64_t)s * PSTEP + (uint64_t)threadIdx.x * PVEC;
    if (p < n) cnt += count_nl16(load16(buf, p, n));
  }
  uint32_t tot;
  (void)block_excl_scan<PBLOCK>(cnt, lds, tot);
  if (threadIdx.x == 0) blk_nl[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(PBLOCK) k_nl_write(const uint8_t* __restrict__ buf, uint64_t n,
                                                     const unsigned long long* __restrict__ blk_off,
                                                     long long* __restrict__ nl_pos) {
  __shared__ uint32_t lds[PBLOCK / 64];
  const uint64_t base = (uint64_t)blockIdx.x * PCHUNK;
  uint64_t run = blk_off[blockIdx.x];
  for (int s = 0; s < PSTEPS; ++s) {
    uint64_t p = base + (uint64_t)s * PSTEP + (uint64_t)threadIdx.x * PVEC;
    if (base + (uint64_t)s * PSTEP >= n) break;          // block-uniform
    uint4 v = p < n ? load16(buf, p, n) : make_uint4(0, 0, 0, 0);
    uint32_t c = p < n ? count_nl16(v) : 0u;
    uint32_t tot;
    uint32_t pre = block_excl_scan<PBLOCK>(c, lds, tot);
    if (c) {
      uint64_t o = run + pre;
      for (int j = 0; j < 16; ++j)
        if (byte_of(v, j) == 10u) nl_pos[o++] = (long long)(p + j);
    }
    run += tot;
  }
}

__global__ void k_lines(const uint8_t* __restrict__ buf, const long long* __restrict__ nl_pos,
                        uint64_t L, long long* __restrict__ line_start,
                        unsigned long long* __restrict__ contrib, uint8_t* __restrict__ hdr) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < L;
       i += (uint64_t)gridDim.x * blockDim.x) {
    long long st = i == 0 ? 0 : nl_pos[i - 1] + 1;
    long long term = nl_pos[i];
    bool h = buf[st] == 62;                                  // line[0] == 62 (:155)
    line_start[i] = st;
    hdr[i] = h;
    contrib[i] = h ? 0ull : (unsigned long long)(term - st);   // line[:-1]
  }
}

__global__ void k_records(const long long* __restrict__ hdr_lines, uint64_t R,
                          const unsigned long long* __restrict__ line_off,
                          const long long* __restrict__ line_start,
                          const long long* __restrict__ nl_pos, uint64_t L, uint64_t total,
                          long long* __restrict__ rec_start, long long* __restrict__ rec_len,
                          long long* __restrict__ rec_hdr, long long* __restrict__ rec_ptr) {
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < R;
       r += (uint64_t)gridDim.x * blockDim.x) {
    long long h = hdr_lines[r];
    long long s = (long long)line_off[h];
    long long e = r + 1 < R ? (long long)line_off[hdr_lines[r + 1]] : (long long)total;
    rec_start[r] = s;
    rec_len[r] = e - s;
    rec_hdr[2 * r] = line_start[h];                          // qid = line[:-1] (:160)
    rec_hdr[2 * r + 1] = nl_pos[h] - line_start[h];
    // seqio's ptr[0] when this record is yielded: the next header line's
    // start, or the last line's start at EOF (:153, :170-172)
    rec_ptr[r] = r + 1 < R ? line_start[hdr_lines[r + 1]] : line_start[L - 1];
  }
}

__constant__ uint8_t c_byte_class[256];

__global__ void __launch_bounds__(PBLOCK) k_copy(const uint8_t* __restrict__ buf, uint64_t n,
                                                 const unsigned long long* __restrict__ blk_off,
                                                 uint64_t L, int has_tail,
                                                 const long long* __restrict__ line_start,
                                                 const unsigned long long* __restrict__ line_off,
                                                 const uint8_t* __restrict__ hdr,
                                                 uint8_t* __restrict__ out) {
  // Compaction keeps byte order, so one 4 KiB input step's content bytes form
  // one contiguous output range: stage their class codes in LDS at their
  // offset in that range, then write the range with aligned 16-byte stores.
  __shared__ uint32_t lds[PBLOCK / 64];
  __shared__ uint8_t cls[256];
  __shared__ unsigned long long s_lo[PBLOCK / 64], s_hi[PBLOCK / 64];
  __shared__ __attribute__((aligned(16))) uint8_t stage[PSTEP];
  cls[threadIdx.x] = c_byte_class[threadIdx.x];
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t base = (uint64_t)blockIdx.x * PCHUNK;
  uint64_t run = blk_off[blockIdx.x];
  for (int s = 0; s < PSTEPS; ++s) {
    uint64_t p = base + (uint64_t)s * PSTEP + (uint64_t)threadIdx.x * PVEC;
    if (base + (uint64_t)s * PSTEP >= n) break;
    uint4 v = p < n ? load16(buf, p, n) : make_uint4(0, 0, 0, 0);
    uint32_t c = p < n ? count_nl16(v) : 0u;
    uint32_t tot;
    uint32_t pre = block_excl_scan<PBLOCK>(c, lds, tot);
    // output offset of each content byte (~0 for none)
    unsigned long long off[16];
    uint8_t code[16];
    unsigned long long mylo = ~0ull, myhi = 0;
    {
      uint64_t li = run + pre;
      uint64_t cur = ~0ull;
      long long ls = 0; unsigned long long lo = 0; bool lh = true;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        off[j] = ~0ull;
        code[j] = 0;
        const uint32_t b = byte_of(v, j);
        const uint64_t pos = p + j;
        if (pos < n) {
          const bool term = (b == 10u) || (has_tail && pos == n - 1);
          if (li < L && !term) {
            if (li != cur) { cur = li; ls = line_start[li]; lo = line_off[li]; lh = hdr[li] != 0; }
            if (!lh) {
              off[j] = lo + (pos - (uint64_t)ls);
              code[j] = cls[b];
              mylo = off[j] < mylo ? off[j] : mylo;
              myhi = off[j] + 1 > myhi ? off[j] + 1 : myhi;
            }
          }
          if (b == 10u) ++li;
        }
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long a = __shfl_xor(mylo, o, 64), b2 = __shfl_xor(myhi, o, 64);
      mylo = a < mylo ? a : mylo;
      myhi = b2 > myhi ? b2 : myhi;
    }
    if (lane == 0) { s_lo[wid] = mylo; s_hi[wid] = myhi; }
    __syncthreads();
    unsigned long long olo = ~0ull, ohi = 0;
    for (int w = 0; w < PBLOCK / 64; ++w) {
      olo = s_lo[w] < olo ? s_lo[w] : olo;
      ohi = s_hi[w] > ohi ? s_hi[w] : ohi;
    }
    if (olo < ohi) {                                   // block-uniform
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (off[j] != ~0ull) stage[off[j] - olo] = code[j];
      __syncthreads();
      // 16-byte aligned global chunks covering [olo, ohi)
      const unsigned long long g0 = olo & ~15ull;
      for (unsigned long long g = g0 + 16ull * threadIdx.x; g < ohi; g += 16ull * PBLOCK) {
        if (g >= olo && g + 16 <= ohi) {
          uint32_t w[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint64_t i0 = g + 4 * q - olo;
            w[q] = (uint32_t)stage[i0] | ((uint32_t)stage[i0 + 1] << 8) | ((uint32_t)stage[i0 + 2] << 16) |
                   ((uint32_t)stage[i0 + 3] << 24);
          }
          *reinterpret_cast<uint4*>(out + g) = make_uint4(w[0], w[1], w[2], w[3]);
        } else {
          for (int j = 0; j < 16; ++j)
            if (g + j >= olo && g + j < ohi) out[g + j] = stage[g + j - olo];
        }
      }
    }
    __syncthreads();                                   // stage / s_lo reused next step
    run += tot;
  }
}

static void upload_byte_class() {
  static bool done = false;
  if (done) return;
  uint8_t t[256];
  for (int i = 0; i < 256; ++i) t[i] = CLS_OTHER;
  const char* s = "ACGTN";
  const uint8_t c[5] = {CLS_A, CLS_C, CLS_G, CLS_T, CLS_N};
  for (int i = 0; i < 5; ++i) { t[(uint8_t)s[i]] = c[i]; t[(uint8_t)(s[i] | 0x20)] = c[i]; }
  t[(uint8_t)'$'] = CLS_DOLLAR;
  PG_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_byte_class), t, 256));
  done = true;
}

template <class F>
static void with_temp(Ctx& c, F&& f) {
  size_t bytes = 0;
  PG_HIP(f((void*)nullptr, bytes));
  c.scratch.reserve(bytes + 16);
  bytes = c.scratch.cap;
  PG_HIP(f(c.scratch.p, bytes));
}

void parse_fasta(Ctx& c) {
  upload_byte_class();
  hipStream_t st = c.stream;
  const uint64_t n = c.n_bytes;
  c.parsed = false;
  c.n_lines = c.n_records = c.n_bases = c.n_nl = 0;
  c.h_rec_start.clear(); c.h_rec_len.clear(); c.h_rec_hdr_start.clear();
  c.h_rec_hdr_len.clear(); c.h_rec_ptr.clear();
  if (n == 0) { c.parsed = true; return; }

  const uint64_t nblk = (n + PCHUNK - 1) / PCHUNK;
  c.blk_nl.reserve(8 * (nblk + 1));
  c.blk_nl_off.reserve(8 * (nblk + 1));
  c.n_sel.reserve(64);
  hipLaunchKernelGGL(k_nl_count, dim3((unsigned)nblk), dim3(PBLOCK), 0, st, c.d_fasta, n,
                     c.blk_nl.as<unsigned long long>());
  PG_HIP(hipGetLastError());
  auto* bn = c.blk_nl.as<unsigned long long>();
  auto* bo = c.blk_nl_off.as<unsigned long long>();
  with_temp(c, [&](void* tmp, size_t& bytes) {
    return rocprim::exclusive_scan(tmp, bytes, bn, bo, 0ull, (size_t)nblk,
                                   rocprim::plus<unsigned long long>(), st);
  });
  unsigned long long last[2];
  PG_HIP(hipMemcpyAsync(&last[0], bo + nblk - 1, 8, hipMemcpyDeviceToHost, st));
  PG_HIP(hipMemcpyAsync(&last[1], bn + nblk - 1, 8, hipMemcpyDeviceToHost, st));
  c.sync();
  const uint64_t n_nl = last[0] + last[1];
  c.n_nl = n_nl;
  c.nl_pos.reserve(8 * (n_nl + 2));
  auto* nl = c.nl_pos.as<long long>();
  if (n_nl) {
    hipLaunchKernelGGL(k_nl_write, dim3((unsigned)nblk), dim3(PBLOCK), 0, st, c.d_fasta, n, bo, nl);
    PG_HIP(hipGetLastError());
  }
  // tail line (:131-132): `end > start > 0` with end = n-1, start = last '\n' + 1
  int has_tail = 0;
  if (n_nl) {
    long long lastnl = 0;
    PG_HIP(hipMemcpyAsync(&lastnl, nl + n_nl - 1, 8, hipMemcpyDeviceToHost, st));
    c.sync();
    long long start = lastnl + 1;
    if ((long long)n - 1 > start) {
      has_tail = 1;
      long long v = (long long)n - 1;
      PG_HIP(hipMemcpyAsync(nl + n_nl, &v, 8, hipMemcpyHostToDevice, st));
    }
  }
  const uint64_t L = n_nl + has_tail;
  c.n_lines = L;
  if (L == 0) { c.sync(); c.parsed = true; return; }

  c.line_start.reserve(8 * L);
  c.line_off.reserve(8 * L);
  c.line_contrib.reserve(8 * L);
  c.line_hdr.reserve(L);
  auto* ls = c.line_start.as<long long>();
  auto* lo = c.line_off.as<unsigned long long>();
  auto* lc = c.line_contrib.as<unsigned long long>();
  auto* lh = c.line_hdr.as<uint8_t>();
  hipLaunchKernelGGL(k_lines, dim3(grid_for(L, 256)), dim3(256), 0, st, c.d_fasta, nl, L, ls, lc, lh);
  PG_HIP(hipGetLastError());
  with_temp(c, [&](void* tmp, size_t& bytes) {
    return rocprim::exclusive_scan(tmp, bytes, lc, lo, 0ull, (size_t)L,
                                   rocprim::plus<unsigned long long>(), st);
  });
  c.hdr_lines.reserve(8 * L);
  auto* hl = c.hdr_lines.as<long long>();
  auto* nsel = c.n_sel.as<unsigned long long>();
  rocprim::counting_iterator<long long> idx(0);
  with_temp(c, [&](void* tmp, size_t& bytes) {
    return rocprim::select(tmp, bytes, idx, lh, hl, nsel, (size_t)L, st);
  });
  unsigned long long meta[3];
  PG_HIP(hipMemcpyAsync(&meta[0], nsel, 8, hipMemcpyDeviceToHost, st));
  PG_HIP(hipMemcpyAsync(&meta[1], lo + L - 1, 8, hipMemcpyDeviceToHost, st));
  PG_HIP(hipMemcpyAsync(&meta[2], lc + L - 1, 8, hipMemcpyDeviceToHost, st));
  c.sync();
  const uint64_t R = meta[0];
  const uint64_t total = meta[1] + meta[2];
  c.n_records = R;
  c.cls.reserve(total + 64);
  if (total) {
    hipLaunchKernelGGL(k_copy, dim3((unsigned)nblk), dim3(PBLOCK), 0, st, c.d_fasta, n, bo, L, has_tail,
                       ls, lo, lh, c.cls.as<uint8_t>());
    PG_HIP(hipGetLastError());
  }
  if (R) {
    c.rec_start.reserve(8 * R);
    c.rec_len.reserve(8 * R);
    c.rec_hdr.reserve(16 * R);
    c.rec_ptr.reserve(8 * R);
    c.rec_flag.reserve(R);
    hipLaunchKernelGGL(k_records, dim3(grid_for(R, 256)), dim3(256), 0, st, hl, R, lo, ls, nl, L, total,
                       c.rec_start.as<long long>(), c.rec_len.as<long long>(),
                       c.rec_hdr.as<long long>(), c.rec_ptr.as<long long>());
    PG_HIP(hipGetLastError());
    c.h_rec_start.resize(R); c.h_rec_len.resize(R); c.h_rec_ptr.resize(R);
    std::vector<int64_t> hdr(2 * R);
    PG_HIP(hipMemcpyAsync(c.h_rec_start.data(), c.rec_start.p, 8 * R, hipMemcpyDeviceToHost, st));
    PG_HIP(hipMemcpyAsync(c.h_rec_len.data(), c.rec_len.p, 8 * R, hipMemcpyDeviceToHost, st));
    PG_HIP(hipMemcpyAsync(c.h_rec_ptr.data(), c.rec_ptr.p, 8 * R, hipMemcpyDeviceToHost, st));
    PG_HIP(hipMemcpyAsync(hdr.data(), c.rec_hdr.p, 16 * R, hipMemcpyDeviceToHost, st));
    c.sync();
    c.h_rec_hdr_start.resize(R); c.h_rec_hdr_len.resize(R);
    uint64_t nb = 0;
    for (uint64_t r = 0; r < R; ++r) {
      c.h_rec_hdr_start[r] = hdr[2 * r];
      c.h_rec_hdr_len[r] = hdr[2 * r + 1];
      nb += (uint64_t)c.h_rec_len[r];
    }
    c.n_bases = nb;
  }
  c.sync();
  c.parsed = true;
}

}  // namespace pg
