// pg_abi.hip — extern "C" entry points of include/pangenome.h.
#include <chrono>
#include <cstring>
#include <string>

#include "../../include/pangenome.h"
#include "pg_internal.h"

struct pg_ctx {
  pg::Ctx c;
};

static thread_local std::string g_err;

template <class F>
static int guard(F&& f) {
  try {
    f();
    return PG_OK;
  } catch (const pg::Error& e) {
    g_err = e.what();
    return e.code;
  } catch (const std::bad_alloc&) {
    g_err = "out of host memory";
    return PG_ENOMEM;
  } catch (const std::exception& e) {
    g_err = e.what();
    return PG_EDEVICE;
  }
}

static void fill_stats(const pg::Ctx& c, pg_stats* s) {
  if (!s) return;
  s->n_bytes = c.n_bytes;
  s->n_records = c.n_records;
  s->n_bases = c.n_bases;
  s->n_windows = c.windows_total;
  s->n_dbg = c.n_dbg;
  s->n_rdbg = c.n_rdbg;
  s->n_slots = c.n_canon;
  s->table_capacity = c.cap;
  s->ms_parse = c.ms_parse;
  s->ms_clear = c.ms_clear;
  s->ms_insert = c.ms_insert;
  s->ms_scan = c.ms_scan;
  s->n_records_a = c.n_records_a;
  s->ms_split = c.ms_split;
  s->ms_range = c.ms_range;
  s->sentinel = c.sentinel;
  s->build_flags = (c.early_split_used ? 1u : 0u) | ((uint64_t)std::min(255, std::max(0, c.bc_attempts - 1)) << 8) |
                   ((uint64_t)std::min(255, std::max(0, c.split_passes)) << 16);
  s->n_work_items = c.work_items;
}

extern "C" {

const char* pg_last_error(void) { return g_err.c_str(); }

int pg_create(pg_ctx** out, int device, int k) {
  return guard([&] {
    if (!out) throw pg::Error(PG_EINVAL, "pg_create: out is NULL");
    int n = 0;
    PG_HIP(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) throw pg::Error(PG_EINVAL, "pg_create: no HIP device " + std::to_string(device));
    PG_HIP(hipSetDevice(device));
    auto* x = new pg_ctx();
    x->c.device = device;
    x->c.k = k < 1 ? 1 : (k > 27 ? 27 : k);
    PG_HIP(hipStreamCreateWithFlags(&x->c.stream, hipStreamNonBlocking));
    PG_HIP(hipStreamCreateWithFlags(&x->c.stream2, hipStreamNonBlocking));
    PG_HIP(hipStreamCreateWithFlags(&x->c.stream3, hipStreamNonBlocking));
    {
      int lo = 0, hi = 0;
      PG_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
      PG_HIP(hipStreamCreateWithPriority(&x->c.stream_hi, hipStreamNonBlocking, hi));
    }
    for (auto& e : x->c.ev) PG_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto& e : x->c.cev) PG_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    PG_HIP(hipEventCreateWithFlags(&x->c.rec_ev, hipEventDisableTiming));
    PG_HIP(hipEventCreateWithFlags(&x->c.ext_ev, hipEventDisableTiming));
    PG_HIP(hipDeviceGetAttribute(&x->c.n_cu, hipDeviceAttributeMultiprocessorCount, device));
    *out = x;
  });
}

void pg_destroy(pg_ctx* x) {
  if (!x) return;
  pg::Ctx& c = x->c;
  (void)hipSetDevice(c.device);
  (void)hipStreamSynchronize(c.stream);
  pg::DevBuf* bufs[] = {&c.fasta_own, &c.span_sum, &c.span_start, &c.n_sel, &c.rec_start, &c.rec_len,
                        &c.rec_hdr, &c.rec_ptr, &c.rec_flag, &c.cls, &c.p2, &c.e16, &c.scratch, &c.table, &c.ovf, &c.flags,
                        &c.recA_key, &c.recA_mw, &c.ctrA, &c.recS_key[0], &c.recS_key[1], &c.recS_mw[0],
                        &c.recS_mw[1], &c.ctrS, &c.snapA, &c.rseg, &c.k5_ctr, &c.tile_sched, &c.tile_desc, &c.k3_queue,
                        &c.k3_hint, &c.part_cnt, &c.tile_cnt, &c.tile_off, &c.occ, &c.edge_tab, &c.pair_tab,
                        &c.edge_out, &c.edge_exp, &c.lab_tab, &c.lab_list, &c.rows_buf, &c.text_len, &c.text_off,
                        &c.text_buf, &c.text_names, &c.preload,
                        &c.dump_cnt};
  for (auto* b : bufs) b->release();
  pg::pool_destroy(c);
  c.stage_pin.release();
  c.rec_pack.release();
  c.h_pin.release();
  c.h_out.release();
  c.tile_pin.release();
  for (auto& b : c.dump_pin) b.release();
  c.t0.destroy();
  c.t1.destroy();
  c.t6.destroy();
  for (auto& e : c.ev)
    if (e) (void)hipEventDestroy(e);
  for (auto e : c.cev)
    if (e) (void)hipEventDestroy(e);
  if (c.rec_ev) (void)hipEventDestroy(c.rec_ev);
  if (c.ext_ev) (void)hipEventDestroy(c.ext_ev);
  if (c.stream_hi) (void)hipStreamDestroy(c.stream_hi);
  (void)hipStreamDestroy(c.stream3);
  (void)hipStreamDestroy(c.stream2);
  (void)hipStreamDestroy(c.stream);
  delete x;
}

int pg_get_k(const pg_ctx* x) { return x ? x->c.k : -1; }

int pg_stream_wait(pg_ctx* x, void* stream) {
  return guard([&] {
    if (!x) throw pg::Error(PG_EINVAL, "pg_stream_wait: ctx is NULL");
    pg::Ctx& c = x->c;
    PG_HIP(hipSetDevice(c.device));
    PG_HIP(hipEventRecord(c.ext_ev, reinterpret_cast<hipStream_t>(stream)));
    for (hipStream_t s : {c.stream, c.stream2, c.stream3, c.stream_hi})
      if (s) PG_HIP(hipStreamWaitEvent(s, c.ext_ev, 0));
  });
}

int pg_set_fasta(pg_ctx* x, const uint8_t* host, uint64_t n) {
  return guard([&] {
    if (!x || (!host && n)) throw pg::Error(PG_EINVAL, "pg_set_fasta: bad arguments");
    pg::Ctx& c = x->c;
    PG_HIP(hipSetDevice(c.device));
    c.fasta_own.reserve(n + 64);
    {                                          // pageable input through the pinned staging ring
      pg::Upload up(c, c.fasta_own.as<uint8_t>(), host, n, c.h2d_chunk);
      for (uint64_t i = 0; i < up.chunks(); ++i) {
        up.wait_queued(i);
        PG_HIP(hipStreamWaitEvent(c.stream, c.cev[i & 15], 0));
        up.consumed(i);
      }
      up.finish();
    }
    c.sync();
    c.d_fasta = c.fasta_own.as<uint8_t>();
    c.n_bytes = n;
    c.parsed = c.built = c.reduced = false;
  });
}

int pg_set_fasta_device(pg_ctx* x, const uint8_t* dev, uint64_t n) {
  return guard([&] {
    if (!x || (!dev && n)) throw pg::Error(PG_EINVAL, "pg_set_fasta_device: bad arguments");
    pg::Ctx& c = x->c;
    PG_HIP(hipSetDevice(c.device));
    if (reinterpret_cast<uintptr_t>(dev) % 16 != 0) {
      c.fasta_own.reserve(n + 64);
      PG_HIP(hipMemcpyAsync(c.fasta_own.p, dev, n, hipMemcpyDeviceToDevice, c.stream));
      c.sync();
      c.d_fasta = c.fasta_own.as<uint8_t>();
    } else {
      c.d_fasta = dev;
    }
    c.n_bytes = n;
    c.parsed = c.built = c.reduced = false;
  });
}

int pg_parse_host(pg_ctx* x, const uint8_t* host, uint64_t n, uint64_t* n_records, uint64_t* n_bases) {
  return guard([&] {
    if (!x || (!host && n)) throw pg::Error(PG_EINVAL, "pg_parse_host: bad arguments");
    pg::Ctx& c = x->c;
    PG_HIP(hipSetDevice(c.device));
    auto t0 = std::chrono::steady_clock::now();
    c.fasta_own.reserve(n + 64);
    c.d_fasta = c.fasta_own.as<uint8_t>();
    c.n_bytes = n;
    c.parsed = c.built = c.reduced = false;
    pg::parse_fasta(c, host);
    c.sync();                                  // (the emission may still run when parse_fasta returns)
    c.ms_parse = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (n_records) *n_records = c.n_records;
    if (n_bases) *n_bases = c.n_bases;
  });
}

int pg_parse(pg_ctx* x, uint64_t* n_records, uint64_t* n_bases) {
  return guard([&] {
    if (!x) throw pg::Error(PG_EINVAL, "pg_parse: ctx is NULL");
    pg::Ctx& c = x->c;
    PG_HIP(hipSetDevice(c.device));
    if (!c.d_fasta && c.n_bytes) throw pg::Error(PG_EINVAL, "pg_parse: no FASTA set");
    auto t0 = std::chrono::steady_clock::now();
    pg::parse_fasta(c);
    c.sync();                                  // (the emission may still run when parse_fasta returns)
    c.ms_parse = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    c.built = c.reduced = false;
    if (n_records) *n_records = c.n_records;
    if (n_bases) *n_bases = c.n_bases;
  });
}

int pg_records(const pg_ctx* x, int64_t* seq_len, int64_t* hdr_start, int64_t* hdr_len, int64_t* ptr) {
  return guard([&] {
    if (!x || !x->c.parsed) throw pg::Error(PG_EINVAL, "pg_records: not parsed");
    const pg::Ctx& c = x->c;
    const size_t R = c.n_records;
    if (seq_len && R) std::memcpy(seq_len, c.h_rec_len.data(), 8 * R);
    if (hdr_start && R) std::memcpy(hdr_start, c.h_rec_hdr_start.data(), 8 * R);
    if (hdr_len && R) std::memcpy(hdr_len, c.h_rec_hdr_len.data(), 8 * R);
    if (ptr && R) std::memcpy(ptr, c.h_rec_ptr.data(), 8 * R);
  });
}

int pg_build_dbg(pg_ctx* x, const uint8_t* rec_flags, int extra_empty, int rc0, pg_stats* stats) {
  return guard([&] {
    if (!x) throw pg::Error(PG_EINVAL, "pg_build_dbg: ctx is NULL");
    PG_HIP(hipSetDevice(x->c.device));
    pg::build_dbg(x->c, rec_flags, extra_empty, rc0 != 0);
    fill_stats(x->c, stats);
  });
}

int pg_build_rdbg(pg_ctx* x, uint64_t* n_rdbg, pg_stats* stats) {
  return guard([&] {
    if (!x) throw pg::Error(PG_EINVAL, "pg_build_rdbg: ctx is NULL");
    PG_HIP(hipSetDevice(x->c.device));
    pg::build_rdbg(x->c);
    if (n_rdbg) *n_rdbg = x->c.n_rdbg;
    fill_stats(x->c, stats);
  });
}

int pg_build(pg_ctx* x, const uint8_t* rec_flags, int extra_empty, int rc0, uint64_t* n_rdbg, pg_stats* stats) {
  return guard([&] {
    if (!x) throw pg::Error(PG_EINVAL, "pg_build: ctx is NULL");
    PG_HIP(hipSetDevice(x->c.device));
    pg::build_dbg(x->c, rec_flags, extra_empty, rc0 != 0);
    pg::build_rdbg(x->c);                      // (the degree scan ran inside the build)
    if (n_rdbg) *n_rdbg = x->c.n_rdbg;
    fill_stats(x->c, stats);
  });
}

int pg_build_device(pg_ctx* x, const uint8_t* dev, uint64_t n, int rc0, uint64_t* n_rdbg, pg_stats* stats) {
  return guard([&] {
    if (!x || (!dev && n)) throw pg::Error(PG_EINVAL, "pg_build_device: bad arguments");
    pg::Ctx& c = x->c;
    PG_HIP(hipSetDevice(c.device));
    if (reinterpret_cast<uintptr_t>(dev) % 16 != 0) {
      c.fasta_own.reserve(n + 64);
      PG_HIP(hipMemcpyAsync(c.fasta_own.p, dev, n, hipMemcpyDeviceToDevice, c.stream));
      c.d_fasta = c.fasta_own.as<uint8_t>();
    } else {
      c.d_fasta = dev;
    }
    c.n_bytes = n;
    c.parsed = c.built = c.reduced = false;
    pg::parse_fasta(c);
    pg::build_dbg(c, nullptr, 0, rc0 != 0);
    pg::build_rdbg(c);
    // K1 on the stream (HIP events; the emission overlaps the host); an empty
    // input returns from parse_fasta before its events are recorded
    c.ms_parse = n ? c.t0.ms() : 0.0;
    if (n_rdbg) *n_rdbg = c.n_rdbg;
    fill_stats(c, stats);
  });
}

int pg_build_host(pg_ctx* x, const uint8_t* host, uint64_t n, int rc0, uint64_t* n_rdbg, pg_stats* stats) {
  return guard([&] {
    if (!x || (!host && n)) throw pg::Error(PG_EINVAL, "pg_build_host: bad arguments");
    pg::Ctx& c = x->c;
    PG_HIP(hipSetDevice(c.device));
    auto t0 = std::chrono::steady_clock::now();
    c.fasta_own.reserve(n + 64);
    c.d_fasta = c.fasta_own.as<uint8_t>();
    c.n_bytes = n;
    c.parsed = c.built = c.reduced = false;
    pg::build_host(c, host, n, rc0 != 0);
    c.ms_parse = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (n_rdbg) *n_rdbg = c.n_rdbg;
    fill_stats(c, stats);
  });
}

int pg_tune(pg_ctx* x, int what, int64_t value) {
  return guard([&] {
    if (!x) throw pg::Error(PG_EINVAL, "pg_tune: ctx is NULL");
    switch (what) {
      case PG_TUNE_K3_CHUNKS:
        if (value < 0 || value > 6) throw pg::Error(PG_EINVAL, "pg_tune: K3 chunks must be in [0, 6]");
        x->c.k3_chunks = (int)value;
        break;
      case PG_TUNE_K3_COVER:
#ifdef PG_COVER_LEGACY
        if (value < 0 || value > 2) throw pg::Error(PG_EINVAL, "pg_tune: K3 cover form must be 0, 1 or 2");
#else
        if (value != 0)
          throw pg::Error(PG_EINVAL, "pg_tune: K3 cover form must be 0 (the class-byte forms 1 and 2 are built only "
                                     "with PG_COVER_LEGACY)");
#endif
        x->c.k3_cover = (int)value;
        break;
      case PG_TUNE_K3_WBLK:
        if (value < 0 || value > 255) throw pg::Error(PG_EINVAL, "pg_tune: K3 work blocks must be in [0, 255]");
        x->c.k3_wblk = (int)value;
        break;
      case PG_TUNE_TIMERS:
        if (value < 0 || value > 7) throw pg::Error(PG_EINVAL, "pg_tune: timers must be in [0, 7]");
        x->c.t0.off = !(value & 1);
        x->c.t1.off = !(value & 2);
        x->c.t6.off = !(value & 4);
        break;
      case PG_TUNE_K3_ANCHORS:
        if (value != 0 && (value < 3 || value > 6) && value != 8)
          throw pg::Error(PG_EINVAL, "pg_tune: K3 anchors must be 3, 4, 5, 6 or 8 (0 = the default)");
        x->c.k3_anchors = (int)value;
        break;
      case PG_TUNE_K1:
        if (value < 0 || value > 7) throw pg::Error(PG_EINVAL, "pg_tune: K1 form must be in [0, 7]");
        x->c.k1_form = (int)value;
        break;
      case PG_TUNE_K3_EMIT:
        if (value < 0 || value > 1) throw pg::Error(PG_EINVAL, "pg_tune: K3 emit form must be 0 or 1");
        x->c.k3_emit = (int)value;
        break;
      case PG_TUNE_K3_TAIL:
        if (value < 0 || value > 64) throw pg::Error(PG_EINVAL, "pg_tune: K3 tail must be in [0, 64]");
        x->c.k3_tail = (int)value;
        break;
      case PG_TUNE_K3_HEAD:
        if (value < 0 || value > 64) throw pg::Error(PG_EINVAL, "pg_tune: K3 head must be in [0, 64]");
        x->c.k3_head = (int)value;
        break;
      case PG_TUNE_H2D_TAIL:
        if (value < 0) throw pg::Error(PG_EINVAL, "pg_tune: H2D tail must be >= 0");
        x->c.h2d_tail = (uint64_t)value;
        break;
      case PG_TUNE_EARLY_SPLIT:
        if (value < 0 || value > 1) throw pg::Error(PG_EINVAL, "pg_tune: early split must be 0 or 1");
        x->c.early_split = (int)value;
        break;
      case PG_TUNE_BUCKET_SHIFT:
        if (value < 0 || value > 8) throw pg::Error(PG_EINVAL, "pg_tune: bucket shift must be in [0, 8]");
        x->c.bb_shift = (int)value;
        break;
      case PG_TUNE_REGION_CAP:
        if (value < 0) throw pg::Error(PG_EINVAL, "pg_tune: region size must be >= 0");
        x->c.region_cap_force = (uint64_t)value;
        break;
      case PG_TUNE_H2D_CHUNK:
        if (value < 0) throw pg::Error(PG_EINVAL, "pg_tune: H2D chunk must be >= 0");
        x->c.h2d_chunk = value ? (uint64_t)value : (64ull << 20);
        break;
      case PG_TUNE_HOST_THREADS:
        if (value < 0 || value > 64) throw pg::Error(PG_EINVAL, "pg_tune: host threads must be in [0, 64]");
        x->c.host_threads = (int)value;
        break;
      case PG_TUNE_STAGE_PIECE:
        if (value < 0 || (value && value < 4096)) throw pg::Error(PG_EINVAL, "pg_tune: staging piece must be 0 or >= 4096");
        x->c.stage_piece = value ? (uint64_t)value : (32ull << 20);
        break;
      case PG_TUNE_HOST_REGISTER:
        if (value < 0 || value > 1) throw pg::Error(PG_EINVAL, "pg_tune: host register must be 0 or 1");
        x->c.host_register = (int)value;
        break;
      case PG_TUNE_DEVICE_CAP:
        if (value < 0) throw pg::Error(PG_EINVAL, "pg_tune: device cap must be >= 0");
        pg::DevBytes::cap().store((uint64_t)value);
        pg::DevBytes::peak().store(pg::DevBytes::cur().load());
        break;
      case PG_TUNE_POISON:
        if (value < -1 || value > 255) throw pg::Error(PG_EINVAL, "pg_tune: poison byte must be in [-1, 255]");
        pg::DevBytes::poison().store((int)value);
        break;
      case PG_TUNE_STAGE_SLOTS:
        if (value < 0 || value == 1 || value > 8) throw pg::Error(PG_EINVAL, "pg_tune: staging slots must be 0 or 2..8");
        x->c.stage_slots = value ? (uint64_t)value : 4;
        break;
      default:
        throw pg::Error(PG_EINVAL, "pg_tune: unknown parameter " + std::to_string(what));
    }
  });
}

uint64_t pg_device_bytes(int peak) {
  return peak ? pg::DevBytes::peak().load() : pg::DevBytes::cur().load();
}

int pg_get_stats(const pg_ctx* x, pg_stats* stats) {
  return guard([&] {
    if (!x || !stats) throw pg::Error(PG_EINVAL, "pg_get_stats: bad arguments");
    fill_stats(x->c, stats);
  });
}

int pg_dbg_export(pg_ctx* x, uint64_t* keys, uint16_t* masks, uint64_t cap, uint64_t* n) {
  return guard([&] {
    if (!x || !n) throw pg::Error(PG_EINVAL, "pg_dbg_export: bad arguments");
    PG_HIP(hipSetDevice(x->c.device));
    const uint64_t total = pg::export_dbg(x->c, nullptr, nullptr, 0);
    *n = total;
    if (keys) {
      if (cap < total || !masks) throw pg::Error(PG_ERANGE, "pg_dbg_export: buffer too small");
      pg::export_dbg(x->c, keys, masks, cap);
    }
  });
}

int pg_rdbg_export(pg_ctx* x, uint64_t* keys, uint64_t cap, uint64_t* n) {
  return guard([&] {
    if (!x || !n) throw pg::Error(PG_EINVAL, "pg_rdbg_export: bad arguments");
    PG_HIP(hipSetDevice(x->c.device));
    *n = pg::export_rdbg(x->c, nullptr, 0);
    if (keys) {
      if (cap < *n) throw pg::Error(PG_ERANGE, "pg_rdbg_export: buffer too small");
      pg::export_rdbg(x->c, keys, cap);
    }
  });
}

int pg_dbg_dump(pg_ctx* x, uint64_t* capacity, uint64_t* keys, uint16_t* values, uint8_t* counts, uint64_t* size) {
  return guard([&] {
    if (!x || !capacity || !size) throw pg::Error(PG_EINVAL, "pg_dbg_dump: bad arguments");
    PG_HIP(hipSetDevice(x->c.device));
    *size = pg::dbg_dump(x->c, *capacity, keys, values, counts);
  });
}

int pg_dbg_dump_fd(pg_ctx* x, uint64_t* capacity, int fd, const uint64_t* offsets, uint32_t* crcs, uint64_t* size) {
  return guard([&] {
    if (!x || !capacity || !size) throw pg::Error(PG_EINVAL, "pg_dbg_dump_fd: bad arguments");
    PG_HIP(hipSetDevice(x->c.device));
    *size = pg::dbg_dump_fd(x->c, *capacity, fd, offsets, crcs);
  });
}

int pg_dbg_load(pg_ctx* x, const uint64_t* keys, const uint16_t* masks, const uint8_t* counts, uint64_t n) {
  return guard([&] {
    if (!x || (n && !keys)) throw pg::Error(PG_EINVAL, "pg_dbg_load: bad arguments");
    PG_HIP(hipSetDevice(x->c.device));
    pg::dbg_load(x->c, keys, masks, counts, n);
  });
}

uint64_t pg_oakht_capacity(uint64_t size) {
  try {
    return pg::oakht_capacity(size);
  } catch (...) {
    return 0;
  }
}

int pg_dbg_partition(pg_ctx* x, int nparts, void* d_out, uint64_t out_cap, uint64_t* counts) {
  return guard([&] {
    if (!x || !counts) throw pg::Error(PG_EINVAL, "pg_dbg_partition: bad arguments");
    PG_HIP(hipSetDevice(x->c.device));
    // the scatter reuses the counts of a count pass over the same table
    const bool counted = x->c.part_gen == x->c.build_gen && x->c.part_nparts == nparts;
    const uint64_t total = d_out && counted ? x->c.part_total : pg::partition_dbg(x->c, nparts, nullptr, 0, counts);
    if (d_out) {
      if (out_cap < total) throw pg::Error(PG_ERANGE, "pg_dbg_partition: output too small");
      pg::partition_dbg(x->c, nparts, d_out, out_cap, counts);
    }
  });
}

int pg_dbg_merge(pg_ctx* x, const void* d_records, uint64_t n, uint64_t cap_hint, int sentinel) {
  return guard([&] {
    if (!x || (!d_records && n)) throw pg::Error(PG_EINVAL, "pg_dbg_merge: bad arguments");
    PG_HIP(hipSetDevice(x->c.device));
    x->c.merge_sum = x->c.merge_rows = 0;
    pg::merge_dbg(x->c, d_records, n, cap_hint, sentinel);
  });
}

int pg_dbg_partition_sums(pg_ctx* x, int nparts, uint64_t* sums) {
  return guard([&] {
    if (!x || !sums || nparts < 1 || nparts > 64) throw pg::Error(PG_EINVAL, "pg_dbg_partition_sums: bad arguments");
    if (x->c.part_nparts != nparts) throw pg::Error(PG_EINVAL, "pg_dbg_partition_sums: no scatter into that many parts");
    for (int i = 0; i < nparts; ++i) sums[i] = x->c.part_sums[i];
  });
}

int pg_rows_checksum(pg_ctx* x, const void* d_rows, const uint64_t* seg_off, uint64_t nseg, uint64_t* sums) {
  return guard([&] {
    if (!x || !seg_off || (nseg && !sums) || (!d_rows && nseg && seg_off[nseg] > seg_off[0]))
      throw pg::Error(PG_EINVAL, "pg_rows_checksum: bad arguments");
    PG_HIP(hipSetDevice(x->c.device));
    pg::rows_checksum(x->c, d_rows, seg_off, nseg, sums);
  });
}

int pg_route_rows_checksum(pg_ctx* x, const void* d_rows, const uint64_t* seg_off, uint64_t nseg, uint64_t* sums) {
  return guard([&] {
    if (!x || !seg_off || (nseg && !sums) || (!d_rows && nseg && seg_off[nseg] > seg_off[0]))
      throw pg::Error(PG_EINVAL, "pg_route_rows_checksum: bad arguments");
    if (reinterpret_cast<uintptr_t>(d_rows) & 3u) throw pg::Error(PG_EINVAL, "pg_route_rows_checksum: rows not 4-byte aligned");
    PG_HIP(hipSetDevice(x->c.device));
    pg::rows_checksum(x->c, d_rows, seg_off, nseg, sums, true);
  });
}

static int route_lg(int nparts, const char* what) {
  if (nparts < 1 || nparts > 64 || (nparts & (nparts - 1)))
    throw pg::Error(PG_EINVAL, std::string(what) + ": nparts must be a power of two in [1, 64]");
  return __builtin_ctz((unsigned)nparts);
}

int pg_route_stage_a(pg_ctx* x, const uint8_t* rec_flags, int extra_empty, int rc0, int nparts, uint64_t* counts,
                     int* sentinel) {
  return guard([&] {
    if (!x || !counts) throw pg::Error(PG_EINVAL, "pg_route_stage_a: bad arguments");
    const int lg = route_lg(nparts, "pg_route_stage_a");
    PG_HIP(hipSetDevice(x->c.device));
    x->c.route_req = true;
    try {
      pg::build_dbg(x->c, rec_flags, extra_empty, rc0 != 0);
    } catch (...) {
      x->c.route_req = false;
      throw;
    }
    if (!x->c.route_ready) throw pg::Error(PG_EINVAL, "pg_route_stage_a: the build did not hold its records");
    pg::route_counts(x->c, lg, counts);
    if (sentinel) *sentinel = x->c.route_sentinel ? 1 : 0;
  });
}

int pg_route_scatter(pg_ctx* x, int nparts, void* d_out, uint64_t out_cap, uint64_t* sums) {
  return guard([&] {
    if (!x || !sums || (!d_out && out_cap)) throw pg::Error(PG_EINVAL, "pg_route_scatter: bad arguments");
    const int lg = route_lg(nparts, "pg_route_scatter");
    PG_HIP(hipSetDevice(x->c.device));
    pg::route_scatter(x->c, lg, d_out, out_cap, sums);
  });
}

int pg_route_finish(pg_ctx* x, uint64_t* n_rdbg, pg_stats* stats) {
  return guard([&] {
    if (!x) throw pg::Error(PG_EINVAL, "pg_route_finish: ctx is NULL");
    PG_HIP(hipSetDevice(x->c.device));
    pg::route_finish(x->c);
    if (n_rdbg) *n_rdbg = x->c.n_rdbg;
    fill_stats(x->c, stats);
  });
}

int pg_route_merge(pg_ctx* x, const void* d_rows, uint64_t n, int nparts, int sentinel, uint64_t* n_rdbg,
                   pg_stats* stats) {
  return guard([&] {
    if (!x || (!d_rows && n)) throw pg::Error(PG_EINVAL, "pg_route_merge: bad arguments");
    const int lg = route_lg(nparts, "pg_route_merge");
    PG_HIP(hipSetDevice(x->c.device));
    if (lg > x->c.cbits && x->c.cbits) throw pg::Error(PG_EINVAL, "pg_route_merge: more owners than coarse bins");
    x->c.merge_sum = x->c.merge_rows = 0;
    pg::merge_dbg(x->c, d_rows, n, 0, sentinel, lg);
    if (n_rdbg) *n_rdbg = x->c.n_rdbg;
    fill_stats(x->c, stats);
  });
}

int pg_route_merge_segs(pg_ctx* x, const void* const* d_segs, const uint64_t* n, int nseg, int nparts, int sentinel,
                       uint64_t* n_rdbg, pg_stats* stats) {
  return guard([&] {
    if (!x || nseg < 0 || (nseg && (!d_segs || !n))) throw pg::Error(PG_EINVAL, "pg_route_merge_segs: bad arguments");
    for (int s = 0; s < nseg; ++s)
      if (n[s] && !d_segs[s]) throw pg::Error(PG_EINVAL, "pg_route_merge_segs: a non-empty segment has no rows");
    const int lg = route_lg(nparts, "pg_route_merge_segs");
    PG_HIP(hipSetDevice(x->c.device));
    if (lg > x->c.cbits && x->c.cbits) throw pg::Error(PG_EINVAL, "pg_route_merge_segs: more owners than coarse bins");
    x->c.merge_sum = x->c.merge_rows = 0;
    pg::merge_dbg_segs(x->c, d_segs, n, nseg, sentinel, lg);
    if (n_rdbg) *n_rdbg = x->c.n_rdbg;
    fill_stats(x->c, stats);
  });
}

int pg_dbg_merge_check(const pg_ctx* x, uint64_t* rows, uint64_t* sum) {
  return guard([&] {
    if (!x || !rows || !sum) throw pg::Error(PG_EINVAL, "pg_dbg_merge_check: bad arguments");
    *rows = x->c.merge_rows;
    *sum = x->c.merge_sum;
  });
}

int pg_edges(pg_ctx* x, const uint8_t* rec_flags, int rc1, uint64_t* n_edges) {
  return guard([&] {
    if (!x) throw pg::Error(PG_EINVAL, "pg_edges: ctx is NULL");
    PG_HIP(hipSetDevice(x->c.device));
    const uint64_t n = pg::walk_edges(x->c, rec_flags, rc1 != 0);
    if (n_edges) *n_edges = n;
  });
}

int pg_edges_export(pg_ctx* x, uint64_t* tuples, int64_t* counts, int64_t* first_walk, uint64_t cap) {
  return guard([&] {
    if (!x || !tuples || !counts || !first_walk) throw pg::Error(PG_EINVAL, "pg_edges_export: bad arguments");
    if (cap < x->c.n_edges) throw pg::Error(PG_ERANGE, "pg_edges_export: buffer too small");
    PG_HIP(hipSetDevice(x->c.device));
    pg::export_edges(x->c, tuples, counts, first_walk, cap);
  });
}

int pg_set_labels(pg_ctx* x, const int64_t* key, const int64_t* value, const int64_t* label, uint64_t n) {
  return guard([&] {
    if (!x || (n && (!key || !value || !label))) throw pg::Error(PG_EINVAL, "pg_set_labels: bad arguments");
    PG_HIP(hipSetDevice(x->c.device));
    pg::set_labels(x->c, key, value, label, n);
  });
}

int pg_rows(pg_ctx* x, const uint8_t* rec_flags, int rc1, uint64_t* n_rows) {
  return guard([&] {
    if (!x) throw pg::Error(PG_EINVAL, "pg_rows: ctx is NULL");
    PG_HIP(hipSetDevice(x->c.device));
    const uint64_t n = pg::walk_rows(x->c, rec_flags, rc1 != 0);
    if (n_rows) *n_rows = n;
  });
}

int pg_rows_export(pg_ctx* x, int64_t* rows5, uint64_t cap) {
  return guard([&] {
    if (!x || !rows5) throw pg::Error(PG_EINVAL, "pg_rows_export: bad arguments");
    if (cap < x->c.n_rows) throw pg::Error(PG_ERANGE, "pg_rows_export: buffer too small");
    PG_HIP(hipSetDevice(x->c.device));
    pg::export_rows(x->c, rows5, cap);
  });
}

int pg_edges_format(pg_ctx* x, char* out, uint64_t cap, uint64_t* n_bytes) {
  return guard([&] {
    if (!x || !n_bytes) throw pg::Error(PG_EINVAL, "pg_edges_format: bad arguments");
    PG_HIP(hipSetDevice(x->c.device));
    *n_bytes = pg::format_edges(x->c, out, cap);
  });
}

int pg_edges_format_fd(pg_ctx* x, int fd, uint64_t* n_bytes) {
  return guard([&] {
    if (!x || !n_bytes || fd < 0) throw pg::Error(PG_EINVAL, "pg_edges_format_fd: bad arguments");
    PG_HIP(hipSetDevice(x->c.device));
    *n_bytes = pg::format_edges(x->c, nullptr, 0, fd);
  });
}

int pg_labels_from_edges(pg_ctx* x, const uint64_t* tuples, uint64_t n_edges, const int64_t* mcl_key,
                         const int64_t* mcl_value, const int64_t* mcl_label, uint64_t n_mcl, int64_t next_label,
                         uint64_t* n_labels) {
  return guard([&] {
    if (!x || (n_mcl && (!mcl_key || !mcl_value || !mcl_label)) || (tuples == nullptr && n_edges))
      throw pg::Error(PG_EINVAL, "pg_labels_from_edges: bad arguments");
    PG_HIP(hipSetDevice(x->c.device));
    const uint64_t n = pg::labels_from_edges(x->c, tuples, n_edges, mcl_key, mcl_value, mcl_label, n_mcl, next_label);
    if (n_labels) *n_labels = n;
  });
}

int pg_labels_export(pg_ctx* x, int64_t* key, int64_t* value, int64_t* label, uint64_t cap) {
  return guard([&] {
    if (!x || !key || !value || !label) throw pg::Error(PG_EINVAL, "pg_labels_export: bad arguments");
    PG_HIP(hipSetDevice(x->c.device));
    pg::export_labels(x->c, key, value, label, cap);
  });
}

int pg_rows_format(pg_ctx* x, const char* names, const int64_t* name_off, uint64_t n_names, char* out, uint64_t cap,
                   uint64_t* n_bytes) {
  return guard([&] {
    if (!x || !n_bytes || !name_off) throw pg::Error(PG_EINVAL, "pg_rows_format: bad arguments");
    PG_HIP(hipSetDevice(x->c.device));
    if (n_names < x->c.n_records) throw pg::Error(PG_EINVAL, "pg_rows_format: fewer names than records");
    *n_bytes = pg::format_rows_text(x->c, names, name_off, n_names, out, cap);
  });
}

int pg_rows_format_fd(pg_ctx* x, const char* names, const int64_t* name_off, uint64_t n_names, int fd,
                      uint64_t* n_bytes) {
  return guard([&] {
    if (!x || !n_bytes || !name_off || fd < 0) throw pg::Error(PG_EINVAL, "pg_rows_format_fd: bad arguments");
    PG_HIP(hipSetDevice(x->c.device));
    if (n_names < x->c.n_records) throw pg::Error(PG_EINVAL, "pg_rows_format_fd: fewer names than records");
    *n_bytes = pg::format_rows_text(x->c, names, name_off, n_names, nullptr, 0, fd);
  });
}

// ---- text of the side file and the region rows (host only, no device work)
static inline char* put_u64(char* o, uint64_t v) {
  char t[24];
  int n = 0;
  do { t[n++] = (char)('0' + v % 10); v /= 10; } while (v);
  while (n) *o++ = t[--n];
  return o;
}
static inline char* put_i64(char* o, int64_t v) {
  if (v < 0) { *o++ = '-'; return put_u64(o, (uint64_t)0 - (uint64_t)v); }
  return put_u64(o, (uint64_t)v);
}

uint64_t pg_format_xyz(const uint64_t* t, const int64_t* counts, uint64_t n, char* out, uint64_t cap) {
  if (!out) return n * 106;                               // upper bound: 4 x 20 digits + count + 5 separators
  if (cap < n * 106) return 0;
  char* o = out;
  for (uint64_t i = 0; i < n; ++i) {
    o = put_u64(o, t[4 * i]); *o++ = '_'; o = put_u64(o, t[4 * i + 1]); *o++ = '\t';
    o = put_u64(o, t[4 * i + 2]); *o++ = '_'; o = put_u64(o, t[4 * i + 3]); *o++ = '\t';
    o = put_i64(o, counts[i]); *o++ = '\n';
  }
  return (uint64_t)(o - out);
}

uint64_t pg_format_rows(const int64_t* rows5, uint64_t n, const char* names, const int64_t* name_off, char* out,
                        uint64_t cap) {
  uint64_t need = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const int64_t r = rows5[5 * i];
    need += (uint64_t)(name_off[r + 1] - name_off[r]) + 3 * 21 + 6;
  }
  if (!out) return need;
  if (cap < need) return 0;
  char* o = out;
  for (uint64_t i = 0; i < n; ++i) {
    const int64_t* w = rows5 + 5 * i;
    const int64_t r = w[0];
    std::memcpy(o, names + name_off[r], (size_t)(name_off[r + 1] - name_off[r]));
    o += name_off[r + 1] - name_off[r];
    *o++ = '\t'; o = put_i64(o, w[1]); *o++ = '\t'; o = put_i64(o, w[2]);
    *o++ = '\t'; *o++ = w[3] == 1 ? '+' : '-'; *o++ = '\t'; o = put_i64(o, w[4]); *o++ = '\n';
  }
  return (uint64_t)(o - out);
}

}  // extern "C"
