/*
 * pangenome.h — C ABI of libpangenome_hip.so, the MI355X (gfx950) build of
 * Rinoahu/pangenome's k-mer -> dBG -> rdBG -> region-table hot path.
 *
 * The reference (kmer_numba.py) has no FFI: its seams are Python functions.
 * Each entry point below replaces one of them; the Python host
 * (pangenome_amd/kmer.py) binds this header through ctypes and keeps the
 * reference's CLI, file contracts and printing.  INTEGRATION.md shows the
 * binding a maintainer of the reference would add.
 *
 * Conventions
 *   - every int-returning call returns PG_OK (0) or a negative error code and
 *     records a message for pg_last_error() (thread-local); no exception or
 *     abort crosses the ABI;
 *   - calls are synchronous: results are on the host (or in the caller's
 *     device buffer) when they return;
 *   - a pg_ctx owns all device working memory (one HIP stream on one device);
 *     it is not re-entrant — use one per thread / per GPU;
 *   - host arrays are caller-owned; `*_cap` arguments give their capacity in
 *     elements and the call fails with PG_ERANGE if it is too small (query
 *     sizes first with a NULL pointer where documented).
 */
#ifndef PANGENOME_H
#define PANGENOME_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PG_OK 0
#define PG_EINVAL (-22)
#define PG_ENOMEM (-12)
#define PG_ERANGE (-34)
#define PG_EDEVICE (-5)

typedef struct pg_ctx pg_ctx;

/* What one build did, for throughput and roofline accounting.  Kernel times
 * are HIP-event durations on the context's stream. */
typedef struct pg_stats {
  uint64_t n_bytes;        /* FASTA bytes parsed                                  */
  uint64_t n_records;      /* records (header lines)                              */
  uint64_t n_bases;        /* sequence bases over all records (forward strand)     */
  uint64_t n_windows;      /* k-mer windows inserted (both strands when rc)        */
  uint64_t n_dbg;          /* dBG keys (reference's non-canonical count)           */
  uint64_t n_rdbg;         /* rdBG keys                                            */
  uint64_t n_slots;        /* occupied canonical slots                             */
  uint64_t table_capacity; /* slots in the device hash table                       */
  double ms_parse;         /* K1 wall (host-timed, includes its small D2H syncs)  */
  double ms_clear;         /* (0: the table is written whole, never cleared)      */
  double ms_insert;        /* K3 stage A: coverage + work passes (record emission)*/
  double ms_scan;          /* K3 stages B + C: partition merge with the fused K5  */
  uint64_t sentinel;       /* 1 if the n<k key (2^64-1) is in the dBG              */
  uint64_t n_records_a;    /* K3 stage A records (windows the coverage pass kept)  */
  double ms_split;         /* K3 stage B: k_split pass(es)                         */
  double ms_range;         /* K3 stage C: k_build_range (table + fused K5)         */
  uint64_t build_flags;    /* bit 0: the last pg_build_host split its records into
                              the table's partitions chunk by chunk under the upload
                              (PG_TUNE_EARLY_SPLIT) and stage C read them; bits
                              8..15: stages B/C re-runs of the last build (a plan
                              or a capacity that did not hold); bits 16..23: the
                              k_split passes of stage B (0 when split under the
                              upload)                                             */
  uint64_t n_work_items;   /* K3 stage A work-pass items: 16-window segments the
                              coverage pass left, 64 class bytes read each        */
} pg_stats;

/* Context on HIP device `device` for k-mer length k (clamped to [1, 27] as
 * seq2rdbg does, kmer_numba.py:1236). */
int pg_create(pg_ctx** out, int device, int k);
void pg_destroy(pg_ctx* ctx);
const char* pg_last_error(void);
int pg_get_k(const pg_ctx* ctx);
/* Order this context after a caller's stream: every stream of the context
 * waits (on the device, hipStreamWaitEvent; the host does not block) for
 * the work queued on `stream` (a hipStream_t; NULL = the null stream) when
 * the call is made.  For callers whose allocator hands out memory that
 * work still queued on their stream may touch (a torch caching-allocator
 * block freed behind a queued copy or collective) before they pass it to
 * an entry point that writes or reads it.  Every entry point returns with
 * its own device work complete, so the other direction needs nothing. */
int pg_stream_wait(pg_ctx* ctx, void* stream);

/* ---- input: the mmapped FASTA the reference reads with seq2bytes
 *      (kmer_numba.py:117-119).  Host bytes are copied to HBM; device bytes
 *      (16-byte aligned) are used in place and must outlive the parse. */
int pg_set_fasta(pg_ctx* ctx, const uint8_t* host_bytes, uint64_t nbytes);
int pg_set_fasta_device(pg_ctx* ctx, const uint8_t* device_bytes, uint64_t nbytes);

/* K1: readline_jit_ + seqio_jit_ (kmer_numba.py:122-172) on the device. */
int pg_parse(pg_ctx* ctx, uint64_t* n_records, uint64_t* n_bases);
/* pg_set_fasta + pg_parse for host bytes in one call (seq2bytes + seqio_jit_,
 * :117-172): the copy to HBM goes in chunks (PG_TUNE_H2D_CHUNK, 64 MiB) on a
 * side stream and K1 runs on each chunk once it has landed, so the parse of
 * all but the last chunk hides under the PCIe transfer.  Pinned host memory
 * is DMA'd directly; pageable memory (the np.memmap the reference reads) is
 * copied by a few host threads into a ring of pinned slots that the DMA
 * drains (PG_TUNE_HOST_THREADS).  The bytes are read until the call returns. */
int pg_parse_host(pg_ctx* ctx, const uint8_t* host_bytes, uint64_t nbytes, uint64_t* n_records,
                  uint64_t* n_bases);
/* pg_parse_host + pg_build of every record (seq2rdbg + dbg2rdbg,
 * kmer_numba.py:1234-1321, for an input no -n limit or 2^33-base checkpoint
 * touches) with the build's first stage streamed under the upload: the
 * records a chunk completes go through the coverage / emission pass while
 * the next chunk is copied.  Results equal pg_parse + pg_build(NULL, 0, rc0);
 * the record table is available afterwards (pg_records). */
int pg_build_host(pg_ctx* ctx, const uint8_t* host_bytes, uint64_t nbytes, int rc0, uint64_t* n_rdbg,
                  pg_stats* stats);
/* pg_set_fasta_device + pg_parse + pg_build(NULL, 0, rc0) in one call, for a
 * FASTA already in HBM (seq2rdbg + dbg2rdbg, kmer_numba.py:1234-1321, no -n
 * limit or checkpoint): the host step between the parse and the build runs
 * in C++ with no return to the caller.  The bytes must outlive the call;
 * the record table is available afterwards (pg_records). */
int pg_build_device(pg_ctx* ctx, const uint8_t* device_bytes, uint64_t nbytes, int rc0, uint64_t* n_rdbg,
                    pg_stats* stats);
/* Per-record table (arrays of n_records): compacted sequence length, header
 * byte span (qid = bytes[hdr_start : hdr_start+hdr_len], '>' included,
 * :160) and seqio's resume pointer (:153). Any pointer may be NULL. */
int pg_records(const pg_ctx* ctx, int64_t* seq_len, int64_t* hdr_start, int64_t* hdr_len, int64_t* ptr);

/* K3: seq2rdbg's dBG pass (kmer_numba.py:1234-1268 -> seq2dbg_jit_ :1202-1230
 * -> build_dbg :1052-1090 -> add_kmer :1036-1047).  rec_flags (NULL = all)
 * holds one byte per record: bit0 = record is part of the pass (the host
 * applies -n and the checkpoint/resume rules); extra_empty = number of extra
 * empty records the reference's resume yields (each adds the n<k sentinel).
 * rc0 != 0 inserts the reverse strand too (-c bit 1, :2110). */
int pg_build_dbg(pg_ctx* ctx, const uint8_t* rec_flags, int extra_empty, int rc0, pg_stats* stats);

/* K5: dbg2rdbg (kmer_numba.py:1313-1321 -> build_rdbg_jit_ :1292-1309).
 * The degree scan runs inside pg_build_dbg (every key's masks are final when
 * its table partition is merged; the rdBG keys are materialised there), so
 * this only reports it. */
int pg_build_rdbg(pg_ctx* ctx, uint64_t* n_rdbg, pg_stats* stats);

/* seq2rdbg then dbg2rdbg (kmer_numba.py:1234-1268, :1313-1321) in one call:
 * pg_build_dbg + pg_build_rdbg. */
int pg_build(pg_ctx* ctx, const uint8_t* rec_flags, int extra_empty, int rc0, uint64_t* n_rdbg, pg_stats* stats);

/* dump()'s keys/values (kmer_numba.py:243-261) of the dBG, sorted by key
 * (on the device).  keys == NULL: only *n is set. */
int pg_dbg_export(pg_ctx* ctx, uint64_t* keys, uint16_t* masks, uint64_t cap, uint64_t* n);
/* rdBG keys, sorted. keys == NULL: only *n is set. */
int pg_rdbg_export(pg_ctx* ctx, uint64_t* keys, uint64_t cap, uint64_t* n);

/* ---- npz persistence: dump() / load_on_disk() (kmer_numba.py:243-335).
 * pg_dbg_dump writes the last build's dBG as an oakht slot layout that
 * load_on_disk (:289-335) and oakht.pointer (:521-538) accept: FNV-1a over the
 * key's low 4 bytes mod a prime capacity, probes j, j, j+1, j+4, j+9, ...;
 * keys[capacity] uint64, values[capacity] uint16 (12-bit mask), counts
 * [capacity] uint8 = occurrences of the oriented key, saturating at 255
 * (__setitem__ :556; counted by an extra window pass over the build).
 * *capacity == 0 picks the reference's growth chain (find_prime(2^20), then
 * find_prime(cap * 1.62) while size > 0.75 * cap, :423-474).  keys == NULL
 * only sets *capacity and *size (call again with arrays of *capacity). */
int pg_dbg_dump(pg_ctx* ctx, uint64_t* capacity, uint64_t* keys, uint16_t* values, uint8_t* counts, uint64_t* size);
/* pg_dbg_dump straight into an open file (dump() :243-261 without a host
 * copy of the slot arrays): the keys / values / counts arrays (8, 2 and 1 B
 * per slot) are written at file offsets offsets[0..2] of descriptor fd
 * (pwrite, in 16 MiB pieces streamed from the device through pinned buffers
 * by up to 16 host threads) and crcs[0..2] receive each array's CRC-32.  The
 * .npy headers and the zip framing around them are the caller's
 * (host.write_db_npz).  fd < 0 only sets *capacity and *size. */
int pg_dbg_dump_fd(pg_ctx* ctx, uint64_t* capacity, int fd, const uint64_t* offsets, uint32_t* crcs,
                   uint64_t* size);
/* Stage (oriented key, 12-bit mask, count) pairs — the counts > 0 slots of a
 * loaded npz — to be OR-merged into every following pg_build_dbg (-d: a dBG
 * with no records inserted; -D: rdBG keys with mask 0, members by the rdBG
 * rule; -r: a checkpoint the build resumes onto).  Key 2^64-1 is the n<k
 * sentinel.  counts may be NULL (1 each); n == 0 clears the stage. */
int pg_dbg_load(pg_ctx* ctx, const uint64_t* keys, const uint16_t* masks, const uint8_t* counts, uint64_t n);
/* The reference's final oakht capacity for `size` keys (host only). */
uint64_t pg_oakht_capacity(uint64_t size);

/* ---- multi-GPU exchange (one process per GPU; the caller moves the bytes
 *      with RCCL).  Replaces nothing in the reference, which is single-core.
 *      Device pointers the caller passes (d_out, d_records, d_rows) must be
 *      ready when the call is made: the library's streams do not wait on the
 *      caller's (synchronise the caller's streams first). */
/* Owner-partition this rank's local dBG into `nparts` contiguous runs of
 * 16-byte records (d_out device buffer, capacity out_cap records).
 * counts[nparts] receives run lengths; d_out == NULL only counts. */
int pg_dbg_partition(pg_ctx* ctx, int nparts, void* d_out, uint64_t out_cap, uint64_t* counts);
/* Integrity sums of the last pg_dbg_partition scatter: sums[i] = the sum
 * mod 2^64 of a 64-bit hash of each 16-byte record of run i (the hash is
 * row_check in pangenome_amd/csrc/pg_common.h; order-free, so the
 * receiver's pg_rows_checksum of the same records must equal it). */
int pg_dbg_partition_sums(pg_ctx* ctx, int nparts, uint64_t* sums);
/* The same sums over nseg segments of 16-byte records at device address
 * d_rows: segment s = records [seg_off[s], seg_off[s+1]). */
int pg_rows_checksum(pg_ctx* ctx, const void* d_rows, const uint64_t* seg_off, uint64_t nseg, uint64_t* sums);
/* OR-merge received 16-byte records (device pointer) into a fresh owner
 * table (the rdBG of the owner's keys is built with it); sentinel != 0 adds
 * the n<k key.  capacity_hint is ignored (the table is sized exactly). */
int pg_dbg_merge(pg_ctx* ctx, const void* d_records, uint64_t n, uint64_t capacity_hint, int sentinel);
/* What the last pg_dbg_merge read: non-empty records and the sum of their
 * hashes (pg_dbg_partition_sums' hash over all n records). */
int pg_dbg_merge_check(const pg_ctx* ctx, uint64_t* rows, uint64_t* sum);
/* Routed exchange: the owners build once.  Instead of a local dBG that is
 * partitioned and merged again, a rank's stage A records (h = the table
 * hash of the canonical key, the 26-bit mask word) go to their owners, and
 * only the owners run stages B and C.  The owner of a record is the top
 * log2(nparts) bits of h (nparts a power of two, at most 64), so a rank's
 * records for one owner are whole stage A regions.
 * pg_route_stage_a: after pg_parse / pg_set_fasta(_device) + pg_parse, stage
 * A of the build pg_build_dbg would run (same arguments), held for routing;
 * counts[nparts] = records per owner, *sentinel = the n<k sentinel seen. */
int pg_route_stage_a(pg_ctx* ctx, const uint8_t* rec_flags, int extra_empty, int rc0, int nparts, uint64_t* counts,
                     int* sentinel);
/* The held records as 12-byte rows {h as two little-endian 32-bit words,
 * mask word} grouped by owner into d_out (device, 4-byte aligned, capacity
 * out_cap rows; owner o's run after owner o-1's); sums[nparts] = each run's
 * integrity sum: the hash of the 16-byte {h, mask word, 0} form, as
 * pg_dbg_partition_sums (round 6: 16-byte rows before, a quarter more bytes
 * on the wire). */
int pg_route_scatter(pg_ctx* ctx, int nparts, void* d_out, uint64_t out_cap, uint64_t* sums);
/* pg_rows_checksum over 12-byte routed rows (the receiver's check of what
 * pg_route_scatter's sums say was sent). */
int pg_route_rows_checksum(pg_ctx* ctx, const void* d_rows, const uint64_t* seg_off, uint64_t nseg, uint64_t* sums);
/* World 1: stages B and C on the held records where they lie (this rank
 * owns them all) - the dBG and rdBG of pg_build_dbg, no copy. */
int pg_route_finish(pg_ctx* ctx, uint64_t* n_rdbg, pg_stats* stats);
/* Owner `part` of `nparts`: a fresh table from the n received 12-byte rows (every
 * rank's run for this owner, device pointer), stages A (re-binning), B and
 * C; sentinel != 0 adds the n<k key.  pg_dbg_merge_check reports what it
 * read.  The table's hash domain is h rotated left by log2(nparts) bits:
 * pg_dbg_export / pg_rdbg_export return plain keys. */
int pg_route_merge(pg_ctx* ctx, const void* d_rows, uint64_t n, int nparts, int sentinel, uint64_t* n_rdbg,
                   pg_stats* stats);
/* pg_route_merge over nseg segments of rows (segment s: n[s] rows at the
 * device pointer d_segs[s]) as one owner table: a sub-log received as one
 * run per round and source, merged without concatenating it first.
 * pg_dbg_merge_check reports the rows of every segment together. */
int pg_route_merge_segs(pg_ctx* ctx, const void* const* d_segs, const uint64_t* n, int nseg, int nparts, int sentinel,
                        uint64_t* n_rdbg, pg_stats* stats);

/* ---- edge pass: rdbg_edge_weight_jit_ (kmer_numba.py:1808-1827) ->
 *      rdbg_edge_weight (:1446-1518).  rec_flags as above (walked records);
 *      rc1 != 0 also walks the reverse strand (-c bit 0, :2141). */
int pg_edges(pg_ctx* ctx, const uint8_t* rec_flags, int rc1, uint64_t* n_edges);
/* Edges ordered by first occurrence: 4 x uint64 (n0, v0, n1, v1) per edge,
 * the number of walks containing it, and the walk of its first occurrence
 * (2 * record + strand) — what the host needs to emulate the order reversal
 * of the reference's dump/reload checkpoints (kmer_numba.py:1881-1887). */
int pg_edges_export(pg_ctx* ctx, uint64_t* tuples, int64_t* counts, int64_t* first_walk, uint64_t cap);

/* The `.xyz` text of the last pg_edges, "%d_%d\t%d_%d\t%d\n" per edge in
 * first-occurrence order (seq2graph :1893-1904), formatted on the device.
 * out == NULL: only *n_bytes (the size) is set; otherwise cap >= that size. */
int pg_edges_format(pg_ctx* ctx, char* out, uint64_t cap, uint64_t* n_bytes);
/* The same text written to descriptor fd at its position, which then follows
 * it (the reference writes it to `<qry>_rdbg_weight.xyz`, :1893-1904): a
 * regular file opened without O_APPEND takes 16 MiB pieces in parallel
 * (pwrite from per-thread pinned buffers), anything else in order (write).
 * *n_bytes = the bytes written.  Host-side buffered writers on fd must be
 * flushed first. */
int pg_edges_format_fd(pg_ctx* ctx, int fd, uint64_t* n_bytes);

/* seq2graph's label dictionary (kmer_numba.py:1918-1944) built on the device:
 * the `.mcl` entries (key, value) -> line index as the host's dict holds them
 * (a later line wins), then every `.xyz` node - n0_v0, then n1_v1 of each
 * edge in file order - the .mcl did not label, numbered next_label,
 * next_label + 1, ... in order of first appearance (next_label = the number
 * of .mcl lines).  tuples: the edges as the .xyz lists them (n_edges x 4
 * uint64), or NULL for the last pg_edges in first-occurrence order.  The
 * table replaces any pg_set_labels table for the following pg_rows. */
int pg_labels_from_edges(pg_ctx* ctx, const uint64_t* tuples, uint64_t n_edges, const int64_t* mcl_key,
                         const int64_t* mcl_value, const int64_t* mcl_label, uint64_t n_mcl, int64_t next_label,
                         uint64_t* n_labels);
/* The label table in insertion order: the .mcl entries, then the new ones
 * by label (cap >= n_labels). */
int pg_labels_export(pg_ctx* ctx, int64_t* key, int64_t* value, int64_t* label, uint64_t cap);

/* ---- region rows: seqs2path_jit_ (kmer_numba.py:1830-1849) -> seq2path_jit_
 *      (:1523-1573).  Labels are the host-built label_dct (:1918-1944):
 *      (key, value) -> label. */
int pg_set_labels(pg_ctx* ctx, const int64_t* key, const int64_t* value, const int64_t* label, uint64_t n);
int pg_rows(pg_ctx* ctx, const uint8_t* rec_flags, int rc1, uint64_t* n_rows);
/* rows: 5 x int64 per row (record index, start, end, strand +1/-1, label),
 * in print order. */
int pg_rows_export(pg_ctx* ctx, int64_t* rows5, uint64_t cap);
/* The text of the last pg_rows, "qid\tstart\tend\t+|-\tlabel\n" per row in
 * print order (:1946-1949), formatted on the device; qid of record r is
 * names[name_off[r] .. name_off[r+1]) (n_names >= records, n_names + 1
 * offsets).  out == NULL: only *n_bytes is set. */
int pg_rows_format(pg_ctx* ctx, const char* names, const int64_t* name_off, uint64_t n_names, char* out, uint64_t cap,
                   uint64_t* n_bytes);
/* The same text written to descriptor fd (the reference prints it to
 * stdout, :1946-1949), as pg_edges_format_fd writes. */
int pg_rows_format_fd(pg_ctx* ctx, const char* names, const int64_t* name_off, uint64_t n_names, int fd,
                      uint64_t* n_bytes);

/* ---- text output (host only; no context).  The reference formats these in
 *      Python loops (kmer_numba.py:1893-1904, :1946-1949).
 * pg_format_xyz: "%d_%d\t%d_%d\t%d\n" per edge (tuples as unsigned).
 * pg_format_rows: "qid\tstart\tend\t+|-\tlabel\n" per row; qid of record r
 * is names[name_off[r] .. name_off[r+1]).  With out == NULL both return the
 * buffer size they need; otherwise the bytes written, 0 if cap is short. */
uint64_t pg_format_xyz(const uint64_t* tuples, const int64_t* counts, uint64_t n, char* out, uint64_t cap);
uint64_t pg_format_rows(const int64_t* rows5, uint64_t n, const char* names, const int64_t* name_off, char* out,
                        uint64_t cap);

/* Tuning (tests and experiments; the defaults are the product setting).
 * PG_TUNE_K3_CHUNKS: chunks of the K3 tile list whose work pass overlaps the
 * next chunk's coverage pass, 1..6, or 0 = by tile count (3 when the list
 * has >= 3072 coverage groups, else 1). */
#define PG_TUNE_K3_CHUNKS 1
/* PG_TUNE_K3_COVER: form of the K3 coverage pass, 0 (default) = K1's packed
 * 2-bit base stream compared word by word, exact per base (round 4); 1 =
 * class bytes staged in LDS (round 2); 2 = class bytes compared 16 at a time
 * from registers, per dword (round 3).  The results are the same, only the
 * records left to the work pass differ. */
#define PG_TUNE_K3_COVER 10
/* PG_TUNE_K3_WBLK: blocks per CU of the K3 work passes when the tile list
 * runs in chunks: low 4 bits for every chunk but the last, high 4 bits for
 * the last (0 = 2 and the same as the others). */
#define PG_TUNE_K3_WBLK 11
/* PG_TUNE_K3_EMIT: form of the K3 work pass, 0 (default) = each queued
 * segment's records computed and emitted in two halves, 1 = at once. */
#define PG_TUNE_K3_EMIT 12
/* PG_TUNE_K3_TAIL: size of the last K3 chunk in 16ths of the others (1..64,
 * 0 = 10: the work pass left behind the last coverage pass is smaller). */
#define PG_TUNE_K3_TAIL 13
/* PG_TUNE_EARLY_SPLIT: pg_build_host's stage B under the upload, 1 (default)
 * = the records of each landed chunk split into the table's fine partitions
 * as soon as its stage A share is done (geometry from the last build; a
 * mismatch at the end re-splits everything), 0 = after the last chunk. */
#define PG_TUNE_EARLY_SPLIT 14
/* PG_TUNE_K3_HEAD: size of the first K3 chunk in 16ths of the middle ones
 * (1..64, 0 = 16: the coverage pass that runs before any work pass). */
#define PG_TUNE_K3_HEAD 15
/* PG_TUNE_H2D_TAIL: bytes of pg_build_host's last H2D chunk (0, the default:
 * every chunk PG_TUNE_H2D_CHUNK bytes).  A small last chunk puts two chunks'
 * K1, record round trip and stage A share behind the last copy (C3: 9.91 ms
 * at 8 MiB, 9.86 at 16, 9.80 uniform). */
#define PG_TUNE_H2D_TAIL 16
/* PG_TUNE_BUCKET_SHIFT: size the table 2^value times smaller than the record
 * count asks (0..8): exercises the overflow set, its spill and the re-run
 * with more buckets (results are unchanged). */
#define PG_TUNE_BUCKET_SHIFT 2
/* PG_TUNE_REGION_CAP: first stage A region size in records (0 = estimated):
 * a small value exercises the stage A re-run (results are unchanged). */
#define PG_TUNE_REGION_CAP 3
/* PG_TUNE_H2D_CHUNK: bytes per pg_parse_host chunk, rounded down to whole
 * 16 KiB K1 spans (0 = 64 MiB): small values exercise the pipeline. */
#define PG_TUNE_H2D_CHUNK 4
/* PG_TUNE_HOST_THREADS: host threads that copy a pageable input (an mmap)
 * into the pinned staging ring of pg_parse_host / pg_build_host / pg_set_fasta
 * (1..64, 0 = half the CPUs the process may run on, at most 8). */
#define PG_TUNE_HOST_THREADS 5
/* PG_TUNE_STAGE_PIECE / PG_TUNE_STAGE_SLOTS: bytes per slot of that ring (one
 * DMA each; 0 = 32 MiB) and its slot count (2..8, 0 = 4); the first pieces
 * of an upload are smaller (2, 4, 8 ... MiB). */
#define PG_TUNE_STAGE_PIECE 6
#define PG_TUNE_STAGE_SLOTS 7
/* PG_TUNE_HOST_REGISTER: 1 (default) = a pageable input's page-aligned
 * chunks are registered (hipHostRegister, read-only) for the duration of the
 * upload and DMA'd directly, falling back to the staging ring for the rest
 * when a chunk cannot be; 0 = staging ring only. */
#define PG_TUNE_HOST_REGISTER 8
/* PG_TUNE_DEVICE_CAP: the most device bytes the library's buffers may hold
 * in this process, over all contexts (0 = no cap): an allocation past it
 * fails with PG_ENOMEM.  Setting it also restarts pg_device_bytes' peak.
 * PROCESS-WIDE: although it is set through one context's pg_tune, the cap
 * and the peak it restarts are shared by every context of the process (and
 * every device).  For tests of a path's memory budget at a scaled-down size. */
#define PG_TUNE_DEVICE_CAP 9
/* PG_TUNE_POISON (debug, PROCESS-WIDE like PG_TUNE_DEVICE_CAP): every device
 * buffer the library allocates from now on is filled with this byte value
 * (0..255; -1, the default, = off), so that a kernel reading memory nothing
 * wrote gives a different result instead of inheriting an earlier run's. */
#define PG_TUNE_POISON 17
/* PG_TUNE_K1: K1 form bits.  Bit 0: the span pass, 0 = per-step form (fast
 * or general 1 KiB step), 1 = whole-span form (a 16 KiB span without '>' and
 * below the last byte counted in one pass of SWAR sums, its newline positions
 * found afterwards; the spans left over by a step-parallel per-step pass).
 * Bit 1: the emission keeps two wave steps of loads in flight (else one).
 * Bit 2: the record table (header pass, k_records, its copy to the host) on
 * the context's stream ahead of the emission, instead of beside it on the
 * high-priority stream. */
#define PG_TUNE_K1 18
/* PG_TUNE_TIMERS: which stage spans of pg_stats are timed with HIP events on
 * the stream (each timing event costs the stream a few us): bit 0 K1
 * (ms_parse), bit 1 stage A (ms_insert), bit 2 stages B/C (ms_split,
 * ms_range); 7 (default) = all, 0 = none (the spans read 0). */
#define PG_TUNE_TIMERS 19
/* PG_TUNE_K3_ANCHORS: anchors per tile and reference of the packed coverage
 * pass (3, 4, 5, 6 or 8; 0 = 4).  More anchors find the drift of more of the
 * short runs between two indels, so fewer windows go to the work pass as
 * records (C3: 27.6 M stage A records with 3, 24.2 M with 4, 21.8 M with 8),
 * at a dearer drift search (C3 step: 4 is the fastest). */
#define PG_TUNE_K3_ANCHORS 20
int pg_tune(pg_ctx* ctx, int what, int64_t value);

/* Device bytes the library's buffers hold in this process now (peak == 0)
 * or at most since the last PG_TUNE_DEVICE_CAP (peak != 0). */
uint64_t pg_device_bytes(int peak);

/* Timings and counters of the last build (see pg_stats). */
int pg_get_stats(const pg_ctx* ctx, pg_stats* stats);

#ifdef __cplusplus
}
#endif
#endif /* PANGENOME_H */
