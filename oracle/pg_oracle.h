/*
 * pg_oracle.h — CPU restatement of Rinoahu/pangenome kmer_numba.py's
 * k-mer -> dBG -> rdBG -> edges -> region-row path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or the timed CPU baseline); the product path (libpangenome_hip.so) never
 * links or calls it.
 *
 * Pinned against the reference's own behaviour: tests/golden/ holds vectors
 * produced by running /root/reference/kmer_numba.py itself (pure-Python mode,
 * tests/golden/make_goldens.py); tests/test_oracle_golden.py checks every one.
 *
 * The dBG is kept in a faithful restatement of the reference's `oakht`
 * (kmer_numba.py:340-679): FNV-1a-64 over the key's low 4 bytes, prime
 * capacity from find_prime(2^20), probe j0, j0, j0+1, j0+4, ..., growth x1.62
 * at load 0.75, and add_kmer's three probe sequences per occurrence
 * (has_key, get, push; :1036-1047).  That makes it the honest single-core
 * CPU baseline ("kind": "port") as well as the parity oracle.
 */
#ifndef PG_ORACLE_H
#define PG_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pgo_result pgo_result;

/* Run the reference's dBG pass (seq2rdbg :1234-1268, with seq2dbg_jit_'s
 * chunk checkpoints :1224-1225 and their resume quirks), then dbg2rdbg
 * (:1313-1321).  ns_never != 0 emulates the default -n 2**63 (never hit).
 * Returns 0 on success. */
int pgo_build_graph(const uint8_t* buf, int64_t n, int k, int rc0,
                    int64_t ns, int ns_never, int64_t chunk, pgo_result** out);

/* Edge pass (seq2graph :1853-1904 -> rdbg_edge_weight_jit_ :1808-1827 ->
 * rdbg_edge_weight :1446-1518) over the same buffer, in reference order
 * (typed-Dict insertion order, reversed at every dump/reload checkpoint). */
int pgo_edges(pgo_result* r, const uint8_t* buf, int64_t n, int rc1,
              int64_t ns, int ns_never, int64_t chunk);

/* Region rows (seqs2path_jit_ :1830-1849 -> seq2path_jit_ :1523-1573) given
 * a label table {(lab_key[i], lab_val[i]) -> lab_id[i]}. */
int pgo_rows(pgo_result* r, const uint8_t* buf, int64_t n, int rc1,
             int64_t ns, int ns_never,
             const int64_t* lab_key, const int64_t* lab_val, const int64_t* lab_id,
             int64_t n_labels);

int64_t pgo_n_dbg(const pgo_result* r);
int64_t pgo_n_rdbg(const pgo_result* r);
int64_t pgo_n_edges(const pgo_result* r);
int64_t pgo_n_rows(const pgo_result* r);
int64_t pgo_n_bases(const pgo_result* r);     /* fw bases seen by the dBG pass (N of :1212) */
int64_t pgo_n_records(const pgo_result* r);
double pgo_seconds_dbg(const pgo_result* r);   /* stage timers mirroring :2107-2135 */
double pgo_seconds_rdbg(const pgo_result* r);

/* Copy-outs, in the oakht's slot order (dBG, rdBG) or reference order. */
void pgo_get_dbg(const pgo_result* r, uint64_t* keys, uint16_t* masks);
void pgo_get_dbg_counts(const pgo_result* r, uint8_t* counts);   /* saturating occurrence counts */
int64_t pgo_dbg_capacity(const pgo_result* r);
void pgo_get_rdbg(const pgo_result* r, uint64_t* keys);
/* edges: 4 x uint64 per edge (n0, v0, n1, v1) and the walk count */
void pgo_get_edges(const pgo_result* r, uint64_t* tuples, int64_t* counts);
/* rows: (header_start, header_len, start, end, strand(+1/-1), label) per row;
 * header bytes are buf[header_start : header_start+header_len] and include '>'. */
void pgo_get_rows(const pgo_result* r, int64_t* rows6);

/* Replace the rdBG key set (what load_on_disk of a -D file gives seq2graph,
 * :2093): the edge and row passes then query exactly these keys.  Used by the
 * multi-GPU tests, where every rank walks its records against the rdBG
 * gathered from all owners. */
void pgo_set_rdbg(pgo_result* r, const uint64_t* keys, int64_t n);

void pgo_free(pgo_result* r);

/* The dBG entries whose key lies in [lo, hi) (hi = 2^64-1: the n<k sentinel
 * included), sorted by key, of the same dBG pass as pgo_build_graph, by
 * sorting the range's occurrences instead of an oakht (inputs too big for
 * one in-memory table are digested range by range).  Returns the entry
 * count, or -1 when out of memory; *keys / *masks are freed with
 * pgo_free_buf. */
int64_t pgo_dbg_range(const uint8_t* buf, int64_t n, int k, int rc0, int64_t ns, int ns_never, int64_t chunk,
                      uint64_t lo, uint64_t hi, uint64_t** keys, uint16_t** masks);
void pgo_free_buf(void* p);

#ifdef __cplusplus
}
#endif
#endif
