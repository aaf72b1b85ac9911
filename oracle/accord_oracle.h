/*
 * accord_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference (aweisberg/cassandra-accord @ 2025-03-04) algorithms on the
 * dependency-calculation path. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this; the product path (libaccord_amd.so) never links or calls it.
 *
 * Parity status:
 *   - KeyDeps.Builder / linearUnion / KeyDeps.merge: pinned by the reference's own property tests
 *     (KeyDepsTest.testMergedProperty, builder, testSimpleEquality), restated as committed fixtures.
 *   - CommandsForKey.mapReduceActive: the reference has NO test for it (CommandsForKey.java:126
 *     "TODO (required): randomised testing"); the Java cannot be built here (no JDK, Gradle needs
 *     network). Its parity is pinned only by this line-by-line restatement cross-checked against the
 *     independent Python model in oracle/canonical.py ("parity unpinned" by the reference itself).
 */
#ifndef ACCORD_ORACLE_H
#define ACCORD_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_keydeps_result {
    uint32_t  n_txn;
    uint64_t *arena_off;  int32_t  *arena;
    uint64_t *kd_off;     uint32_t *key_idx;
    uint64_t *u_off;      uint32_t *dep_txn;
    uint64_t  total_edges;
    uint64_t  visited;    /* entries visited by the O(prefix) scans (work counter) */
    uint64_t  queried_pairs; /* (txn, key) pairs evaluated as queries */
    double    build_s;    /* seconds spent building the CommandsForKey snapshot */
    double    query_s;    /* seconds spent in the per-txn calculatePartialDeps loop */
    int       error;      /* 0 ok, -1 IllegalArgument, -2 IllegalState */
    char      message[256];
    uint64_t *kd_key;     /* [kd_off[n]] KeyDeps.keys as key codes */
} orc_keydeps_result;

/* Batch PreAccept.calculatePartialDeps over one CommandsForKey snapshot (SURVEY.md §8 batch
 * semantics). n_shards > 1 evaluates it the way CommandStores do: EvenSplit of the key-code domain
 * into contiguous shards, per-shard calculatePartialDeps, then the PreAccept.reduce fold of
 * PartialDeps.with in shard order (PreAccept.java:141-156, CommandStores.java:575-592).
 * query_lo/query_hi/query_stride restrict which txns are evaluated as queries (t in [lo, hi) with
 * (t - lo) % stride == 0); all txns stay CFK entries; results for other txns are empty. */
orc_keydeps_result *orc_keydeps_batch(uint32_t n,
                                      const uint64_t *tmsb, const uint64_t *tlsb, const int32_t *tnode,
                                      const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                                      const uint8_t *status, const uint32_t *key_off, const uint64_t *key_code,
                                      uint32_t n_shards, uint32_t query_lo, uint32_t query_hi,
                                      uint32_t query_stride);
/* The same with an explicit query set: txn t is evaluated iff query_mask[t] != 0 (one snapshot build for a scattered
 * sample). */
orc_keydeps_result *orc_keydeps_batch_qmask(uint32_t n,
                                            const uint64_t *tmsb, const uint64_t *tlsb, const int32_t *tnode,
                                            const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                                            const uint8_t *status, const uint32_t *key_off, const uint64_t *key_code,
                                            const uint8_t *query_mask);
/* The same over a mixed key/range batch (rng_* as orc_rangedeps_batch): range-domain txns are no CommandsForKey
 * members; as queries they scan every CFK whose key lies in their (store-sliced) ranges
 * (InMemoryCommandStore.mapReduceForKey :274-289). For a range txn, key_idx indexes the list of CFK keys its
 * ranges cover (range order); kd_key holds the key codes for every txn. */
orc_keydeps_result *orc_keydeps_mixed(uint32_t n,
                                      const uint64_t *tmsb, const uint64_t *tlsb, const int32_t *tnode,
                                      const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                                      const uint8_t *status, const uint32_t *key_off, const uint64_t *key_code,
                                      const uint32_t *rng_off, const uint64_t *rng_start, const uint64_t *rng_end,
                                      int end_inclusive, uint32_t n_shards, uint32_t query_lo, uint32_t query_hi,
                                      uint32_t query_stride);
/* orc_keydeps_mixed with an explicit query set (query_mask[t] != 0). */
orc_keydeps_result *orc_keydeps_mixed_qmask(uint32_t n,
                                            const uint64_t *tmsb, const uint64_t *tlsb, const int32_t *tnode,
                                            const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                                            const uint8_t *status, const uint32_t *key_off, const uint64_t *key_code,
                                            const uint32_t *rng_off, const uint64_t *rng_start, const uint64_t *rng_end,
                                            int end_inclusive, const uint8_t *query_mask);
void orc_keydeps_free(orc_keydeps_result *r);

/* KeyDeps.merge (KeyDeps.java:115-135) over groups of replies in the acc_merge_in layout
 * (integer key codes, u32 TxnId order ranks). Output arrays are malloc'd; free with orc_merge_free. */
typedef struct orc_merge_result {
    uint32_t  n_groups;
    uint64_t *key_off; uint64_t *key_code;
    uint64_t *val_off; uint32_t *txn_rank;
    uint64_t *k2v_off; int32_t  *k2v;
    int       error;
    char      message[256];
} orc_merge_result;

orc_merge_result *orc_keydeps_merge(uint32_t n_groups, const uint64_t *grp_off,
                                    const uint64_t *key_off, const uint64_t *key_code,
                                    const uint64_t *val_off, const uint32_t *txn_rank,
                                    const uint64_t *k2v_off, const int32_t *k2v);
void orc_merge_free(orc_merge_result *r);

/* Deterministic levelisation restatement. */
int orc_levelise(uint32_t n, const uint64_t *off, const uint32_t *dep, const uint32_t *exec_rank,
                 uint32_t *level, uint32_t *order, uint32_t *n_levels);

/* RangeDeps of a mixed key/range batch (SURVEY.md §8 A8 range part, config 4). Txns whose TxnId domain bit
 * (lsb & 1, TxnId.java:124-157) is Range are range commands with the ranges [rng_off[t], rng_off[t+1]);
 * key txns list keys as in orc_keydeps_batch. For every queried txn T, restates
 * InMemoryCommandStore.mapReduceRangesInternal (InMemoryCommandStore.java:883-1016) as called by
 * mapReduceActive (:863-870) from PreAccept.calculatePartialDeps (PreAccept.java:245-265): range commands
 * in TxnId order, TxnId < T.executeAt, kind witnessed by T, status not INVALID (saveStatus < Erased),
 * each of their ranges intersecting T's keys/ranges collected per Range (Range::compare order), p1
 * excluded, then RangeDeps.Builder. end_inclusive = 1: Range.EndInclusive (s, e]; 0: StartInclusive [s, e).
 * Ranges are reported as ids into the dictionary of distinct stored ranges sorted by (start, end). */
typedef struct orc_rangedeps_result {
    uint32_t  n_txn;
    uint32_t  n_ranges;   uint64_t *rng_start; uint64_t *rng_end;   /* dictionary */
    uint64_t *arena_off;  int32_t  *arena;      /* Java rangesToTxnIds per txn */
    uint64_t *rd_off;     uint32_t *range_id;   /* per txn: dictionary ids, ascending */
    uint64_t *u_off;      uint32_t *dep_txn;    /* per txn: batch indices in TxnId order */
    uint64_t  total_edges;
    uint64_t  visited;    /* range-command entries examined (work counter) */
    uint64_t  queried;    /* txns evaluated */
    double    query_s;
    int       error;
    char      message[256];
} orc_rangedeps_result;

orc_rangedeps_result *orc_rangedeps_batch(uint32_t n,
                                          const uint64_t *tmsb, const uint64_t *tlsb, const int32_t *tnode,
                                          const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                                          const uint8_t *status, const uint32_t *key_off, const uint64_t *key_code,
                                          const uint32_t *rng_off, const uint64_t *rng_start, const uint64_t *rng_end,
                                          int end_inclusive, uint32_t query_lo, uint32_t query_hi, uint32_t query_stride);
/* orc_rangedeps_batch with an explicit query set (query_mask[t] != 0). */
orc_rangedeps_result *orc_rangedeps_batch_qmask(uint32_t n,
                                                const uint64_t *tmsb, const uint64_t *tlsb, const int32_t *tnode,
                                                const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                                                const uint8_t *status, const uint32_t *key_off, const uint64_t *key_code,
                                                const uint32_t *rng_off, const uint64_t *rng_start,
                                                const uint64_t *rng_end, int end_inclusive, const uint8_t *query_mask);
void orc_rangedeps_free(orc_rangedeps_result *r);

/* InMemorySafeStore.mapReduceRangesInternal (impl/InMemoryCommandStore.java:883-1016), the range-command half of the
 * BeginRecovery scans, per query into a Deps.Builder; table and queries as acc_map_reduce_full_ranges
 * (include/accord_amd.h). Results per query in the orc_rangedeps_result layout (dep_txn = first table index). */
orc_rangedeps_result *orc_map_reduce_full_ranges(uint32_t n,
                                                 const uint64_t *tmsb, const uint64_t *tlsb, const int32_t *tnode,
                                                 const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                                                 const uint8_t *status, const uint8_t *flags,
                                                 const uint32_t *rng_off, const uint64_t *rng_start, const uint64_t *rng_end,
                                                 int end_inclusive, const uint32_t *dep_off, const uint64_t *dmsb,
                                                 const uint64_t *dlsb, const int32_t *dnode, const uint64_t *dep_start,
                                                 const uint64_t *dep_end, const uint8_t *dep_is_key,
                                                 uint32_t nq, const uint64_t *qmsb, const uint64_t *qlsb, const int32_t *qnode,
                                                 const uint8_t *part_is_range, const uint32_t *part_off,
                                                 const uint64_t *part_start, const uint64_t *part_end,
                                                 int started_at, int test_dep, int test_status, int test_kinds, int exec_after);

/* ---- accord_oracle_rmm.c: RelationMultiMap operations on whole deps objects over raw values ---- */

/* KeyDeps.merge / RangeDeps.merge (LinearMerger fold of linearUnion) per group of replies with raw TxnId columns;
 * keys are (key_a, 0) codes or (key_a, key_b) = (start, end) ranges (is_range). val_src = input slot of the TxnId
 * instance the Java keeps (SortedArrays.linearUnion / RelationMultiMap.linearUnion identity rules). */
typedef struct orc_rmm_merge_result {
    uint32_t  n_groups;
    uint64_t *key_off;  uint64_t *key_a; uint64_t *key_b;
    uint64_t *val_off;  uint64_t *val_src; uint64_t *val_msb; uint64_t *val_lsb; int32_t *val_node;
    uint64_t *k2v_off;  int32_t  *k2v;
    int       error;
    char      message[256];
} orc_rmm_merge_result;
orc_rmm_merge_result *orc_rmm_merge(uint32_t n_groups, const uint64_t *grp_off, int is_range,
                                    const uint64_t *key_off, const uint64_t *key_a, const uint64_t *key_b,
                                    const uint64_t *val_off, const uint64_t *vmsb, const uint64_t *vlsb, const int32_t *vnode,
                                    const uint64_t *k2v_off, const int32_t *k2v);
void orc_rmm_merge_free(orc_rmm_merge_result *r);

/* RelationMultiMap.invert, batched (trg_off[n_groups+1], trg sized sum(ntrg + entries)). Returns 0 / -1. */
int orc_invert(uint32_t n_groups, const uint64_t *src_off, const int32_t *src, const uint64_t *nsrc, const uint64_t *ntrg,
               uint64_t *trg_off, int32_t *trg);

/* KeyDeps.slice / RangeDeps.slice + trimUnusedValues per group (select ranges sel[sel_off[g]..sel_off[g+1])). */
typedef struct orc_slice_result {
    uint32_t  n_groups;
    uint64_t *key_off; uint32_t *key_idx;   /* selected key indices (into the group's keys) */
    uint64_t *val_off; uint32_t *val_idx;   /* kept TxnId indices (into the group's txnIds) */
    uint64_t *k2v_off; int32_t  *k2v;
} orc_slice_result;
orc_slice_result *orc_rmm_slice(uint32_t n_groups, int is_range, int end_inclusive,
                                const uint64_t *key_off, const uint64_t *key_a, const uint64_t *key_b,
                                const uint64_t *val_off, const uint64_t *k2v_off, const int32_t *k2v,
                                const uint64_t *sel_off, const uint64_t *sel_s, const uint64_t *sel_e);
void orc_slice_free(orc_slice_result *r);

/* RelationMultiMap.remove = KeyDeps/RangeDeps.without per group, remove = membership in the group's set a or b
 * (Deps::contains); kind[g]: 0 from, 1 none, 2 rebuilt. Free with orc_slice_free. */
orc_slice_result *orc_rmm_without(uint32_t n_groups, const uint64_t *key_off, const uint64_t *val_off,
                                  const uint64_t *k2v_off, const int32_t *k2v,
                                  const uint64_t *vm, const uint64_t *vl, const int32_t *vn,
                                  const uint64_t *a_off, const uint64_t *am, const uint64_t *al, const int32_t *an,
                                  const uint64_t *b_off, const uint64_t *bm, const uint64_t *bl, const int32_t *bn,
                                  uint8_t *kind);

/* Stabbing queries over built RangeDeps: per query the ascending indices of group grp[q]'s ranges containing the
 * key qs[q] (is_key_query) or intersecting [qs[q], qe[q]). */
typedef struct orc_stab_result { uint64_t *off; uint32_t *idx; } orc_stab_result;
orc_stab_result *orc_rmm_stab(uint32_t n_queries, const uint32_t *grp, const uint64_t *qs, const uint64_t *qe,
                              int is_key_query, int end_inclusive, const uint64_t *rng_off, const uint64_t *rs,
                              const uint64_t *re);
void orc_stab_free(orc_stab_result *r);

/* Timestamp.compareTo (Timestamp.java:208-217) — exported for tests. */
int orc_ts_compare(uint64_t amsb, uint64_t alsb, int32_t anode, uint64_t bmsb, uint64_t blsb, int32_t bnode);

#ifdef __cplusplus
}
#endif

/* ---- accord_oracle_cfk.c: CommandsForKey.update with the command's deps (missing[], TRANSITIVELY_KNOWN additions) ----
 * Key-major CommandsForKey snapshot (key k: entries [ent_off[k], ent_off[k+1]) sorted by TxnId, each with executeAt,
 * InternalStatus and missing[] = [miss_off[e], miss_off[e+1]) sorted), then n_upd command updates applied in order to
 * every key they list (ust = new InternalStatus, 0xFF = none; uflags bit 0 = acceptedOrCommitted changed; per (update,
 * key) pair the command's partialDeps().keyDeps.txnIds(key) in [udep_off[j], udep_off[j+1])). Result key-major. */
typedef struct orc_cfk_result {
    uint32_t n_keys;
    uint64_t *key; uint32_t *ent_off;
    uint64_t *emsb, *elsb; int32_t *enode;
    uint64_t *xmsb, *xlsb; int32_t *xnode;
    uint8_t *status;
    uint32_t *miss_off;
    uint64_t *mmsb, *mlsb; int32_t *mnode;
    uint64_t n_entries, n_missing;
    int error; char message[256];
} orc_cfk_result;

orc_cfk_result *orc_cfk_apply(uint32_t n_keys, const uint64_t *key, const uint32_t *ent_off,
                              const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                              const uint64_t *xmsb, const uint64_t *xlsb, const int32_t *xnode, const uint8_t *est,
                              const uint32_t *miss_off, const uint64_t *mmsb, const uint64_t *mlsb, const int32_t *mnode,
                              uint32_t n_upd, const uint64_t *umsb, const uint64_t *ulsb, const int32_t *unode,
                              const uint64_t *uxmsb, const uint64_t *uxlsb, const int32_t *uxnode, const uint8_t *ust,
                              const uint8_t *uflags, const uint32_t *ukey_off, const uint64_t *ukey,
                              const uint32_t *udep_off, const uint64_t *dmsb, const uint64_t *dlsb, const int32_t *dnode);
void orc_cfk_free(orc_cfk_result *r);

/* MaxConflicts.get + the PreAccept fast-path test for each query (accord_oracle_cfk.c); layout as acc_max_conflicts */
int orc_max_conflicts(uint32_t n_upd, const uint64_t *xmsb, const uint64_t *xlsb, const int32_t *xnode,
                      const uint32_t *key_off, const uint64_t *key, const uint32_t *rng_off, const uint64_t *rs,
                      const uint64_t *re, int end_inclusive, uint32_t nq, const uint64_t *qmsb, const uint64_t *qlsb,
                      const int32_t *qnode, const uint8_t *is_range, const uint32_t *part_off, const uint64_t *ps,
                      const uint64_t *pe, uint64_t *omsb, uint64_t *olsb, int32_t *onode, uint8_t *fast);

#endif
