/*
 * accord_amd.h — C ABI of the MI355X-native Accord dependency-calculation path.
 *
 * This is the drop-in boundary a JVM shim (JNI for Java 11, FFM for Java >= 22) binds; see
 * INTEGRATION.md for the binding stubs. Plain pointers and sizes only: no C++, no torch types.
 *
 * Reference interfaces replaced (paths relative to accord-core/src/main/java/accord/):
 *
 *   acc_keydeps_batch      PreAccept.calculatePartialDeps            messages/PreAccept.java:245-265
 *                          -> SafeCommandStore.mapReduceActive        local/SafeCommandStore.java:279
 *                          -> InMemorySafeStore.mapReduceActive       impl/InMemoryCommandStore.java:863-870
 *                          -> CommandsForKey.mapReduceActive          local/CommandsForKey.java:614-650
 *                          -> KeyDeps.Builder / AbstractBuilder.build utils/RelationMultiMap.java:88-260
 *                          evaluated for every txn of a batch against one CommandsForKey snapshot
 *                          (batch semantics: SURVEY.md §8 "Batch semantics").
 *   acc_keydeps_merge      KeyDeps.merge(List, getter, getter)       primitives/KeyDeps.java:115-135
 *                          (LinearMerger fold of linearUnion,         utils/RelationMultiMap.java:284-406,561-816)
 *                          batched over many coordinated txns (Deps.merge primitives/Deps.java:256-260).
 *   acc_rangedeps_batch    the range-command part of InMemorySafeStore.mapReduceActive impl/InMemoryCommandStore.java:863-870
 *                          -> mapReduceRangesInternal                 impl/InMemoryCommandStore.java:883-1016
 *                          -> RangeDeps.Builder                       primitives/RangeDeps.java:873-891
 *                          for every txn of a mixed key/range batch (PreAccept.calculatePartialDeps
 *                          messages/PreAccept.java:245-265; SearchableRangeList stabbing core/utils/SearchableRangeList.java:89-116).
 *   acc_shard_pack /       per-node reduce of per-CommandStore PartialDeps across GPUs (PreAccept.reduce
 *   acc_shard_merge        messages/PreAccept.java:141-156, CommandStores.mapReduce local/CommandStores.java:575-592):
 *                          fragments to the txn's home GPU (all-to-all(v) by the host over RCCL), then KeyDeps.with
 *                          folded in shard order = the batched KeyDeps.merge below.
 *   acc_partial_deps_batch both halves of PartialDeps of a mixed batch in one call (KeyDeps + RangeDeps through
 *                          PartialDeps.Builder primitives/PartialDeps.java:31-45), one shared dictionary pass.
 *   acc_map_reduce_full    the recovery scans of BeginRecovery        messages/BeginRecovery.java:334-378
 *                          -> SafeCommandStore.mapReduceFull          local/SafeCommandStore.java:285
 *                          -> InMemorySafeStore.mapReduceFull         impl/InMemoryCommandStore.java:874-881 (key part)
 *                          -> CommandsForKey.mapReduceFull            local/CommandsForKey.java:553-612
 *                          -> Deps.Builder                            primitives/Deps.java:46-96
 *                          for a batch of recovery queries against one CommandsForKey snapshot.
 *   acc_map_reduce_full_ranges  the range-command half of the same scans  impl/InMemoryCommandStore.java:883-1016
 *   acc_latest_deps_merge  LatestDeps.mergeProposal / mergeCommit     primitives/LatestDeps.java:306-326
 *                          (Recover.java:295-355): the interval fold of the replies, then KeyDeps/RangeDeps.slice of
 *                          every selected deps object to its interval and the batched Deps.merge of the slices.
 *   acc_deps_from_json /   Json.DEPS_ADAPTER read / write             accord-maelstrom/.../maelstrom/Json.java:316-398
 *   acc_deps_to_json       (the in-tree Deps wire format) parsed / written on device, with the KeyDeps / RangeDeps Builder.
 *   acc_cfk_*              CommandsForKey.update for batches of commands   local/CommandsForKey.java:652-706
 *                          against a CFK store kept in HBM (SafeCommandStore.updateCommandsForKey :217-240).
 *   acc_levelise           execution-order restatement of Commands.updateWaitingOn local/Commands.java:776-830
 *                          (deterministic wavefront schedule).
 *
 * Array-level seams mirrored: KeyDeps.SerializerSupport.create(Keys, TxnId[], int[])
 * (primitives/KeyDeps.java:55-73): every per-txn result is emitted as the exact Java `keysToTxnIds`
 * int[] plus the key subset and the TxnId array (as batch indices).
 *
 * Error model (utils/Invariants.java:98-205): IllegalArgumentException -> ACC_E_ARG,
 * IllegalStateException / AssertionError -> ACC_E_STATE. Device failures have their own codes.
 * acc_last_error(ctx) returns the message of the last failing call on that context.
 *
 * Threading (local/SafeCommandStore.java:50-55): one acc_ctx per host thread / CommandStore shard;
 * calls on one ctx are not re-entrant; distinct contexts run on independent HIP streams.
 */
#ifndef ACCORD_AMD_H
#define ACCORD_AMD_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* A Ranges: sorted, deoverlapped Range (start, end) key codes of one bound type (primitives/Ranges.java). */
typedef struct acc_rlist {
    const uint64_t *start;
    const uint64_t *end;
    uint32_t n;
    uint32_t reserved;
} acc_rlist;

/* ---- error codes ---- */
#define ACC_OK          0
#define ACC_E_ARG      (-1)   /* IllegalArgumentException class */
#define ACC_E_STATE    (-2)   /* IllegalStateException / invariant violation */
#define ACC_E_NOMEM    (-3)   /* device allocation failed */
#define ACC_E_DEVICE   (-4)   /* HIP runtime error */
#define ACC_E_CAP      (-5)   /* caller buffer too small; required sizes were written */

/* ---- InternalStatus ordinals (local/CommandsForKey.java:194-203) ---- */
#define ACC_ST_TRANSITIVELY_KNOWN   0
#define ACC_ST_HISTORICAL           1
#define ACC_ST_PREACCEPTED          2
#define ACC_ST_ACCEPTED             3
#define ACC_ST_COMMITTED            4
#define ACC_ST_STABLE               5
#define ACC_ST_APPLIED              6
#define ACC_ST_INVALID_OR_TRUNCATED 7

/* ---- Txn.Kind ordinals (primitives/Txn.java:53-113); kind = (lsb >> 1) & 7 (TxnId.java:149-152) ---- */
#define ACC_KIND_READ                 0
#define ACC_KIND_WRITE                1
#define ACC_KIND_EPHEMERAL_READ       2
#define ACC_KIND_SYNC_POINT           3
#define ACC_KIND_EXCLUSIVE_SYNC_POINT 4
#define ACC_KIND_LOCAL_ONLY           5

/* ---- memory placement of caller arrays ---- */
#define ACC_MEM_HOST   0
#define ACC_MEM_DEVICE 1

/* ---- context options ---- */
#define ACC_OPT_TIMING 0x1u   /* record per-kernel HIP events (bench / profiling) */
#define ACC_OPT_FORCE_REPLAY 0x2u  /* always take the exact FAST-bisection replay path (testing) */
#define ACC_OPT_NO_WINDOW_TIER 0x4u  /* KeyDeps: the sorting build tiers instead of the window tier (testing) */
#define ACC_OPT_RD_WIDE_SORT 0x8u    /* RangeDeps: 64-bit sort keys in the lane-group build tiers (testing) */
#define ACC_OPT_PD_SERIAL 0x10u      /* acc_partial_deps_batch: both halves in order on this context (one buffer set:
                                        less device memory, no overlap) */

/* levelise walk (acc_opts.lv_tier); AUTO picks the whole-graph LDS walk up to 65,535 txns, the windowed walk beyond */
#define ACC_LV_AUTO     0u
#define ACC_LV_LDS_WALK 1u
#define ACC_LV_WINDOWED 2u
#define ACC_LV_WAVES    3u

typedef struct acc_ctx acc_ctx;

/* Context options, fixed at acc_create (the library reads no environment): flags plus the knobs the tests use to force
 * a code path; zero everywhere = the defaults. */
typedef struct acc_opts {
    uint32_t flags;           /* ACC_OPT_* */
    uint32_t reserved;
    uint32_t cfk_hot;         /* acc_cfk_apply: keys with more than this many sorted elements take the closed form
                                 of the replay (0: 64) */
    uint32_t lv_tier;         /* ACC_LV_* */
    uint32_t lv_chunk;        /* the LDS walk's dependency chunk cap in entries (0: as large as the LDS allows) */
    uint32_t reserved2;
} acc_opts;

/* Timestamp / TxnId as three SoA columns: Timestamp.msb, Timestamp.lsb, Node.Id.id
 * (primitives/Timestamp.java:77-79). Order = Timestamp.compareTo (:208-217), identity = equals (:244-249). */
typedef struct acc_ts_cols {
    const uint64_t *msb;
    const uint64_t *lsb;
    const int32_t  *node;
} acc_ts_cols;

/* One batch = one CommandsForKey snapshot of one CommandStore. Every txn of the batch is both an
 * entry of the CFK of each of its keys and a query T evaluated with startedBefore = T.executeAt and
 * testKind = T.kind().witnesses(); p1 = (executeAt.equals(txnId) ? null : txnId). */
typedef struct acc_batch_in {
    uint32_t    n_txn;        /* N */
    uint32_t    mem;          /* ACC_MEM_HOST or ACC_MEM_DEVICE for every pointer below */
    uint64_t    n_pairs;      /* P = key_off[N]; must be < 2^32 */
    acc_ts_cols txn_id;       /* [N] TxnIds, pairwise distinct under Timestamp.equals */
    acc_ts_cols execute_at;   /* [N] executeAt (== txnId for PREACCEPTED-style entries) */
    const uint8_t  *status;   /* [N] InternalStatus ordinal */
    const uint32_t *key_off;  /* [N+1] CSR offsets into key_code */
    const uint64_t *key_code; /* [P] order-preserving key codes, sorted unique within each txn (Keys) */
} acc_batch_in;

/* Result view of the last acc_keydeps_batch on a context. Pointers are DEVICE pointers owned by
 * the context and valid until the next compute call on it. For txn t:
 *   arena[arena_off[t] .. arena_off[t+1])  = Java KeyDeps.keysToTxnIds (int[]) of t's PartialDeps
 *   key_idx[kd_off[t] .. kd_off[t+1])      = KeyDeps.keys as indices into t's input keys
 *   dep_txn[u_off[t] .. u_off[t+1])        = KeyDeps.txnIds as batch indices, ascending TxnId order */
typedef struct acc_keydeps_view {
    uint32_t n_txn;
    uint64_t total_arena, total_keys, total_deps, total_edges; /* Σ(Kd+E), ΣKd, ΣU, ΣE */
    const uint64_t *arena_off;
    const int32_t  *arena;
    const uint64_t *kd_off;
    const uint32_t *key_idx;
    const uint64_t *u_off;
    const uint32_t *dep_txn;
    const uint64_t *kd_key;   /* [total_keys] KeyDeps.keys as key codes (acc_keydeps_mixed; null after acc_keydeps_batch) */
} acc_keydeps_view;

/* Caller-owned output buffers (two-call sizing: capacities in elements; a call with null offset
 * arrays, or with a capacity below the requirement, returns ACC_E_CAP after writing the required
 * totals to need_*, and touches nothing else). */
typedef struct acc_keydeps_out {
    uint32_t  mem;            /* ACC_MEM_HOST or ACC_MEM_DEVICE */
    uint64_t  cap_arena, cap_keys, cap_deps;
    uint64_t  need_arena, need_keys, need_deps;  /* written */
    uint64_t *arena_off;      /* [N+1] */
    int32_t  *arena;          /* [cap_arena] */
    uint64_t *kd_off;         /* [N+1] */
    uint32_t *key_idx;        /* [cap_keys] */
    uint64_t *u_off;          /* [N+1] */
    uint32_t *dep_txn;        /* [cap_deps] */
    uint64_t *kd_key;         /* optional [cap_keys]: key codes, copied when non-null and the result has them */
} acc_keydeps_out;

/* ---- context ---- */
int         acc_create(int device, const acc_opts *opts, acc_ctx **out_ctx);
void        acc_destroy(acc_ctx *ctx);
const char *acc_last_error(const acc_ctx *ctx);
int         acc_sync(acc_ctx *ctx);
/* HIP stream (hipStream_t) the context launches on, as an opaque handle. */
void       *acc_stream(acc_ctx *ctx);
const char *acc_version(void);

/* ---- KeyDeps batch: CommandsForKey conflict scan + KeyDeps.Builder for all txns of a batch ---- */
int acc_keydeps_batch(acc_ctx *ctx, const acc_batch_in *in, acc_keydeps_view *out_view);
int acc_keydeps_copy_out(acc_ctx *ctx, acc_keydeps_out *out);

/* ---- RangeDeps batch: range-command stabbing + RangeDeps.Builder for all txns of a mixed batch ----
 * Txns whose TxnId domain bit (lsb & 1, TxnId.java:124-157) is Range are range commands/queries with Ranges
 * rng_start/rng_end[rng_off[t] .. rng_off[t+1]) (sorted and deoverlapped, start < end); key-domain txns list keys
 * in key_off/key_code exactly as acc_batch_in and no ranges. A range txn whose status is INVALID_OR_TRUNCATED is
 * an erased range command (saveStatus >= Erased, InMemoryCommandStore.java:892-893) and contributes no deps. */
typedef struct acc_range_batch_in {
    uint32_t    n_txn;
    uint32_t    mem;           /* ACC_MEM_HOST or ACC_MEM_DEVICE for every pointer below */
    uint64_t    n_pairs;       /* P = key_off[N] */
    uint64_t    n_ranges;      /* R = rng_off[N]; P + R < 2^32 */
    acc_ts_cols txn_id;
    acc_ts_cols execute_at;
    const uint8_t  *status;
    const uint32_t *key_off;   /* [N+1] */
    const uint64_t *key_code;  /* [P] */
    const uint32_t *rng_off;   /* [N+1] */
    const uint64_t *rng_start; /* [R] order-preserving codes of Range.start() */
    const uint64_t *rng_end;   /* [R] order-preserving codes of Range.end() */
    uint32_t    end_inclusive; /* 1: Range.EndInclusive (s, e]; 0: Range.StartInclusive [s, e) (Range.java:40-138) */
    uint32_t    reserved;
} acc_range_batch_in;

/* Result of the last acc_rangedeps_batch (device pointers owned by the context). Ranges are ids into the
 * dictionary of distinct stored ranges (the ranges of non-erased range commands) sorted by Range::compare
 * (start, then end; Range.java:309-317). For txn t:
 *   arena[arena_off[t] .. arena_off[t+1])      = Java RangeDeps.rangesToTxnIds (int[])
 *   range_id[rd_off[t] .. rd_off[t+1])        = RangeDeps.ranges as dictionary ids (ascending)
 *   dep_txn[u_off[t] .. u_off[t+1])           = RangeDeps.txnIds as batch indices, ascending TxnId order */
typedef struct acc_rangedeps_view {
    uint32_t n_txn;
    uint32_t n_ranges;                  /* dictionary size */
    uint64_t total_arena, total_ranges, total_deps, total_edges;
    const uint64_t *rng_start, *rng_end;   /* [n_ranges] dictionary */
    const uint64_t *arena_off;  const int32_t  *arena;
    const uint64_t *rd_off;     const uint32_t *range_id;
    const uint64_t *u_off;      const uint32_t *dep_txn;
} acc_rangedeps_view;

typedef struct acc_rangedeps_out {
    uint32_t  mem;
    uint64_t  cap_arena, cap_ranges, cap_deps, cap_dict;
    uint64_t  need_arena, need_ranges, need_deps, need_dict;   /* written */
    uint64_t *rng_start, *rng_end;      /* [cap_dict] */
    uint64_t *arena_off;  int32_t  *arena;     /* [N+1], [cap_arena] */
    uint64_t *rd_off;     uint32_t *range_id;  /* [N+1], [cap_ranges] */
    uint64_t *u_off;      uint32_t *dep_txn;   /* [N+1], [cap_deps] */
} acc_rangedeps_out;

int acc_rangedeps_batch(acc_ctx *ctx, const acc_range_batch_in *in, acc_rangedeps_view *out_view);

/* KeyDeps of every txn of a mixed key/range batch (the same input as acc_rangedeps_batch). Key txns: exactly
 * acc_keydeps_batch. A range-domain txn is no CommandsForKey member (SafeCommandStore.updateCommandsForKey registers
 * key txns only, local/SafeCommandStore.java:217-240); as a query it runs CommandsForKey.mapReduceActive on every CFK
 * whose key lies in its ranges with the Range bound inclusivity (InMemoryCommandStore.mapReduceForKey,
 * impl/InMemoryCommandStore.java:274-289). Replaces the key part of PreAccept.calculatePartialDeps for range txns
 * (messages/PreAccept.java:245-265). The view is acc_keydeps_view with kd_key filled for every txn; for a range txn,
 * key_idx indexes the list of CFK keys its ranges cover (range order). Copy out with acc_keydeps_copy_out. */
int acc_keydeps_mixed(acc_ctx *ctx, const acc_range_batch_in *in, acc_keydeps_view *out_view);
int acc_rangedeps_copy_out(acc_ctx *ctx, acc_rangedeps_out *out);
/* The whole PartialDeps of every txn of a mixed batch in one call (PreAccept.calculatePartialDeps,
 * messages/PreAccept.java:245-265, routing each emitted (key | range, TxnId) through PartialDeps.Builder,
 * primitives/PartialDeps.java:31-45 / Deps.AbstractBuilder.add primitives/Deps.java:56-71): the KeyDeps half of
 * acc_keydeps_mixed and the RangeDeps half of acc_rangedeps_batch, sharing one dictionary pass (and its validation) and
 * the staged inputs. Both views stay valid until the next compute call; acc_keydeps_copy_out / acc_rangedeps_copy_out
 * copy them. The RangeDeps half runs concurrently on a child context created on first use (own stream and its own
 * grow-only device buffers, held until acc_destroy of ctx; environment ACC_PD_SERIAL=1 keeps both halves on ctx). */
int acc_partial_deps_batch(acc_ctx *ctx, const acc_range_batch_in *in, acc_keydeps_view *key_view,
                           acc_rangedeps_view *range_view);

/* ---- Deps.merge over many replies per txn ----
 * Input: R = n_groups groups (one coordinated txn each); group g owns replies
 * [grp_off[g], grp_off[g+1]); reply r is a KeyDeps in Java layout over integer ids:
 *   keys:   key_code[key_off[r] .. key_off[r+1])          (sorted unique)
 *   txnIds: txn_rank[val_off[r] .. val_off[r+1])          (sorted unique u32 order ranks of TxnIds)
 *   keysToTxnIds: k2v[k2v_off[r] .. k2v_off[r+1])         (Java int[] verbatim)
 * Output per group: the KeyDeps.merge result (== canonical union, KeyDepsTest.java:275-283) in the
 * same three-array layout, device-resident in the context. */
typedef struct acc_merge_in {
    uint32_t mem;
    uint32_t n_groups;
    uint64_t n_replies;
    const uint64_t *grp_off;   /* [n_groups+1] into replies */
    const uint64_t *key_off;   /* [n_replies+1] */
    const uint64_t *key_code;  /* [key_off[n_replies]] */
    const uint64_t *val_off;   /* [n_replies+1] */
    const uint32_t *txn_rank;  /* [val_off[n_replies]] */
    const uint64_t *k2v_off;   /* [n_replies+1] */
    const int32_t  *k2v;       /* [k2v_off[n_replies]] */
} acc_merge_in;

typedef struct acc_merge_view {
    uint32_t n_groups;
    uint64_t total_keys, total_vals, total_k2v, total_in_entries;
    const uint64_t *key_off;  const uint64_t *key_code;
    const uint64_t *val_off;  const uint32_t *txn_rank;
    const uint64_t *k2v_off;  const int32_t  *k2v;
} acc_merge_view;

int acc_keydeps_merge(acc_ctx *ctx, const acc_merge_in *in, acc_merge_view *out_view);

/* Caller-owned copy of the last merge result (two-call sizing as acc_keydeps_out). */
typedef struct acc_merge_out {
    uint32_t  mem;
    uint64_t  cap_keys, cap_vals, cap_k2v;
    uint64_t  need_keys, need_vals, need_k2v;   /* written */
    uint64_t *key_off;  uint64_t *key_code;     /* [n_groups+1], [cap_keys] */
    uint64_t *val_off;  uint32_t *txn_rank;     /* [n_groups+1], [cap_vals] */
    uint64_t *k2v_off;  int32_t  *k2v;          /* [n_groups+1], [cap_k2v] */
} acc_merge_out;

int acc_merge_copy_out(acc_ctx *ctx, acc_merge_out *out);

/* ---- Deps.merge over raw deps objects ----
 * Deps.merge(List, getter) (primitives/Deps.java:256-260) = KeyDeps.merge (primitives/KeyDeps.java:115-135) and
 * RangeDeps.merge (primitives/RangeDeps.java:101-134) of the replies of each coordinated txn (group g owns replies
 * [grp_off[g], grp_off[g+1])), folded left to right by a LinearMerger (utils/RelationMultiMap.java:284-406), empty
 * replies skipped. Each reply half is given as the arrays KeyDeps/RangeDeps.SerializerSupport expose
 * (primitives/KeyDeps.java:55-73, primitives/RangeDeps.java:55-73): keys (or ranges), the TxnId[] as raw columns and the
 * Java keysToTxnIds / rangesToTxnIds int[] verbatim. TxnIds are ranked on device (Timestamp.compareTo / equals); an
 * equals-tie whose raw bits differ (flags outside IDENTITY_LSB) keeps the instance the Java fold keeps
 * (SortedArrays.linearUnion utils/SortedArrays.java:152-281, RelationMultiMap.linearUnion :561-816). */
typedef struct acc_rmm_in {
    const uint64_t *key_off;   /* [n_replies+1]; null: the half is absent (every result is NONE) */
    const uint64_t *key_a;     /* KeyDeps: key codes; RangeDeps: Range.start codes */
    const uint64_t *key_b;     /* RangeDeps: Range.end codes (Range::compare = (start, end), Range.java:310-317); KeyDeps: null */
    const uint64_t *val_off;   /* [n_replies+1] */
    acc_ts_cols     txn;       /* TxnId[] of every reply, raw */
    const uint64_t *k2v_off;   /* [n_replies+1] */
    const int32_t  *k2v;       /* keysToTxnIds / rangesToTxnIds int[] of every reply */
} acc_rmm_in;

typedef struct acc_deps_merge_in {
    uint32_t mem;              /* ACC_MEM_HOST or ACC_MEM_DEVICE for every pointer */
    uint32_t n_groups;
    uint64_t n_replies;
    const uint64_t *grp_off;   /* [n_groups+1] */
    acc_rmm_in key_deps;
    acc_rmm_in range_deps;
} acc_deps_merge_in;

/* A merged half per group g (device pointers owned by the context, valid until its next compute call):
 * keys/ranges key_a[key_off[g]..key_off[g+1]) (+ key_b), TxnIds txn_*[val_off[g]..], ints k2v[k2v_off[g]..].
 * txn_src = an input slot (index into the half's TxnId columns) holding the kept instance's raw bits. */
typedef struct acc_rmm_view {
    uint64_t total_keys, total_vals, total_k2v;
    const uint64_t *key_off;  const uint64_t *key_a;  const uint64_t *key_b;
    const uint64_t *val_off;  const uint64_t *txn_msb; const uint64_t *txn_lsb; const int32_t *txn_node;
    const uint32_t *txn_src;
    const uint64_t *k2v_off;  const int32_t  *k2v;
} acc_rmm_view;

typedef struct acc_deps_merge_view {
    uint32_t n_groups;
    uint64_t total_in_entries;          /* keysToTxnIds + rangesToTxnIds entries over every reply */
    acc_rmm_view key_deps, range_deps;
} acc_deps_merge_view;

int acc_deps_merge(acc_ctx *ctx, const acc_deps_merge_in *in, acc_deps_merge_view *out_view);

/* Copy any acc_rmm_view of this context into caller buffers (two-call sizing: null offset arrays or a capacity below
 * the need -> ACC_E_CAP after writing need_*). key_b / txn_src are copied when both the view and the caller have them. */
typedef struct acc_rmm_out {
    uint32_t  mem;
    uint64_t  cap_keys, cap_vals, cap_k2v;
    uint64_t  need_keys, need_vals, need_k2v;   /* written */
    uint64_t *key_off;  uint64_t *key_a;  uint64_t *key_b;        /* [n_groups+1], [cap_keys] x2 */
    uint64_t *val_off;  uint64_t *txn_msb; uint64_t *txn_lsb; int32_t *txn_node; uint32_t *txn_src;   /* [cap_vals] */
    uint64_t *k2v_off;  int32_t  *k2v;                            /* [cap_k2v] */
} acc_rmm_out;

int acc_rmm_copy_out(acc_ctx *ctx, uint32_t n_groups, const acc_rmm_view *view, acc_rmm_out *out);

/* ---- RelationMultiMap helpers over a batch of built deps objects (one KeyDeps or RangeDeps per group) ----
 * The arrays of KeyDeps/RangeDeps.SerializerSupport (primitives/KeyDeps.java:55-73, primitives/RangeDeps.java:55-73);
 * the TxnIds themselves are not needed (val_off gives their count per group). key_b null = KeyDeps (key codes),
 * non-null = RangeDeps (Range start/end codes sorted by Range::compare). */
typedef struct acc_rmm_batch {
    uint32_t mem;              /* ACC_MEM_HOST or ACC_MEM_DEVICE for every pointer (and for acc_ranges_in) */
    uint32_t n_groups;
    const uint64_t *key_off;   /* [n_groups+1] */
    const uint64_t *key_a;     /* key codes | Range.start codes */
    const uint64_t *key_b;     /* null | Range.end codes */
    const uint64_t *val_off;   /* [n_groups+1] TxnIds per group */
    const uint64_t *k2v_off;   /* [n_groups+1] */
    const int32_t  *k2v;       /* keysToTxnIds / rangesToTxnIds int[] per group */
} acc_rmm_batch;

/* Per-group int[] result (device pointers owned by the context): ints[off[g] .. off[g+1]). */
typedef struct acc_csr_view {
    uint32_t n_groups;
    uint64_t total;
    const uint64_t *off;
    const int32_t  *ints;
} acc_csr_view;

/* RelationMultiMap.invert (utils/RelationMultiMap.java:907-938) of every group: KeyDeps.txnIdsToKeys
 * (primitives/KeyDeps.java:350-362) / RangeDeps txnIdsToRanges: per group the Java int[] of nv end offsets (from nv)
 * followed by the key indices of each TxnId in ascending key order. */
int acc_rmm_invert(acc_ctx *ctx, const acc_rmm_batch *in, acc_csr_view *out_view);

/* Ranges per group (sorted, deoverlapped; Ranges.ofSortedAndDeoverlapped): [off[g], off[g+1]) of start/end. */
typedef struct acc_ranges_in {
    const uint64_t *off;       /* [n_groups+1] */
    const uint64_t *start;
    const uint64_t *end;
    uint32_t end_inclusive;    /* Range.EndInclusive (s, e] = 1; StartInclusive [s, e) = 0 (Range.java:40-138) */
    uint32_t reserved;
} acc_ranges_in;

/* Slice result per group: the selected key indices (into the group's keys, ascending), the kept TxnId indices (into
 * the group's txnIds, ascending) and the new keysToTxnIds int[] over the kept TxnIds. */
typedef struct acc_slice_view {
    uint32_t n_groups;
    uint64_t total_keys, total_vals, total_k2v;
    const uint64_t *key_off;  const uint32_t *key_idx;
    const uint64_t *val_off;  const uint32_t *val_idx;
    const uint64_t *k2v_off;  const int32_t  *k2v;
} acc_slice_view;

/* KeyDeps.slice(Ranges) (primitives/KeyDeps.java:189-236: keys contained in the ranges) / RangeDeps.slice(Ranges)
 * (primitives/RangeDeps.java:545-565: ranges intersecting them) with trimUnusedValues
 * (utils/RelationMultiMap.java:491-532), each group against its own select Ranges; the reference's short cuts are kept
 * (empty input, nothing selected, everything selected = `return this` without trimming). */
int acc_rmm_slice(acc_ctx *ctx, const acc_rmm_batch *in, const acc_ranges_in *select, acc_slice_view *out_view);

/* RelationMultiMap.remove (utils/RelationMultiMap.java:843-905) = KeyDeps.without (primitives/KeyDeps.java:255-259) /
 * RangeDeps.without (primitives/RangeDeps.java:584-588) of every group, with the predicate of the recovery callers
 * (`without(earlierCommittedWitness::contains)`, messages/BeginRecovery.java:180-183, coordinate/Recover.java:322):
 * remove(t) = Deps.contains(t) = KeyDeps.contains || RangeDeps.contains (primitives/Deps.java:107-110), each an
 * Arrays.binarySearch over that deps object's sorted TxnIds (Timestamp.compareTo == 0). The group's TxnId set(s) to
 * test against: set_a and set_b (either may be absent: off null), each sorted ascending by Timestamp.compareTo
 * without duplicates per group (ACC_E_ARG otherwise). The input half's TxnIds are `txn` ([val_off[n_groups]] raw).
 * Result per group, exactly as the Java returns:
 *   ACC_WITHOUT_FROM — `return from` (isEmpty(): no entries; or nothing removed): the input object itself;
 *   ACC_WITHOUT_NONE — `return none` (every TxnId removed): KeyDeps.NONE / RangeDeps.NONE, no keys;
 *   ACC_WITHOUT_NEW  — rebuilt: every key kept (keys whose lists emptied stay, :877-891), the kept TxnIds in order,
 *                      the new keysToTxnIds int[].
 * The view is an acc_slice_view over the input (key_idx: kept key indices, val_idx: kept TxnId indices, k2v: the
 * group's int[]; FROM groups list everything with the input int[] verbatim) plus the kind per group. */
#define ACC_WITHOUT_FROM 0
#define ACC_WITHOUT_NONE 1
#define ACC_WITHOUT_NEW  2

typedef struct acc_txn_sets {
    const uint64_t *off;       /* [n_groups+1]; null: every set is empty */
    acc_ts_cols     txn;       /* sorted unique TxnIds of every group's set */
} acc_txn_sets;

typedef struct acc_without_view {
    acc_slice_view sl;
    const uint8_t *kind;       /* [n_groups] ACC_WITHOUT_* */
    uint64_t n_from, n_none, n_new;
} acc_without_view;

int acc_rmm_without(acc_ctx *ctx, const acc_rmm_batch *in, const acc_ts_cols *txn, const acc_txn_sets *set_a,
                    const acc_txn_sets *set_b, acc_without_view *out_view);

/* The recovery reply reduce of the deps the recovery coordinator folds (coordinate/Recover.java:320-322; pairwise as
 * BeginRecovery.RecoverOk.reduce, messages/BeginRecovery.java:180-183): per recovered txn (group),
 *   earlierCommittedWitness  = Deps.merge(replies' earlierCommittedWitness)           -> committed_view,
 *   earlierAcceptedNoWitness = Deps.merge(replies' earlierAcceptedNoWitness)
 *                                .without(earlierCommittedWitness::contains)            -> accepted_merged + accepted_*.
 * Both merges as acc_deps_merge (same input layout; the replies in the order the Java folds them); the without runs on
 * the merged accepted halves with each group's merged committed key and range TxnIds as the two sets. accepted_key /
 * accepted_range index into accepted_merged's halves (val_idx into its TxnIds, key_idx into its keys / ranges).
 * Views are device pointers owned by the context, valid until its next compute call. */
typedef struct acc_recovery_deps_view {
    acc_deps_merge_view committed;        /* earlierCommittedWitness per group */
    acc_deps_merge_view accepted_merged;  /* Deps.merge of earlierAcceptedNoWitness per group (before the without) */
    acc_without_view accepted_key;        /* KeyDeps.without over accepted_merged.key_deps */
    acc_without_view accepted_range;      /* RangeDeps.without over accepted_merged.range_deps */
} acc_recovery_deps_view;

int acc_recovery_deps_reduce(acc_ctx *ctx, const acc_deps_merge_in *committed_witness,
                             const acc_deps_merge_in *accepted_no_witness, acc_recovery_deps_view *out_view);

/* Stabbing queries over built RangeDeps (SearchableRangeList.forEach, utils/SearchableRangeList.java:89-116;
 * RangeDeps.forEach / computeTxnIds, primitives/RangeDeps.java:152-412, 629-643): query q against group grp[q]:
 * a key (q_end null: Range.contains with the bound type) or a range [q_start, q_end) (compareIntersecting == 0). */
typedef struct acc_stab_in {
    uint32_t mem;
    uint32_t n_queries;
    const uint32_t *grp;       /* [n_queries] */
    const uint64_t *q_start;   /* [n_queries] key codes | range starts */
    const uint64_t *q_end;     /* [n_queries] range ends, or null for key queries */
    uint32_t end_inclusive;
    uint32_t want_txns;        /* also produce computeTxnIds (sorted unique TxnId indices) */
} acc_stab_in;

typedef struct acc_stab_view {
    uint32_t n_queries;
    uint64_t total_ranges, total_txns;
    const uint64_t *range_off; const uint32_t *range_idx;   /* ascending range indices per query */
    const uint64_t *txn_off;   const uint32_t *txn_idx;     /* want_txns: ascending TxnId indices per query */
} acc_stab_view;

int acc_rangedeps_stab(acc_ctx *ctx, const acc_rmm_batch *range_deps, const acc_stab_in *queries, acc_stab_view *out_view);

/* Copy `bytes` from a device pointer of a result view into caller memory (mem = ACC_MEM_HOST / ACC_MEM_DEVICE), on the
 * context stream, synchronously: lets a host without HIP bindings read any view. */
int acc_copy_out(acc_ctx *ctx, void *dst, const void *src_device, size_t bytes, uint32_t mem);

/* ---- Key-range CommandStore shards across GPUs (PreAccept.reduce) ----
 * acc_shard_pack: the last acc_keydeps_batch result of this shard (the same `in`) as fragments for the txns' home
 * ranks (home(t) = t mod world, t the global index). A fragment = header (t, nk, nv, no) + nk key codes + nv TxnIds (batch indices) +
 * no Java keysToTxnIds ints; only txns with a non-empty shard KeyDeps send one (PartialDeps.with skips empties).
 * Streams are destination-major: destination d owns elements [x_off[d], x_off[d+1]) of each stream. The caller
 * supplies the four stream buffers (two-call sizing: with a capacity below the need, ACC_E_CAP after writing the
 * four host offset arrays, whose last entries are the totals) and four HOST offset arrays of world+1 entries. */
typedef struct acc_frag_streams {
    uint32_t  world;
    uint32_t  mem;                                   /* placement of hdr/keys/vals/k2v */
    uint64_t  cap_frag, cap_keys, cap_vals, cap_k2v; /* capacities: fragments (hdr = 4 u32 each), elements */
    uint32_t *hdr;
    uint64_t *keys;
    uint32_t *vals;
    int32_t  *k2v;
    uint64_t *frag_off, *key_off, *val_off, *k2v_off;   /* host [world+1], written */
    const uint32_t *txn_global; /* optional [N], placement of the batch: global index of each batch txn (a store's
                                   batch holds only the txns touching its keys, in TxnId order); null = identity */
} acc_frag_streams;

int acc_shard_pack(acc_ctx *ctx, const acc_batch_in *in, acc_frag_streams *out);

/* acc_shard_merge: what this rank received, the four streams concatenated in source-rank (= shard) order, with the
 * per-source element counts (host arrays of `world` entries). Result: the merged KeyDeps of every home txn
 * t = rank + g * world (group g), in the acc_merge_view layout (txn ranks = batch indices). */
typedef struct acc_frag_recv {
    uint32_t mem;              /* placement of hdr/keys/vals/k2v */
    uint32_t world, rank, n_txn;
    const uint64_t *n_frag, *n_keys, *n_vals, *n_k2v;   /* host [world] */
    const uint32_t *hdr;
    const uint64_t *keys;
    const uint32_t *vals;
    const int32_t  *k2v;
} acc_frag_recv;

int acc_shard_merge(acc_ctx *ctx, const acc_frag_recv *in, acc_merge_view *out_view);

/* ---- The exchange between CommandStores on different GPUs, behind the ABI ----
 * acc_comm: a communicator of `world` ranks (one GPU and one acc_ctx each). Two transports:
 *   RCCL (acc_comm_init_rccl): rank 0 makes an id with acc_comm_unique_id and the host distributes the 128 bytes
 *     (any channel); device buffers move point to point over xGMI;
 *   host (acc_comm_init_host): the caller's all-to-all(v) of host bytes (e.g. a JVM node's own messaging): fn gets
 *     send[] with send_bytes[d] bytes for rank d (concatenated in rank order) and fills recv[] with recv_bytes[s]
 *     bytes from each rank s; returns 0 on success.
 * acc_shard_reduce: PreAccept.reduce of the store KeyDeps (messages/PreAccept.java:141-156, PartialDeps.with) for the
 * last acc_keydeps_batch on ctx over `in` (the same batch): acc_shard_pack, one exchange of the element counts, one
 * all-to-all(v) of the four fragment streams, acc_shard_merge; every rank calls it (collective). txn_global / n_global
 * as acc_frag_streams.txn_global and the global txn count; the result is acc_shard_merge's view. */
#define ACC_COMM_ID_BYTES 128
typedef struct acc_comm acc_comm;
typedef int (*acc_alltoallv_fn)(void *user, const void *send, const uint64_t *send_bytes, void *recv,
                                const uint64_t *recv_bytes);
int  acc_comm_unique_id(uint8_t *id_out);   /* [ACC_COMM_ID_BYTES]; ACC_E_DEVICE without RCCL */
int  acc_comm_init_rccl(acc_ctx *ctx, uint32_t world, uint32_t rank, const uint8_t *id, acc_comm **out);
int  acc_comm_init_host(acc_ctx *ctx, uint32_t world, uint32_t rank, acc_alltoallv_fn fn, void *user, acc_comm **out);
void acc_comm_destroy(acc_comm *comm);
int  acc_shard_reduce(acc_ctx *ctx, acc_comm *comm, const acc_batch_in *in, const uint32_t *txn_global, uint32_t n_global,
                      acc_merge_view *out_view);
/* PartialDeps.covering (primitives/PartialDeps.java:31-58, 80-86). A store's txns all carry the store's Ranges as
 * covering (PreAccept.calculatePartialDeps: new PartialDeps.Builder(ranges), messages/PreAccept.java:245-265); the
 * reduced PartialDeps of a home txn carries the fold that.covering.with(this.covering) over the stores that replied
 * for it (every store whose batch holds the txn), in store order. Per home txn: cov_id into a table of the distinct
 * coverings (device memory owned by the context, valid until the next reduce) and the mask of the stores that replied.
 * Both calls check the PartialDeps constructor's invariants covering.containsAll(keyDeps.keys) and
 * rangeDeps.isCoveredBy(covering) for every txn (PartialDeps.java:52-58) -> ACC_E_STATE. */
typedef struct acc_covering_view {
    uint32_t n_groups;             /* home txns, as the reduce's key view */
    uint32_t n_coverings;          /* distinct coverings in the table */
    const uint32_t *cov_id;        /* [n_groups] */
    const uint64_t *cov_off;       /* [n_coverings+1] into cov_start / cov_end */
    const uint64_t *cov_start;
    const uint64_t *cov_end;
    const uint64_t *store_mask;    /* [n_groups] bit s: store (rank) s replied for the txn */
    uint64_t total_ranges;
} acc_covering_view;

/* The store's `covering` (sorted, deoverlapped; the batch's bound type) for the last acc_partial_deps_batch on ctx over
 * `in` (the same batch): the invariant checks of every txn's PartialDeps(covering, keyDeps, rangeDeps). */
int  acc_partial_deps_covering(acc_ctx *ctx, const acc_range_batch_in *in, const acc_rlist *covering);

/* acc_partial_deps_reduce: PreAccept.reduce of a store's whole PartialDeps (messages/PreAccept.java:141-156;
 * PartialDeps.with = KeyDeps.with + RangeDeps.with, primitives/PartialDeps.java:80-86) for the last
 * acc_partial_deps_batch on ctx over `in` (the same mixed batch): the KeyDeps fragments (as acc_shard_reduce) and the
 * RangeDeps fragments (ranges as (start, end) codes, TxnIds raw, rangesToTxnIds) of both halves in ONE size exchange
 * and ONE grouped all-to-all(v); on the home rank the KeyDeps.with fold (key_view, as acc_shard_reduce) and the
 * RangeDeps.with fold in store order (RangeDeps.java:567-582; the range half of range_view, raw TxnIds; its key half is
 * absent). A range command is stored sliced to each store's ranges (impl/InMemoryCommandStore.java:739-761), so the
 * result depends on the store split exactly as the reference's does. With `covering` (this store's Ranges; null: no
 * covering), the same exchange carries the store's txns and covering, and covering_view receives every home txn's
 * PartialDeps.covering (above). Collective over comm. */
int  acc_partial_deps_reduce(acc_ctx *ctx, acc_comm *comm, const acc_range_batch_in *in, const uint32_t *txn_global,
                             uint32_t n_global, const acc_rlist *covering, acc_merge_view *key_view,
                             acc_deps_merge_view *range_view, acc_covering_view *covering_view);

/* ---- Recovery scans: CommandsForKey.mapReduceFull over a batch of queries (SURVEY.md §8(f) N3 = A7) ----
 * The snapshot is an acc_batch_in (one CommandsForKey per key, as for acc_keydeps_batch) plus, per input pair j
 * (txn t, key k), the entry's TxnInfoWithMissing.missing (local/CommandsForKey.java:385-410): the TxnIds of that CFK
 * the txn's deps do not include, as batch indices sorted by TxnId, missing_txn[missing_off[j] .. missing_off[j+1]).
 * Every query q is one (testTxnId, keys) call of SafeCommandStore.mapReduceFull with the call-wide tests:
 *   started_at  TestStartedAt ordinal: 0 STARTED_BEFORE (txnId < testTxnId), 1 STARTED_AFTER (from the binarySearch
 *               insert position, testTxnId itself included when it is on the key), 2 ANY
 *   test_dep    TestDep ordinal: 0 WITH, 1 WITHOUT (testTxnId absent / present in missing), 2 ANY_DEPS; WITH and
 *               WITHOUT also need InternalStatus.hasInfo and executeAt > testTxnId; WITH skips keys where testTxnId
 *               is no CFK member
 *   test_status TestStatus ordinal: 0 ANY_STATUS (not TRANSITIVELY_KNOWN), 1 IS_PROPOSED (ACCEPTED, COMMITTED),
 *               2 IS_STABLE (STABLE, APPLIED)
 *   test_kinds  Kinds as a mask over Kind ordinals, or -1 for testTxnId.kind().witnessedBy() (Txn.java:247-262)
 *   flags       ACC_FULL_EXECUTES_AFTER: the map keeps only executeAt > testTxnId (BeginRecovery.java:339-341)
 * The result per query is the Deps.Builder KeyDeps of every (key, txnId) the map visited, in the acc_keydeps_view
 * layout (key_idx into the query's keys, dep_txn = batch indices); the boolean recovery predicates
 * (hasAcceptedOrCommittedStartedAfterWithoutWitnessing, hasStableExecutesAfterWithoutWitnessing) are
 * u_off[q+1] > u_off[q]. acc_keydeps_copy_out copies it. The range commands' half of the same call is
 * acc_map_reduce_full_ranges below. */
#define ACC_STARTED_BEFORE 0
#define ACC_STARTED_AFTER  1
#define ACC_STARTED_ANY    2
#define ACC_DEP_WITH       0
#define ACC_DEP_WITHOUT    1
#define ACC_DEP_ANY        2
#define ACC_STATUS_ANY         0
#define ACC_STATUS_IS_PROPOSED 1
#define ACC_STATUS_IS_STABLE   2
#define ACC_FULL_EXECUTES_AFTER 1u

typedef struct acc_recovery_in {
    uint32_t    n_query;
    uint32_t    mem;            /* placement of the query arrays and of missing_off / missing_txn */
    acc_ts_cols test_txn;       /* [n_query] testTxnId of each query (any TxnId, batch member or not) */
    const uint32_t *key_off;    /* [n_query+1] */
    const uint64_t *key_code;   /* keys of each query, sorted unique (Keys) */
    const uint32_t *missing_off;/* [n_pairs+1] of the snapshot */
    const uint32_t *missing_txn;/* [n_missing] batch indices */
    uint64_t    n_missing;
    uint8_t     started_at, test_dep, test_status, flags;
    int32_t     test_kinds;
} acc_recovery_in;

int acc_map_reduce_full(acc_ctx *ctx, const acc_batch_in *snapshot, const acc_recovery_in *q, acc_keydeps_view *out_view);

/* ---- Recovery scans, range-command half: InMemorySafeStore.mapReduceRangesInternal
 * (impl/InMemoryCommandStore.java:883-1016), the second half of SafeCommandStore.mapReduceFull (:874-881) ----
 * The store's range commands are a table of n_cmd entries sorted by TxnId (non-decreasing): the rangeCommands map (a
 * TreeMap by TxnId) and, flagged ACC_RCMD_HISTORICAL, the historicalRangeCommands map (a TxnId may be in both). Entry c:
 *   txn_id, execute_at  Command.executeAt() (executeAtOrTxnId where it is null; a historical entry: its TxnId)
 *   status              Status ordinal (local/Status.java:47-86: NotDefined 0 .. Accepted 3, PreCommitted 4,
 *                       Committed 5, Stable 6, PreApplied 7, Applied 8, Truncated 9, Invalidated 10)
 *   flags               ACC_RCMD_ERASED: saveStatus >= Erased, never visited (:891-893); ACC_RCMD_HAS_DEPS:
 *                       known().deps.hasProposedOrDecidedDeps() (Status.java:601-612); ACC_RCMD_HISTORICAL (:962-1004):
 *                       visited only when test_status = ANY_STATUS and test_dep = ANY_DEPS, with executeAt = TxnId
 *   ranges              [rng_off[c], rng_off[c+1]): sorted, non-overlapping, start < end, bound type end_inclusive
 *   deps                its PartialDeps flattened to (TxnId, participant) pairs sorted by TxnId: dep_txn[dep_off[c] ..
 *                       dep_off[c+1]), a KeyDeps entry with dep_is_key = 1 and its key in dep_start, a RangeDeps entry
 *                       with its range [dep_start, dep_end). The WITH / WITHOUT test is Deps.intersects(testTxnId,
 *                       the entry's ranges) (primitives/Deps.java:112-115, KeyDeps.java:266-285, RangeDeps.java:468-495)
 * Query q = one (testTxnId, keysOrRanges.slice(slice)) call: participants [part_off[q], part_off[q+1]), keys
 * (part_is_range[q] = 0: part_start sorted unique) or ranges (1: part_start / part_end sorted, non-overlapping). The
 * call-wide tests are those of acc_recovery_in (started_at, test_dep, test_status, test_kinds, flags).
 * Result per query: the RangeDeps of every (range of the command, TxnId) the map visited, built by Deps.Builder, as an
 * acc_rangedeps_view with query q in place of txn q: the range dictionary is the distinct ranges of the table, dep_txn
 * the first table index holding that TxnId. The boolean recovery predicates are u_off[q+1] > u_off[q]. Copy out with
 * acc_rangedeps_copy_out; the view is valid until the next compute call. */
#define ACC_RCMD_ERASED     1u
#define ACC_RCMD_HAS_DEPS   2u
#define ACC_RCMD_HISTORICAL 4u

typedef struct acc_range_cmds_in {
    uint32_t    n_cmd;
    uint32_t    mem;             /* placement of every array below */
    uint32_t    end_inclusive;   /* 1: Range.EndInclusive (s, e]; 0: Range.StartInclusive [s, e) */
    acc_ts_cols txn_id, execute_at;
    const uint8_t  *status, *flags;
    const uint32_t *rng_off;     /* [n_cmd+1] */
    const uint64_t *rng_start, *rng_end;
    const uint32_t *dep_off;     /* [n_cmd+1] */
    acc_ts_cols     dep_txn;
    const uint64_t *dep_start, *dep_end;
    const uint8_t  *dep_is_key;
} acc_range_cmds_in;

typedef struct acc_recovery_ranges_in {
    uint32_t    n_query;
    uint32_t    mem;
    acc_ts_cols test_txn;        /* [n_query] */
    const uint8_t  *part_is_range;   /* [n_query] */
    const uint32_t *part_off;        /* [n_query+1] */
    const uint64_t *part_start, *part_end;
    uint8_t     started_at, test_dep, test_status, flags;
    int32_t     test_kinds;
} acc_recovery_ranges_in;

int acc_map_reduce_full_ranges(acc_ctx *ctx, const acc_range_cmds_in *cmds, const acc_recovery_ranges_in *q,
                               acc_rangedeps_view *out_view);

/* ---- Recovery merge of LatestDeps replies ----
 * Group g = one recovering txn with replies [grp_off[g], grp_off[g+1]), each a LatestDeps (primitives/LatestDeps.java):
 * reply r owns intervals [iv_off[r], iv_off[r+1]) = RoutingKey ranges [iv_start, iv_end) ascending and disjoint (gaps =
 * null entries), each with a KnownDeps ordinal (local/Status.java:539-578: DepsUnknown 0, DepsProposed 1,
 * DepsCommitted 2, DepsErased 3, DepsKnown 4, NoDeps 5), a Ballot and its coordinatedDeps / localDeps as ids of deps
 * objects (-1 = null). Ids stand for Java object identity: MergeBuilder.tryMergeEqual compares deps by reference
 * (LatestDeps.java:420-435), so equal ids must mean the same object. Deps object d = key_deps / range_deps reply slot d
 * in the acc_rmm_in layout of Deps.merge (n_deps slots). The interval descriptors are host arrays; the deps arrays are in
 * deps_mem. mode ACC_LATEST_PROPOSAL = mergeProposal (:350-358), ACC_LATEST_COMMIT = mergeCommit(txn_id[g],
 * execute_at[g]) (:360-369), which also yields sufficientFor. Ranges are end_inclusive (s, e] or [s, e). */
#define ACC_LATEST_PROPOSAL 0u
#define ACC_LATEST_COMMIT   1u
typedef struct acc_latest_in {
    uint32_t n_groups;
    uint32_t mode;
    const uint32_t *grp_off;          /* [n_groups+1] */
    const uint32_t *iv_off;           /* [n_replies+1] */
    const uint64_t *iv_start, *iv_end;
    const uint8_t  *known;
    acc_ts_cols     ballot;
    const int32_t  *coord_deps;       /* coordinatedDeps id per interval, -1 = null */
    const int32_t  *local_deps;       /* localDeps id per interval, -1 = null */
    acc_ts_cols     txn_id, execute_at;   /* [n_groups], ACC_LATEST_COMMIT only */
    uint32_t        end_inclusive;
    uint32_t        deps_mem;
    uint32_t        n_deps;
    acc_rmm_in      key_deps, range_deps;
} acc_latest_in;

/* deps: per group the merged Deps (device views as acc_deps_merge, copied with acc_rmm_copy_out); sufficientFor per group
 * (mergeCommit): ranges sufficient_start/end[sufficient_off[g] .. sufficient_off[g+1]), HOST pointers owned by the
 * context, valid until its next call. */
typedef struct acc_latest_view {
    acc_deps_merge_view deps;
    uint64_t        total_sufficient;
    const uint64_t *sufficient_off;
    const uint64_t *sufficient_start, *sufficient_end;
} acc_latest_view;

int acc_latest_deps_merge(acc_ctx *ctx, const acc_latest_in *in, acc_latest_view *out_view);

/* ---- Deps wire format: Maelstrom JSON <-> device ----
 * acc_deps_from_json: a batch of JSON documents, each one Deps as Json.DEPS_ADAPTER writes it
 * (accord-maelstrom/.../Json.java:316-398: {"keyDeps":[[datum,[msb,lsb,node]],...],"rangeDeps":[[start,end,[msb,lsb,node]],...]})
 * concatenated in bytes[doc_off[d] .. doc_off[d+1]), parsed on device and built per document (KeyDeps / RangeDeps
 * Builder, Json.java:356-392) into the per-document Deps of `deps` (acc_rmm_view halves; copy with acc_rmm_copy_out).
 * Keys are datums (mael/Datum.java); their codes in `deps` are dense ranks of every datum of the batch in
 * Datum.compareTo order (hash first, COMPARE_BY_HASH), with the dictionary rank -> (Datum.Kind ordinal, null, value,
 * hash). Every Datum.Kind: LONG and DOUBLE as Gson reads a number (nextLong, else nextDouble; the decimal conversion
 * is Double.parseDouble's exactly rounded fast path, other literals give ACC_E_ARG), HASH, and STRING (ASCII text, JSON
 * escapes resolved; two different texts with one hash and equal first 16 characters give ACC_E_ARG). DOUBLE egress is
 * Double.toString (shortest round-trip digits, JDK >= 19), STRING egress Gson's HTML-safe escaping.
 * acc_deps_to_json: the inverse for any acc_rmm_view pair of this context whose key codes index such a dictionary
 * (e.g. a Deps.merge of ingested replies): Gson's compact DEPS_ADAPTER text per group, two-call sizing on need_bytes. */
typedef struct acc_json_in {
    uint32_t mem;
    uint32_t n_docs;
    const uint8_t  *bytes;
    const uint64_t *doc_off;   /* [n_docs+1] */
} acc_json_in;

typedef struct acc_json_deps_view {
    uint32_t n_docs;
    acc_deps_merge_view deps;
    uint64_t n_dict;
    const uint8_t  *dict_kind;   /* Datum.Kind ordinal: STRING 0, LONG 1, DOUBLE 2, HASH 3 */
    const uint8_t  *dict_null;   /* value == null (the +Inf sentinel) */
    const uint64_t *dict_value;  /* LONG: the long; HASH: the hash as u32; DOUBLE: Double.doubleToLongBits;
                                    STRING: byte offset of its text in dict_str */
    const int32_t  *dict_hash;   /* Datum.hash(value) */
    const uint32_t *dict_len;    /* STRING: text length in bytes (ASCII); else 0 */
    const uint8_t  *dict_str;    /* the STRING texts */
} acc_json_deps_view;

int acc_deps_from_json(acc_ctx *ctx, const acc_json_in *in, acc_json_deps_view *out_view);

typedef struct acc_json_out_in {
    uint32_t n_groups;
    acc_rmm_view key_deps, range_deps;      /* device views (key_off null = absent half) */
    uint64_t n_dict;
    const uint8_t  *dict_kind, *dict_null;  /* device */
    const uint64_t *dict_value;
    const uint32_t *dict_len;               /* device; STRING datums need both (as acc_json_deps_view) */
    const uint8_t  *dict_str;
} acc_json_out_in;

typedef struct acc_json_out {
    uint32_t  mem;
    uint64_t  cap_bytes;
    uint64_t  need_bytes;      /* written */
    uint8_t  *bytes;           /* [cap_bytes] */
    uint64_t *doc_off;         /* [n_groups+1] */
} acc_json_out;

int acc_deps_to_json(acc_ctx *ctx, const acc_json_out_in *in, acc_json_out *out);

/* ---- A device-resident CommandsForKey store, updated incrementally ----
 * acc_cfk_update applies CommandsForKey.update(prev, next) (local/CommandsForKey.java:652-706) for every key of every
 * command of `delta`, as SafeCommandStore.updateCommandsForKey does (local/SafeCommandStore.java:217-240; key-domain,
 * globally visible kinds only, others are ignored): an absent TxnId is inserted (executeAt = txnId unless the status
 * carries info), a present one is updated in place and registered on any new keys; a status lower than the stored one
 * is the reference's stale-status IllegalStateException (ACC_E_STATE), an equal status without info changes nothing.
 * The store stays in HBM between calls; acc_cfk_view describes it as an acc_batch_in of DEVICE pointers (txns in TxnId
 * order, keys ascending per txn) that acc_keydeps_batch / acc_map_reduce_full / acc_shard_pack take as they are. The
 * view is valid until the next acc_cfk_update on that store. One store is used by one context at a time. */
typedef struct acc_cfk acc_cfk;
int  acc_cfk_create(acc_ctx *ctx, acc_cfk **out);
void acc_cfk_destroy(acc_cfk *cfk);
int  acc_cfk_update(acc_ctx *ctx, acc_cfk *cfk, const acc_batch_in *delta);
int  acc_cfk_view(acc_ctx *ctx, acc_cfk *cfk, acc_batch_in *out);

/* ---- CommandsForKey.update with each command's deps (local/CommandsForKey.java:657-1149) ----
 * The missing[] and TRANSITIVELY_KNOWN half of CommandsForKey maintenance, on a key-major snapshot: key k (sorted unique
 * codes) holds its TxnInfos [ent_off[k], ent_off[k+1]) in TxnId order (TxnId, executeAt, InternalStatus) and each
 * TxnInfo its TxnInfoWithMissing.missing [miss_off[e], miss_off[e+1]) (sorted raw TxnIds). A batch of command updates
 * is applied in array order to every key each lists, as SafeCommandStore.updateCommandsForKey calls
 * CommandsForKey.update(prev, next) (local/SafeCommandStore.java:217-240): status = the new InternalStatus (0xFF: the
 * save status maps to none, no change), flags bit 0 = acceptedOrCommitted changed since the previous update (the
 * reference returns the CFK unchanged for an equal status otherwise), flags bit 1 = next.status() == AcceptedInvalidate
 * (Commands.acceptInvalidate may move an Accepted command to AcceptedInvalidateWithDefinition = PREACCEPTED: no stale
 * status check, the CFK stays unchanged, CommandsForKey.java:681-688), execute_at = Command.executeAt(), and per
 * (update, key) pair the command's partialDeps().keyDeps.txnIds(key) [dep_off[j], dep_off[j+1]) sorted. Deps the CFK
 * lacks become TRANSITIVELY_KNOWN entries; TxnIds it holds (uncommitted, witnessed) that a dep list lacks go to that
 * TxnInfo's missing[]; committing removes a TxnId from every missing[]. A status going back is ACC_E_STATE (the
 * reference's IllegalStateException) unless flags bit 1 is set. RedundantBefore is empty. The result (keys without entries dropped) is
 * device-resident until the next compute call, and its missing[] is what acc_map_reduce_full's WITH / WITHOUT tests
 * read. */
typedef struct acc_cfk_snap {
    uint32_t mem, n_keys;
    uint64_t n_entries, n_missing;
    const uint64_t *key;         /* [n_keys] */
    const uint32_t *ent_off;     /* [n_keys+1] */
    acc_ts_cols txn_id, execute_at;
    const uint8_t *status;       /* [n_entries] InternalStatus ordinals */
    const uint32_t *miss_off;    /* [n_entries+1] */
    acc_ts_cols missing;         /* [n_missing] */
} acc_cfk_snap;

typedef struct acc_cfk_updates {
    uint32_t mem, n_upd;
    uint64_t n_pairs, n_deps;
    acc_ts_cols txn_id, execute_at;
    const uint8_t *status, *flags;
    const uint32_t *key_off;     /* [n_upd+1] */
    const uint64_t *key;         /* [n_pairs] sorted unique per update */
    const uint32_t *dep_off;     /* [n_pairs+1] */
    acc_ts_cols deps;            /* [n_deps] */
} acc_cfk_updates;

typedef struct acc_cfk_snap_view {
    uint32_t n_keys;
    uint64_t n_entries, n_missing;
    const uint64_t *key;
    const uint32_t *ent_off;
    acc_ts_cols txn_id, execute_at;
    const uint8_t *status;
    const uint32_t *miss_off;
    acc_ts_cols missing;
} acc_cfk_snap_view;

int  acc_cfk_apply(acc_ctx *ctx, const acc_cfk_snap *snap, const acc_cfk_updates *updates, acc_cfk_snap_view *out_view);

/* The key-major CommandsForKey state as the txn-major snapshot acc_map_reduce_full scans, without leaving HBM (the
 * recovery scan of SafeCommandStore.mapReduceFull reads the store's CFKs, local/CommandsForKey.java:553-612): each
 * distinct TxnId of snap is one batch txn (TxnId order) whose keys are the keys holding it, with the executeAt and
 * InternalStatus its TxnInfos carry — equal on every key, as a store's CFKs all see the command's one status, else
 * ACC_E_STATE — and each (txn, key) pair's TxnInfoWithMissing.missing becomes batch indices (a missing TxnId that is no
 * entry of the store: ACC_E_STATE). snap may be an acc_cfk_apply result (mem = ACC_MEM_DEVICE). The output is DEVICE
 * memory owned by the context, valid until the next acc_cfk_snap_to_batch; acc_map_reduce_full reads it in place
 * (its acc_recovery_in with mem = ACC_MEM_DEVICE and this missing_off / missing_txn). */
typedef struct acc_cfk_batch_view {
    acc_batch_in    batch;        /* mem = ACC_MEM_DEVICE */
    const uint32_t *missing_off;  /* [batch.n_pairs+1] */
    const uint32_t *missing_txn;  /* [n_missing] batch indices, sorted per pair */
    uint64_t        n_missing;
} acc_cfk_batch_view;

int  acc_cfk_snap_to_batch(acc_ctx *ctx, const acc_cfk_snap *snap, acc_cfk_batch_view *out_view);

/* One CommandsForKey store for the update with deps and every scan (the reference keeps one
 * CommandsForKey per key that CommandsForKey.update writes and mapReduceActive / mapReduceFull read,
 * local/CommandsForKey.java:614-706, 1085-1149): acc_cfk_apply_deps applies a batch of updates with deps to the acc_cfk
 * store itself — acc_cfk_apply over the store's key-major state, then the store's txn-major view and its per-pair
 * missing[] as txn indices rebuilt from the result — so acc_cfk_view (acc_keydeps_batch, acc_shard_pack), acc_cfk_missing
 * (acc_map_reduce_full: its batch and acc_recovery_in's missing_off / missing_txn with mem = ACC_MEM_DEVICE) and
 * acc_cfk_state (the key-major state in the acc_cfk_apply layout, DEVICE memory) read one state in place, valid until
 * the next update of the store. A rejected batch (ACC_E_STATE / ACC_E_ARG) leaves the store unchanged. A store keeps
 * missing[] from its first acc_cfk_apply_deps on; acc_cfk_update (status-only, no missing[]) is then ACC_E_STATE, and
 * acc_cfk_apply_deps on a store holding acc_cfk_update state is ACC_E_STATE. The store adopts the call's result
 * arrays from the context (no copies) and hands its previous arrays to the context for its next results. Keys with
 * many updates in one batch (more than ACC_CFK_HOT, default 64, snapshot + update elements) are computed by the
 * data-parallel closed form of the replay (acc_cfk_apply too); results are the same. */
int  acc_cfk_apply_deps(acc_ctx *ctx, acc_cfk *cfk, const acc_cfk_updates *updates);
int  acc_cfk_state(acc_ctx *ctx, acc_cfk *cfk, acc_cfk_snap *out);
int  acc_cfk_missing(acc_ctx *ctx, acc_cfk *cfk, acc_cfk_batch_view *out);

/* ---- MaxConflicts and the PreAccept executeAt proposal (local/MaxConflicts.java:31-96,
 * local/CommandStore.java:280-290 updateMaxConflicts, :320-345 preaccept) ----
 * A CommandStore's MaxConflicts is the pointwise max of every (keysOrRanges, executeAt) update it received
 * (MaxConflicts.merge(map, create(keysOrRanges, executeAt)), a ReducingRangeMap folded with Timestamp::max; a key k
 * enters as its asRange(), which holds exactly k), so MaxConflicts.get(q) is the max executeAt over the updates whose
 * keys / ranges intersect q's keys / ranges (Range.contains for a key, compareIntersecting for two ranges).
 * Input: the updates (Command.executeAt() and keys or ranges each; updateMaxConflicts skips an update whose executeAt
 * does not exceed the previous one, which the max already absorbs). Output per query (a PreAccept of txn_id over its
 * sliced keys or ranges): max = minNonConflicting = MaxConflicts.get(keys) (all zero = Timestamp.NONE when nothing
 * intersects) and fast_path = txnId.compareTo(minNonConflicting) >= 0 (preaccept then returns txnId when
 * permitFastPath and the epoch check hold, the caller's part; otherwise time.uniqueNow(minNonConflicting)). Among
 * compare-equal timestamps with different raw flag bits, which instance is returned is unspecified. */
typedef struct acc_conflicts_in {
    uint32_t mem, n_upd, end_inclusive;
    uint64_t n_keys, n_ranges;
    acc_ts_cols execute_at;      /* [n_upd] */
    const uint32_t *key_off;     /* [n_upd+1] */
    const uint64_t *key;         /* [n_keys] sorted unique per update */
    const uint32_t *rng_off;     /* [n_upd+1] */
    const uint64_t *rng_start, *rng_end;   /* [n_ranges] sorted, non-overlapping per update */
} acc_conflicts_in;

typedef struct acc_preaccept_in {
    uint32_t mem, n_query;
    uint64_t n_parts;
    acc_ts_cols txn_id;          /* [n_query] */
    const uint8_t *is_range;     /* [n_query] 0: keys, 1: ranges */
    const uint32_t *part_off;    /* [n_query+1] */
    const uint64_t *part_start, *part_end;
} acc_preaccept_in;

typedef struct acc_preaccept_out {
    uint32_t mem;
    uint64_t *max_msb, *max_lsb;
    int32_t  *max_node;
    uint8_t  *fast_path;         /* all [n_query], caller-owned */
} acc_preaccept_out;

int  acc_max_conflicts(acc_ctx *ctx, const acc_conflicts_in *updates, const acc_preaccept_in *queries,
                       acc_preaccept_out *out);

/* A CommandStore's MaxConflicts kept on the device across calls (the store's one map, CommandStore.maxConflicts,
 * local/CommandStore.java:270-290): disjoint intervals over the key codes with a Timestamp each (ReducingRangeMap).
 * acc_maxconflicts_update merges a batch of commands' (keysOrRanges, executeAt) into it (MaxConflicts.update =
 * ReducingIntervalMap.merge with Timestamp::max; a batch equals its commands applied one by one in any order);
 * acc_maxconflicts_get answers PreAccept queries as acc_max_conflicts does, in O(log map) per key or range (the
 * acc_max_conflicts form rebuilds the map from the store's whole update history on every call). end_inclusive fixes
 * the map's Range bound type; updates must carry the same. Not thread-safe; one context at a time. */
typedef struct acc_maxconflicts acc_maxconflicts;
int  acc_maxconflicts_create(acc_ctx *ctx, uint32_t end_inclusive, acc_maxconflicts **out);
void acc_maxconflicts_destroy(acc_maxconflicts *map);
int  acc_maxconflicts_update(acc_ctx *ctx, acc_maxconflicts *map, const acc_conflicts_in *updates);
int  acc_maxconflicts_get(acc_ctx *ctx, acc_maxconflicts *map, const acc_preaccept_in *queries, acc_preaccept_out *out);
/* intervals currently held (ReducingRangeMap.size) */
uint64_t acc_maxconflicts_size(const acc_maxconflicts *map);

/* ---- Levelisation of a dependency graph by executeAt ----
 * Graph over n txns: deps of txn t = dep[off[t] .. off[t+1]) (batch indices); exec_rank[t] = order
 * rank of t.executeAt. Edges whose dep has exec_rank >= exec_rank[t] are ignored (Commands.java:804-810).
 * level[t] = 0 without remaining preds, else 1 + max level(pred); order = txns sorted by
 * (level, exec_rank, index). Outputs are caller buffers of n elements in `mem`. */
typedef struct acc_graph_in {
    uint32_t mem;
    uint32_t n;
    const uint64_t *off;       /* [n+1] */
    const uint32_t *dep;       /* [off[n]] */
    const uint32_t *exec_rank; /* [n] */
} acc_graph_in;

int acc_levelise(acc_ctx *ctx, const acc_graph_in *in, uint32_t *level, uint32_t *order, uint32_t *n_levels);

/* ---- Ranges algebra (host code, no context; primitives/Ranges.java, AbstractRanges.java) ----
 * A Ranges is a sorted, deoverlapped list of Range (start, end) key codes of one bound type (Range.EndInclusive (s, e]
 * or Range.StartInclusive [s, e), Range.java:40-138); operations on ranges alone do not depend on the bound type.
 * Results go to caller arrays of `cap` entries; *out_n is always the result size (ACC_E_CAP when > cap; bounds:
 * with / subtract <= a.n + b.n, merge_touching <= a.n, select <= k, of <= in.n). Inputs that must be sorted and
 * deoverlapped are checked (Ranges.ofSortedAndDeoverlapped: IllegalArgumentException -> ACC_E_ARG). */
/* (acc_rlist is declared at the top of this header) */

/* Ranges.of(Range...)                          AbstractRanges.java:689-707 (sort by Range::compare, merge overlaps) */
int acc_ranges_of(const acc_rlist *in, uint64_t *out_start, uint64_t *out_end, uint32_t cap, uint32_t *out_n);
/* a.with(b) = union(MERGE_OVERLAPPING)         Ranges.java:119-127, AbstractRanges.java:439-585 */
int acc_ranges_with(const acc_rlist *a, const acc_rlist *b, uint64_t *out_start, uint64_t *out_end, uint32_t cap,
                    uint32_t *out_n);
/* a.subtract(b)                                AbstractRanges.java:223-287 */
int acc_ranges_subtract(const acc_rlist *a, const acc_rlist *b, uint64_t *out_start, uint64_t *out_end, uint32_t cap,
                        uint32_t *out_n);
/* a.mergeTouching()                            AbstractRanges.java:637-675 */
int acc_ranges_merge_touching(const acc_rlist *a, uint64_t *out_start, uint64_t *out_end, uint32_t cap, uint32_t *out_n);
/* a.select(int[] indexes)                      Ranges.java:76-82 */
int acc_ranges_select(const acc_rlist *a, const uint32_t *idx, uint32_t k, uint64_t *out_start, uint64_t *out_end,
                      uint32_t cap, uint32_t *out_n);
/* a.indexOf(key): index, or -(insertion point) - 1   AbstractRanges.java:51-54 (SortedArrays FAST search) */
int acc_ranges_index_of(const acc_rlist *a, uint32_t end_inclusive, uint64_t key, int64_t *out_index);
/* a.containsAll(Keys) (sorted unique key codes) AbstractRanges.java:86-91; a.containsAll(Ranges) :96-101 */
int acc_ranges_contains_all_keys(const acc_rlist *a, uint32_t end_inclusive, const uint64_t *keys, uint32_t n_keys,
                                 int32_t *out);
int acc_ranges_contains_all(const acc_rlist *a, const acc_rlist *b, int32_t *out);
/* RangeDeps.isCoveredBy(covering) over a RangeDeps' ranges (sorted by Range::compare) primitives/RangeDeps.java:595-613 */
int acc_rangedeps_is_covered_by(const acc_rlist *range_deps_ranges, const acc_rlist *covering, int32_t *out);

/* ---- timing (ACC_OPT_TIMING) ---- */
/* Per-kernel accumulated device time since the last reset: name[i], total ms, launch count. */
int  acc_timing_count(acc_ctx *ctx);
int  acc_timing_get(acc_ctx *ctx, int i, const char **name, double *total_ms, uint64_t *launches);
void acc_timing_reset(acc_ctx *ctx);
/* Restrict the per-kernel events to the launches whose tag is in the comma-separated list (NULL or "" = every launch).
   Each timed launch adds two event records to the stream; a bench times its step with only the kernel it reports. */
int  acc_timing_filter(acc_ctx *ctx, const char *tags_csv);

/* ---- counters of the last call (e.g. "keydeps.path_replay", "keydeps.big_txns", "keydeps.big_entries") ---- */
int acc_stats_count(acc_ctx *ctx);
int acc_stats_get(acc_ctx *ctx, int i, const char **name, uint64_t *value);

#ifdef __cplusplus
}
#endif
#endif /* ACCORD_AMD_H */
