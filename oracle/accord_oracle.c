/*
 * accord_oracle.c — TEST INFRASTRUCTURE ONLY (see accord_oracle.h header for the rules).
 *
 * Plain-C restatement of the reference Java, function by function. Paths are relative to
 * /root/reference/accord-core/src/main/java/accord/. The O(prefix) CommandsForKey scan and the
 * object-style builder are kept on purpose: this file is also the CPU baseline ("port").
 */
#define _GNU_SOURCE
#include "accord_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* ------------------------------------------------------------------ Timestamp / TxnId */

typedef struct ts { uint64_t msb, lsb; int32_t node; } ts;

/* Timestamp.IDENTITY_LSB / IDENTITY_FLAGS (Timestamp.java:41-42) */
#define IDENTITY_LSB   0xFFFFFFFFFFFF001EULL
#define IDENTITY_FLAGS 0x001EULL

/* Timestamp.compareTo (Timestamp.java:208-217): unsigned msb, then lowHlc = lsb>>>16 (signed long
 * compare of a non-negative value), then lsb & IDENTITY_FLAGS, then Node.Id.compareTo (signed int,
 * local/Node.java:136-139). */
static inline int ts_cmp(const ts *a, const ts *b)
{
    if (a->msb != b->msb) return a->msb < b->msb ? -1 : 1;
    uint64_t ah = a->lsb >> 16, bh = b->lsb >> 16;
    if (ah != bh) return ah < bh ? -1 : 1;
    uint64_t af = a->lsb & IDENTITY_FLAGS, bf = b->lsb & IDENTITY_FLAGS;
    if (af != bf) return af < bf ? -1 : 1;
    if (a->node != b->node) return a->node < b->node ? -1 : 1;
    return 0;
}

/* Timestamp.equals (Timestamp.java:244-249) */
static inline int ts_eq(const ts *a, const ts *b)
{
    return a->msb == b->msb && ((a->lsb ^ b->lsb) & IDENTITY_LSB) == 0 && a->node == b->node;
}

int orc_ts_compare(uint64_t amsb, uint64_t alsb, int32_t anode, uint64_t bmsb, uint64_t blsb, int32_t bnode)
{
    ts a = { amsb, alsb, anode }, b = { bmsb, blsb, bnode };
    return ts_cmp(&a, &b);
}

/* TxnId.kind(): rwOrdinal = (flags >> 1) & 7 (TxnId.java:149-152) */
static inline int ts_kind(const ts *t) { return (int)((t->lsb >> 1) & 7); }

/* Txn.Kind ordinals (Txn.java:53-113) */
enum { K_READ = 0, K_WRITE = 1, K_EREAD = 2, K_SYNC = 3, K_XSYNC = 4, K_LOCAL = 5, K_COUNT = 6 };
/* Kinds predicates as bitmasks over Kind ordinals (Txn.java:125-153) */
#define KINDS_WS           (1u << K_WRITE)
#define KINDS_RS_OR_WS     ((1u << K_READ) | (1u << K_WRITE))
#define KINDS_ANY_VISIBLE  ((1u << K_READ) | (1u << K_WRITE) | (1u << K_SYNC) | (1u << K_XSYNC))

/* Kind.witnesses() (Txn.java:221-236). Returns -1 for kinds whose witnesses() throws. */
static int kind_witnesses(int kind)
{
    switch (kind) {
    case K_EREAD: case K_READ: return (int)KINDS_WS;
    case K_WRITE: case K_SYNC: return (int)KINDS_RS_OR_WS;
    case K_XSYNC:              return (int)KINDS_ANY_VISIBLE;
    default:                   return -1;   /* LocalOnly: AssertionError; >5: ofOrdinal out of range */
    }
}

/* CommandsForKey.InternalStatus ordinals (CommandsForKey.java:194-203) */
enum { ST_TK = 0, ST_HIST = 1, ST_PRE = 2, ST_ACC = 3, ST_COMMITTED = 4, ST_STABLE = 5, ST_APPLIED = 6, ST_INVALID = 7 };

/* ------------------------------------------------------------------ error plumbing */

typedef struct err { int code; char msg[256]; } err;
static void set_err(err *e, int code, const char *m)
{
    if (e->code) return;
    e->code = code;
    snprintf(e->msg, sizeof e->msg, "%s", m);
}

/* ------------------------------------------------------------------ growable buffers */

typedef struct ivec { int64_t *v; size_t n, cap; } ivec;
static void iv_push(ivec *a, int64_t x)
{
    if (a->n == a->cap) { a->cap = a->cap ? a->cap * 2 : 16; a->v = realloc(a->v, a->cap * sizeof *a->v); }
    a->v[a->n++] = x;
}

/* ------------------------------------------------------------------ stable merge sort of indices */

typedef int (*icmp_fn)(int64_t a, int64_t b, const void *ctx);

/* Stable (like java.util.Arrays.sort on Objects / TimSort: equal elements keep input order). */
static void stable_sort(int64_t *a, size_t n, icmp_fn cmp, const void *ctx)
{
    if (n < 2) return;
    int64_t *tmp = malloc(n * sizeof *tmp);
    for (size_t w = 1; w < n; w *= 2) {
        for (size_t lo = 0; lo < n; lo += 2 * w) {
            size_t mid = lo + w < n ? lo + w : n, hi = lo + 2 * w < n ? lo + 2 * w : n;
            size_t i = lo, j = mid, k = lo;
            while (i < mid && j < hi) tmp[k++] = cmp(a[j], a[i], ctx) < 0 ? a[j++] : a[i++];
            while (i < mid) tmp[k++] = a[i++];
            while (j < hi) tmp[k++] = a[j++];
        }
        memcpy(a, tmp, n * sizeof *a);
    }
    free(tmp);
}

/* Stable LSD radix sort of index array a (entries index key[]) by the u64 key (16-bit digits): the same order as
 * stable_sort with an unsigned key comparator, in O(n) passes (the batch grouping of 10^8 pairs). */
static void radix_sort_by_u64(int64_t *a, size_t n, const uint64_t *key)
{
    if (n < 2) return;
    uint64_t mx = 0;
    for (size_t i = 0; i < n; ++i) mx |= key[a[i]];
    int64_t *tmp = malloc(n * sizeof *tmp);
    size_t *cnt = malloc(65537 * sizeof *cnt);
    for (int shift = 0; shift < 64 && (mx >> shift); shift += 16) {
        memset(cnt, 0, 65537 * sizeof *cnt);
        for (size_t i = 0; i < n; ++i) cnt[((key[a[i]] >> shift) & 0xFFFF) + 1]++;
        for (int d = 0; d < 65536; ++d) cnt[d + 1] += cnt[d];
        for (size_t i = 0; i < n; ++i) tmp[cnt[(key[a[i]] >> shift) & 0xFFFF]++] = a[i];
        memcpy(a, tmp, n * sizeof *a);
    }
    free(tmp);
    free(cnt);
}

/* ------------------------------------------------------------------ batch data */

typedef struct batch {
    uint32_t n;
    ts *id, *ex;
    const uint8_t *status;
    const uint32_t *key_off;
    const uint64_t *key_code;
} batch;

static int cmp_txn_by_id(int64_t a, int64_t b, const void *c)
{
    const batch *B = c; return ts_cmp(&B->id[a], &B->id[b]);
}
static int cmp_txn_by_exec(int64_t a, int64_t b, const void *c)
{
    const batch *B = c; return ts_cmp(&B->ex[a], &B->ex[b]);
}

/* ------------------------------------------------------------------ CommandsForKey */

/* One key's summary: txns sorted by TxnId (CommandsForKey.java:403-404) and committed[] = entries
 * with COMMITTED <= status < INVALID_OR_TRUNCATED sorted by executeAt with a stable sort
 * (ctor, CommandsForKey.java:459-469). Entries are batch txn indices. */
typedef struct cfk {
    uint64_t key;
    int64_t *txns; size_t ntxns;
    int64_t *committed; size_t ncommitted;
} cfk;

static int is_sorted_by(const int64_t *a, size_t n, icmp_fn cmp, const void *ctx)
{
    for (size_t i = 1; i < n; ++i)
        if (cmp(a[i - 1], a[i], ctx) > 0) return 0;
    return 1;
}

static void cfk_init(cfk *c, const batch *B)
{
    /* a stable sort leaves a sorted input as it is: skip the O(n log n) pass for batches handed over in TxnId order */
    if (!is_sorted_by(c->txns, c->ntxns, cmp_txn_by_id, B)) stable_sort(c->txns, c->ntxns, cmp_txn_by_id, B);
    c->committed = malloc((c->ntxns ? c->ntxns : 1) * sizeof *c->committed);
    c->ncommitted = 0;
    for (size_t i = 0; i < c->ntxns; ++i) {
        int s = B->status[c->txns[i]];
        if (s >= ST_COMMITTED && s != ST_INVALID) c->committed[c->ncommitted++] = c->txns[i];
    }
    if (!is_sorted_by(c->committed, c->ncommitted, cmp_txn_by_exec, B))
        stable_sort(c->committed, c->ncommitted, cmp_txn_by_exec, B);
}

/* SortedArrays.binarySearch(..., FAST) (SortedArrays.java:992-1027) with the comparator
 * (f, v) -> f.compareTo(v.executeAt) used by CommandsForKey.mapReduceActive (:619). */
static long bsearch_fast_exec(const cfk *c, const batch *B, const ts *find)
{
    long from = 0, to = (long)c->ncommitted;
    while (from < to) {
        long i = (long)(((unsigned long)from + (unsigned long)to) >> 1);
        int cc = ts_cmp(find, &B->ex[c->committed[i]]);
        if (cc < 0) to = i;
        else if (cc > 0) from = i + 1;
        else return i;
    }
    return -1 - to;
}

/* java.util.Arrays.binarySearch(Object[], from, to, key) with Comparable (TxnInfo extends
 * Timestamp): midVal.compareTo(key); used by CommandsForKey.insertPos (:1698-1703). */
static long insert_pos(const cfk *c, const batch *B, const ts *key)
{
    long low = 0, high = (long)c->ntxns - 1;
    while (low <= high) {
        long mid = (long)(((unsigned long)low + (unsigned long)high) >> 1);
        int cc = ts_cmp(&B->id[c->txns[mid]], key);
        if (cc < 0) low = mid + 1;
        else if (cc > 0) high = mid - 1;
        else return mid;
    }
    return low;   /* i < 0 ? -1 - i : i  ==  low */
}

/* ------------------------------------------------------------------ KeyDeps.Builder */

/* RelationMultiMap.AbstractBuilder<Key, TxnId, KeyDeps> (RelationMultiMap.java:88-260) with keys as
 * u64 codes (unsigned order = RoutableKey.compareTo via the host's order-preserving encoding) and
 * values as batch txn indices compared by TxnId (KeyDeps.ADAPTER valueComparator = TxnId::compareTo). */
typedef struct builder {
    const batch *B;
    uint64_t *keys; size_t keys_cap;
    int64_t *key_limits;
    int64_t *vals; size_t vals_cap;
    size_t key_count, key_offset, total_count;
    int has_ordered_keys, has_ordered_values;
} builder;

static void b_init(builder *b, const batch *B)
{
    memset(b, 0, sizeof *b);
    b->B = B;
    b->keys_cap = 16; b->keys = malloc(16 * sizeof *b->keys); b->key_limits = malloc(16 * sizeof *b->key_limits);
    b->vals_cap = 16; b->vals = malloc(16 * sizeof *b->vals);
    b->has_ordered_keys = 1; b->has_ordered_values = 1;
}
static void b_reset(builder *b)
{
    b->key_count = b->key_offset = b->total_count = 0;
    b->has_ordered_keys = 1; b->has_ordered_values = 1;
}
static void b_free(builder *b) { free(b->keys); free(b->key_limits); free(b->vals); }

/* AbstractBuilder.finishKey (:147-171) */
static void b_finish_key(builder *b)
{
    if (b->total_count == b->key_offset && b->key_count > 0) { --b->key_count; return; }
    if (b->key_count == 0) return;
    if (!b->has_ordered_values) {
        stable_sort(b->vals + b->key_offset, b->total_count - b->key_offset, cmp_txn_by_id, b->B);
        size_t removed = 0;
        for (size_t i = b->key_offset + 1; i < b->total_count; ++i) {
            if (ts_eq(&b->B->id[b->vals[i - 1]], &b->B->id[b->vals[i]])) ++removed;
            else if (removed > 0) b->vals[i - removed] = b->vals[i];
        }
        b->total_count -= removed;
    }
    b->key_limits[b->key_count - 1] = (int64_t)b->total_count;
    b->key_offset = b->total_count;
}

/* AbstractBuilder.nextKey (:125-145) */
static void b_next_key(builder *b, uint64_t key)
{
    if (b->key_count > 0 && b->keys[b->key_count - 1] >= key) b->has_ordered_keys = 0;
    b_finish_key(b);
    if (b->key_count == b->keys_cap) {
        b->keys_cap *= 2;
        b->keys = realloc(b->keys, b->keys_cap * sizeof *b->keys);
        b->key_limits = realloc(b->key_limits, b->keys_cap * sizeof *b->key_limits);
    }
    b->keys[b->key_count++] = key;
    b->has_ordered_values = 1;
}

/* AbstractBuilder.add(V) (:183-199) */
static void b_add_value(builder *b, int64_t v)
{
    if (b->has_ordered_values && b->total_count > b->key_offset
        && ts_cmp(&b->B->id[b->vals[b->total_count - 1]], &b->B->id[v]) >= 0)
        b->has_ordered_values = 0;
    if (b->total_count >= b->vals_cap) { b->vals_cap *= 2; b->vals = realloc(b->vals, b->vals_cap * sizeof *b->vals); }
    b->vals[b->total_count++] = v;
}

/* AbstractBuilder.add(K, V) (:173-178) */
static void b_add(builder *b, uint64_t key, int64_t v)
{
    if (b->key_count == 0 || b->keys[b->key_count - 1] != key) b_next_key(b, key);
    b_add_value(b, v);
}

/* A built KeyDeps over batch indices: keys (codes), txnIds (batch idx), keysToTxnIds (Java int[]). */
typedef struct kdeps {
    uint64_t *keys; size_t nkeys;
    int64_t  *vals; size_t nvals;
    int32_t  *k2v;  size_t nk2v;
} kdeps;

static void kd_free(kdeps *d) { free(d->keys); free(d->vals); free(d->k2v); memset(d, 0, sizeof *d); }

static int cmp_u64(int64_t a, int64_t b, const void *c)
{
    const uint64_t *k = c; return k[a] < k[b] ? -1 : k[a] > k[b];
}

/* SortedArrays.findNextIntersection / foldlIntersection (SortedArrays.java:1148-1173,1271-1292):
 * indices (into `values`) of the members of the sorted key list, written to out. */
static size_t fold_intersection(const batch *B, const int64_t *values, size_t nvalues,
                                const int64_t *list, size_t from, size_t to, int32_t *out)
{
    size_t ai = 0, bi = from, n = 0;
    while (ai < nvalues && bi < to) {
        int c = ts_cmp(&B->id[values[ai]], &B->id[list[bi]]);
        if (c == 0) { out[n++] = (int32_t)ai; ++ai; ++bi; }
        else if (c < 0) ++ai;
        else ++bi;
    }
    return n;
}

/* AbstractBuilder.build (:201-260). Returns 0 / -1 (IllegalArgumentException: duplicate key). */
static int b_build(builder *b, kdeps *out, err *e)
{
    memset(out, 0, sizeof *out);
    if (b->total_count == 0) return 0;          /* none() = KeyDeps.NONE */
    b_finish_key(b);

    size_t total = b->total_count;
    int64_t *uv = malloc(total * sizeof *uv);
    memcpy(uv, b->vals, total * sizeof *uv);
    stable_sort(uv, total, cmp_txn_by_id, b->B);
    size_t vc = 1;
    for (size_t i = 1; i < total; ++i)
        if (!ts_eq(&b->B->id[uv[vc - 1]], &b->B->id[uv[i]])) uv[vc++] = uv[i];

    size_t kc = b->key_count;
    int64_t *sorted_idx = NULL;          /* sortedKeyIndexes[sorted pos] = original key index */
    uint64_t *skeys = malloc((kc ? kc : 1) * sizeof *skeys);
    if (b->has_ordered_keys) {
        memcpy(skeys, b->keys, kc * sizeof *skeys);
    } else {
        int64_t *perm = malloc(kc * sizeof *perm);
        for (size_t i = 0; i < kc; ++i) perm[i] = (int64_t)i;
        stable_sort(perm, kc, cmp_u64, b->keys);
        for (size_t i = 0; i < kc; ++i) skeys[i] = b->keys[perm[i]];
        for (size_t i = 1; i < kc; ++i)
            if (skeys[i - 1] == skeys[i]) {
                free(perm); free(skeys); free(uv);
                set_err(e, -1, "Key has been visited more than once (AbstractBuilder.build)");
                return -1;
            }
        sorted_idx = perm;
    }

    int32_t *res = malloc((kc + total) * sizeof *res);
    size_t offset = kc;
    for (size_t ki = 0; ki < kc; ++ki) {
        size_t k = sorted_idx ? (size_t)sorted_idx[ki] : ki;
        size_t from = k == 0 ? 0 : (size_t)b->key_limits[k - 1];
        size_t to = (size_t)b->key_limits[k];
        offset += fold_intersection(b->B, uv, vc, b->vals, from, to, res + offset);
        res[ki] = (int32_t)offset;
    }
    free(sorted_idx);
    out->keys = skeys; out->nkeys = kc;
    out->vals = realloc(uv, (vc ? vc : 1) * sizeof *uv); out->nvals = vc;
    out->k2v = res; out->nk2v = offset;
    return 0;
}

/* ------------------------------------------------------------------ linearUnion (KeyDeps.with) */

/* RelationMultiMap.linearUnion (RelationMultiMap.java:561-816), general path. Its fast paths
 * (:583-730) return an input unchanged only when it already equals the union, so the value result is
 * always the canonical union (KeyDepsTest.testMergedProperty). Value identity on ties keeps the
 * LEFT element (SortedArrays.linearUnion :250-255). cmpv compares two value handles. */
typedef int (*vcmp_fn)(int64_t a, int64_t b, const void *ctx);

static void kd_union(const kdeps *L, const kdeps *R, kdeps *out, vcmp_fn cmpv, const void *ctx)
{
    /* SortedArrays.linearUnion of keys and of values (:152-281) */
    uint64_t *ok = malloc((L->nkeys + R->nkeys + 1) * sizeof *ok); size_t nok = 0;
    { size_t i = 0, j = 0;
      while (i < L->nkeys && j < R->nkeys) {
          if (L->keys[i] < R->keys[j]) ok[nok++] = L->keys[i++];
          else if (L->keys[i] > R->keys[j]) ok[nok++] = R->keys[j++];
          else { ok[nok++] = L->keys[i++]; ++j; }
      }
      while (i < L->nkeys) ok[nok++] = L->keys[i++];
      while (j < R->nkeys) ok[nok++] = R->keys[j++]; }
    int64_t *ov = malloc((L->nvals + R->nvals + 1) * sizeof *ov); size_t nov = 0;
    int32_t *remapL = malloc((L->nvals + 1) * sizeof *remapL), *remapR = malloc((R->nvals + 1) * sizeof *remapR);
    { size_t i = 0, j = 0;
      while (i < L->nvals && j < R->nvals) {
          int c = cmpv(L->vals[i], R->vals[j], ctx);
          if (c < 0) { remapL[i] = (int32_t)nov; ov[nov++] = L->vals[i++]; }
          else if (c > 0) { remapR[j] = (int32_t)nov; ov[nov++] = R->vals[j++]; }
          else { remapL[i] = remapR[j] = (int32_t)nov; ov[nov++] = L->vals[i++]; ++j; }
      }
      while (i < L->nvals) { remapL[i] = (int32_t)nov; ov[nov++] = L->vals[i++]; }
      while (j < R->nvals) { remapR[j] = (int32_t)nov; ov[nov++] = R->vals[j++]; } }

    int32_t *o = malloc((L->nk2v + R->nk2v + 1) * sizeof *o);
    size_t lk = 0, rk = 0, okk = 0, l = L->nkeys, r = R->nkeys, olen = nok;
    while (lk < L->nkeys && rk < R->nkeys) {
        if (L->keys[lk] < R->keys[rk]) {
            while (l < (size_t)L->k2v[lk]) o[olen++] = remapL[L->k2v[l++]];
            o[okk++] = (int32_t)olen; lk++;
        } else if (L->keys[lk] > R->keys[rk]) {
            while (r < (size_t)R->k2v[rk]) o[olen++] = remapR[R->k2v[r++]];
            o[okk++] = (int32_t)olen; rk++;
        } else {
            while (l < (size_t)L->k2v[lk] && r < (size_t)R->k2v[rk]) {
                int32_t nl = remapL[L->k2v[l]], nr = remapR[R->k2v[r]];
                if (nl <= nr) { o[olen++] = nl; l += 1; r += nl == nr ? 1 : 0; }
                else { o[olen++] = nr; ++r; }
            }
            while (l < (size_t)L->k2v[lk]) o[olen++] = remapL[L->k2v[l++]];
            while (r < (size_t)R->k2v[rk]) o[olen++] = remapR[R->k2v[r++]];
            o[okk++] = (int32_t)olen; rk++; lk++;
        }
    }
    while (lk < L->nkeys) { while (l < (size_t)L->k2v[lk]) o[olen++] = remapL[L->k2v[l++]]; o[okk++] = (int32_t)olen; lk++; }
    while (rk < R->nkeys) { while (r < (size_t)R->k2v[rk]) o[olen++] = remapR[R->k2v[r++]]; o[okk++] = (int32_t)olen; rk++; }
    free(remapL); free(remapR);
    out->keys = ok; out->nkeys = nok; out->vals = ov; out->nvals = nov; out->k2v = o; out->nk2v = olen;
}

static int cmp_vals_by_id(int64_t a, int64_t b, const void *c)
{
    const batch *B = c; return ts_cmp(&B->id[a], &B->id[b]);
}

/* KeyDeps.isEmpty (KeyDeps.java:292-295): no entries (keys without values may remain). */
static int kd_is_empty(const kdeps *d) { return d->nk2v == d->nkeys; }

/* KeyDeps.with (KeyDeps.java:238-253): empty operands short-circuit (isEmpty() ? that : this). */
static void kd_with(kdeps *acc, const kdeps *that, vcmp_fn cmpv, const void *ctx)
{
    if (!kd_is_empty(acc) && kd_is_empty(that)) return;
    if (kd_is_empty(acc)) {
        kd_free(acc);
        acc->keys = malloc(that->nkeys * sizeof *acc->keys); memcpy(acc->keys, that->keys, that->nkeys * sizeof *acc->keys); acc->nkeys = that->nkeys;
        acc->vals = malloc((that->nvals + 1) * sizeof *acc->vals); memcpy(acc->vals, that->vals, that->nvals * sizeof *acc->vals); acc->nvals = that->nvals;
        acc->k2v = malloc(that->nk2v * sizeof *acc->k2v); memcpy(acc->k2v, that->k2v, that->nk2v * sizeof *acc->k2v); acc->nk2v = that->nk2v;
        return;
    }
    kdeps u; kd_union(acc, that, &u, cmpv, ctx);
    kd_free(acc); *acc = u;
}

/* ------------------------------------------------------------------ the batch */


/* CommandsForKey.mapReduceActive (CommandsForKey.java:614-650) feeding the calculatePartialDeps
 * map function (PreAccept.java:253-259): emits (key, txn) into the builder. */
static uint64_t cfk_map_reduce_active(const cfk *c, const batch *B, const ts *started_before,
                                      unsigned test_kinds, long p1, builder *b, err *e)
{
    long i = bsearch_fast_exec(c, B, started_before);
    if (i < 0) i = -2 - i; else --i;
    while (i >= 0 && ts_kind(&B->id[c->committed[i]]) != K_WRITE) --i;   /* TxnInfo.kind(): kind of the TxnId */
    const ts *max_committed_before = i < 0 ? NULL : &B->ex[c->committed[i]];
    long end = insert_pos(c, B, started_before);
    uint64_t visited = 0;
    for (long k = 0; k < end; ++k) {
        int64_t t = c->txns[k];
        ++visited;
        int kind = ts_kind(&B->id[t]);
        if (kind >= K_COUNT) { set_err(e, -1, "Kind.ofOrdinal: invalid kind ordinal"); return visited; }
        if (!((test_kinds >> kind) & 1u)) continue;
        switch (B->status[t]) {
        case ST_COMMITTED: case ST_STABLE: case ST_APPLIED:
            if (max_committed_before == NULL || ts_cmp(&B->ex[t], max_committed_before) >= 0) break;
            continue;
        case ST_TK: case ST_INVALID:
            continue;
        default: break;
        }
        if (p1 < 0 || !ts_eq(&B->id[t], &B->id[p1])) b_add(b, c->key, t);
    }
    return visited;
}

/* Range.contains bounds over the sorted CFK keys (InMemoryCommandStore.mapReduceForKey :274-289:
 * commandsForKey.subMap(start, startInclusive, end, endInclusive)): first CFK index with key inside / past the
 * range. EndInclusive (s, e]: keys > s up to <= e; StartInclusive [s, e): keys >= s up to < e. */
static size_t cfk_lower(const cfk *cfks, size_t ncfk, uint64_t bound, int strictly_above)
{
    size_t a = 0, z = ncfk;
    while (a < z) {
        size_t m = (a + z) / 2;
        if (strictly_above ? cfks[m].key <= bound : cfks[m].key < bound) a = m + 1; else z = m;
    }
    return a;
}

static void keydeps_impl(orc_keydeps_result *R, uint32_t n,
                         const uint64_t *tmsb, const uint64_t *tlsb, const int32_t *tnode,
                         const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                         const uint8_t *status, const uint32_t *key_off, const uint64_t *key_code,
                         const uint32_t *rng_off, const uint64_t *rng_start, const uint64_t *rng_end, int end_inclusive,
                         uint32_t n_shards, uint32_t query_lo, uint32_t query_hi, uint32_t query_stride,
                         const uint8_t *qmask);

orc_keydeps_result *orc_keydeps_batch(uint32_t n,
                                      const uint64_t *tmsb, const uint64_t *tlsb, const int32_t *tnode,
                                      const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                                      const uint8_t *status, const uint32_t *key_off, const uint64_t *key_code,
                                      uint32_t n_shards, uint32_t query_lo, uint32_t query_hi,
                                      uint32_t query_stride)
{
    orc_keydeps_result *R = calloc(1, sizeof *R);
    keydeps_impl(R, n, tmsb, tlsb, tnode, emsb, elsb, enode, status, key_off, key_code, NULL, NULL, NULL, 1,
                 n_shards, query_lo, query_hi, query_stride, NULL);
    return R;
}

orc_keydeps_result *orc_keydeps_batch_qmask(uint32_t n,
                                            const uint64_t *tmsb, const uint64_t *tlsb, const int32_t *tnode,
                                            const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                                            const uint8_t *status, const uint32_t *key_off, const uint64_t *key_code,
                                            const uint8_t *query_mask)
{
    orc_keydeps_result *R = calloc(1, sizeof *R);
    keydeps_impl(R, n, tmsb, tlsb, tnode, emsb, elsb, enode, status, key_off, key_code, NULL, NULL, NULL, 1,
                 1, 0, n, 1, query_mask);
    return R;
}

orc_keydeps_result *orc_keydeps_mixed(uint32_t n,
                                      const uint64_t *tmsb, const uint64_t *tlsb, const int32_t *tnode,
                                      const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                                      const uint8_t *status, const uint32_t *key_off, const uint64_t *key_code,
                                      const uint32_t *rng_off, const uint64_t *rng_start, const uint64_t *rng_end,
                                      int end_inclusive, uint32_t n_shards, uint32_t query_lo, uint32_t query_hi,
                                      uint32_t query_stride)
{
    orc_keydeps_result *R = calloc(1, sizeof *R);
    keydeps_impl(R, n, tmsb, tlsb, tnode, emsb, elsb, enode, status, key_off, key_code, rng_off, rng_start, rng_end,
                 end_inclusive, n_shards, query_lo, query_hi, query_stride, NULL);
    return R;
}

orc_keydeps_result *orc_keydeps_mixed_qmask(uint32_t n,
                                            const uint64_t *tmsb, const uint64_t *tlsb, const int32_t *tnode,
                                            const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                                            const uint8_t *status, const uint32_t *key_off, const uint64_t *key_code,
                                            const uint32_t *rng_off, const uint64_t *rng_start, const uint64_t *rng_end,
                                            int end_inclusive, const uint8_t *query_mask)
{
    orc_keydeps_result *R = calloc(1, sizeof *R);
    keydeps_impl(R, n, tmsb, tlsb, tnode, emsb, elsb, enode, status, key_off, key_code, rng_off, rng_start, rng_end,
                 end_inclusive, 1, 0, n, 1, query_mask);
    return R;
}

static void keydeps_impl(orc_keydeps_result *R, uint32_t n,
                         const uint64_t *tmsb, const uint64_t *tlsb, const int32_t *tnode,
                         const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                         const uint8_t *status, const uint32_t *key_off, const uint64_t *key_code,
                         const uint32_t *rng_off, const uint64_t *rng_start, const uint64_t *rng_end, int end_inclusive,
                         uint32_t n_shards, uint32_t query_lo, uint32_t query_hi, uint32_t query_stride,
                         const uint8_t *qmask)
{
    double t_start = now_s();
    if (query_stride == 0) query_stride = 1;
    err E = { 0, "" };
    batch B = { n, malloc((n + 1) * sizeof(ts)), malloc((n + 1) * sizeof(ts)), status, key_off, key_code };
    for (uint32_t i = 0; i < n; ++i) {
        B.id[i] = (ts){ tmsb[i], tlsb[i], tnode[i] };
        B.ex[i] = (ts){ emsb[i], elsb[i], enode[i] };
    }
    if (n_shards == 0) n_shards = 1;
    if (query_hi > n) query_hi = n;
    uint64_t P = key_off[n];

    /* Input validation (what the reference would reject): Keys sorted unique per txn
     * (Keys.ofSortedUnique), valid kinds/statuses, TxnIds distinct (CFK txns sorted unique). */
    for (uint32_t t = 0; t < n && !E.code; ++t) {
        if (status[t] > ST_INVALID) set_err(&E, -1, "invalid InternalStatus ordinal");
        if (ts_kind(&B.id[t]) >= K_COUNT) set_err(&E, -1, "Kind.ofOrdinal: invalid kind ordinal");
        for (uint32_t j = key_off[t] + 1; j < key_off[t + 1]; ++j)
            if (key_code[j - 1] >= key_code[j]) set_err(&E, -1, "keys of a txn must be sorted and unique");
        if (rng_off) {
            int isr = (int)(tlsb[t] & 1);   /* TxnId.domain() (TxnId.java:134-157) */
            if (isr && key_off[t + 1] != key_off[t]) set_err(&E, -1, "a range txn cannot list keys");
            if (!isr && rng_off[t + 1] != rng_off[t]) set_err(&E, -1, "a key txn cannot list ranges");
            for (uint32_t j = rng_off[t]; j < rng_off[t + 1]; ++j) {
                if (rng_start[j] >= rng_end[j]) set_err(&E, -1, "range start must be below its end");
                if (j > rng_off[t] && rng_end[j - 1] > rng_start[j]) set_err(&E, -1, "ranges of a txn must be sorted and non-overlapping");
            }
        }
    }

    /* Group pairs by key -> one CommandsForKey per key (InMemoryCommandStore.commandsForKey). */
    int64_t *pidx = malloc((P + 1) * sizeof *pidx);
    for (uint64_t j = 0; j < P; ++j) pidx[j] = (int64_t)j;
    radix_sort_by_u64(pidx, P, key_code);   /* = stable_sort(pidx, P, cmp_pair_key, key_code) */
    int64_t *owner = malloc((P + 1) * sizeof *owner);
    for (uint32_t t = 0; t < n; ++t) for (uint32_t j = key_off[t]; j < key_off[t + 1]; ++j) owner[j] = t;
    size_t ncfk = 0, nkeys = 0;
    for (uint64_t s = 0; s < P; ++s) nkeys += s == 0 || key_code[pidx[s]] != key_code[pidx[s - 1]];
    cfk *cfks = calloc(nkeys + 1, sizeof *cfks);
    for (uint64_t s = 0; s < P; ) {
        uint64_t e2 = s;
        while (e2 < P && key_code[pidx[e2]] == key_code[pidx[s]]) ++e2;
        cfk *c = &cfks[ncfk++];
        c->key = key_code[pidx[s]];
        c->ntxns = e2 - s;
        c->txns = malloc(c->ntxns * sizeof *c->txns);
        for (uint64_t q = s; q < e2; ++q) c->txns[q - s] = owner[pidx[q]];
        cfk_init(c, &B);
        for (size_t q = 1; q < c->ntxns; ++q)
            if (ts_eq(&B.id[c->txns[q - 1]], &B.id[c->txns[q]]))
                set_err(&E, -1, "TxnIds of a batch must be distinct (CommandsForKey txns are sorted unique)");
        s = e2;
    }

    /* EvenSplit of the observed key-code domain into n_shards contiguous shards
     * (ShardDistributor.java:106-156). KeyDeps results are invariant to the split. */
    uint64_t klo = ncfk ? cfks[0].key : 0, khi = ncfk ? cfks[ncfk - 1].key : 0;
    unsigned __int128 span = (unsigned __int128)(khi - klo) + 1;
    uint64_t *shard_lo = malloc((n_shards + 1) * sizeof *shard_lo);
    for (uint32_t s = 0; s < n_shards; ++s) shard_lo[s] = klo + (uint64_t)(span * s / n_shards);

    R->build_s = now_s() - t_start;
    double t_query = now_s();
    R->n_txn = n;
    R->arena_off = calloc(n + 1, sizeof(uint64_t));
    R->kd_off = calloc(n + 1, sizeof(uint64_t));
    R->u_off = calloc(n + 1, sizeof(uint64_t));
    ivec arena = { 0 }, kidx = { 0 }, deps = { 0 }, kkey = { 0 };
    builder b; b_init(&b, &B);

    for (uint32_t t = 0; t < n && !E.code; ++t) {
        R->arena_off[t] = arena.n; R->kd_off[t] = kidx.n; R->u_off[t] = deps.n;
        if (t < query_lo || t >= query_hi || (t - query_lo) % query_stride) continue;
        if (qmask && !qmask[t]) continue;
        R->queried_pairs += key_off[t + 1] - key_off[t];
        int wk = kind_witnesses(ts_kind(&B.id[t]));
        if (wk < 0) { set_err(&E, -2, "Kind.witnesses(): unhandled kind (AssertionError)"); break; }
        /* p1 = executeAt.equals(txnId) ? null : txnId (PreAccept.java:259) */
        long p1 = ts_eq(&B.ex[t], &B.id[t]) ? -1 : (long)t;
        kdeps acc = { 0 };
        for (uint32_t sh = 0; sh < n_shards && !E.code; ++sh) {
            uint64_t lo = shard_lo[sh];
            int last = sh + 1 == n_shards;
            uint64_t hi = last ? 0 : shard_lo[sh + 1];
            b_reset(&b);
            /* InMemoryCommandStore.mapReduceForKey (:257-272): keys of T in this slice, ascending. */
            for (uint32_t j = key_off[t]; j < key_off[t + 1]; ++j) {
                uint64_t k = key_code[j];
                if (k < lo || (!last && k >= hi)) continue;
                size_t a = 0, z = ncfk;
                while (a < z) { size_t m = (a + z) / 2; if (cfks[m].key < k) a = m + 1; else z = m; }
                R->visited += cfk_map_reduce_active(&cfks[a], &B, &B.ex[t], (unsigned)wk, p1, &b, &E);
            }
            /* Range domain (:274-289): ranges.slice(store) in order, every CommandsForKey of the subMap. A range
             * txn is no CFK member (SafeCommandStore.updateCommandsForKey registers key txns only). */
            if (rng_off)
                for (uint32_t r = rng_off[t]; r < rng_off[t + 1]; ++r) {
                    size_t a = cfk_lower(cfks, ncfk, rng_start[r], end_inclusive);
                    size_t z = cfk_lower(cfks, ncfk, rng_end[r], end_inclusive);
                    for (size_t c = a; c < z; ++c) {
                        uint64_t k = cfks[c].key;
                        if (k < lo || (!last && k >= hi)) continue;
                        R->visited += cfk_map_reduce_active(&cfks[c], &B, &B.ex[t], (unsigned)wk, p1, &b, &E);
                    }
                }
            kdeps part; if (b_build(&b, &part, &E)) break;
            /* PreAccept.reduce -> PartialDeps.with -> KeyDeps.with (PreAccept.java:141-156) */
            kd_with(&acc, &part, cmp_vals_by_id, &B);
            kd_free(&part);
        }
        /* Emit in the ABI layout: key indices into T's keys, deps as batch indices. */
        for (size_t q = 0; q < acc.nk2v; ++q) iv_push(&arena, acc.k2v[q]);
        for (size_t q = 0; q < acc.nkeys; ++q) {
            iv_push(&kkey, (int64_t)acc.keys[q]);
            if (rng_off && rng_off[t + 1] > rng_off[t]) {
                /* range txn: index among the CFK keys its ranges cover, in range order */
                uint64_t idx = 0;
                for (uint32_t r = rng_off[t]; r < rng_off[t + 1]; ++r) {
                    size_t a = cfk_lower(cfks, ncfk, rng_start[r], end_inclusive);
                    size_t z = cfk_lower(cfks, ncfk, rng_end[r], end_inclusive);
                    if (z > a && cfks[z - 1].key >= acc.keys[q]) {
                        while (a < z) { size_t m = (a + z) / 2; if (cfks[m].key < acc.keys[q]) a = m + 1; else z = m; }
                        idx += a - cfk_lower(cfks, ncfk, rng_start[r], end_inclusive);
                        break;
                    }
                    idx += z - a;
                }
                iv_push(&kidx, (int64_t)idx);
                continue;
            }
            uint32_t a = key_off[t], z = key_off[t + 1];
            while (a < z) { uint32_t m = (a + z) / 2; if (key_code[m] < acc.keys[q]) a = m + 1; else z = m; }
            iv_push(&kidx, (int64_t)(a - key_off[t]));
        }
        for (size_t q = 0; q < acc.nvals; ++q) iv_push(&deps, acc.vals[q]);
        R->total_edges += acc.nk2v - acc.nkeys;
        kd_free(&acc);
    }
    R->arena_off[n] = arena.n; R->kd_off[n] = kidx.n; R->u_off[n] = deps.n;
    R->query_s = now_s() - t_query;
    R->arena = malloc((arena.n + 1) * sizeof(int32_t));
    for (size_t q = 0; q < arena.n; ++q) R->arena[q] = (int32_t)arena.v[q];
    R->key_idx = malloc((kidx.n + 1) * sizeof(uint32_t));
    for (size_t q = 0; q < kidx.n; ++q) R->key_idx[q] = (uint32_t)kidx.v[q];
    R->dep_txn = malloc((deps.n + 1) * sizeof(uint32_t));
    for (size_t q = 0; q < deps.n; ++q) R->dep_txn[q] = (uint32_t)deps.v[q];
    R->kd_key = malloc((kkey.n + 1) * sizeof(uint64_t));
    for (size_t q = 0; q < kkey.n; ++q) R->kd_key[q] = (uint64_t)kkey.v[q];
    R->error = E.code;
    snprintf(R->message, sizeof R->message, "%s", E.msg);

    b_free(&b);
    free(arena.v); free(kidx.v); free(deps.v); free(kkey.v);
    for (size_t c = 0; c < ncfk; ++c) { free(cfks[c].txns); free(cfks[c].committed); }
    free(cfks); free(pidx); free(owner); free(shard_lo); free(B.id); free(B.ex);
}

void orc_keydeps_free(orc_keydeps_result *r)
{
    if (!r) return;
    free(r->arena_off); free(r->arena); free(r->kd_off); free(r->key_idx); free(r->u_off); free(r->dep_txn);
    free(r->kd_key);
    free(r);
}

/* ------------------------------------------------------------------ KeyDeps.merge */

static int cmp_u32_rank(int64_t a, int64_t b, const void *c)
{
    (void)c; return a < b ? -1 : a > b;
}

/* KeyDeps.merge(List, getter, getter) (KeyDeps.java:115-135): skip null/empty, LinearMerger.update
 * folds linearUnion left to right (RelationMultiMap.java:333-373). Values are u32 TxnId ranks. */
orc_merge_result *orc_keydeps_merge(uint32_t n_groups, const uint64_t *grp_off,
                                    const uint64_t *key_off, const uint64_t *key_code,
                                    const uint64_t *val_off, const uint32_t *txn_rank,
                                    const uint64_t *k2v_off, const int32_t *k2v)
{
    orc_merge_result *R = calloc(1, sizeof *R);
    R->n_groups = n_groups;
    R->key_off = calloc(n_groups + 1, sizeof(uint64_t));
    R->val_off = calloc(n_groups + 1, sizeof(uint64_t));
    R->k2v_off = calloc(n_groups + 1, sizeof(uint64_t));
    ivec ok = { 0 }, ov = { 0 }, o = { 0 };
    for (uint32_t g = 0; g < n_groups; ++g) {
        kdeps acc = { 0 };
        for (uint64_t r = grp_off[g]; r < grp_off[g + 1]; ++r) {
            kdeps in;
            in.nkeys = key_off[r + 1] - key_off[r];
            if (k2v_off[r + 1] - k2v_off[r] == in.nkeys) continue;   /* deps.isEmpty() (KeyDeps.java:292-295) */
            in.keys = (uint64_t *)(key_code + key_off[r]);
            in.nvals = val_off[r + 1] - val_off[r];
            in.vals = malloc((in.nvals + 1) * sizeof *in.vals);
            for (size_t q = 0; q < in.nvals; ++q) in.vals[q] = txn_rank[val_off[r] + q];
            in.nk2v = k2v_off[r + 1] - k2v_off[r];
            in.k2v = (int32_t *)(k2v + k2v_off[r]);
            /* KeyDeps ctor check (KeyDeps.java:184-185) */
            if ((uint64_t)in.k2v[in.nkeys - 1] != in.nk2v && !R->error) {
                R->error = -1; snprintf(R->message, sizeof R->message, "Last key in keyToTxnId does not point to the end of the array");
            }
            kd_with(&acc, &in, cmp_u32_rank, NULL);
            free(in.vals);
        }
        R->key_off[g] = ok.n; R->val_off[g] = ov.n; R->k2v_off[g] = o.n;
        for (size_t q = 0; q < acc.nkeys; ++q) iv_push(&ok, (int64_t)acc.keys[q]);
        for (size_t q = 0; q < acc.nvals; ++q) iv_push(&ov, acc.vals[q]);
        for (size_t q = 0; q < acc.nk2v; ++q) iv_push(&o, acc.k2v[q]);
        kd_free(&acc);
    }
    R->key_off[n_groups] = ok.n; R->val_off[n_groups] = ov.n; R->k2v_off[n_groups] = o.n;
    R->key_code = malloc((ok.n + 1) * sizeof(uint64_t));
    for (size_t q = 0; q < ok.n; ++q) R->key_code[q] = (uint64_t)ok.v[q];
    R->txn_rank = malloc((ov.n + 1) * sizeof(uint32_t));
    for (size_t q = 0; q < ov.n; ++q) R->txn_rank[q] = (uint32_t)ov.v[q];
    R->k2v = malloc((o.n + 1) * sizeof(int32_t));
    for (size_t q = 0; q < o.n; ++q) R->k2v[q] = (int32_t)o.v[q];
    free(ok.v); free(ov.v); free(o.v);
    return R;
}

void orc_merge_free(orc_merge_result *r)
{
    if (!r) return;
    free(r->key_off); free(r->key_code); free(r->val_off); free(r->txn_rank); free(r->k2v_off); free(r->k2v);
    free(r);
}

/* ------------------------------------------------------------------ levelisation */

static int cmp_exec_rank(int64_t a, int64_t b, const void *c)
{
    const uint32_t *er = c; return er[a] < er[b] ? -1 : er[a] > er[b];
}
typedef struct lvl_ctx { const uint32_t *level, *exec_rank; } lvl_ctx;
static int cmp_level_order(int64_t a, int64_t b, const void *c)
{
    const lvl_ctx *L = c;
    if (L->level[a] != L->level[b]) return L->level[a] < L->level[b] ? -1 : 1;
    if (L->exec_rank[a] != L->exec_rank[b]) return L->exec_rank[a] < L->exec_rank[b] ? -1 : 1;
    return a < b ? -1 : a > b;
}

/* A txn waits on each dep whose executeAt is earlier than its own (Commands.updateWaitingOn
 * drops deps with a later executeAt, Commands.java:804-810). level = 0 without such deps, else
 * 1 + max(level of dep). Processing in executeAt order makes every dep's level final first. */
int orc_levelise(uint32_t n, const uint64_t *off, const uint32_t *dep, const uint32_t *exec_rank,
                 uint32_t *level, uint32_t *order, uint32_t *n_levels)
{
    int64_t *idx = malloc((n + 1) * sizeof *idx);
    for (uint32_t i = 0; i < n; ++i) idx[i] = i;
    stable_sort(idx, n, cmp_exec_rank, exec_rank);
    uint32_t maxl = 0;
    for (uint32_t q = 0; q < n; ++q) {
        uint32_t t = (uint32_t)idx[q], l = 0;
        for (uint64_t e = off[t]; e < off[t + 1]; ++e) {
            uint32_t d = dep[e];
            if (d >= n) { free(idx); return -1; }
            if (exec_rank[d] < exec_rank[t] && level[d] + 1 > l) l = level[d] + 1;
        }
        level[t] = l;
        if (l + 1 > maxl) maxl = l + 1;
    }
    for (uint32_t i = 0; i < n; ++i) idx[i] = i;
    lvl_ctx L = { level, exec_rank };
    stable_sort(idx, n, cmp_level_order, &L);
    for (uint32_t i = 0; i < n; ++i) order[i] = (uint32_t)idx[i];
    *n_levels = n ? maxl : 0;
    free(idx);
    return 0;
}

/* ------------------------------------------------------------------ RangeDeps (range commands) */

/* TxnId.domain(): flags & 1, Key = 0, Range = 1 (TxnId.java:134-157, Routable.Domain ordinals) */
static inline int ts_is_range(const ts *t) { return (int)(t->lsb & 1); }

typedef struct rng_dict { const uint64_t *s, *e; } rng_dict;
static int cmp_range(int64_t a, int64_t b, const void *c)
{
    /* Range.compare (Range.java:309-317): by start, then end */
    const rng_dict *D = c;
    if (D->s[a] != D->s[b]) return D->s[a] < D->s[b] ? -1 : 1;
    if (D->e[a] != D->e[b]) return D->e[a] < D->e[b] ? -1 : 1;
    return 0;
}

/* Range.contains(key) for the two bound types (Range.java:40-138): EndInclusive (s, e], StartInclusive [s, e) */
static inline int range_contains(uint64_t s, uint64_t e, uint64_t k, int end_inclusive)
{
    return end_inclusive ? (s < k && k <= e) : (s <= k && k < e);
}
/* Range.compareIntersecting == 0 (Range.java:296-305) */
static inline int ranges_intersect(uint64_t as, uint64_t ae, uint64_t bs, uint64_t be)
{
    return as < be && ae > bs;
}

typedef struct rd_item { int64_t rid, txn; } rd_item;
typedef struct rd_ctx { const batch *B; const rd_item *it; } rd_ctx;
static int cmp_rd_item(int64_t a, int64_t b, const void *c)
{
    /* TreeMap<Range, List> by Range::compare, lists in the order range commands are visited (TxnId) */
    const rd_ctx *X = c;
    if (X->it[a].rid != X->it[b].rid) return X->it[a].rid < X->it[b].rid ? -1 : 1;
    return ts_cmp(&X->B->id[X->it[a].txn], &X->B->id[X->it[b].txn]);
}

static orc_rangedeps_result *rangedeps_impl(uint32_t n,
                                          const uint64_t *tmsb, const uint64_t *tlsb, const int32_t *tnode,
                                          const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                                          const uint8_t *status, const uint32_t *key_off, const uint64_t *key_code,
                                          const uint32_t *rng_off, const uint64_t *rng_start, const uint64_t *rng_end,
                                          int end_inclusive, uint32_t query_lo, uint32_t query_hi, uint32_t query_stride,
                                          const uint8_t *qmask);

orc_rangedeps_result *orc_rangedeps_batch(uint32_t n,
                                          const uint64_t *tmsb, const uint64_t *tlsb, const int32_t *tnode,
                                          const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                                          const uint8_t *status, const uint32_t *key_off, const uint64_t *key_code,
                                          const uint32_t *rng_off, const uint64_t *rng_start, const uint64_t *rng_end,
                                          int end_inclusive, uint32_t query_lo, uint32_t query_hi, uint32_t query_stride)
{
    return rangedeps_impl(n, tmsb, tlsb, tnode, emsb, elsb, enode, status, key_off, key_code, rng_off, rng_start,
                          rng_end, end_inclusive, query_lo, query_hi, query_stride, NULL);
}

orc_rangedeps_result *orc_rangedeps_batch_qmask(uint32_t n,
                                                const uint64_t *tmsb, const uint64_t *tlsb, const int32_t *tnode,
                                                const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                                                const uint8_t *status, const uint32_t *key_off, const uint64_t *key_code,
                                                const uint32_t *rng_off, const uint64_t *rng_start,
                                                const uint64_t *rng_end, int end_inclusive, const uint8_t *query_mask)
{
    return rangedeps_impl(n, tmsb, tlsb, tnode, emsb, elsb, enode, status, key_off, key_code, rng_off, rng_start,
                          rng_end, end_inclusive, 0, n, 1, query_mask);
}

static orc_rangedeps_result *rangedeps_impl(uint32_t n,
                                          const uint64_t *tmsb, const uint64_t *tlsb, const int32_t *tnode,
                                          const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                                          const uint8_t *status, const uint32_t *key_off, const uint64_t *key_code,
                                          const uint32_t *rng_off, const uint64_t *rng_start, const uint64_t *rng_end,
                                          int end_inclusive, uint32_t query_lo, uint32_t query_hi, uint32_t query_stride,
                                          const uint8_t *qmask)
{
    orc_rangedeps_result *R = calloc(1, sizeof *R);
    if (query_stride == 0) query_stride = 1;
    if (query_hi > n) query_hi = n;
    err E = { 0, "" };
    batch B = { n, malloc((n + 1) * sizeof(ts)), malloc((n + 1) * sizeof(ts)), status, key_off, key_code };
    for (uint32_t i = 0; i < n; ++i) {
        B.id[i] = (ts){ tmsb[i], tlsb[i], tnode[i] };
        B.ex[i] = (ts){ emsb[i], elsb[i], enode[i] };
    }
    /* validation: Keys / Ranges of a txn sorted and deoverlapped (Keys.ofSortedUnique,
     * Ranges.ofSortedAndDeoverlapped), start < end, a txn's participants match its domain */
    for (uint32_t t = 0; t < n && !E.code; ++t) {
        if (status[t] > ST_INVALID) set_err(&E, -1, "invalid InternalStatus ordinal");
        if (ts_kind(&B.id[t]) >= K_COUNT) set_err(&E, -1, "Kind.ofOrdinal: invalid kind ordinal");
        int isr = ts_is_range(&B.id[t]);
        if (isr && key_off[t + 1] != key_off[t]) set_err(&E, -1, "a range txn cannot list keys");
        if (!isr && rng_off[t + 1] != rng_off[t]) set_err(&E, -1, "a key txn cannot list ranges");
        for (uint32_t j = key_off[t] + 1; j < key_off[t + 1]; ++j)
            if (key_code[j - 1] >= key_code[j]) set_err(&E, -1, "keys of a txn must be sorted and unique");
        for (uint32_t j = rng_off[t]; j < rng_off[t + 1]; ++j) {
            if (rng_start[j] >= rng_end[j]) set_err(&E, -1, "range start must be below its end");
            if (j > rng_off[t] && rng_end[j - 1] > rng_start[j]) set_err(&E, -1, "ranges of a txn must be sorted and non-overlapping");
        }
    }
    /* Range commands (InMemoryCommandStore.rangeCommands, a TreeMap by TxnId): range-domain txns whose
     * saveStatus is below Erased (INVALID here is the erased/invalidated class), in TxnId order. */
    ivec cmds = { 0 };
    for (uint32_t t = 0; t < n; ++t)
        if (ts_is_range(&B.id[t]) && status[t] != ST_INVALID && rng_off[t + 1] > rng_off[t]) iv_push(&cmds, t);
    stable_sort(cmds.v, cmds.n, cmp_txn_by_id, &B);
    for (size_t q = 1; q < cmds.n && !E.code; ++q)
        if (ts_eq(&B.id[cmds.v[q - 1]], &B.id[cmds.v[q]])) set_err(&E, -1, "TxnIds of a batch must be distinct");
    /* dictionary of the distinct stored ranges in Range::compare order */
    ivec all = { 0 };
    for (size_t q = 0; q < cmds.n; ++q)
        for (uint32_t j = rng_off[cmds.v[q]]; j < rng_off[cmds.v[q] + 1]; ++j) iv_push(&all, j);
    rng_dict D = { rng_start, rng_end };
    stable_sort(all.v, all.n, cmp_range, &D);
    size_t nd = 0;
    uint64_t *ds = malloc((all.n + 1) * sizeof *ds), *de = malloc((all.n + 1) * sizeof *de);
    int64_t *rid_of = malloc((rng_off[n] + 1) * sizeof *rid_of);
    for (size_t q = 0; q < all.n; ++q) {
        uint64_t s = rng_start[all.v[q]], e = rng_end[all.v[q]];
        if (nd == 0 || ds[nd - 1] != s || de[nd - 1] != e) { ds[nd] = s; de[nd] = e; ++nd; }
        rid_of[all.v[q]] = (int64_t)nd - 1;
    }
    R->n_txn = n; R->n_ranges = (uint32_t)nd; R->rng_start = ds; R->rng_end = de;
    R->arena_off = calloc(n + 1, sizeof(uint64_t));
    R->rd_off = calloc(n + 1, sizeof(uint64_t));
    R->u_off = calloc(n + 1, sizeof(uint64_t));
    ivec arena = { 0 }, rids = { 0 }, deps = { 0 };
    builder b; b_init(&b, &B);
    rd_item *items = NULL; size_t items_cap = 0;
    int64_t *order = NULL; size_t order_cap = 0;
    double t_query = now_s();
    for (uint32_t t = 0; t < n && !E.code; ++t) {
        R->arena_off[t] = arena.n; R->rd_off[t] = rids.n; R->u_off[t] = deps.n;
        if (t < query_lo || t >= query_hi || (t - query_lo) % query_stride) continue;
        if (qmask && !qmask[t]) continue;
        ++R->queried;
        int wk = kind_witnesses(ts_kind(&B.id[t]));
        if (wk < 0) { set_err(&E, -2, "Kind.witnesses(): unhandled kind (AssertionError)"); break; }
        long p1 = ts_eq(&B.ex[t], &B.id[t]) ? -1 : (long)t;   /* PreAccept.java:259 */
        const int isr = ts_is_range(&B.id[t]);
        size_t ni = 0;
        /* commandStore.rangeCommands.forEach (:888-960) */
        for (size_t q = 0; q < cmds.n; ++q) {
            int64_t c = cmds.v[q];
            ++R->visited;
            if (ts_cmp(&B.id[c], &B.ex[t]) >= 0) continue;                 /* STARTED_BEFORE (:897-898) */
            if (!(((unsigned)wk >> ts_kind(&B.id[c])) & 1u)) continue;     /* testKind (:926-927) */
            /* Routables.foldl(rangeCommand.ranges, sliced, ...) (:950-959): each of C's ranges that
             * intersects T's keys (Range.contains) or T's ranges (compareIntersecting) */
            for (uint32_t j = rng_off[c]; j < rng_off[c + 1]; ++j) {
                int hit = 0;
                if (isr) {
                    for (uint32_t u = rng_off[t]; u < rng_off[t + 1] && !hit; ++u)
                        hit = ranges_intersect(rng_start[j], rng_end[j], rng_start[u], rng_end[u]);
                } else {
                    for (uint32_t u = key_off[t]; u < key_off[t + 1] && !hit; ++u)
                        hit = range_contains(rng_start[j], rng_end[j], key_code[u], end_inclusive);
                }
                if (!hit) continue;
                if (ni == items_cap) { items_cap = items_cap ? 2 * items_cap : 64; items = realloc(items, items_cap * sizeof *items); }
                items[ni++] = (rd_item){ rid_of[j], c };
            }
        }
        /* TreeMap iteration: Range order, then the per-range list in visit (TxnId) order; the list
         * dedupes consecutive equal TxnIds (:953-955) */
        if (ni > order_cap) { order_cap = ni; order = realloc(order, order_cap * sizeof *order); }
        for (size_t q = 0; q < ni; ++q) order[q] = (int64_t)q;
        rd_ctx X = { &B, items };
        stable_sort(order, ni, cmp_rd_item, &X);
        b_reset(&b);
        for (size_t q = 0; q < ni; ++q) {
            const rd_item *it = &items[order[q]];
            if (q > 0 && items[order[q - 1]].rid == it->rid && items[order[q - 1]].txn == it->txn) continue;
            /* calculatePartialDeps map: skip p1 (PreAccept.java:253-259) -> RangeDeps.Builder.add */
            if (p1 >= 0 && ts_eq(&B.id[it->txn], &B.id[p1])) continue;
            b_add(&b, (uint64_t)it->rid, it->txn);
        }
        kdeps part; if (b_build(&b, &part, &E)) break;
        for (size_t q = 0; q < part.nk2v; ++q) iv_push(&arena, part.k2v[q]);
        for (size_t q = 0; q < part.nkeys; ++q) iv_push(&rids, (int64_t)part.keys[q]);
        for (size_t q = 0; q < part.nvals; ++q) iv_push(&deps, part.vals[q]);
        R->total_edges += part.nk2v - part.nkeys;
        kd_free(&part);
    }
    R->arena_off[n] = arena.n; R->rd_off[n] = rids.n; R->u_off[n] = deps.n;
    R->query_s = now_s() - t_query;
    R->arena = malloc((arena.n + 1) * sizeof(int32_t));
    for (size_t q = 0; q < arena.n; ++q) R->arena[q] = (int32_t)arena.v[q];
    R->range_id = malloc((rids.n + 1) * sizeof(uint32_t));
    for (size_t q = 0; q < rids.n; ++q) R->range_id[q] = (uint32_t)rids.v[q];
    R->dep_txn = malloc((deps.n + 1) * sizeof(uint32_t));
    for (size_t q = 0; q < deps.n; ++q) R->dep_txn[q] = (uint32_t)deps.v[q];
    R->error = E.code;
    snprintf(R->message, sizeof R->message, "%s", E.msg);
    b_free(&b);
    free(items); free(order); free(arena.v); free(rids.v); free(deps.v); free(cmds.v); free(all.v); free(rid_of);
    free(B.id); free(B.ex);
    return R;
}

void orc_rangedeps_free(orc_rangedeps_result *r)
{
    if (!r) return;
    free(r->rng_start); free(r->rng_end); free(r->arena_off); free(r->arena); free(r->rd_off); free(r->range_id);
    free(r->u_off); free(r->dep_txn);
    free(r);
}

/* ------------------------------------------------------------------ recovery scan (mapReduceFull) */

/* Kind.witnessedBy() (Txn.java:247-262) as a Kinds mask; -1 where it throws (LocalOnly, invalid ordinals). */
static int kind_witnessed_by(int kind)
{
    switch (kind) {
    case K_EREAD:              return 0;                                                   /* Nothing */
    case K_READ:               return (1 << K_WRITE) | (1 << K_SYNC) | (1 << K_XSYNC);     /* WsOrSyncPoints */
    case K_WRITE:              return (int)KINDS_ANY_VISIBLE;                              /* AnyGloballyVisible */
    case K_SYNC: case K_XSYNC: return 1 << K_XSYNC;                                        /* ExclusiveSyncPoints */
    default:                   return -1;
    }
}

/* java.util.Arrays.binarySearch over a TxnId-sorted list of batch indices: found? */
static int txn_list_contains(const batch *B, const uint32_t *list, size_t nl, const ts *key)
{
    long low = 0, high = (long)nl - 1;
    while (low <= high) {
        long mid = (long)(((unsigned long)low + (unsigned long)high) >> 1);
        int c = ts_cmp(&B->id[list[mid]], key);
        if (c < 0) low = mid + 1;
        else if (c > 0) high = mid - 1;
        else return 1;
    }
    return 0;
}

/* CommandsForKey.mapReduceFull (CommandsForKey.java:553-612) for one key, feeding a Deps.Builder with the map
 * functions of BeginRecovery (messages/BeginRecovery.java:334-378): every visited txn is added, or (exec_after) only
 * those with executeAt > testTxnId. missing(t) = the TxnInfoWithMissing.missing of this CFK's entry for t. */
static void cfk_map_reduce_full(const cfk *c, const batch *B, const ts *test, unsigned test_kinds, int started_at,
                                int test_dep, int test_status, int exec_after, const uint32_t *miss_off,
                                const uint32_t *miss_txn, builder *b)
{
    /* Arrays.binarySearch(txns, testTxnId) */
    long low = 0, high = (long)c->ntxns - 1, found = -1;
    while (low <= high) {
        long mid = (long)(((unsigned long)low + (unsigned long)high) >> 1);
        int cc = ts_cmp(&B->id[c->txns[mid]], test);
        if (cc < 0) low = mid + 1;
        else if (cc > 0) high = mid - 1;
        else { found = mid; break; }
    }
    int is_known = found >= 0;
    if (!is_known && test_dep == 0 /* WITH */) return;
    long insert_pos = is_known ? found : low;
    long start, end;
    switch (started_at) {
    case 0:  start = 0; end = insert_pos; break;                     /* STARTED_BEFORE */
    case 1:  start = insert_pos; end = (long)c->ntxns; break;        /* STARTED_AFTER */
    default: start = 0; end = (long)c->ntxns; break;                 /* ANY */
    }
    for (long i = start; i < end; ++i) {
        int64_t t = c->txns[i];
        int kind = ts_kind(&B->id[t]);
        if (!((test_kinds >> kind) & 1u)) continue;
        int s = B->status[t];
        switch (test_status) {
        case 1: if (s == ST_ACC || s == ST_COMMITTED) break; else continue;       /* IS_PROPOSED */
        case 2: if (s >= ST_STABLE && s < ST_INVALID) break; else continue;       /* IS_STABLE */
        default: if (s == ST_TK) continue; break;                                 /* ANY_STATUS */
        }
        const ts *ex = &B->ex[t];
        if (test_dep != 2 /* ANY_DEPS */) {
            int has_info = s >= ST_ACC && s <= ST_APPLIED;                         /* InternalStatus.hasInfo */
            if (!has_info) continue;
            if (ts_cmp(ex, test) <= 0) continue;
            /* the pair (t, key) of this CFK: t's keys are sorted, so a binary search finds it */
            uint32_t a = B->key_off[t], z = B->key_off[t + 1];
            while (a < z) { uint32_t m = (a + z) / 2; if (B->key_code[m] < c->key) a = m + 1; else z = m; }
            int has_as_dep = !txn_list_contains(B, miss_txn + miss_off[a], miss_off[a + 1] - miss_off[a], test);
            if (has_as_dep != (test_dep == 0)) continue;
        }
        if (exec_after && ts_cmp(ex, test) <= 0) continue;
        b_add(b, c->key, t);
    }
}

orc_keydeps_result *orc_map_reduce_full(uint32_t n,
                                        const uint64_t *tmsb, const uint64_t *tlsb, const int32_t *tnode,
                                        const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                                        const uint8_t *status, const uint32_t *key_off, const uint64_t *key_code,
                                        const uint32_t *miss_off, const uint32_t *miss_txn,
                                        uint32_t nq, const uint64_t *qmsb, const uint64_t *qlsb, const int32_t *qnode,
                                        const uint32_t *qkey_off, const uint64_t *qkey_code,
                                        int started_at, int test_dep, int test_status, int test_kinds, int exec_after)
{
    orc_keydeps_result *R = calloc(1, sizeof *R);
    double t0 = now_s();
    err E = { 0, "" };
    batch B = { n, malloc((n + 1) * sizeof(ts)), malloc((n + 1) * sizeof(ts)), status, key_off, key_code };
    for (uint32_t i = 0; i < n; ++i) {
        B.id[i] = (ts){ tmsb[i], tlsb[i], tnode[i] };
        B.ex[i] = (ts){ emsb[i], elsb[i], enode[i] };
        if (status[i] > ST_INVALID) set_err(&E, -1, "invalid InternalStatus ordinal");
    }
    uint64_t P = n ? key_off[n] : 0;
    for (uint64_t j = 0; j < P && !E.code; ++j)
        for (uint32_t x = miss_off[j]; x < miss_off[j + 1]; ++x) {
            if (miss_txn[x] >= n) { set_err(&E, -1, "missing[] entry is not a batch txn"); break; }
            if (x > miss_off[j] && ts_cmp(&B.id[miss_txn[x - 1]], &B.id[miss_txn[x]]) >= 0) {
                set_err(&E, -1, "missing[] must be sorted unique by TxnId"); break;
            }
        }
    int64_t *pidx = malloc((P + 1) * sizeof *pidx);
    for (uint64_t j = 0; j < P; ++j) pidx[j] = (int64_t)j;
    radix_sort_by_u64(pidx, P, key_code);
    size_t ncfk = 0, nkeys = 0;
    for (uint64_t s = 0; s < P; ++s) nkeys += s == 0 || key_code[pidx[s]] != key_code[pidx[s - 1]];
    cfk *cfks = calloc(nkeys + 1, sizeof *cfks);
    int64_t *owner = malloc((P + 1) * sizeof *owner);
    for (uint32_t t = 0; t < n; ++t) for (uint32_t j = key_off[t]; j < key_off[t + 1]; ++j) owner[j] = t;
    for (uint64_t s = 0; s < P; ) {
        uint64_t e2 = s;
        while (e2 < P && key_code[pidx[e2]] == key_code[pidx[s]]) ++e2;
        cfk *c = &cfks[ncfk++];
        c->key = key_code[pidx[s]];
        c->ntxns = e2 - s;
        c->txns = malloc(c->ntxns * sizeof *c->txns);
        for (uint64_t q = s; q < e2; ++q) c->txns[q - s] = owner[pidx[q]];
        cfk_init(c, &B);
        s = e2;
    }
    R->build_s = now_s() - t0;
    double t1 = now_s();
    R->n_txn = nq;
    R->arena_off = calloc(nq + 1, sizeof(uint64_t));
    R->kd_off = calloc(nq + 1, sizeof(uint64_t));
    R->u_off = calloc(nq + 1, sizeof(uint64_t));
    ivec arena = { 0 }, kidx = { 0 }, deps = { 0 };
    builder b; b_init(&b, &B);
    for (uint32_t q = 0; q < nq && !E.code; ++q) {
        R->arena_off[q] = arena.n; R->kd_off[q] = kidx.n; R->u_off[q] = deps.n;
        ts test = { qmsb[q], qlsb[q], qnode[q] };
        int kinds = test_kinds >= 0 ? test_kinds : kind_witnessed_by(ts_kind(&test));
        if (kinds < 0) { set_err(&E, -2, "Kind.witnessedBy(): unhandled kind (AssertionError)"); break; }
        for (uint32_t j = qkey_off[q] + 1; j < qkey_off[q + 1]; ++j)
            if (qkey_code[j - 1] >= qkey_code[j]) set_err(&E, -1, "keys of a query must be sorted and unique");
        b_reset(&b);
        for (uint32_t j = qkey_off[q]; j < qkey_off[q + 1] && !E.code; ++j) {
            size_t a = 0, z = ncfk;
            while (a < z) { size_t m = (a + z) / 2; if (cfks[m].key < qkey_code[j]) a = m + 1; else z = m; }
            if (a == ncfk || cfks[a].key != qkey_code[j]) continue;     /* no CommandsForKey for this key */
            ++R->queried_pairs;
            cfk_map_reduce_full(&cfks[a], &B, &test, (unsigned)kinds, started_at, test_dep, test_status, exec_after,
                                miss_off, miss_txn, &b);
        }
        kdeps d; if (b_build(&b, &d, &E)) break;
        for (size_t x = 0; x < d.nk2v; ++x) iv_push(&arena, d.k2v[x]);
        for (size_t x = 0; x < d.nkeys; ++x) {
            uint32_t a = qkey_off[q], z = qkey_off[q + 1];
            while (a < z) { uint32_t m = (a + z) / 2; if (qkey_code[m] < d.keys[x]) a = m + 1; else z = m; }
            iv_push(&kidx, (int64_t)(a - qkey_off[q]));
        }
        for (size_t x = 0; x < d.nvals; ++x) iv_push(&deps, d.vals[x]);
        R->total_edges += d.nk2v - d.nkeys;
        kd_free(&d);
    }
    R->arena_off[nq] = arena.n; R->kd_off[nq] = kidx.n; R->u_off[nq] = deps.n;
    R->query_s = now_s() - t1;
    R->arena = malloc((arena.n + 1) * sizeof(int32_t));
    for (size_t x = 0; x < arena.n; ++x) R->arena[x] = (int32_t)arena.v[x];
    R->key_idx = malloc((kidx.n + 1) * sizeof(uint32_t));
    for (size_t x = 0; x < kidx.n; ++x) R->key_idx[x] = (uint32_t)kidx.v[x];
    R->dep_txn = malloc((deps.n + 1) * sizeof(uint32_t));
    for (size_t x = 0; x < deps.n; ++x) R->dep_txn[x] = (uint32_t)deps.v[x];
    R->error = E.code;
    snprintf(R->message, sizeof R->message, "%s", E.msg);
    b_free(&b);
    free(arena.v); free(kidx.v); free(deps.v);
    for (size_t c = 0; c < ncfk; ++c) { free(cfks[c].txns); free(cfks[c].committed); }
    free(cfks); free(pidx); free(owner); free(B.id); free(B.ex);
    return R;
}

/* ------------------------------------------------------------------ recovery scan, range-command half */

/* Status ordinals (local/Status.java:47-86) */
enum { S_ACCEPTED = 3, S_PRECOMMITTED = 4, S_COMMITTED = 5, S_STABLE = 6, S_TRUNCATED = 9, S_MAX = 10 };
enum { RC_ERASED = 1, RC_HAS_DEPS = 2, RC_HISTORICAL = 4 };

typedef struct rr_table {
    const batch *B;                 /* id = TxnId, ex = executeAt of each entry */
    const uint8_t *status, *flags;
    const uint32_t *rng_off; const uint64_t *rs, *re;
    const uint32_t *dep_off; const ts *dep; const uint64_t *ds, *de; const uint8_t *dk;
    int ei;
} rr_table;

/* Deps.intersects(X, ranges) (primitives/Deps.java:112-115): KeyDeps.intersects (KeyDeps.java:266-285) - a key of
 * X's KeyDeps entries inside one of the ranges - or RangeDeps.intersects (RangeDeps.java:468-495) - a range of X's
 * RangeDeps entries intersecting one of them; over the command's PartialDeps flattened to (TxnId, participant) pairs */
static int rr_deps_intersects(const rr_table *T, uint32_t c, const ts *x)
{
    for (uint32_t j = T->dep_off[c]; j < T->dep_off[c + 1]; ++j) {
        if (!ts_eq(&T->dep[j], x)) continue;
        for (uint32_t r = T->rng_off[c]; r < T->rng_off[c + 1]; ++r) {
            if (T->dk[j] ? range_contains(T->rs[r], T->re[r], T->ds[j], T->ei)
                         : ranges_intersect(T->rs[r], T->re[r], T->ds[j], T->de[j]))
                return 1;
        }
    }
    return 0;
}

/* does range (s, e) intersect the sliced participants of the query (Routables.foldl(rangeCommand.ranges, sliced)) */
static int rr_hits(uint64_t s, uint64_t e, int is_range, const uint64_t *ps, const uint64_t *pe, uint32_t p0, uint32_t p1, int ei)
{
    for (uint32_t u = p0; u < p1; ++u)
        if (is_range ? ranges_intersect(s, e, ps[u], pe[u]) : range_contains(s, e, ps[u], ei)) return 1;
    return 0;
}

typedef struct rr_item { int64_t rid, seq, c; ts ex; } rr_item;
static int cmp_rr_item(int64_t a, int64_t b, const void *ctx)
{
    const rr_item *it = ctx;
    if (it[a].rid != it[b].rid) return it[a].rid < it[b].rid ? -1 : 1;
    return it[a].seq < it[b].seq ? -1 : it[a].seq > it[b].seq;
}

/* InMemorySafeStore.mapReduceRangesInternal (impl/InMemoryCommandStore.java:883-1016) for each recovery query, into a
 * Deps.Builder with the map functions of BeginRecovery (messages/BeginRecovery.java:334-378): every visited
 * (range, TxnId) is added, or (exec_after) only those with executeAt > testTxnId. The table holds the rangeCommands
 * entries and, flagged historical, the historicalRangeCommands entries, sorted by TxnId. */
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
                                                 int started_at, int test_dep, int test_status, int test_kinds, int exec_after)
{
    orc_rangedeps_result *R = calloc(1, sizeof *R);
    err E = { 0, "" };
    batch B = { n, malloc((n + 1) * sizeof(ts)), malloc((n + 1) * sizeof(ts)), NULL, NULL, NULL };
    for (uint32_t i = 0; i < n; ++i) {
        B.id[i] = (ts){ tmsb[i], tlsb[i], tnode[i] };
        B.ex[i] = (ts){ emsb[i], elsb[i], enode[i] };
        if (status[i] > S_MAX || (flags[i] & ~7u)) set_err(&E, -1, "invalid Status ordinal or flags");
        if (i > 0 && ts_cmp(&B.id[i - 1], &B.id[i]) > 0) set_err(&E, -1, "the range-command table must be sorted by TxnId");
    }
    const uint64_t ND = n ? dep_off[n] : 0;
    ts *dep = malloc((ND + 1) * sizeof *dep);
    for (uint64_t j = 0; j < ND; ++j) dep[j] = (ts){ dmsb[j], dlsb[j], dnode[j] };
    rr_table T = { &B, status, flags, rng_off, rng_start, rng_end, dep_off, dep, dep_start, dep_end, dep_is_key, end_inclusive };
    /* first table index of each TxnId (the reported dependency) */
    int64_t *first = malloc((n + 1) * sizeof *first);
    for (uint32_t i = 0; i < n; ++i) first[i] = (i > 0 && ts_eq(&B.id[i - 1], &B.id[i])) ? first[i - 1] : (int64_t)i;
    /* the distinct ranges of the table in Range::compare order */
    const uint64_t NR = n ? rng_off[n] : 0;
    int64_t *all = malloc((NR + 1) * sizeof *all);
    for (uint64_t j = 0; j < NR; ++j) all[j] = (int64_t)j;
    rng_dict D = { rng_start, rng_end };
    stable_sort(all, NR, cmp_range, &D);
    uint64_t *ds = malloc((NR + 1) * sizeof *ds), *de = malloc((NR + 1) * sizeof *de);
    int64_t *rid_of = malloc((NR + 1) * sizeof *rid_of);
    size_t nd = 0;
    for (uint64_t q = 0; q < NR; ++q) {
        uint64_t s = rng_start[all[q]], e = rng_end[all[q]];
        if (nd == 0 || ds[nd - 1] != s || de[nd - 1] != e) { ds[nd] = s; de[nd] = e; ++nd; }
        rid_of[all[q]] = (int64_t)nd - 1;
    }
    R->n_txn = nq; R->n_ranges = (uint32_t)nd; R->rng_start = ds; R->rng_end = de;
    R->arena_off = calloc(nq + 1, sizeof(uint64_t));
    R->rd_off = calloc(nq + 1, sizeof(uint64_t));
    R->u_off = calloc(nq + 1, sizeof(uint64_t));
    ivec arena = { 0 }, rids = { 0 }, deps = { 0 };
    builder b; b_init(&b, &B);
    rr_item *items = NULL; size_t items_cap = 0;
    int64_t *order = NULL; size_t order_cap = 0;
    int64_t *last = malloc((nd + 1) * sizeof *last);   /* per range: table index of its list's last TxnInfo */
    for (uint32_t q = 0; q < nq && !E.code; ++q) {
        R->arena_off[q] = arena.n; R->rd_off[q] = rids.n; R->u_off[q] = deps.n;
        const ts x = { qmsb[q], qlsb[q], qnode[q] };
        int kinds = test_kinds >= 0 ? test_kinds : kind_witnessed_by(ts_kind(&x));
        if (kinds < 0) { set_err(&E, ts_kind(&x) == K_LOCAL ? -2 : -1, "Kind.witnessedBy(): unhandled kind"); break; }
        const uint32_t p0 = part_off[q], p1 = part_off[q + 1];
        const int isr = part_is_range[q];
        for (size_t r = 0; r < nd; ++r) last[r] = -1;
        size_t ni = 0;
        for (int pass = 0; pass < 2; ++pass) {
            /* pass 0: commandStore.rangeCommands.forEach (:888-960); pass 1: historicalRangeCommands (:962-1004) */
            if (pass == 1 && !(test_status == 0 && test_dep == 2)) break;
            for (uint32_t c = 0; c < n; ++c) {
                const int hist = (flags[c] & RC_HISTORICAL) != 0;
                if (hist != pass) continue;
                const ts *id = &B.id[c];
                if (!hist) {
                    if (flags[c] & RC_ERASED) continue;                            /* saveStatus >= Erased */
                    int skip = 0;
                    switch (started_at) {
                    case 1: skip = ts_cmp(id, &x) <= 0; break;                     /* STARTED_AFTER */
                    case 0: if (ts_cmp(id, &x) >= 0) { skip = 1; break; }         /* STARTED_BEFORE ... */
                        /* fall through */
                    default: skip = test_dep != 2 && ts_cmp(&B.ex[c], &x) < 0;   /* ... and ANY */
                    }
                    if (skip) continue;
                    const int st = status[c];
                    if (test_status == 1 && !(st == S_PRECOMMITTED || st == S_COMMITTED || st == S_ACCEPTED)) continue;
                    if (test_status == 2 && (st < S_STABLE || st >= S_TRUNCATED)) continue;
                    if (!((kinds >> ts_kind(id)) & 1)) continue;
                    if (test_dep != 2) {
                        if (!(flags[c] & RC_HAS_DEPS)) continue;                   /* hasProposedOrDecidedDeps */
                        if ((test_dep == 0) == !rr_deps_intersects(&T, c, &x)) continue;
                    }
                } else {
                    if (started_at == 1 && ts_cmp(id, &x) <= 0) continue;
                    if (started_at == 0 && ts_cmp(id, &x) >= 0) continue;
                    if (!((kinds >> ts_kind(id)) & 1)) continue;
                }
                for (uint32_t j = rng_off[c]; j < rng_off[c + 1]; ++j) {
                    if (!rr_hits(rng_start[j], rng_end[j], isr, part_start, part_end, p0, p1, end_inclusive)) continue;
                    const int64_t rid = rid_of[j];
                    /* list.isEmpty() || !list.get(last).txnId.equals(txnId) */
                    if (last[rid] >= 0 && ts_eq(&B.id[last[rid]], id)) continue;
                    last[rid] = c;
                    if (ni == items_cap) { items_cap = items_cap ? 2 * items_cap : 64; items = realloc(items, items_cap * sizeof *items); }
                    items[ni] = (rr_item){ rid, (int64_t)ni, c, hist ? *id : B.ex[c] };   /* TxnInfo.executeAt */
                    ++ni;
                }
            }
        }
        /* TreeMap<Range, List<TxnInfo>> iteration: range order, each list in insertion order; the map */
        if (ni > order_cap) { order_cap = ni; order = realloc(order, order_cap * sizeof *order); }
        for (size_t u = 0; u < ni; ++u) order[u] = (int64_t)u;
        stable_sort(order, ni, cmp_rr_item, items);
        b_reset(&b);
        for (size_t u = 0; u < ni; ++u) {
            const rr_item *it = &items[order[u]];
            if (exec_after && ts_cmp(&it->ex, &x) <= 0) continue;
            b_add(&b, (uint64_t)it->rid, first[it->c]);
        }
        kdeps part; if (b_build(&b, &part, &E)) break;
        for (size_t u = 0; u < part.nk2v; ++u) iv_push(&arena, part.k2v[u]);
        for (size_t u = 0; u < part.nkeys; ++u) iv_push(&rids, (int64_t)part.keys[u]);
        for (size_t u = 0; u < part.nvals; ++u) iv_push(&deps, part.vals[u]);
        R->total_edges += part.nk2v - part.nkeys;
        kd_free(&part);
    }
    R->arena_off[nq] = arena.n; R->rd_off[nq] = rids.n; R->u_off[nq] = deps.n;
    R->arena = malloc((arena.n + 1) * sizeof(int32_t));
    for (size_t u = 0; u < arena.n; ++u) R->arena[u] = (int32_t)arena.v[u];
    R->range_id = malloc((rids.n + 1) * sizeof(uint32_t));
    for (size_t u = 0; u < rids.n; ++u) R->range_id[u] = (uint32_t)rids.v[u];
    R->dep_txn = malloc((deps.n + 1) * sizeof(uint32_t));
    for (size_t u = 0; u < deps.n; ++u) R->dep_txn[u] = (uint32_t)deps.v[u];
    R->error = E.code;
    snprintf(R->message, sizeof R->message, "%s", E.msg);
    b_free(&b);
    free(items); free(order); free(last); free(arena.v); free(rids.v); free(deps.v); free(all); free(rid_of);
    free(first); free(dep); free(B.id); free(B.ex);
    return R;
}
