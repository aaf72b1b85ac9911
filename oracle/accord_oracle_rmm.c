/*
 * accord_oracle_rmm.c — TEST INFRASTRUCTURE ONLY (rules in accord_oracle.h).
 *
 * Plain-C restatement of the RelationMultiMap operations on whole deps objects, over raw values:
 *   - RelationMultiMap.LinearMerger fold of RelationMultiMap.linearUnion (utils/RelationMultiMap.java:284-406,
 *     561-816) with SortedArrays.linearUnion (utils/SortedArrays.java:152-281) and remapToSuperset (:1196-1223),
 *     tracking value INSTANCES (input slots) so that equals-ties keep the instance the Java keeps;
 *     = KeyDeps.merge (primitives/KeyDeps.java:115-135), RangeDeps.merge (primitives/RangeDeps.java:101-134),
 *     Deps.merge (primitives/Deps.java:256-260) when run on both parts;
 *   - RelationMultiMap.invert (utils/RelationMultiMap.java:907-938);
 *   - KeyDeps.slice (primitives/KeyDeps.java:189-236) / RangeDeps.slice (primitives/RangeDeps.java:545-565) with
 *     trimUnusedValues (utils/RelationMultiMap.java:491-532);
 *   - stabbing queries over a built RangeDeps (SearchableRangeList.forEach, utils/SearchableRangeList.java:89-116;
 *     RangeDeps.forEach(key), primitives/RangeDeps.java:152-412): range indices in ascending order.
 * Paths are relative to /root/reference/accord-core/src/main/java/accord/.
 */
#define _GNU_SOURCE
#include "accord_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct rts { uint64_t msb, lsb; int32_t node; } rts;

#define R_IDENTITY_LSB   0xFFFFFFFFFFFF001EULL
#define R_IDENTITY_FLAGS 0x001EULL

/* Timestamp.compareTo / equals (primitives/Timestamp.java:208-217, 244-249) */
static int rts_cmp(const rts *a, const rts *b)
{
    if (a->msb != b->msb) return a->msb < b->msb ? -1 : 1;
    uint64_t ah = a->lsb >> 16, bh = b->lsb >> 16;
    if (ah != bh) return ah < bh ? -1 : 1;
    uint64_t af = a->lsb & R_IDENTITY_FLAGS, bf = b->lsb & R_IDENTITY_FLAGS;
    if (af != bf) return af < bf ? -1 : 1;
    if (a->node != b->node) return a->node < b->node ? -1 : 1;
    return 0;
}
static int rts_eq(const rts *a, const rts *b)
{
    return a->msb == b->msb && ((a->lsb ^ b->lsb) & R_IDENTITY_LSB) == 0 && a->node == b->node;
}

/* A key: u64 code (a, 0) for KeyDeps, Range (start, end) for RangeDeps; Range::compare = start then end
 * (primitives/Range.java:310-317); codes are order preserving, so unsigned compare. */
typedef struct okey { uint64_t a, b; } okey;
static int okey_cmp(const okey *x, const okey *y)
{
    if (x->a != y->a) return x->a < y->a ? -1 : 1;
    if (x->b != y->b) return x->b < y->b ? -1 : 1;
    return 0;
}

/* A RelationMultiMap: keys, values as instance handles (input slots into the value table), keysToValues. `id`
 * identifies the arrays (Java object identity of the key/value arrays: 0 = a freshly built array). */
typedef struct rmm {
    okey *keys; size_t nk; int kid;
    int64_t *vals; size_t nv; int vid;
    int32_t *k2v; size_t no;
} rmm;

typedef struct rctx { const rts *tab; } rctx;

static void rmm_free(rmm *m) { free(m->keys); free(m->vals); free(m->k2v); memset(m, 0, sizeof *m); }

/* SortedArrays.linearUnion (utils/SortedArrays.java:152-281) over values (handles compared by TxnId order).
 * *which = 1: the result IS the left array, 2: the right array, 0: a new array. */
static int64_t *sa_union_vals(const int64_t *left, size_t ln, const int64_t *right, size_t rn, const rts *tab,
                              size_t *nout, int *which)
{
    size_t li = 0, ri = 0, rs = 0;
    int64_t *res = malloc((ln + rn + 1) * sizeof *res);
    *which = 0;
    int built = 0;
    if (ln >= rn) {
        while (li < ln && ri < rn) {
            int c = left[li] == right[ri] ? 0 : rts_cmp(&tab[left[li]], &tab[right[ri]]);
            if (c <= 0) { li += 1; ri += c == 0 ? 1 : 0; }
            else {
                memcpy(res, left, li * sizeof *res); rs = li;
                res[rs++] = right[ri++];
                built = 1;
                break;
            }
        }
        if (!built) {
            if (ri == rn) { memcpy(res, left, ln * sizeof *res); *nout = ln; *which = 1; return res; }
            memcpy(res, left, li * sizeof *res); rs = li;
        }
    } else {
        while (li < ln && ri < rn) {
            int c = left[li] == right[ri] ? 0 : rts_cmp(&tab[left[li]], &tab[right[ri]]);
            if (c >= 0) { ri += 1; li += c == 0 ? 1 : 0; }
            else {
                memcpy(res, right, ri * sizeof *res); rs = ri;
                res[rs++] = left[li++];
                built = 1;
                break;
            }
        }
        if (!built) {
            if (li == ln) { memcpy(res, right, rn * sizeof *res); *nout = rn; *which = 2; return res; }
            memcpy(res, right, ri * sizeof *res); rs = ri;
        }
    }
    while (li < ln && ri < rn) {
        int c = left[li] == right[ri] ? 0 : rts_cmp(&tab[left[li]], &tab[right[ri]]);
        if (c == 0) { res[rs++] = left[li]; li++; ri++; }
        else if (c < 0) res[rs++] = left[li++];
        else res[rs++] = right[ri++];
    }
    while (li < ln) res[rs++] = left[li++];
    while (ri < rn) res[rs++] = right[ri++];
    *nout = rs;
    return res;
}

/* The same over keys (Range::compare / key order). */
static okey *sa_union_keys(const okey *left, size_t ln, const okey *right, size_t rn, size_t *nout, int *which)
{
    size_t li = 0, ri = 0, rs = 0;
    okey *res = malloc((ln + rn + 1) * sizeof *res);
    *which = 0;
    int built = 0;
    if (ln >= rn) {
        while (li < ln && ri < rn) {
            int c = okey_cmp(&left[li], &right[ri]);
            if (c <= 0) { li += 1; ri += c == 0 ? 1 : 0; }
            else { memcpy(res, left, li * sizeof *res); rs = li; res[rs++] = right[ri++]; built = 1; break; }
        }
        if (!built) {
            if (ri == rn) { memcpy(res, left, ln * sizeof *res); *nout = ln; *which = 1; return res; }
            memcpy(res, left, li * sizeof *res); rs = li;
        }
    } else {
        while (li < ln && ri < rn) {
            int c = okey_cmp(&left[li], &right[ri]);
            if (c >= 0) { ri += 1; li += c == 0 ? 1 : 0; }
            else { memcpy(res, right, ri * sizeof *res); rs = ri; res[rs++] = left[li++]; built = 1; break; }
        }
        if (!built) {
            if (li == ln) { memcpy(res, right, rn * sizeof *res); *nout = rn; *which = 2; return res; }
            memcpy(res, right, ri * sizeof *res); rs = ri;
        }
    }
    while (li < ln && ri < rn) {
        int c = okey_cmp(&left[li], &right[ri]);
        if (c == 0) { res[rs++] = left[li]; li++; ri++; }
        else if (c < 0) res[rs++] = left[li++];
        else res[rs++] = right[ri++];
    }
    while (li < ln) res[rs++] = left[li++];
    while (ri < rn) res[rs++] = right[ri++];
    *nout = rs;
    return res;
}

/* SortedArrays.remapToSuperset (:1196-1223): null (here: NULL) when the lengths are equal. */
static int32_t *remap_to_superset(const int64_t *src, size_t sn, const int64_t *trg, size_t tn, const rts *tab)
{
    if (sn == tn) return NULL;
    int32_t *res = malloc((sn + 1) * sizeof *res);
    size_t i = 0, j = 0;
    while (i < sn && j < tn) {
        if (src[i] != trg[j] && !rts_eq(&tab[src[i]], &tab[trg[j]])) {
            while (j < tn && rts_cmp(&tab[trg[j]], &tab[src[i]]) < 0) ++j;   /* exponentialSearch FAST (found) */
        }
        res[i++] = (int32_t)j++;
    }
    return res;
}
static inline int32_t remap(int32_t i, const int32_t *rm) { return rm ? rm[i] : i; }

/* RelationMultiMap.linearUnion (utils/RelationMultiMap.java:561-816). Returns 1 when the result is `left` as is,
 * 2 when it is `right` as is, 0 when `out` was built. */
static int rmm_union(const rmm *L, const rmm *R, rmm *out, const rts *tab)
{
    size_t nko, nvo;
    int kw, vw;
    okey *outKeys = sa_union_keys(L->keys, L->nk, R->keys, R->nk, &nko, &kw);
    int64_t *outVals = sa_union_vals(L->vals, L->nv, R->vals, R->nv, tab, &nvo, &vw);
    int32_t *remapLeft = remap_to_superset(L->vals, L->nv, outVals, nvo, tab);
    int32_t *remapRight = remap_to_superset(R->vals, R->nv, outVals, nvo, tab);
    int result = -1;
    int32_t *o = NULL;
    size_t lk = 0, rk = 0, ok = 0, l = L->nk, r = R->nk, olen = nko;
    const int32_t *left = L->k2v, *right = R->k2v;

    if (!remapLeft && !remapRight && L->no == R->no && L->nk == R->nk
        && memcmp(L->k2v, R->k2v, R->no * sizeof *L->k2v) == 0) {
        int eq = 1;
        for (size_t i = 0; i < R->nk && eq; ++i) eq = okey_cmp(&L->keys[i], &R->keys[i]) == 0;
        if (eq) { result = 1; goto done; }
    }
    if (!remapLeft && kw == 1) {
        /* "this" knows all the TxnId and Keys already (:592-651) */
        int conflict = 0;
        while (lk < L->nk && rk < R->nk && !conflict) {
            int ck = okey_cmp(&L->keys[lk], &R->keys[rk]);
            if (ck < 0) { olen += (size_t)left[lk] - l; l = (size_t)left[lk]; ok++; lk++; }
            else if (ck > 0) { result = -2; goto done; }   /* throwUnexpectedMissingKeyException */
            else {
                while (l < (size_t)left[lk] && r < (size_t)right[rk]) {
                    int32_t nl = left[l], nr = remap(right[r], remapRight);
                    if (nl < nr) { olen++; l++; }
                    else if (nr < nl) { conflict = 1; break; }
                    else { olen++; l++; r++; }
                }
                if (conflict) break;
                if (l < (size_t)left[lk]) { olen += (size_t)left[lk] - l; l = (size_t)left[lk]; }
                else if (r < (size_t)right[rk]) { conflict = 1; break; }
                ok++; rk++; lk++;
            }
        }
        if (!conflict) { result = 1; goto done; }
        o = malloc((L->no + R->no + 1) * sizeof *o);
        memcpy(o, left, olen * sizeof *o);
    } else if (!remapRight && kw == 2) {
        /* "that" knows all the TxnId and keys already (:652-711) */
        int conflict = 0;
        while (lk < L->nk && rk < R->nk && !conflict) {
            int ck = okey_cmp(&L->keys[lk], &R->keys[rk]);
            if (ck < 0) { result = -2; goto done; }
            else if (ck > 0) { olen += (size_t)right[rk] - r; r = (size_t)right[rk]; ok++; rk++; }
            else {
                while (l < (size_t)left[lk] && r < (size_t)right[rk]) {
                    int32_t nl = remap(left[l], remapLeft), nr = right[r];
                    if (nl < nr) { conflict = 1; break; }
                    else if (nr < nl) { olen++; r++; }
                    else { olen++; l++; r++; }
                }
                if (conflict) break;
                if (l < (size_t)left[lk]) { conflict = 1; break; }
                else if (r < (size_t)right[rk]) { olen += (size_t)right[rk] - r; r = (size_t)right[rk]; }
                ok++; rk++; lk++;
            }
        }
        if (!conflict) { result = 2; goto done; }
        o = malloc((L->no + R->no + 1) * sizeof *o);
        memcpy(o, right, olen * sizeof *o);
    } else {
        o = malloc((L->no + R->no + 1) * sizeof *o);
    }
    /* general merge (:713-795) */
    while (lk < L->nk && rk < R->nk) {
        int ck = okey_cmp(&L->keys[lk], &R->keys[rk]);
        if (ck < 0) {
            while (l < (size_t)left[lk]) o[olen++] = remap(left[l++], remapLeft);
            o[ok++] = (int32_t)olen; lk++;
        } else if (ck > 0) {
            while (r < (size_t)right[rk]) o[olen++] = remap(right[r++], remapRight);
            o[ok++] = (int32_t)olen; rk++;
        } else {
            while (l < (size_t)left[lk] && r < (size_t)right[rk]) {
                int32_t nl = remap(left[l], remapLeft), nr = remap(right[r], remapRight);
                if (nl <= nr) { o[olen++] = nl; l += 1; r += nl == nr ? 1 : 0; }
                else { o[olen++] = nr; ++r; }
            }
            while (l < (size_t)left[lk]) o[olen++] = remap(left[l++], remapLeft);
            while (r < (size_t)right[rk]) o[olen++] = remap(right[r++], remapRight);
            o[ok++] = (int32_t)olen; rk++; lk++;
        }
    }
    while (lk < L->nk) { while (l < (size_t)left[lk]) o[olen++] = remap(left[l++], remapLeft); o[ok++] = (int32_t)olen; lk++; }
    while (rk < R->nk) { while (r < (size_t)right[rk]) o[olen++] = remap(right[r++], remapRight); o[ok++] = (int32_t)olen; rk++; }
    out->keys = outKeys; out->nk = nko; out->kid = 0;
    out->vals = outVals; out->nv = nvo; out->vid = 0;
    out->k2v = o; out->no = olen;
    free(remapLeft); free(remapRight);
    return 0;
done:
    free(outKeys); free(outVals); free(remapLeft); free(remapRight); free(o);
    return result;
}

static void rmm_copy(rmm *dst, const rmm *src)
{
    dst->keys = malloc((src->nk + 1) * sizeof *dst->keys); memcpy(dst->keys, src->keys, src->nk * sizeof *dst->keys);
    dst->vals = malloc((src->nv + 1) * sizeof *dst->vals); memcpy(dst->vals, src->vals, src->nv * sizeof *dst->vals);
    dst->k2v = malloc((src->no + 1) * sizeof *dst->k2v); memcpy(dst->k2v, src->k2v, src->no * sizeof *dst->k2v);
    dst->nk = src->nk; dst->nv = src->nv; dst->no = src->no; dst->kid = src->kid; dst->vid = src->vid;
}

typedef struct rivec { int64_t *v; size_t n, cap; } rivec;
static void rpush(rivec *a, int64_t x)
{
    if (a->n == a->cap) { a->cap = a->cap ? a->cap * 2 : 64; a->v = realloc(a->v, a->cap * sizeof *a->v); }
    a->v[a->n++] = x;
}

static void set_msg(int *err, char *msg, int code, const char *m)
{
    if (*err) return;
    *err = code;
    snprintf(msg, 256, "%s", m);
}

/* Validation of one input object (KeyDeps ctor :179-186 last offset; RelationMultiMap.checkValid :1073-1097 duplicate
 * values; Keys.ofSortedUnique / Range order; txnIds sorted unique). Returns 0 when valid. */
static int validate_rmm(const rmm *m, const rts *tab, int is_range, int *err, char *msg)
{
    for (size_t i = 1; i < m->nk; ++i)
        if (okey_cmp(&m->keys[i - 1], &m->keys[i]) >= 0) { set_msg(err, msg, -1, "keys must be sorted and unique"); return 1; }
    for (size_t i = 0; is_range && i < m->nk; ++i)
        if (m->keys[i].a >= m->keys[i].b) { set_msg(err, msg, -1, "range start must be below its end"); return 1; }
    for (size_t i = 1; i < m->nv; ++i)
        if (rts_cmp(&tab[m->vals[i - 1]], &tab[m->vals[i]]) >= 0) { set_msg(err, msg, -1, "txnIds must be sorted and unique"); return 1; }
    if (m->nk == 0) {
        if (m->no) { set_msg(err, msg, -1, "Last key in keyToTxnId does not point to the end of the array"); return 1; }
        return 0;
    }
    if (m->no < m->nk || (size_t)m->k2v[m->nk - 1] != m->no) {
        set_msg(err, msg, -1, "Last key in keyToTxnId does not point to the end of the array"); return 1;
    }
    size_t prev = m->nk;
    for (size_t k = 0; k < m->nk; ++k) {
        size_t end = (size_t)(uint32_t)m->k2v[k];
        if (end < prev || end > m->no) { set_msg(err, msg, -1, "Last key in keyToTxnId does not point to the end of the array"); return 1; }
        for (size_t q = prev; q < end; ++q) {
            int32_t x = m->k2v[q];
            if (x < 0 || (size_t)x >= m->nv) { set_msg(err, msg, -1, "keyToTxnId entry out of range of txnIds"); return 1; }
            if (q > prev && m->k2v[q - 1] >= x) { set_msg(err, msg, -2, "Duplicate value found for key (RelationMultiMap.checkValid)"); return 1; }
        }
        prev = end;
    }
    return 0;
}

orc_rmm_merge_result *orc_rmm_merge(uint32_t n_groups, const uint64_t *grp_off, int is_range,
                                    const uint64_t *key_off, const uint64_t *key_a, const uint64_t *key_b,
                                    const uint64_t *val_off, const uint64_t *vmsb, const uint64_t *vlsb, const int32_t *vnode,
                                    const uint64_t *k2v_off, const int32_t *k2v)
{
    orc_rmm_merge_result *R = calloc(1, sizeof *R);
    R->n_groups = n_groups;
    uint64_t nrep = grp_off[n_groups];
    uint64_t NV = val_off[nrep];
    rts *tab = malloc((NV + 1) * sizeof *tab);
    for (uint64_t i = 0; i < NV; ++i) tab[i] = (rts){ vmsb[i], vlsb[i], vnode[i] };
    R->key_off = calloc(n_groups + 1, sizeof(uint64_t));
    R->val_off = calloc(n_groups + 1, sizeof(uint64_t));
    R->k2v_off = calloc(n_groups + 1, sizeof(uint64_t));
    rivec ka = { 0 }, kb = { 0 }, vs = { 0 }, oo = { 0 };
    for (uint32_t g = 0; g < n_groups && !R->error; ++g) {
        rmm acc = { 0 };
        int have = 0;
        for (uint64_t r = grp_off[g]; r < grp_off[g + 1] && !R->error; ++r) {
            rmm in = { 0 };
            in.nk = key_off[r + 1] - key_off[r];
            in.nv = val_off[r + 1] - val_off[r];
            in.no = k2v_off[r + 1] - k2v_off[r];
            in.keys = malloc((in.nk + 1) * sizeof *in.keys);
            for (size_t q = 0; q < in.nk; ++q)
                in.keys[q] = (okey){ key_a[key_off[r] + q], key_b ? key_b[key_off[r] + q] : 0 };
            in.vals = malloc((in.nv + 1) * sizeof *in.vals);
            for (size_t q = 0; q < in.nv; ++q) in.vals[q] = (int64_t)(val_off[r] + q);
            in.k2v = (int32_t *)(k2v + k2v_off[r]);
            in.kid = in.vid = (int)(r + 1);
            if (validate_rmm(&in, tab, is_range, &R->error, R->message)) { free(in.keys); free(in.vals); break; }
            /* deps.isEmpty(): keys.length == keysToValues.length (RelationMultiMap.isEmpty :1012-1015) */
            if (in.no == in.nk) { free(in.keys); free(in.vals); continue; }
            if (!have) {   /* LinearMerger.update, first input (:333-344) */
                rmm_copy(&acc, &in);
                have = 1;
            } else {
                rmm u = { 0 };
                int w = rmm_union(&acc, &in, &u, tab);
                if (w == -2) { set_msg(&R->error, R->message, -2, "unexpected missing key"); }
                else if (w == 2) { rmm_free(&acc); rmm_copy(&acc, &in); }
                else if (w == 0) { rmm_free(&acc); acc = u; }
            }
            free(in.keys); free(in.vals);
        }
        R->key_off[g] = ka.n; R->val_off[g] = vs.n; R->k2v_off[g] = oo.n;
        for (size_t q = 0; q < acc.nk; ++q) { rpush(&ka, (int64_t)acc.keys[q].a); rpush(&kb, (int64_t)acc.keys[q].b); }
        for (size_t q = 0; q < acc.nv; ++q) rpush(&vs, acc.vals[q]);
        for (size_t q = 0; q < acc.no; ++q) rpush(&oo, acc.k2v[q]);
        if (have) rmm_free(&acc);
    }
    R->key_off[n_groups] = ka.n; R->val_off[n_groups] = vs.n; R->k2v_off[n_groups] = oo.n;
    R->key_a = malloc((ka.n + 1) * 8); R->key_b = malloc((kb.n + 1) * 8);
    for (size_t q = 0; q < ka.n; ++q) { R->key_a[q] = (uint64_t)ka.v[q]; R->key_b[q] = (uint64_t)kb.v[q]; }
    R->val_src = malloc((vs.n + 1) * 8);
    R->val_msb = malloc((vs.n + 1) * 8); R->val_lsb = malloc((vs.n + 1) * 8); R->val_node = malloc((vs.n + 1) * 4);
    for (size_t q = 0; q < vs.n; ++q) {
        uint64_t s = (uint64_t)vs.v[q];
        R->val_src[q] = s; R->val_msb[q] = tab[s].msb; R->val_lsb[q] = tab[s].lsb; R->val_node[q] = tab[s].node;
    }
    R->k2v = malloc((oo.n + 1) * 4);
    for (size_t q = 0; q < oo.n; ++q) R->k2v[q] = (int32_t)oo.v[q];
    free(ka.v); free(kb.v); free(vs.v); free(oo.v); free(tab);
    return R;
}

void orc_rmm_merge_free(orc_rmm_merge_result *r)
{
    if (!r) return;
    free(r->key_off); free(r->key_a); free(r->key_b); free(r->val_off); free(r->val_src); free(r->val_msb);
    free(r->val_lsb); free(r->val_node); free(r->k2v_off); free(r->k2v);
    free(r);
}

/* ------------------------------------------------------------------ invert */

/* RelationMultiMap.invert (utils/RelationMultiMap.java:907-938), batched over groups: per group g the source CSR
 * src[src_off[g] .. src_off[g+1]) with nsrc[g] = srcKeyCount keys and ntrg[g] = trgKeyCount target keys. */
int orc_invert(uint32_t n_groups, const uint64_t *src_off, const int32_t *src, const uint64_t *nsrc, const uint64_t *ntrg,
               uint64_t *trg_off, int32_t *trg)
{
    uint64_t o = 0;
    for (uint32_t g = 0; g < n_groups; ++g) {
        trg_off[g] = o;
        const int32_t *s = src + src_off[g];
        size_t srcLength = src_off[g + 1] - src_off[g], srcKeyCount = nsrc[g], trgKeyCount = ntrg[g];
        int32_t *t = trg + o;
        size_t len = trgKeyCount + srcLength - srcKeyCount;
        memset(t, 0, len * sizeof *t);
        for (size_t i = srcKeyCount; i < srcLength; ++i) {
            if (s[i] < 0 || (size_t)s[i] >= trgKeyCount) return -1;
            t[s[i]]++;
        }
        if (trgKeyCount) {
            t[0] += (int32_t)trgKeyCount;
            for (size_t i = 1; i < trgKeyCount; ++i) t[i] += t[i - 1];
            memmove(t + 1, t, (trgKeyCount - 1) * sizeof *t);
            t[0] = (int32_t)trgKeyCount;
        }
        size_t k = 0;
        for (size_t i = srcKeyCount; i < srcLength; ++i) {
            while (i == (size_t)s[k]) ++k;
            t[t[s[i]]++] = (int32_t)k;
        }
        o += len;
    }
    trg_off[n_groups] = o;
    return 0;
}

/* ------------------------------------------------------------------ slice + trimUnusedValues */

/* Range.contains(key) with the bound type (primitives/Range.java:40-138); ranges intersect:
 * compareIntersecting == 0 (:296-305). */
static int r_contains(uint64_t s, uint64_t e, uint64_t k, int end_inclusive)
{
    return end_inclusive ? (k > s && k <= e) : (k >= s && k < e);
}
static int r_intersects(uint64_t as, uint64_t ae, uint64_t bs, uint64_t be) { return as < be && ae > bs; }

/* KeyDeps.slice(Ranges) (primitives/KeyDeps.java:189-236) / RangeDeps.slice(Ranges) (primitives/RangeDeps.java:545-565)
 * per group over the same group's select ranges sel[sel_off[g] .. sel_off[g+1]); trimUnusedValues
 * (utils/RelationMultiMap.java:491-532). Keys: key_a (KeyDeps codes) or (key_a, key_b) ranges (is_range). Output per
 * group: the selected key indices (ascending), the kept value indices (ascending) and the new keysToTxnIds. */
orc_slice_result *orc_rmm_slice(uint32_t n_groups, int is_range, int end_inclusive,
                                const uint64_t *key_off, const uint64_t *key_a, const uint64_t *key_b,
                                const uint64_t *val_off, const uint64_t *k2v_off, const int32_t *k2v,
                                const uint64_t *sel_off, const uint64_t *sel_s, const uint64_t *sel_e)
{
    orc_slice_result *R = calloc(1, sizeof *R);
    R->n_groups = n_groups;
    R->key_off = calloc(n_groups + 1, 8); R->val_off = calloc(n_groups + 1, 8); R->k2v_off = calloc(n_groups + 1, 8);
    rivec ks = { 0 }, vs = { 0 }, oo = { 0 };
    for (uint32_t g = 0; g < n_groups; ++g) {
        R->key_off[g] = ks.n; R->val_off[g] = vs.n; R->k2v_off[g] = oo.n;
        size_t nk = key_off[g + 1] - key_off[g], nv = val_off[g + 1] - val_off[g], no = k2v_off[g + 1] - k2v_off[g];
        const int32_t *src = k2v + k2v_off[g];
        if (no == nk) {   /* isEmpty(): KeyDeps returns (keys, txnIds, k2v); RangeDeps (NO_RANGES, txnIds, NO_INTS) */
            if (!is_range) for (size_t k = 0; k < nk; ++k) rpush(&ks, (int64_t)k);
            for (size_t v = 0; v < nv; ++v) rpush(&vs, (int64_t)v);
            if (!is_range) for (size_t q = 0; q < no; ++q) rpush(&oo, src[q]);
            continue;
        }
        /* select: Keys.slice(ranges) = keys contained in any select range; RangeDeps: ranges intersecting any */
        int64_t *sel = malloc((nk + 1) * sizeof *sel);
        size_t ns = 0;
        for (size_t k = 0; k < nk; ++k) {
            uint64_t a = key_a[key_off[g] + k], b = is_range ? key_b[key_off[g] + k] : 0;
            int hit = 0;
            for (uint64_t q = sel_off[g]; q < sel_off[g + 1] && !hit; ++q)
                hit = is_range ? r_intersects(a, b, sel_s[q], sel_e[q]) : r_contains(sel_s[q], sel_e[q], a, end_inclusive);
            if (hit) sel[ns++] = (int64_t)k;
        }
        if (ns == 0) { free(sel); continue; }   /* (Keys.EMPTY | NO_RANGES, NO_TXNIDS, NO_INTS) */
        if (ns == nk) {                         /* return this */
            for (size_t k = 0; k < nk; ++k) rpush(&ks, (int64_t)k);
            for (size_t v = 0; v < nv; ++v) rpush(&vs, (int64_t)v);
            for (size_t q = 0; q < no; ++q) rpush(&oo, src[q]);
            free(sel);
            continue;
        }
        size_t off = ns;
        for (size_t j = 0; j < ns; ++j) { size_t i = (size_t)sel[j]; off += (size_t)src[i] - (i == 0 ? nk : (size_t)src[i - 1]); }
        int32_t *trg = malloc((off + 1) * sizeof *trg);
        off = ns;
        for (size_t j = 0; j < ns; ++j) {
            size_t i = (size_t)sel[j];
            size_t start = i == 0 ? nk : (size_t)src[i - 1], count = (size_t)src[i] - start;
            memcpy(trg + off, src + start, count * sizeof *trg);
            off += count;
            trg[j] = (int32_t)off;
        }
        /* trimUnusedValues */
        char *used = calloc(nv + 1, 1);
        for (size_t q = ns; q < off; ++q) used[trg[q]] = 1;
        int32_t *remapv = malloc((nv + 1) * sizeof *remapv);
        int32_t cnt = 0;
        for (size_t v = 0; v < nv; ++v) remapv[v] = used[v] ? cnt++ : -1;
        if ((size_t)cnt < nv)
            for (size_t q = ns; q < off; ++q) trg[q] = remapv[trg[q]];
        for (size_t j = 0; j < ns; ++j) rpush(&ks, sel[j]);
        for (size_t v = 0; v < nv; ++v) if ((size_t)cnt == nv || used[v]) rpush(&vs, (int64_t)v);
        for (size_t q = 0; q < off; ++q) rpush(&oo, trg[q]);
        free(used); free(remapv); free(trg); free(sel);
    }
    R->key_off[n_groups] = ks.n; R->val_off[n_groups] = vs.n; R->k2v_off[n_groups] = oo.n;
    R->key_idx = malloc((ks.n + 1) * 4); R->val_idx = malloc((vs.n + 1) * 4); R->k2v = malloc((oo.n + 1) * 4);
    for (size_t q = 0; q < ks.n; ++q) R->key_idx[q] = (uint32_t)ks.v[q];
    for (size_t q = 0; q < vs.n; ++q) R->val_idx[q] = (uint32_t)vs.v[q];
    for (size_t q = 0; q < oo.n; ++q) R->k2v[q] = (int32_t)oo.v[q];
    free(ks.v); free(vs.v); free(oo.v);
    return R;
}

/* ------------------------------------------------------------------ without (RelationMultiMap.remove) */

/* Arrays.binarySearch(txnIds, t) >= 0 over a sorted TxnId[] (java.util.Arrays: lo/hi bisection, compareTo) */
static int bsearch_contains(const uint64_t *m, const uint64_t *l, const int32_t *n, uint64_t lo, uint64_t hi, const rts *t)
{
    if (!m) return 0;
    int64_t low = (int64_t)lo, high = (int64_t)hi - 1;
    while (low <= high) {
        int64_t mid = (low + high) >> 1;
        rts x = { m[mid], l[mid], n[mid] };
        int c = rts_cmp(&x, t);
        if (c < 0) low = mid + 1;
        else if (c > 0) high = mid - 1;
        else return 1;
    }
    return 0;
}

/* RelationMultiMap.remove (utils/RelationMultiMap.java:843-905) per group = KeyDeps.without (primitives/KeyDeps.java:
 * 255-259) / RangeDeps.without (primitives/RangeDeps.java:584-588) with remove = Deps::contains over the group's two
 * sets (primitives/Deps.java:107-110: keyDeps.contains || rangeDeps.contains). kind[g]: 0 `return from`, 1 `return
 * none`, 2 the rebuilt object (keys passed through: emptied keys stay). Output as orc_rmm_slice's. */
orc_slice_result *orc_rmm_without(uint32_t n_groups, const uint64_t *key_off, const uint64_t *val_off,
                                  const uint64_t *k2v_off, const int32_t *k2v,
                                  const uint64_t *vm, const uint64_t *vl, const int32_t *vn,
                                  const uint64_t *a_off, const uint64_t *am, const uint64_t *al, const int32_t *an,
                                  const uint64_t *b_off, const uint64_t *bm, const uint64_t *bl, const int32_t *bn,
                                  uint8_t *kind)
{
    orc_slice_result *R = calloc(1, sizeof *R);
    R->n_groups = n_groups;
    R->key_off = calloc(n_groups + 1, 8); R->val_off = calloc(n_groups + 1, 8); R->k2v_off = calloc(n_groups + 1, 8);
    rivec ks = { 0 }, vs = { 0 }, oo = { 0 };
    for (uint32_t g = 0; g < n_groups; ++g) {
        R->key_off[g] = ks.n; R->val_off[g] = vs.n; R->k2v_off[g] = oo.n;
        size_t nk = key_off[g + 1] - key_off[g], nv = val_off[g + 1] - val_off[g], no = k2v_off[g + 1] - k2v_off[g];
        const int32_t *old = k2v + k2v_off[g];
        /* :844-845 if (isEmpty(keys, oldKeysToValues)) return from; */
        int from = no == nk;
        int32_t *remapValue = malloc((nv + 1) * sizeof *remapValue);
        int count = 0;
        if (!from) {
            /* :853-858 remapValue[i] = remove.test(oldValues[i]) ? -1 : count++ */
            for (size_t i = 0; i < nv; ++i) {
                size_t v = val_off[g] + i;
                rts t = { vm[v], vl[v], vn[v] };
                int rm = (a_off && bsearch_contains(am, al, an, a_off[g], a_off[g + 1], &t)) ||
                         (b_off && bsearch_contains(bm, bl, bn, b_off[g], b_off[g + 1], &t));
                remapValue[i] = rm ? -1 : count++;
            }
            /* :862-863 if (count == oldValues.length) return from; */
            if ((size_t)count == nv) from = 1;
        }
        if (from) {
            kind[g] = 0;
            for (size_t k = 0; k < nk; ++k) rpush(&ks, (int64_t)k);
            for (size_t v = 0; v < nv; ++v) rpush(&vs, (int64_t)v);
            for (size_t q = 0; q < no; ++q) rpush(&oo, old[q]);
            free(remapValue);
            continue;
        }
        /* :865-866 if (count == 0) return none; */
        if (count == 0) { kind[g] = 1; free(remapValue); continue; }
        kind[g] = 2;
        /* :868-873 newValues[remapValue[i]] = oldValues[i] */
        for (size_t i = 0; i < nv; ++i) if (remapValue[i] >= 0) rpush(&vs, (int64_t)i);
        /* :875-894 the keysToValues walk, literally */
        int32_t *nkv = malloc((no + 1) * sizeof *nkv);
        size_t k = 0, i = nk, o = nk;
        while (i < no) {
            while (old[k] == (int32_t)i) nkv[k++] = (int32_t)o;
            int32_t remapped = remapValue[old[i]];
            if (remapped >= 0) nkv[o++] = remapped;
            ++i;
        }
        while (k < nk) nkv[k++] = (int32_t)o;
        /* passthrough keys (:904 constructor.construct(passthroughKeys, ...)) */
        for (size_t kk = 0; kk < nk; ++kk) rpush(&ks, (int64_t)kk);
        for (size_t q = 0; q < o; ++q) rpush(&oo, nkv[q]);
        free(nkv); free(remapValue);
    }
    R->key_off[n_groups] = ks.n; R->val_off[n_groups] = vs.n; R->k2v_off[n_groups] = oo.n;
    R->key_idx = malloc((ks.n + 1) * 4); R->val_idx = malloc((vs.n + 1) * 4); R->k2v = malloc((oo.n + 1) * 4);
    for (size_t q = 0; q < ks.n; ++q) R->key_idx[q] = (uint32_t)ks.v[q];
    for (size_t q = 0; q < vs.n; ++q) R->val_idx[q] = (uint32_t)vs.v[q];
    for (size_t q = 0; q < oo.n; ++q) R->k2v[q] = (int32_t)oo.v[q];
    free(ks.v); free(vs.v); free(oo.v);
    return R;
}

void orc_slice_free(orc_slice_result *r)
{
    if (!r) return;
    free(r->key_off); free(r->val_off); free(r->k2v_off); free(r->key_idx); free(r->val_idx); free(r->k2v);
    free(r);
}

/* ------------------------------------------------------------------ stabbing queries over a built RangeDeps */

/* Per query q (against group grp[q]'s ranges): every range index i with ranges[i] containing the key
 * (Range.contains, is_key_query) or intersecting [qs, qe) (compareIntersecting == 0), ascending
 * (SearchableRangeList.forEach, utils/SearchableRangeList.java:89-116; order as SearchableRangeListTest.java:98-112). */
orc_stab_result *orc_rmm_stab(uint32_t n_queries, const uint32_t *grp, const uint64_t *qs, const uint64_t *qe,
                              int is_key_query, int end_inclusive, const uint64_t *rng_off, const uint64_t *rs,
                              const uint64_t *re)
{
    orc_stab_result *R = calloc(1, sizeof *R);
    R->off = calloc(n_queries + 1, 8);
    rivec hits = { 0 };
    for (uint32_t q = 0; q < n_queries; ++q) {
        R->off[q] = hits.n;
        uint32_t g = grp[q];
        for (uint64_t i = rng_off[g]; i < rng_off[g + 1]; ++i) {
            int hit = is_key_query ? r_contains(rs[i], re[i], qs[q], end_inclusive) : r_intersects(rs[i], re[i], qs[q], qe[q]);
            if (hit) rpush(&hits, (int64_t)(i - rng_off[g]));
        }
    }
    R->off[n_queries] = hits.n;
    R->idx = malloc((hits.n + 1) * 4);
    for (size_t q = 0; q < hits.n; ++q) R->idx[q] = (uint32_t)hits.v[q];
    free(hits.v);
    return R;
}

void orc_stab_free(orc_stab_result *r)
{
    if (!r) return;
    free(r->off); free(r->idx); free(r);
}
