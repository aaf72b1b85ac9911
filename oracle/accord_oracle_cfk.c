/*
 * accord_oracle_cfk.c — TEST INFRASTRUCTURE ONLY (rules in accord_oracle.h).
 *
 * Plain-C restatement of CommandsForKey.update with the command's deps, step by step:
 *   update(prev, next, hasPrev)           local/CommandsForKey.java:657-722
 *   insert / update with InfoWithAdditions :736-760
 *   updateOrInsertWithAdditions           :772-863
 *   update(pos, cur, new) / insert(pos, …) :865-897
 *   insertInfoAndOneMissing               :899-944
 *   removeMissing                         :946-972
 *   insertMissing / mergeAndFilterMissing / to  :979-1033
 *   computeInfoAndAdditions               :1057-1149
 *   InternalStatus.hasInfo / hasDeps / depsKnownBefore, TxnInfo.create  :194-330 (depsKnownBefore :260-279)
 * over one CommandsForKey per key, applying a batch of command updates to every key they touch in batch order. The
 * Java's object identities (executeAt == txnId, depsKnownBefore == txn) are restated as flags: an executeAt equal to
 * its TxnId is the TxnId itself (TxnInfo.create), and depsKnownBefore is the txn itself for PREACCEPTED / ACCEPTED
 * or when executeAt is the TxnId. RedundantBefore is empty (NO_REDUNDANT_BEFORE: shardRedundantBefore = TxnId.NONE,
 * so every dep is considered). Paths are relative to /root/reference/accord-core/src/main/java/accord/.
 */
#define _GNU_SOURCE
#include "accord_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct cts { uint64_t msb, lsb; int32_t node; } cts;

/* Timestamp.compareTo / equals (primitives/Timestamp.java:208-217, 244-249) */
static int c_cmp(const cts *a, const cts *b)
{
    if (a->msb != b->msb) return a->msb < b->msb ? -1 : 1;
    uint64_t ah = a->lsb >> 16, bh = b->lsb >> 16;
    if (ah != bh) return ah < bh ? -1 : 1;
    uint64_t af = a->lsb & 0x1EULL, bf = b->lsb & 0x1EULL;
    if (af != bf) return af < bf ? -1 : 1;
    if (a->node != b->node) return a->node < b->node ? -1 : 1;
    return 0;
}
static int c_kind(const cts *t) { return (int)((t->lsb >> 1) & 7); }

/* Kind.witnesses() (primitives/Txn.java:221-236) */
static unsigned c_witnesses(int kind)
{
    switch (kind) {
    case 0: case 2: return 1u << 1;                                   /* Read, EphemeralRead: Ws */
    case 1: case 3: return (1u << 0) | (1u << 1);                     /* Write, SyncPoint: RsOrWs */
    case 4:         return (1u << 0) | (1u << 1) | (1u << 3) | (1u << 4);   /* ExclusiveSyncPoint: AnyGloballyVisible */
    default:        return 0;
    }
}
static int witnesses(const cts *owner, const cts *t) { return (c_witnesses(c_kind(owner)) >> c_kind(t)) & 1u; }

enum { TK = 0, HIST = 1, PRE = 2, ACC = 3, COMMITTED = 4, STABLE = 5, APPLIED = 6, INVALID = 7 };
static int has_info(int st) { return st >= ACC && st <= APPLIED; }   /* InternalStatus(hasInfo) :194-203 */

typedef struct info {
    cts id, ex;
    int ex_self;          /* executeAt == txnId (the same object in the Java) */
    int st;
    cts *miss; size_t nm; /* TxnInfoWithMissing.missing, sorted */
} info;

typedef struct cfk { info *t; size_t n; } cfk;

typedef struct cerr { int code; char msg[200]; } cerr;
static void c_fail(cerr *e, int code, const char *m) { if (!e->code) { e->code = code; snprintf(e->msg, sizeof e->msg, "%s", m); } }

/* TxnInfo.depsKnownBefore() (:322-325 -> InternalStatus.depsKnownBefore :259-279): self (the txn) or its executeAt */
static int dkb_is_self(const info *x) { return x->st == PRE || x->st == ACC || x->ex_self; }
static const cts *dkb(const info *x) { return dkb_is_self(x) ? &x->id : &x->ex; }


static long bsearch_ts(const cts *a, long from, long to, const cts *k)   /* Arrays.binarySearch */
{
    long lo = from, hi = to - 1;
    while (lo <= hi) {
        long mid = (long)(((unsigned long)lo + (unsigned long)hi) >> 1);
        int c = c_cmp(&a[mid], k);
        if (c < 0) lo = mid + 1; else if (c > 0) hi = mid - 1; else return mid;
    }
    return -(lo + 1);
}
static long bsearch_info(const cfk *c, long from, long to, const cts *k)
{
    long lo = from, hi = to - 1;
    while (lo <= hi) {
        long mid = (long)(((unsigned long)lo + (unsigned long)hi) >> 1);
        int r = c_cmp(&c->t[mid].id, k);
        if (r < 0) lo = mid + 1; else if (r > 0) hi = mid - 1; else return mid;
    }
    return -(lo + 1);
}

/* SortedArrays.insert of one TxnId into a sorted missing[] */
static void miss_insert(info *x, const cts *id)
{
    long p = bsearch_ts(x->miss, 0, (long)x->nm, id);
    if (p >= 0) return;
    p = -1 - p;
    cts *r = malloc((x->nm + 1) * sizeof *r);
    memcpy(r, x->miss, (size_t)p * sizeof *r);
    r[p] = *id;
    memcpy(r + p + 1, x->miss + p, (x->nm - (size_t)p) * sizeof *r);
    free(x->miss); x->miss = r; ++x->nm;
}

/* removeMissing (:946-972) */
static void remove_missing(cfk *c, const cts *id)
{
    for (size_t i = 0; i < c->n; ++i) {
        info *x = &c->t[i];
        if (!x->nm) continue;
        long j = bsearch_ts(x->miss, 0, (long)x->nm, id);
        if (j < 0) continue;
        memmove(x->miss + j, x->miss + j + 1, (x->nm - (size_t)j - 1) * sizeof(cts));
        --x->nm;
    }
}

/* mergeAndFilterMissing (:988-1025): additions[0, count) filtered by owner.kind().witnesses(), merged into current */
static void merge_filter_missing(info *owner, const cts *add, size_t count, cerr *e)
{
    unsigned kinds = c_witnesses(c_kind(&owner->id));
    size_t keep = 0;
    for (size_t i = 0; i < count; ++i) keep += (kinds >> c_kind(&add[i])) & 1u;
    if (!keep) return;
    cts *r = malloc((owner->nm + keep) * sizeof *r);
    size_t i = 0, j = 0, n = 0;
    while (i < count && j < owner->nm) {
        if ((kinds >> c_kind(&add[i])) & 1u) {
            if (c_cmp(&add[i], &owner->miss[j]) < 0) r[n++] = add[i++];
            else r[n++] = owner->miss[j++];
        } else ++i;
    }
    for (; i < count; ++i) if ((kinds >> c_kind(&add[i])) & 1u) r[n++] = add[i];
    while (j < owner->nm) r[n++] = owner->miss[j++];
    if (n != owner->nm + keep) c_fail(e, -2, "mergeAndFilterMissing: a missing TxnId was already present");
    free(owner->miss); owner->miss = r; owner->nm = n;
}

/* to (:1027-1033) */
static size_t to_pos(const info *x, const cts *missing_src, size_t missing_count, size_t missing_limit)
{
    if (dkb_is_self(x)) return missing_count;
    long t = bsearch_ts(missing_src, 0, (long)missing_limit, dkb(x));
    if (t < 0) t = -1 - t;
    return (size_t)t;
}

static info mk_info(const cts *id, int st, const cts *ex, int ex_self, cts *miss, size_t nm)
{
    info x; x.id = *id; x.st = st; x.ex_self = ex_self; x.ex = ex_self ? *id : *ex; x.miss = miss; x.nm = nm;
    return x;
}

/* insertInfoAndOneMissing (:899-944) + insert(pos, TxnInfo) (:880-897) */
static void insert_plain(cfk *c, size_t pos, info ins)
{
    info *nt = malloc((c->n + 1) * sizeof *nt);
    if (ins.st >= COMMITTED) {
        memcpy(nt, c->t, pos * sizeof *nt);
        nt[pos] = ins;
        memcpy(nt + pos + 1, c->t + pos, (c->n - pos) * sizeof *nt);
    } else {
        for (size_t i = 0; i < pos; ++i) {
            info x = c->t[i];
            if (has_info(x.st)) {   /* hasDeps() */
                if (c_cmp(dkb(&x), &ins.id) > 0 && witnesses(&x.id, &ins.id)) miss_insert(&x, &ins.id);
            }
            nt[i] = x;
        }
        nt[pos] = ins;
        for (size_t i = pos; i < c->n; ++i) {
            info x = c->t[i];
            if (has_info(x.st) && witnesses(&x.id, &ins.id)) miss_insert(&x, &ins.id);
            nt[i + 1] = x;
        }
    }
    free(c->t); c->t = nt; ++c->n;
}

/* update(pos, txnId, cur, new) (:865-875) */
static void update_plain(cfk *c, size_t pos, info nw)
{
    int crossed = c->t[pos].st < COMMITTED && nw.st >= COMMITTED;
    free(c->t[pos].miss);
    c->t[pos] = nw;
    if (crossed) remove_missing(c, &nw.id);
}

/* computeInfoAndAdditions (:1057-1149): the new TxnInfo (with its missing[]) and the deps this CFK does not know */
static info compute_info(const cfk *c, long insert_pos, long update_pos, const cts *id, int st, const cts *ex_in,
                         const cts *deps, size_t nd, cts **additions, size_t *n_add, cerr *e)
{
    int ex_self = 1;
    cts ex = *id;
    if (has_info(st) && c_cmp(ex_in, id) != 0) { ex = *ex_in; ex_self = 0; }
    /* depsKnownBefore = status.depsKnownBefore(txnId, executeAt) */
    const int self = st == PRE || st == ACC || ex_self;
    const cts *dk = self ? id : &ex;
    long dpos;
    if (self) dpos = insert_pos;
    else {
        dpos = bsearch_info(c, insert_pos, (long)c->n, dk);
        if (dpos >= 0) c_fail(e, -2, "computeInfoAndAdditions: depsKnownBefore matches a TxnId");
        dpos = -1 - dpos;
    }
    cts *miss = malloc((c->n + 1) * sizeof *miss);
    cts *add = malloc((nd + 1) * sizeof *add);
    size_t nm = 0, na = 0, di = 0;
    long ti = 0;
    while (ti < dpos && di < nd) {
        const info *t = &c->t[ti];
        int r = c_cmp(&t->id, &deps[di]);
        if (r == 0) { ++ti; ++di; }
        else if (r < 0) {
            if (ti != update_pos && t->st < COMMITTED && witnesses(id, &t->id)) miss[nm++] = t->id;
            ++ti;
        } else add[na++] = deps[di++];
    }
    while (ti < dpos) {
        const info *t = &c->t[ti];
        if (ti != update_pos && t->st < COMMITTED && witnesses(id, &t->id)) miss[nm++] = t->id;
        ++ti;
    }
    while (di < nd) add[na++] = deps[di++];
    *additions = add; *n_add = na;
    return mk_info(id, st, &ex, ex_self, miss, nm);
}

/* updateOrInsertWithAdditions (:772-863) */
static void update_or_insert_with_additions(cfk *c, long src_insert, long src_update, info winfo, const cts *add,
                                            size_t n_add, cerr *e)
{
    const cts *upd = &winfo.id;
    long aip = bsearch_ts(add, 0, (long)n_add, upd);
    if (aip >= 0) { c_fail(e, -1, "an addition equals the updated TxnId"); return; }
    aip = -1 - aip;
    const size_t target = (size_t)src_insert + (size_t)aip;
    const size_t newn = c->n + n_add + (src_update < 0 ? 1 : 0);
    info *nt = calloc(newn + 1, sizeof *nt);
    const cts *msrc = add;
    cts *owned = NULL;
    const int insert_self_missing = src_update < 0 && winfo.st < COMMITTED;
    size_t i = 0, j = 0, mcount = 0, mlimit = n_add, count = 0;
    while (i < c->n) {
        if (count == target) {
            nt[count] = winfo;
            if ((long)i == src_update) { free(c->t[i].miss); ++i; }
            else if (insert_self_missing) ++mcount;
            ++count;
            continue;
        }
        int r = j == n_add ? -1 : c_cmp(&c->t[i].id, &add[j]);
        if (r < 0) {
            info x = c->t[i];
            if ((long)i == src_update) { free(x.miss); x = winfo; }
            else if (has_info(x.st)) {
                if (insert_self_missing && msrc == add &&
                    (mcount != j || (!dkb_is_self(&x) && c_cmp(dkb(&x), upd) > 0))) {
                    /* insertMissing (:979-986): the additions plus the inserted TxnId */
                    owned = malloc((n_add + 1) * sizeof *owned);
                    memcpy(owned, add, (size_t)aip * sizeof *owned);
                    owned[aip] = *upd;
                    memcpy(owned + aip + 1, add + aip, (n_add - (size_t)aip) * sizeof *owned);
                    msrc = owned;
                    ++mlimit;
                }
                size_t to = to_pos(&x, msrc, mcount, mlimit);
                if (to > 0) merge_filter_missing(&x, msrc, to, e);
            }
            nt[count] = x;
            ++i;
        } else if (r > 0) {
            cts a = add[j++];
            nt[count] = mk_info(&a, TK, &a, 1, NULL, 0);   /* TxnInfo.create(txnId, TRANSITIVELY_KNOWN, txnId) */
            ++mcount;
        } else {
            c_fail(e, -2, "an addition matched an existing TxnId");
            ++i;
        }
        ++count;
    }
    if (j < n_add) {
        if (count <= target) {
            while (count < target) { cts a = add[j++]; nt[count++] = mk_info(&a, TK, &a, 1, NULL, 0); }
            nt[target] = winfo;
            count = target + 1;
        }
        while (j < n_add) { cts a = add[j++]; nt[count++] = mk_info(&a, TK, &a, 1, NULL, 0); }
    } else if (count == target) {
        nt[target] = winfo;
        ++count;
    }
    free(owned);
    free(c->t);
    c->t = nt;
    c->n = count;
}

/* fl: bit 0 = acceptedOrCommitted changed since the previous update, bit 1 = next.status() == AcceptedInvalidate */
static void apply_one(cfk *c, const cts *id, const cts *ex, int st, int fl, const cts *deps, size_t nd, cerr *e)
{
    long pos = bsearch_info(c, 0, (long)c->n, id);
    if (pos < 0) {
        pos = -1 - pos;
        if (has_info(st)) {
            cts *add; size_t na;
            info ni = compute_info(c, pos, -1, id, st, ex, deps, nd, &add, &na, e);
            if (na == 0) insert_plain(c, (size_t)pos, ni);
            else update_or_insert_with_additions(c, pos, -1, ni, add, na, e);
            free(add);
        } else {
            insert_plain(c, (size_t)pos, mk_info(id, st, id, 1, NULL, 0));
        }
        return;
    }
    info *cur = &c->t[pos];
    if (st <= cur->st) {
        /* Invariants.checkState(cur.status == newStatus || next.status() == AcceptedInvalidate) (:681-686) */
        if (cur->st != st && !(fl & 2)) { c_fail(e, -2, "stale status update to CommandsForKey (IllegalStateException)"); return; }
        if (!has_info(st) || !(fl & 1)) return;            /* acceptedOrCommitted unchanged: this (:687-688) */
    }
    const int prev_st = cur->st;
    if (has_info(st)) {
        cts *add; size_t na;
        info ni = compute_info(c, pos, pos, id, st, ex, deps, nd, &add, &na, e);
        if (na == 0) update_plain(c, (size_t)pos, ni);
        else {
            update_or_insert_with_additions(c, pos, pos, ni, add, na, e);
            if (prev_st < COMMITTED && st >= COMMITTED) remove_missing(c, id);
        }
        free(add);
    } else {
        update_plain(c, (size_t)pos, mk_info(id, st, id, 1, NULL, 0));
    }
}

static int cmp_u64p(const void *a, const void *b)
{
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

orc_cfk_result *orc_cfk_apply(uint32_t n_keys, const uint64_t *key, const uint32_t *ent_off,
                              const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                              const uint64_t *xmsb, const uint64_t *xlsb, const int32_t *xnode, const uint8_t *est,
                              const uint32_t *miss_off, const uint64_t *mmsb, const uint64_t *mlsb, const int32_t *mnode,
                              uint32_t n_upd, const uint64_t *umsb, const uint64_t *ulsb, const int32_t *unode,
                              const uint64_t *uxmsb, const uint64_t *uxlsb, const int32_t *uxnode, const uint8_t *ust,
                              const uint8_t *uflags, const uint32_t *ukey_off, const uint64_t *ukey,
                              const uint32_t *udep_off, const uint64_t *dmsb, const uint64_t *dlsb, const int32_t *dnode)
{
    orc_cfk_result *R = calloc(1, sizeof *R);
    cerr E = { 0, "" };
    /* the union of snapshot keys and update keys */
    size_t nu_keys = n_upd ? ukey_off[n_upd] : 0;
    uint64_t *all = malloc((n_keys + nu_keys + 1) * sizeof *all);
    memcpy(all, key, n_keys * sizeof *all);
    memcpy(all + n_keys, ukey, nu_keys * sizeof *all);
    qsort(all, n_keys + nu_keys, sizeof *all, cmp_u64p);
    size_t nk = 0;
    for (size_t i = 0; i < n_keys + nu_keys; ++i) if (nk == 0 || all[nk - 1] != all[i]) all[nk++] = all[i];
    cfk *cs = calloc(nk + 1, sizeof *cs);
    for (uint32_t k = 0; k < n_keys; ++k) {
        if (k && key[k - 1] >= key[k]) c_fail(&E, -1, "snapshot keys must be sorted unique");
        size_t a = 0, z = nk;
        while (a < z) { size_t m = (a + z) / 2; if (all[m] < key[k]) a = m + 1; else z = m; }
        cfk *c = &cs[a];
        c->n = ent_off[k + 1] - ent_off[k];
        c->t = calloc(c->n + 1, sizeof *c->t);
        for (size_t i = 0; i < c->n; ++i) {
            uint32_t x = ent_off[k] + (uint32_t)i;
            cts id = { emsb[x], elsb[x], enode[x] }, ex = { xmsb[x], xlsb[x], xnode[x] };
            int self = c_cmp(&ex, &id) == 0;
            size_t nm = miss_off[x + 1] - miss_off[x];
            cts *mm = malloc((nm + 1) * sizeof *mm);
            for (size_t q = 0; q < nm; ++q) mm[q] = (cts){ mmsb[miss_off[x] + q], mlsb[miss_off[x] + q], mnode[miss_off[x] + q] };
            c->t[i] = mk_info(&id, est[x], &ex, self, mm, nm);
            if (est[x] > INVALID) c_fail(&E, -1, "invalid InternalStatus ordinal");
            if (i && c_cmp(&c->t[i - 1].id, &id) >= 0) c_fail(&E, -1, "CommandsForKey entries must be sorted unique by TxnId");
        }
    }
    /* every update, to each of its keys, in batch order (SafeCommandStore.updateCommandsForKey) */
    for (uint32_t u = 0; u < n_upd && !E.code; ++u) {
        cts id = { umsb[u], ulsb[u], unode[u] }, ex = { uxmsb[u], uxlsb[u], uxnode[u] };
        if (ust[u] == 0xFF) continue;                        /* InternalStatus.from(saveStatus) == null */
        if (ust[u] > INVALID) { c_fail(&E, -1, "invalid InternalStatus ordinal"); break; }
        for (uint32_t j = ukey_off[u]; j < ukey_off[u + 1] && !E.code; ++j) {
            if (j > ukey_off[u] && ukey[j - 1] >= ukey[j]) { c_fail(&E, -1, "keys of an update must be sorted unique"); break; }
            size_t a = 0, z = nk;
            while (a < z) { size_t m = (a + z) / 2; if (all[m] < ukey[j]) a = m + 1; else z = m; }
            size_t nd = udep_off[j + 1] - udep_off[j];
            cts *deps = malloc((nd + 1) * sizeof *deps);
            for (size_t q = 0; q < nd; ++q) deps[q] = (cts){ dmsb[udep_off[j] + q], dlsb[udep_off[j] + q], dnode[udep_off[j] + q] };
            for (size_t q = 1; q < nd; ++q) if (c_cmp(&deps[q - 1], &deps[q]) >= 0) c_fail(&E, -1, "deps must be sorted unique");
            if (!E.code) apply_one(&cs[a], &id, &ex, ust[u], uflags[u], deps, nd, &E);
            free(deps);
        }
    }
    /* output, key-major */
    size_t ne = 0, nmiss = 0, nkeys_out = 0;
    for (size_t k = 0; k < nk; ++k) {
        if (!cs[k].n) continue;
        ++nkeys_out; ne += cs[k].n;
        for (size_t i = 0; i < cs[k].n; ++i) nmiss += cs[k].t[i].nm;
    }
    R->n_keys = (uint32_t)nkeys_out;
    R->key = malloc((nkeys_out + 1) * sizeof(uint64_t));
    R->ent_off = malloc((nkeys_out + 1) * sizeof(uint32_t));
    R->emsb = malloc((ne + 1) * 8); R->elsb = malloc((ne + 1) * 8); R->enode = malloc((ne + 1) * 4);
    R->xmsb = malloc((ne + 1) * 8); R->xlsb = malloc((ne + 1) * 8); R->xnode = malloc((ne + 1) * 4);
    R->status = malloc(ne + 1);
    R->miss_off = malloc((ne + 1) * sizeof(uint32_t));
    R->mmsb = malloc((nmiss + 1) * 8); R->mlsb = malloc((nmiss + 1) * 8); R->mnode = malloc((nmiss + 1) * 4);
    size_t ko = 0, eo = 0, mo = 0;
    R->ent_off[0] = 0; R->miss_off[0] = 0;
    for (size_t k = 0; k < nk; ++k) {
        cfk *c = &cs[k];
        if (c->n) {
            R->key[ko++] = all[k];
            for (size_t i = 0; i < c->n; ++i, ++eo) {
                info *x = &c->t[i];
                R->emsb[eo] = x->id.msb; R->elsb[eo] = x->id.lsb; R->enode[eo] = x->id.node;
                R->xmsb[eo] = x->ex.msb; R->xlsb[eo] = x->ex.lsb; R->xnode[eo] = x->ex.node;
                R->status[eo] = (uint8_t)x->st;
                for (size_t q = 0; q < x->nm; ++q, ++mo) { R->mmsb[mo] = x->miss[q].msb; R->mlsb[mo] = x->miss[q].lsb; R->mnode[mo] = x->miss[q].node; }
                R->miss_off[eo + 1] = (uint32_t)mo;
            }
            R->ent_off[ko] = (uint32_t)eo;
        }
        for (size_t i = 0; i < c->n; ++i) free(c->t[i].miss);
        free(c->t);
    }
    R->n_entries = ne; R->n_missing = nmiss;
    R->error = E.code;
    snprintf(R->message, sizeof R->message, "%s", E.msg);
    free(cs); free(all);
    return R;
}

void orc_cfk_free(orc_cfk_result *r)
{
    if (!r) return;
    free(r->key); free(r->ent_off); free(r->emsb); free(r->elsb); free(r->enode); free(r->xmsb); free(r->xlsb);
    free(r->xnode); free(r->status); free(r->miss_off); free(r->mmsb); free(r->mlsb); free(r->mnode);
    free(r);
}

/* ------------------------------------------------------------------ MaxConflicts (local/MaxConflicts.java:31-96) */

/* MaxConflicts.get(keysOrRanges) after merge(create(keysOrRanges_u, executeAt_u)) of every update u, restated
 * point-wise: the ReducingRangeMap's value at a point is the Timestamp::max of the updates covering it (a key enters
 * as asRange(), covering exactly itself), and foldl over the query's keys / ranges visits every map entry they
 * intersect; then CommandStore.preaccept's test txnId.compareTo(minNonConflicting) >= 0 (CommandStore.java:320-345). */
static int mc_range_contains(uint64_t s, uint64_t e, uint64_t k, int ei) { return ei ? (s < k && k <= e) : (s <= k && k < e); }

int orc_max_conflicts(uint32_t n_upd, const uint64_t *xmsb, const uint64_t *xlsb, const int32_t *xnode,
                      const uint32_t *key_off, const uint64_t *key, const uint32_t *rng_off, const uint64_t *rs,
                      const uint64_t *re, int end_inclusive, uint32_t nq, const uint64_t *qmsb, const uint64_t *qlsb,
                      const int32_t *qnode, const uint8_t *is_range, const uint32_t *part_off, const uint64_t *ps,
                      const uint64_t *pe, uint64_t *omsb, uint64_t *olsb, int32_t *onode, uint8_t *fast)
{
    for (uint32_t q = 0; q < nq; ++q) {
        int have = 0;
        cts best = { 0, 0, 0 };
        for (uint32_t u = 0; u < n_upd; ++u) {
            int hit = 0;
            for (uint32_t p = part_off[q]; p < part_off[q + 1] && !hit; ++p) {
                if (is_range[q]) {
                    for (uint32_t j = key_off[u]; j < key_off[u + 1] && !hit; ++j)
                        hit = mc_range_contains(ps[p], pe[p], key[j], end_inclusive);
                    for (uint32_t j = rng_off[u]; j < rng_off[u + 1] && !hit; ++j)
                        hit = rs[j] < pe[p] && re[j] > ps[p];
                } else {
                    for (uint32_t j = key_off[u]; j < key_off[u + 1] && !hit; ++j) hit = key[j] == ps[p];
                    for (uint32_t j = rng_off[u]; j < rng_off[u + 1] && !hit; ++j)
                        hit = mc_range_contains(rs[j], re[j], ps[p], end_inclusive);
                }
            }
            if (!hit) continue;
            cts x = { xmsb[u], xlsb[u], xnode[u] };
            if (!have || c_cmp(&best, &x) < 0) best = x;   /* Timestamp.max */
            have = 1;
        }
        omsb[q] = best.msb; olsb[q] = best.lsb; onode[q] = best.node;
        cts id = { qmsb[q], qlsb[q], qnode[q] };
        fast[q] = (uint8_t)(c_cmp(&id, &best) >= 0);
    }
    return 0;
}
