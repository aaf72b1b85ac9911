// cfk.hip — a device-resident CommandsForKey store maintained incrementally:
// CommandsForKey.update(prev, next) (local/CommandsForKey.java:652-706), as SafeCommandStore.updateCommandsForKey calls it
// for every key of a command (local/SafeCommandStore.java:217-240), applied to a batch of commands at once.
//
// The store keeps the snapshot that acc_keydeps_batch / acc_map_reduce_full / acc_shard_* read, resident in HBM across
// batches: per txn (sorted by TxnId) TxnId, executeAt, InternalStatus and its keys (txn-major CSR, keys ascending).
// An update of D commands costs O(n + P) streaming passes plus O(D log n) searches instead of re-staging the whole
// snapshot from the host:
//   1. delta TxnIds dense-ranked (Timestamp.compareTo) -> sorted delta order (duplicates -> ACC_E_ARG);
//   2. each delta txn searched among the stored TxnIds: present -> update in place (the status must not go back:
//      newStatus < cur is the reference's IllegalStateException "stale status"; equal status without info is a no-op;
//      executeAt = txnId when the new status has no info, TxnInfo.create :669-670), absent -> insert;
//   3. stored txn j moves to j + #(inserted TxnIds below it); inserted txn m (delta order) lands at its insert position
//      + m; key lists merge (a command registers on keys it was not yet on);
//   4. key offsets by one scan, then every column is written once into the other buffer set, and the sets swap.
#include "dict.hpp"

struct acc_cfk {
    int device = 0;
    uint32_t n = 0;
    uint64_t P = 0;
    struct Set {
        uint64_t *tm = nullptr, *tl = nullptr, *em = nullptr, *el = nullptr, *key_code = nullptr;
        int32_t *tn = nullptr, *en = nullptr;
        uint8_t *status = nullptr;
        uint32_t *key_off = nullptr;
        size_t cap_n = 0, cap_p = 0;
        // byte sizes of the arrays above in declaration order (tm tl em el key_code tn en status key_off): they differ
        // once acc_cfk_apply_deps has adopted a call's result arrays
        size_t bytes[9] = {};
    } set[2];
    int cur = 0;
    // acc_cfk_apply_deps: the same store with every TxnInfo's missing[] — the key-major CommandsForKey state (what
    // acc_cfk_apply maintains) and, beside the txn-major view above, each (txn, key) pair's missing[] as txn indices
    // (what acc_map_reduce_full reads). Both are rewritten by every acc_cfk_apply_deps, so the scans and the next update
    // read the one state in place.
    bool deps = false;
    struct KeyMajor {
        uint32_t nk = 0;
        uint64_t ne = 0, nm = 0;
        uint64_t *key = nullptr, *em = nullptr, *el = nullptr, *xm = nullptr, *xl = nullptr, *mm = nullptr, *ml = nullptr;
        int32_t *en = nullptr, *xn = nullptr, *mn = nullptr;
        uint8_t *st = nullptr;
        uint32_t *ent_off = nullptr, *miss_off = nullptr;
        // byte sizes (key ent_off em el en xm xl xn st miss_off mm ml mn): adopted result arrays (acc_cfk_apply_deps)
        size_t bytes[13] = {};
    } km;
    uint32_t *bmiss_off = nullptr, *bmiss_txn = nullptr;   // [P + 1], [bnm]
    uint64_t bnm = 0;
    size_t bytes_bmo = 0, bytes_bmt = 0;
};

namespace acc {

namespace cf {

constexpr uint64_t IDENTITY_LSB = 0xFFFFFFFFFFFF001EULL;
enum : uint64_t { E_STATUS = 1, E_KIND = 2, E_KEYS = 4, E_STALE = 8, E_OFF = 16, E_DUP = 32 };

__device__ __forceinline__ int ts_cmp(uint64_t am, uint64_t al, int32_t an, uint64_t bm, uint64_t bl, int32_t bn)
{
    if (am != bm) return am < bm ? -1 : 1;
    const uint64_t a1 = al & IDENTITY_LSB, b1 = bl & IDENTITY_LSB;
    if (a1 != b1) return a1 < b1 ? -1 : 1;
    if (an != bn) return an < bn ? -1 : 1;
    return 0;
}

__host__ __device__ inline bool has_info(uint32_t s) { return s >= ACC_ST_ACCEPTED && s <= ACC_ST_APPLIED; }

struct Delta {
    const uint64_t *tm, *tl, *em, *el, *key_code;
    const int32_t *tn, *en;
    const uint8_t *status;
    const uint32_t *key_off;
    uint32_t D;
};

struct Store {
    const uint64_t *tm, *tl, *em, *el, *key_code;
    const int32_t *tn, *en;
    const uint8_t *status;
    const uint32_t *key_off;
    uint32_t n;
};

struct Out {
    uint64_t *tm, *tl, *em, *el, *key_code;
    int32_t *tn, *en;
    uint8_t *status;
    uint32_t *key_off;
};

}  // namespace cf

using namespace cf;

// the key loop stays inside [0, Pd) whatever key_off holds: offsets must start at 0, not decrease and stay within Pd
__global__ __launch_bounds__(BLOCK) void k_cf_validate(Delta d, uint32_t Pd, uint64_t *__restrict__ errs, uint64_t *__restrict__ w0,
                                                       uint64_t *__restrict__ w1, uint64_t *__restrict__ w2)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= d.D) return;
    uint64_t e = 0;
    if (d.status[i] > ACC_ST_INVALID_OR_TRUNCATED) e |= E_STATUS;
    if (((d.tl[i] >> 1) & 7u) > ACC_KIND_LOCAL_ONLY) e |= E_KIND;
    const uint32_t k0 = d.key_off[i], k1 = d.key_off[i + 1];
    if (k1 < k0 || k1 > Pd || (i == 0 && k0 != 0)) e |= E_OFF;
    else
        for (uint32_t j = k0 + 1; j < k1; ++j)
            if (d.key_code[j - 1] >= d.key_code[j]) { e |= E_KEYS; break; }
    w0[i] = d.tm[i];
    w1[i] = d.tl[i] & IDENTITY_LSB;
    w2[i] = (uint64_t)((uint32_t)d.tn[i] ^ 0x80000000u);
    if (e) atomicOr((unsigned long long *)errs, (unsigned long long)e);
}

__global__ __launch_bounds__(BLOCK) void k_cf_order(uint32_t D, const uint32_t *__restrict__ rank, uint32_t *__restrict__ ord)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < D) ord[rank[i]] = i;
}

// sorted delta txn k: its lower bound among the stored TxnIds, found or not, the status rule, the new-txn flag
__global__ __launch_bounds__(BLOCK) void k_cf_locate(Delta d, Store s, const uint32_t *__restrict__ ord, uint32_t *__restrict__ pos,
                                                     uint32_t *__restrict__ isnew, int32_t *__restrict__ upd_of_old,
                                                     uint64_t *__restrict__ errs, uint32_t *__restrict__ skipped)
{
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k >= d.D) return;
    const uint32_t i = ord[k];
    const uint64_t xm = d.tm[i], xl = d.tl[i];
    const int32_t xn = d.tn[i];
    const uint32_t kind = (uint32_t)(xl >> 1) & 7u;
    if ((xl & 1u) || kind == ACC_KIND_EPHEMERAL_READ || kind == ACC_KIND_LOCAL_ONLY) {
        // only key-domain, globally visible txns are CommandsForKey members (SafeCommandStore.java:224)
        pos[k] = 0;
        isnew[k] = 0;
        atomicAdd(skipped, 1u);
        return;
    }
    uint32_t lo = 0, hi = s.n;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (ts_cmp(s.tm[m], s.tl[m], s.tn[m], xm, xl, xn) < 0) lo = m + 1; else hi = m;
    }
    const bool found = lo < s.n && ts_cmp(s.tm[lo], s.tl[lo], s.tn[lo], xm, xl, xn) == 0;
    pos[k] = lo;
    isnew[k] = found ? 0u : 1u;
    if (found) {
        if (d.status[i] < s.status[lo]) atomicOr((unsigned long long *)errs, (unsigned long long)E_STALE);
        upd_of_old[lo] = (int32_t)i;
    }
}

__global__ __launch_bounds__(BLOCK) void k_cf_newpos(uint32_t D, const uint32_t *__restrict__ isnew, const uint32_t *__restrict__ newx,
                                                     const uint32_t *__restrict__ pos, uint32_t *__restrict__ newpos)
{
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k < D && isnew[k]) newpos[newx[k]] = pos[k];
}

__device__ __forceinline__ uint32_t merged_count(const uint64_t *a, uint32_t na, const uint64_t *b, uint32_t nb)
{
    uint32_t i = 0, j = 0, c = 0;
    while (i < na && j < nb) {
        if (a[i] < b[j]) ++i;
        else if (b[j] < a[i]) ++j;
        else { ++i; ++j; }
        ++c;
    }
    return c + (na - i) + (nb - j);
}

// new index and key count of every stored txn (updated or not) and every inserted txn
__global__ __launch_bounds__(BLOCK) void k_cf_counts(Delta d, Store s, const int32_t *__restrict__ upd_of_old, uint32_t nnew,
                                                     const uint32_t *__restrict__ newpos, const uint32_t *__restrict__ ord,
                                                     const uint32_t *__restrict__ isnew, const uint32_t *__restrict__ newx,
                                                     const uint32_t *__restrict__ pos, uint32_t *__restrict__ kcount)
{
    const uint32_t x = blockIdx.x * BLOCK + threadIdx.x;
    if (x < s.n) {
        uint32_t lo = 0, hi = nnew;   // inserted TxnIds below stored txn x: insert positions <= x
        while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (newpos[m] <= x) lo = m + 1; else hi = m; }
        const uint32_t dst = x + lo;
        const uint32_t a0 = s.key_off[x], na = s.key_off[x + 1] - a0;
        const int32_t u = upd_of_old[x];
        kcount[dst] = u < 0 ? na
                            : merged_count(s.key_code + a0, na, d.key_code + d.key_off[u], d.key_off[u + 1] - d.key_off[u]);
    }
    if (x < d.D && isnew[x]) {
        const uint32_t i = ord[x];
        kcount[pos[x] + newx[x]] = d.key_off[i + 1] - d.key_off[i];
    }
}

__device__ __forceinline__ void put_txn(const Out &o, uint32_t t, uint64_t tm, uint64_t tl, int32_t tn, uint64_t em, uint64_t el,
                                        int32_t en, uint8_t st)
{
    o.tm[t] = tm; o.tl[t] = tl; o.tn[t] = tn; o.em[t] = em; o.el[t] = el; o.en[t] = en; o.status[t] = st;
}

__global__ __launch_bounds__(BLOCK) void k_cf_write(Delta d, Store s, const int32_t *__restrict__ upd_of_old, uint32_t nnew,
                                                    const uint32_t *__restrict__ newpos, const uint32_t *__restrict__ ord,
                                                    const uint32_t *__restrict__ isnew, const uint32_t *__restrict__ newx,
                                                    const uint32_t *__restrict__ pos, Out o)
{
    const uint32_t x = blockIdx.x * BLOCK + threadIdx.x;
    if (x < s.n) {
        uint32_t lo = 0, hi = nnew;
        while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (newpos[m] <= x) lo = m + 1; else hi = m; }
        const uint32_t dst = x + lo;
        const uint32_t a0 = s.key_off[x], na = s.key_off[x + 1] - a0;
        const int32_t u = upd_of_old[x];
        uint64_t em = s.em[x], el = s.el[x];
        int32_t en = s.en[x];
        uint8_t st = s.status[x];
        uint64_t *out = o.key_code + o.key_off[dst];
        if (u < 0) {
            for (uint32_t j = 0; j < na; ++j) out[j] = s.key_code[a0 + j];
        } else {
            const uint8_t ns = d.status[u];
            // CommandsForKey.update :674-703: a higher status, or the same status with info, replaces the entry
            if (ns > st || has_info(ns)) {
                st = ns;
                if (has_info(ns)) { em = d.em[u]; el = d.el[u]; en = d.en[u]; }
                else { em = s.tm[x]; el = s.tl[x]; en = s.tn[x]; }
            }
            const uint64_t *b = d.key_code + d.key_off[u];
            const uint32_t nb = d.key_off[u + 1] - d.key_off[u];
            const uint64_t *a = s.key_code + a0;
            uint32_t i = 0, j = 0, c = 0;
            while (i < na || j < nb) {
                if (j >= nb || (i < na && a[i] < b[j])) out[c++] = a[i++];
                else if (i >= na || b[j] < a[i]) out[c++] = b[j++];
                else { out[c++] = a[i++]; ++j; }
            }
        }
        put_txn(o, dst, s.tm[x], s.tl[x], s.tn[x], em, el, en, st);
    }
    if (x < d.D && isnew[x]) {
        const uint32_t i = ord[x], dst = pos[x] + newx[x];
        const uint8_t ns = d.status[i];
        // TxnInfo.create(txnId, status, txnId) for statuses without info (:669-670)
        if (has_info(ns)) put_txn(o, dst, d.tm[i], d.tl[i], d.tn[i], d.em[i], d.el[i], d.en[i], ns);
        else put_txn(o, dst, d.tm[i], d.tl[i], d.tn[i], d.tm[i], d.tl[i], d.tn[i], ns);
        uint64_t *out = o.key_code + o.key_off[dst];
        for (uint32_t j = d.key_off[i]; j < d.key_off[i + 1]; ++j) out[j - d.key_off[i]] = d.key_code[j];
    }
}

namespace {

template <class T>
void realloc_dev(T *&p, size_t count)
{
    if (p) ACC_HIP(hipFree(p));
    p = nullptr;
    ACC_HIP(hipMalloc(&p, count * sizeof(T)));
}

// capacity for n txns (txn columns, n + 1 key offsets) and P key codes; contents are not kept
void reserve(acc_cfk::Set &s, size_t n, size_t P)
{
    if (n + 2 > s.cap_n) {
        const size_t c = n + n / 4 + 64;
        realloc_dev(s.tm, c); realloc_dev(s.tl, c); realloc_dev(s.em, c); realloc_dev(s.el, c);
        realloc_dev(s.tn, c); realloc_dev(s.en, c); realloc_dev(s.status, c); realloc_dev(s.key_off, c);
        s.cap_n = c;
        s.bytes[0] = s.bytes[1] = s.bytes[2] = s.bytes[3] = c * 8;
        s.bytes[5] = s.bytes[6] = s.bytes[8] = c * 4;
        s.bytes[7] = c;
    }
    if (P + 1 > s.cap_p) {
        const size_t c = P + P / 4 + 64;
        realloc_dev(s.key_code, c);
        s.cap_p = c;
        s.bytes[4] = c * 8;
    }
}

}  // namespace

void cfk_update(acc_ctx *ctx, acc_cfk *cfk, const acc_batch_in *in)
{
    if (!cfk || !in) fail(ACC_E_ARG, "null argument");
    if (cfk->deps)
        fail(ACC_E_STATE, "the store holds missing[] (acc_cfk_apply_deps): status-only updates would not maintain it");
    if (in->mem != ACC_MEM_HOST && in->mem != ACC_MEM_DEVICE) fail(ACC_E_ARG, "mem must be ACC_MEM_HOST or ACC_MEM_DEVICE");
    hipStream_t st = ctx->stream;
    const uint32_t D = in->n_txn;
    const size_t Pd = (size_t)in->n_pairs;
    Delta d{};
    d.D = D;
    d.key_off = stage_in(ctx, "cf_key_off", in->key_off, (size_t)D + 1, in->mem);
    d.tm = stage_in(ctx, "cf_tm", in->txn_id.msb, D, in->mem);
    d.tl = stage_in(ctx, "cf_tl", in->txn_id.lsb, D, in->mem);
    d.tn = stage_in(ctx, "cf_tn", in->txn_id.node, D, in->mem);
    d.em = stage_in(ctx, "cf_em", in->execute_at.msb, D, in->mem);
    d.el = stage_in(ctx, "cf_el", in->execute_at.lsb, D, in->mem);
    d.en = stage_in(ctx, "cf_en", in->execute_at.node, D, in->mem);
    d.status = stage_in(ctx, "cf_status", in->status, D, in->mem);
    d.key_code = stage_in(ctx, "cf_key_code", in->key_code, Pd, in->mem);
    if (D == 0) return;
    uint64_t *errs = ctx->get<uint64_t>("cf_errs", 1);
    ACC_HIP(hipMemsetAsync(errs, 0, 8, st));
    uint64_t *w[3] = { ctx->get<uint64_t>("cf_w0", D), ctx->get<uint64_t>("cf_w1", D), ctx->get<uint64_t>("cf_w2", D) };
    launch(ctx, "cf_validate", k_cf_validate, dim3(grid_for(D, BLOCK)), dim3(BLOCK), 0, d, (uint32_t)Pd, errs, w[0], w[1], w[2]);
    const uint64_t *words[3] = { w[0], w[1], w[2] };
    DenseRank dr = dense_rank(ctx, "cf_dr", D, 3, words, nullptr, nullptr, false);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, errs, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, dr.count_dev, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 2, d.key_off + D, 4, hipMemcpyDeviceToHost, st));
    ctx->sync();
    uint64_t e = ctx->pinned[0];
    if (e & E_STATUS) fail(ACC_E_ARG, "invalid InternalStatus ordinal (> INVALID_OR_TRUNCATED)");
    if (e & E_KIND) fail(ACC_E_ARG, "Kind.ofOrdinal: invalid kind ordinal in TxnId flags");
    if (e & E_OFF) fail(ACC_E_ARG, "key_off must start at 0, be non-decreasing and end at n_pairs");
    if (e & E_KEYS) fail(ACC_E_ARG, "keys of a txn must be sorted and unique (Keys.ofSortedUnique)");
    if (ctx->pinned[1] != D) fail(ACC_E_ARG, "TxnIds of one update must be distinct");
    if ((ctx->pinned[2] & 0xFFFFFFFFull) != Pd) fail(ACC_E_ARG, "key_off[n_txn] must equal n_pairs");

    acc_cfk::Set &S = cfk->set[cfk->cur];
    const uint32_t n = cfk->n;
    Store s{ S.tm, S.tl, S.em, S.el, S.key_code, S.tn, S.en, S.status, S.key_off, n };
    uint32_t *ord = ctx->get<uint32_t>("cf_ord", D);
    launch(ctx, "cf_order", k_cf_order, dim3(grid_for(D, BLOCK)), dim3(BLOCK), 0, D, (const uint32_t *)dr.rank, ord);
    uint32_t *pos = ctx->get<uint32_t>("cf_pos", D), *isnew = ctx->get<uint32_t>("cf_isnew", D);
    uint32_t *newx = ctx->get<uint32_t>("cf_newx", (size_t)D + 1);
    int32_t *upd = ctx->get<int32_t>("cf_upd", (size_t)n + 1);
    ACC_HIP(hipMemsetAsync(upd, 0xFF, ((size_t)n + 1) * 4, st));
    uint32_t *skipped = ctx->get<uint32_t>("cf_skipped", 1);
    ACC_HIP(hipMemsetAsync(skipped, 0, 4, st));
    launch(ctx, "cf_locate", k_cf_locate, dim3(grid_for(D, BLOCK)), dim3(BLOCK), 0, d, s, (const uint32_t *)ord, pos, isnew, upd, errs,
           skipped);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, isnew, newx, D, true, newx + D);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, errs, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, newx + D, 4, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 2, skipped, 4, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint32_t nskip = (uint32_t)(ctx->pinned[2] & 0xFFFFFFFFu);
    if (ctx->pinned[0] & E_STALE)
        fail(ACC_E_STATE, "Attempted update to CommandsForKey with a stale status (CommandsForKey.update :680-688)");
    const uint32_t nnew = (uint32_t)(ctx->pinned[1] & 0xFFFFFFFFu);
    uint32_t *newpos = ctx->get<uint32_t>("cf_newpos", (size_t)nnew + 1);
    launch(ctx, "cf_newpos", k_cf_newpos, dim3(grid_for(D, BLOCK)), dim3(BLOCK), 0, D, (const uint32_t *)isnew,
           (const uint32_t *)newx, (const uint32_t *)pos, newpos);
    const uint32_t n2 = n + nnew;
    uint32_t *kcount = ctx->get<uint32_t>("cf_kcount", (size_t)n2 + 1);
    const uint32_t gx = grid_for(std::max(n, D), BLOCK);
    launch(ctx, "cf_counts", k_cf_counts, dim3(gx), dim3(BLOCK), 0, d, s, (const int32_t *)upd, nnew, (const uint32_t *)newpos,
           (const uint32_t *)ord, (const uint32_t *)isnew, (const uint32_t *)newx, (const uint32_t *)pos, kcount);
    acc_cfk::Set &T = cfk->set[cfk->cur ^ 1];
    reserve(T, n2, 0);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, kcount, T.key_off, n2, true, T.key_off + n2);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, T.key_off + n2, 4, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t P2 = ctx->pinned[0] & 0xFFFFFFFFull;
    if (P2 >= 0xFFFFFFFFull - 1) fail(ACC_E_CAP, "CommandsForKey store too large (pairs >= 2^32)");
    reserve(T, n2, P2);
    Out o{ T.tm, T.tl, T.em, T.el, T.key_code, T.tn, T.en, T.status, T.key_off };
    launch(ctx, "cf_write", k_cf_write, dim3(gx), dim3(BLOCK), 0, d, s, (const int32_t *)upd, nnew, (const uint32_t *)newpos,
           (const uint32_t *)ord, (const uint32_t *)isnew, (const uint32_t *)newx, (const uint32_t *)pos, o);
    ctx->sync();
    cfk->cur ^= 1;
    cfk->n = n2;
    cfk->P = P2;
    ctx->stat("cfk.inserted", nnew);
    ctx->stat("cfk.updated", D - nnew - nskip);
    ctx->stat("cfk.skipped", nskip);   // range-domain, EphemeralRead, LocalOnly: no CommandsForKey entry
}

acc_cfk *cfk_new(int device)
{
    acc_cfk *c = new acc_cfk();
    c->device = device;
    return c;
}

void cfk_free(acc_cfk *cfk)
{
    if (!cfk) return;
    (void)hipSetDevice(cfk->device);
    for (auto &s : cfk->set) {
        (void)hipFree(s.tm); (void)hipFree(s.tl); (void)hipFree(s.em); (void)hipFree(s.el); (void)hipFree(s.key_code);
        (void)hipFree(s.tn); (void)hipFree(s.en); (void)hipFree(s.status); (void)hipFree(s.key_off);
    }
    auto &k = cfk->km;
    for (void *p : { (void *)k.key, (void *)k.em, (void *)k.el, (void *)k.xm, (void *)k.xl, (void *)k.mm, (void *)k.ml,
                     (void *)k.en, (void *)k.xn, (void *)k.mn, (void *)k.st, (void *)k.ent_off, (void *)k.miss_off,
                     (void *)cfk->bmiss_off, (void *)cfk->bmiss_txn })
        (void)hipFree(p);
    delete cfk;
}

void cfk_apply(acc_ctx *ctx, const acc_cfk_snap *in, const acc_cfk_updates *up, acc_cfk_snap_view *view);
void cfk_snap_to_batch(acc_ctx *ctx, const acc_cfk_snap *in, acc_cfk_batch_view *view, bool trusted = false);
void cfk_view(acc_cfk *cfk, acc_batch_in *out);

namespace {

acc_cfk_snap km_snap(acc_cfk *cfk)
{
    const acc_cfk::KeyMajor &k = cfk->km;
    return acc_cfk_snap{ ACC_MEM_DEVICE, k.nk, k.ne, k.nm, k.key, k.ent_off, acc_ts_cols{ k.em, k.el, k.en },
                         acc_ts_cols{ k.xm, k.xl, k.xn }, k.st, k.miss_off, acc_ts_cols{ k.mm, k.ml, k.mn } };
}

}  // namespace

// CommandsForKey.update with the command's deps on the store itself (local/CommandsForKey.java:657-1149 per key, as
// SafeCommandStore.updateCommandsForKey calls it, local/SafeCommandStore.java:217-240): acc_cfk_apply over the store's
// key-major state, then the txn-major view and its per-pair missing[] indices rebuilt from the result
// (acc_cfk_snap_to_batch), both copied into the store only when both succeeded — a rejected batch (stale status, bad
// offsets, a TxnId whose keys disagree on its status) leaves the store as it was.
void cfk_apply_deps(acc_ctx *ctx, acc_cfk *cfk, const acc_cfk_updates *up)
{
    if (!cfk || !up) fail(ACC_E_ARG, "null argument");
    if (!cfk->deps && cfk->n)
        fail(ACC_E_STATE, "the store holds status-only state (acc_cfk_update): missing[] is maintained from an empty store");
    acc_cfk::KeyMajor &k = cfk->km;
    if (!k.ent_off) {   // empty state: offsets [0]
        realloc_dev(k.ent_off, 1);
        realloc_dev(k.miss_off, 1);
        k.bytes[1] = k.bytes[9] = 4;
        ACC_HIP(hipMemsetAsync(k.ent_off, 0, 4, ctx->stream));
        ACC_HIP(hipMemsetAsync(k.miss_off, 0, 4, ctx->stream));
    }
    const acc_cfk_snap prev = km_snap(cfk);
    acc_cfk_snap_view v{};
    // stream time of the two halves (stats cfk.apply_us / cfk.view_us: the steady-state bench's view step)
    hipEvent_t ev[3] = { ctx->take_event(), ctx->take_event(), ctx->take_event() };
    struct Give {
        acc_ctx *c; hipEvent_t *e;
        ~Give() { for (int i = 0; i < 3; ++i) c->event_pool.push_back(e[i]); }
    } give{ ctx, ev };
    ACC_HIP(hipEventRecord(ev[0], ctx->stream));
    cfk_apply(ctx, &prev, up, &v);
    ACC_HIP(hipEventRecord(ev[1], ctx->stream));
    const acc_cfk_snap next{ ACC_MEM_DEVICE, v.n_keys, v.n_entries, v.n_missing, v.key, v.ent_off, v.txn_id, v.execute_at,
                             v.status, v.miss_off, v.missing };
    acc_cfk_batch_view bv{};
    cfk_snap_to_batch(ctx, &next, &bv, true);
    ACC_HIP(hipEventRecord(ev[2], ctx->stream));
    // ---- both results become the store's arrays: the context's result buffers and the store's previous arrays trade
    // places (no copies; the context writes its next results into the old arrays)
    auto adopt = [&](const char *name, auto *&p, size_t &bytes) {
        void *v = p;
        ctx->swap_buf(name, v, bytes);
        p = static_cast<std::remove_reference_t<decltype(p)>>(v);
    };
    const acc_batch_in &b = bv.batch;
    // the results must sit in the context's named buffers before any array is adopted: a rejected call leaves the
    // store holding its previous arrays, none of the new ones
    if (ctx->buf_ptr("cd_okey") != v.key || ctx->buf_ptr("cd_oem") != v.txn_id.msb || ctx->buf_ptr("cd_omm") != v.missing.msb ||
        ctx->buf_ptr("cd_omoff") != v.miss_off)
        fail(ACC_E_STATE, "internal: CommandsForKey result buffers moved");
    if (ctx->buf_ptr("cb_tm") != b.txn_id.msb || ctx->buf_ptr("cb_ko") != b.key_off || ctx->buf_ptr("cb_mo") != bv.missing_off)
        fail(ACC_E_STATE, "internal: CommandsForKey view buffers moved");
    const uint32_t nk = v.n_keys;
    const uint64_t ne = v.n_entries, nm = v.n_missing;
    size_t *kb = k.bytes;
    adopt("cd_okey", k.key, kb[0]); adopt("cd_oent_off", k.ent_off, kb[1]);
    adopt("cd_oem", k.em, kb[2]); adopt("cd_oel", k.el, kb[3]); adopt("cd_oen", k.en, kb[4]);
    adopt("cd_oxm", k.xm, kb[5]); adopt("cd_oxl", k.xl, kb[6]); adopt("cd_oxn", k.xn, kb[7]);
    adopt("cd_ost", k.st, kb[8]); adopt("cd_omoff", k.miss_off, kb[9]);
    adopt("cd_omm", k.mm, kb[10]); adopt("cd_oml", k.ml, kb[11]); adopt("cd_omn", k.mn, kb[12]);
    k.nk = nk; k.ne = ne; k.nm = nm;
    const uint32_t n = b.n_txn;
    const uint64_t P = b.n_pairs;
    acc_cfk::Set &S = cfk->set[cfk->cur];
    size_t *sb = S.bytes;
    adopt("cb_tm", S.tm, sb[0]); adopt("cb_tl", S.tl, sb[1]); adopt("cb_xm", S.em, sb[2]); adopt("cb_xl", S.el, sb[3]);
    adopt("cb_kc", S.key_code, sb[4]); adopt("cb_tn", S.tn, sb[5]); adopt("cb_xn", S.en, sb[6]);
    adopt("cb_st", S.status, sb[7]); adopt("cb_ko", S.key_off, sb[8]);
    S.cap_n = S.cap_p = 0;   // (sizes now per array: a status-only reserve would reallocate; deps mode refuses it)
    adopt("cb_mo", cfk->bmiss_off, cfk->bytes_bmo);
    adopt("cb_mt", cfk->bmiss_txn, cfk->bytes_bmt);
    cfk->bnm = bv.n_missing;
    ctx->sync();
    float ms_a = 0, ms_v = 0;
    ACC_HIP(hipEventElapsedTime(&ms_a, ev[0], ev[1]));
    ACC_HIP(hipEventElapsedTime(&ms_v, ev[1], ev[2]));
    ctx->stat("cfk.apply_us", (uint64_t)(ms_a * 1000.0f));
    ctx->stat("cfk.view_us", (uint64_t)(ms_v * 1000.0f));
    cfk->n = n;
    cfk->P = P;
    cfk->deps = true;
}

void cfk_state(acc_cfk *cfk, acc_cfk_snap *out)
{
    if (!cfk || !out) fail(ACC_E_ARG, "null argument");
    if (!cfk->deps) fail(ACC_E_STATE, "the store holds no missing[] state (no acc_cfk_apply_deps yet)");
    *out = km_snap(cfk);
}

void cfk_missing(acc_cfk *cfk, acc_cfk_batch_view *out)
{
    if (!cfk || !out) fail(ACC_E_ARG, "null argument");
    if (!cfk->deps) fail(ACC_E_STATE, "the store holds no missing[] state (no acc_cfk_apply_deps yet)");
    cfk_view(cfk, &out->batch);
    out->missing_off = cfk->bmiss_off;
    out->missing_txn = cfk->bmiss_txn;
    out->n_missing = cfk->bnm;
}

void cfk_view(acc_cfk *cfk, acc_batch_in *out)
{
    if (!cfk || !out) fail(ACC_E_ARG, "null argument");
    acc_cfk::Set &S = cfk->set[cfk->cur];
    if (!S.key_off) {   // empty store: a valid zero-txn batch
        reserve(S, 0, 0);
        ACC_HIP(hipMemset(S.key_off, 0, 4));
    }
    *out = acc_batch_in{ cfk->n, ACC_MEM_DEVICE, cfk->P, acc_ts_cols{ S.tm, S.tl, S.tn }, acc_ts_cols{ S.em, S.el, S.en },
                         S.status, S.key_off, S.key_code };
}

}  // namespace acc
