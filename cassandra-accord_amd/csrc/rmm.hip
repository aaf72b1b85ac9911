// rmm.hip — RelationMultiMap helpers over batches of built deps objects:
//   * invert:  RelationMultiMap.invert (utils/RelationMultiMap.java:907-938) = KeyDeps.txnIdsToKeys / RangeDeps
//              txnIdsToRanges (primitives/KeyDeps.java:350-362): a stable counting sort of every entry by TxnId;
//   * slice:   KeyDeps.slice(Ranges) (primitives/KeyDeps.java:189-236) / RangeDeps.slice(Ranges)
//              (primitives/RangeDeps.java:545-565) with trimUnusedValues (utils/RelationMultiMap.java:491-532);
//   * stab:    SearchableRangeList.forEach(key | range) (utils/SearchableRangeList.java:89-116) and
//              RangeDeps.computeTxnIds (primitives/RangeDeps.java:629-643) over a built RangeDeps: the range indices
//              containing a key / intersecting a range in ascending order (SearchableRangeListTest.java:98-112), and the
//              sorted unique TxnId indices behind them.
// A batch holds one deps object per group in the SerializerSupport layout; results are per group (per query for stab)
// CSRs, device-resident in the context. Integer work only (HBM-bound sorts, scans and binary searches).
#include "dict.hpp"

namespace acc {

namespace {

__device__ __forceinline__ uint64_t ub64(const uint64_t *a, uint64_t lo, uint64_t hi, uint64_t v)   // first a[i] > v
{
    while (lo < hi) { const uint64_t m = (lo + hi) >> 1; if (a[m] <= v) lo = m + 1; else hi = m; }
    return lo;
}

// header slot of entry position `local` (>= nk) of a keysToValues int[]: the key whose end offset first exceeds it
__device__ __forceinline__ uint32_t key_of_entry(const int32_t *h, uint32_t nk, uint32_t local)
{
    uint32_t lo = 0, hi = nk;
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if ((uint32_t)h[m] <= local) lo = m + 1; else hi = m; }
    return lo;
}

struct Batch {
    uint32_t ng;
    const uint64_t *key_off, *val_off, *k2v_off;
    const uint64_t *key_a, *key_b;
    const int32_t *k2v;
    uint64_t NK, NV, NO;
};

// per group: offsets monotone, header end offsets ascending within [nk, no] and == no at the last key (KeyDeps ctor,
// KeyDeps.java:179-186), entry values inside [0, nv). err bits: 1 layout, 2 value range
__global__ __launch_bounds__(BLOCK) void k_b_validate(Batch b, uint64_t *__restrict__ err)
{
    const uint64_t q = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    uint64_t e = 0;
    if (q < b.ng) {
        if (b.key_off[q + 1] < b.key_off[q] || b.val_off[q + 1] < b.val_off[q] || b.k2v_off[q + 1] < b.k2v_off[q] ||
            b.k2v_off[q + 1] - b.k2v_off[q] < b.key_off[q + 1] - b.key_off[q])
            e |= 1;
    }
    if (q < b.NO && !(e & 1)) {
        // entry position q of the flattened ints
        const uint64_t g = ub64(b.k2v_off, 0, (uint64_t)b.ng + 1, q) - 1;
        const uint64_t nk = b.key_off[g + 1] - b.key_off[g], no = b.k2v_off[g + 1] - b.k2v_off[g], nv = b.val_off[g + 1] - b.val_off[g];
        const uint64_t local = q - b.k2v_off[g];
        const int32_t x = b.k2v[q];
        if (local < nk) {
            const uint64_t prev = local == 0 ? nk : (uint64_t)(uint32_t)b.k2v[q - 1];
            if ((uint64_t)(uint32_t)x < prev || (uint64_t)(uint32_t)x > no || (local + 1 == nk && (uint64_t)(uint32_t)x != no)) e |= 1;
        } else if (x < 0 || (uint64_t)x >= nv) e |= 2;
    }
    if (__ballot(e != 0) && e) atomicOr((unsigned long long *)err, (unsigned long long)e);
}

// ---------------------------------------------------------------- invert

// every int of the batch: entries -> (global TxnId slot, key index); header slots -> pad (slot NV sorts last)
__global__ __launch_bounds__(BLOCK) void k_inv_expand(Batch b, uint64_t *__restrict__ slot, uint32_t *__restrict__ key, uint32_t *__restrict__ cnt)
{
    const uint64_t q = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (q >= b.NO) return;
    const uint64_t g = ub64(b.k2v_off, 0, (uint64_t)b.ng + 1, q) - 1;
    const uint32_t nk = (uint32_t)(b.key_off[g + 1] - b.key_off[g]);
    const uint32_t local = (uint32_t)(q - b.k2v_off[g]);
    if (local < nk) { slot[q] = b.NV; key[q] = 0; return; }
    const uint64_t s = b.val_off[g] + (uint32_t)b.k2v[q];
    slot[q] = s;
    key[q] = key_of_entry(b.k2v + b.k2v_off[g], nk, local);
    atomicAdd(&cnt[s], 1u);
}

// header of the inverted int[] of each group: end offset (from nv) of every TxnId's key list
__global__ __launch_bounds__(BLOCK) void k_inv_header(Batch b, const uint32_t *__restrict__ start, const uint32_t *__restrict__ cnt,
                                                      int32_t *__restrict__ out)
{
    const uint64_t s = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (s >= b.NV) return;
    const uint64_t g = ub64(b.val_off, 0, (uint64_t)b.ng + 1, s) - 1;
    const uint64_t v0 = b.val_off[g], nv = b.val_off[g + 1] - v0;
    const uint64_t ebefore = b.k2v_off[g] - b.key_off[g];   // entries of earlier groups (their slots sort first)
    const uint64_t base = v0 + ebefore;                     // the group's output offset
    out[base + (s - v0)] = (int32_t)(nv + (start[s] + cnt[s] - ebefore));
}

// sorted entry p (stable by slot: key order kept within a TxnId) -> its place after the group's header
__global__ __launch_bounds__(BLOCK) void k_inv_entries(Batch b, uint64_t nent, const uint64_t *__restrict__ sslot,
                                                       const uint32_t *__restrict__ skey, int32_t *__restrict__ out)
{
    const uint64_t p = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p >= nent) return;
    const uint64_t s = sslot[p];
    const uint64_t g = ub64(b.val_off, 0, (uint64_t)b.ng + 1, s) - 1;
    const uint64_t v0 = b.val_off[g], nv = b.val_off[g + 1] - v0;
    const uint64_t ebefore = b.k2v_off[g] - b.key_off[g];
    out[v0 + ebefore + nv + (p - ebefore)] = (int32_t)skey[p];
}

__global__ __launch_bounds__(BLOCK) void k_inv_off(Batch b, uint64_t *__restrict__ off)
{
    const uint64_t g = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (g <= b.ng) off[g] = b.val_off[g] + (b.k2v_off[g] - b.key_off[g]);
}

// ---------------------------------------------------------------- slice

struct Sel {
    const uint64_t *off, *s, *e;   // per group: Ranges (sorted, deoverlapped)
    uint32_t end_inclusive;
    uint32_t is_range;
};

// Keys.slice(ranges): key contained in a select range (Range.contains with the bound type, Range.java:40-138);
// RangeDeps: range intersecting one (compareIntersecting == 0, Range.java:296-305).
__global__ __launch_bounds__(BLOCK) void k_sl_select(Batch b, Sel sel, uint32_t *__restrict__ flag, uint64_t *__restrict__ elen)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= b.NK) return;
    const uint64_t g = ub64(b.key_off, 0, (uint64_t)b.ng + 1, i) - 1;
    const uint64_t a0 = sel.off[g], a1 = sel.off[g + 1];
    bool hit = false;
    if (a1 > a0) {
        if (!sel.is_range) {
            const uint64_t c = b.key_a[i];
            // last select range starting below c (EndInclusive: s < c) / at or below c (StartInclusive: s <= c)
            uint64_t lo = a0, hi = a1;
            while (lo < hi) { const uint64_t m = (lo + hi) >> 1; if (sel.end_inclusive ? sel.s[m] < c : sel.s[m] <= c) lo = m + 1; else hi = m; }
            if (lo > a0) {
                const uint64_t e = sel.e[lo - 1];
                hit = sel.end_inclusive ? c <= e : c < e;
            }
        } else {
            const uint64_t s = b.key_a[i], e = b.key_b[i];
            // first select range ending after s (ends ascend: deoverlapped); it intersects iff it starts before e
            uint64_t lo = a0, hi = a1;
            while (lo < hi) { const uint64_t m = (lo + hi) >> 1; if (sel.e[m] <= s) lo = m + 1; else hi = m; }
            hit = lo < a1 && sel.s[lo] < e;
        }
    }
    flag[i] = hit;
    // entries of this key
    const int32_t *h = b.k2v + b.k2v_off[g];
    const uint64_t nk = b.key_off[g + 1] - b.key_off[g], k = i - b.key_off[g];
    const uint64_t start = k == 0 ? nk : (uint64_t)(uint32_t)h[k - 1];
    elen[i] = hit ? (uint64_t)(uint32_t)h[k] - start : 0;
}

enum : uint32_t { SL_SLICE = 0, SL_EMPTY_IN = 1, SL_NONE = 2, SL_ALL = 3 };

struct SlG {
    const uint32_t *sel_excl;   // [NK+1] exclusive count of selected keys
    const uint64_t *ent_excl;   // [NK+1] exclusive count of entries of selected keys
    uint32_t *mode;             // [ng]
    uint64_t *c_keys, *c_k2v;   // [ng] output sizes (values come from the used-value scan)
};

__global__ __launch_bounds__(BLOCK) void k_sl_group(Batch b, Sel sel, SlG x)
{
    const uint64_t g = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (g >= b.ng) return;
    const uint64_t k0 = b.key_off[g], k1 = b.key_off[g + 1];
    const uint64_t nk = k1 - k0, no = b.k2v_off[g + 1] - b.k2v_off[g];
    const uint64_t ns = x.sel_excl[k1] - x.sel_excl[k0], ne = x.ent_excl[k1] - x.ent_excl[k0];
    uint32_t m;
    if (no == nk) m = SL_EMPTY_IN;          // isEmpty(): KeyDeps keeps (keys, txnIds, ints); RangeDeps (NONE, txnIds, NONE)
    else if (ns == 0) m = SL_NONE;          // (EMPTY, NO_TXNIDS, NO_INTS)
    else if (ns == nk) m = SL_ALL;          // `return this`
    else m = SL_SLICE;
    x.mode[g] = m;
    x.c_keys[g] = m == SL_EMPTY_IN ? (sel.is_range ? 0 : nk) : m == SL_NONE ? 0 : m == SL_ALL ? nk : ns;
    x.c_k2v[g] = m == SL_EMPTY_IN ? (sel.is_range ? 0 : no) : m == SL_NONE ? 0 : m == SL_ALL ? no : ns + ne;
}

// used[v]: value kept. SLICE: referenced by an entry of a selected key (trimUnusedValues); EMPTY_IN / ALL: every value
__global__ __launch_bounds__(BLOCK) void k_sl_used_all(Batch b, const uint32_t *__restrict__ mode, uint32_t *__restrict__ used)
{
    const uint64_t s = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (s >= b.NV) return;
    const uint64_t g = ub64(b.val_off, 0, (uint64_t)b.ng + 1, s) - 1;
    const uint32_t m = mode[g];
    used[s] = (m == SL_EMPTY_IN || m == SL_ALL) ? 1u : 0u;
}

__global__ __launch_bounds__(BLOCK) void k_sl_used_entries(Batch b, const uint32_t *__restrict__ mode, const uint32_t *__restrict__ flag,
                                                           uint32_t *__restrict__ used)
{
    const uint64_t q = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (q >= b.NO) return;
    const uint64_t g = ub64(b.k2v_off, 0, (uint64_t)b.ng + 1, q) - 1;
    if (mode[g] != SL_SLICE) return;
    const uint32_t nk = (uint32_t)(b.key_off[g + 1] - b.key_off[g]);
    const uint32_t local = (uint32_t)(q - b.k2v_off[g]);
    if (local < nk) return;
    const uint32_t k = key_of_entry(b.k2v + b.k2v_off[g], nk, local);
    if (flag[b.key_off[g] + k]) used[b.val_off[g] + (uint32_t)b.k2v[q]] = 1u;
}

struct SlOut {
    const uint32_t *mode, *flag, *sel_excl, *used_excl;
    const uint64_t *ent_excl;
    const uint64_t *key_out, *val_out, *k2v_out;   // [ng+1] output offsets
    uint32_t *key_idx, *val_idx;
    int32_t *k2v;
    uint32_t is_range;
};

__global__ __launch_bounds__(BLOCK) void k_sl_write_keys(Batch b, SlOut o)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= b.NK) return;
    const uint64_t g = ub64(b.key_off, 0, (uint64_t)b.ng + 1, i) - 1;
    const uint32_t m = o.mode[g];
    const uint64_t k0 = b.key_off[g], k = i - k0, nk = b.key_off[g + 1] - k0;
    const int32_t *h = b.k2v + b.k2v_off[g];
    const uint64_t ko = o.key_out[g], oo = o.k2v_out[g];
    if ((m == SL_EMPTY_IN && !o.is_range) || m == SL_ALL) {
        o.key_idx[ko + k] = (uint32_t)k;
        o.k2v[oo + k] = h[k];   // header as is
    } else if (m == SL_SLICE && o.flag[i]) {
        const uint64_t j = o.sel_excl[i] - o.sel_excl[k0];
        const uint64_t ns = o.sel_excl[b.key_off[g + 1]] - o.sel_excl[k0];
        o.key_idx[ko + j] = (uint32_t)k;
        o.k2v[oo + j] = (int32_t)(ns + (o.ent_excl[i + 1] - o.ent_excl[k0]));
    }
    (void)nk;
}

__global__ __launch_bounds__(BLOCK) void k_sl_write_vals(Batch b, SlOut o)
{
    const uint64_t s = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (s >= b.NV) return;
    const uint64_t g = ub64(b.val_off, 0, (uint64_t)b.ng + 1, s) - 1;
    if (o.used_excl[s + 1] == o.used_excl[s]) return;
    o.val_idx[o.val_out[g] + (o.used_excl[s] - o.used_excl[b.val_off[g]])] = (uint32_t)(s - b.val_off[g]);
}

__global__ __launch_bounds__(BLOCK) void k_sl_write_entries(Batch b, SlOut o)
{
    const uint64_t q = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (q >= b.NO) return;
    const uint64_t g = ub64(b.k2v_off, 0, (uint64_t)b.ng + 1, q) - 1;
    const uint32_t m = o.mode[g];
    const uint32_t nk = (uint32_t)(b.key_off[g + 1] - b.key_off[g]);
    const uint32_t local = (uint32_t)(q - b.k2v_off[g]);
    if (local < nk) return;
    if (m == SL_ALL) { o.k2v[o.k2v_out[g] + local] = b.k2v[q]; return; }
    if (m != SL_SLICE) return;
    const int32_t *h = b.k2v + b.k2v_off[g];
    const uint32_t k = key_of_entry(h, nk, local);
    const uint64_t i = b.key_off[g] + k;
    if (!o.flag[i]) return;
    const uint64_t k0 = b.key_off[g];
    const uint64_t ns = o.sel_excl[b.key_off[g + 1]] - o.sel_excl[k0];
    const uint32_t start = k == 0 ? nk : (uint32_t)h[k - 1];
    const uint64_t pos = ns + (o.ent_excl[i] - o.ent_excl[k0]) + (local - start);
    const uint64_t v = b.val_off[g] + (uint32_t)b.k2v[q];
    o.k2v[o.k2v_out[g] + pos] = (int32_t)(o.used_excl[v] - o.used_excl[b.val_off[g]]);   // trimUnusedValues remap
}

// ---------------------------------------------------------------- stab

struct Stab {
    const uint32_t *grp;
    const uint64_t *qs, *qe;   // qe null: key queries
    uint32_t nq, end_inclusive;
    const uint64_t *pmax;      // [NK] prefix max of range ends within the group (codes)
};

// candidate window of query q: ranges [lo, hi) of its group; lo = first with prefix-max end reaching the query,
// hi = first starting at or after it
__device__ __forceinline__ void stab_window(const Batch &b, const Stab &s, uint32_t q, uint64_t &lo, uint64_t &hi, uint64_t &g)
{
    g = s.grp[q];
    const uint64_t a0 = b.key_off[g], a1 = b.key_off[g + 1];
    const uint64_t x = s.qs[q];
    const bool key = s.qe == nullptr;
    const uint64_t y = key ? x : s.qe[q];
    // hi: ranges with start < y (EndInclusive key: start < k; StartInclusive key: start <= k; range query: start < end)
    uint64_t l = a0, h = a1;
    const bool incl = key && !s.end_inclusive;
    while (l < h) { const uint64_t m = (l + h) >> 1; if (incl ? b.key_a[m] <= y : b.key_a[m] < y) l = m + 1; else h = m; }
    hi = l;
    // lo: first range whose prefix-max end reaches x (EndInclusive key: end >= k; StartInclusive key: end > k;
    // range query: end > start)
    const bool ge = key && s.end_inclusive;
    l = a0; h = hi;
    while (l < h) { const uint64_t m = (l + h) >> 1; if (ge ? s.pmax[m] < x : s.pmax[m] <= x) l = m + 1; else h = m; }
    lo = l;
}

__device__ __forceinline__ bool stab_hit(const Batch &b, const Stab &s, uint32_t q, uint64_t i)
{
    const uint64_t rs = b.key_a[i], re = b.key_b[i], x = s.qs[q];
    if (s.qe == nullptr) return s.end_inclusive ? (x > rs && x <= re) : (x >= rs && x < re);
    return rs < s.qe[q] && re > x;
}

template <bool EMIT>
__global__ __launch_bounds__(BLOCK) void k_stab(Batch b, Stab s, uint64_t *__restrict__ cnt, const uint64_t *__restrict__ off,
                                                uint32_t *__restrict__ out, uint64_t *__restrict__ tcnt)
{
    const uint32_t q = blockIdx.x * BLOCK + threadIdx.x;
    if (q >= s.nq) return;
    uint64_t lo, hi, g;
    stab_window(b, s, q, lo, hi, g);
    uint64_t c = 0, tc = 0;
    const int32_t *h = b.k2v + b.k2v_off[g];
    const uint64_t a0 = b.key_off[g], nk = b.key_off[g + 1] - a0;
    for (uint64_t i = lo; i < hi; ++i) {
        if (!stab_hit(b, s, q, i)) continue;
        if (EMIT) out[off[q] + c] = (uint32_t)(i - a0);
        else {
            const uint64_t k = i - a0;
            tc += (uint64_t)(uint32_t)h[k] - (k == 0 ? nk : (uint64_t)(uint32_t)h[k - 1]);
        }
        ++c;
    }
    if (!EMIT) { cnt[q] = c; tcnt[q] = tc; }
}

// computeTxnIds: every TxnId index of the hit ranges as (query << vb | index), sorted and de-duplicated afterwards
__global__ __launch_bounds__(BLOCK) void k_stab_txns(Batch b, Stab s, const uint64_t *__restrict__ roff, const uint32_t *__restrict__ ridx,
                                                     const uint64_t *__restrict__ toff, int vb, uint64_t *__restrict__ key)
{
    const uint32_t q = blockIdx.x * BLOCK + threadIdx.x;
    if (q >= s.nq) return;
    const uint64_t g = s.grp[q];
    const int32_t *h = b.k2v + b.k2v_off[g];
    const uint64_t nk = b.key_off[g + 1] - b.key_off[g];
    uint64_t o = toff[q];
    for (uint64_t r = roff[q]; r < roff[q + 1]; ++r) {
        const uint32_t k = ridx[r];
        const uint64_t a = k == 0 ? nk : (uint64_t)(uint32_t)h[k - 1], e = (uint64_t)(uint32_t)h[k];
        for (uint64_t x = a; x < e; ++x) key[o++] = ((uint64_t)q << vb) | (uint32_t)h[x];
    }
}

__global__ __launch_bounds__(BLOCK) void k_stab_uflag(uint64_t n, const uint64_t *__restrict__ sk, int vb, uint32_t *__restrict__ flag,
                                                      uint64_t *__restrict__ ucnt)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const bool f = i == 0 || sk[i] != sk[i - 1];
    flag[i] = f;
    if (f) atomicAdd((unsigned long long *)&ucnt[sk[i] >> vb], 1ull);
}

__global__ __launch_bounds__(BLOCK) void k_stab_uwrite(uint64_t n, const uint64_t *__restrict__ sk, int vb, const uint32_t *__restrict__ flag,
                                                       const uint32_t *__restrict__ incl, uint32_t *__restrict__ out)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < n && flag[i]) out[incl[i] - 1] = (uint32_t)(sk[i] & ((1ull << vb) - 1));
}

// per-group prefix max of range ends, as (group << 32 | end rank + 1) for the segmented max scan
__global__ __launch_bounds__(BLOCK) void k_stab_pm_in(Batch b, const uint32_t *__restrict__ erank, uint64_t *__restrict__ pm)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= b.NK) return;
    const uint64_t g = ub64(b.key_off, 0, (uint64_t)b.ng + 1, i) - 1;
    pm[i] = (g << 32) | ((uint64_t)erank[i] + 1);
}

__global__ __launch_bounds__(BLOCK) void k_stab_pm_out(uint64_t n, const uint64_t *__restrict__ pm, const uint32_t *__restrict__ efirst,
                                                       const uint64_t *__restrict__ key_b, uint64_t *__restrict__ out)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) out[i] = key_b[efirst[(uint32_t)(pm[i] & 0xFFFFFFFFu) - 1]];
}

__global__ __launch_bounds__(BLOCK) void k_gather_u32(size_t n, const uint64_t *__restrict__ idx, const uint32_t *__restrict__ src,
                                                      uint64_t *__restrict__ out)
{
    const size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) out[i] = src[idx[i]];
}

Batch stage_batch(acc_ctx *ctx, const acc_rmm_batch *in, bool need_b)
{
    if (!in) fail(ACC_E_ARG, "null argument");
    if (in->mem != ACC_MEM_HOST && in->mem != ACC_MEM_DEVICE) fail(ACC_E_ARG, "mem must be ACC_MEM_HOST or ACC_MEM_DEVICE");
    hipStream_t st = ctx->stream;
    Batch b{};
    b.ng = in->n_groups;
    b.key_off = stage_in(ctx, "rb_key_off", in->key_off, (size_t)b.ng + 1, in->mem);
    b.val_off = stage_in(ctx, "rb_val_off", in->val_off, (size_t)b.ng + 1, in->mem);
    b.k2v_off = stage_in(ctx, "rb_k2v_off", in->k2v_off, (size_t)b.ng + 1, in->mem);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, b.key_off + b.ng, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, b.val_off + b.ng, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 2, b.k2v_off + b.ng, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    b.NK = ctx->pinned[0]; b.NV = ctx->pinned[1]; b.NO = ctx->pinned[2];
    if (b.NK >= 0xFFFFFFFFull || b.NV >= 0xFFFFFFFFull || b.NO >= 0xFFFFFFFFull) fail(ACC_E_CAP, "deps batch too large");
    b.key_a = (in->key_a || b.NK) ? stage_in(ctx, "rb_key_a", in->key_a, b.NK, in->mem) : nullptr;
    b.key_b = need_b ? stage_in(ctx, "rb_key_b", in->key_b, b.NK, in->mem) : nullptr;
    b.k2v = stage_in(ctx, "rb_k2v", in->k2v, b.NO, in->mem);
    uint64_t *err = ctx->get<uint64_t>("rb_err", 1);
    ACC_HIP(hipMemsetAsync(err, 0, 8, st));
    launch(ctx, "rb_validate", k_b_validate, dim3(grid_for(std::max<uint64_t>(b.NO, b.ng), BLOCK)), dim3(BLOCK), 0, b, err);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, err, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    if (ctx->pinned[0] & 1) fail(ACC_E_ARG, "Last key in keyToTxnId does not point to the end of the array (or offsets not monotone)");
    if (ctx->pinned[0] & 2) fail(ACC_E_ARG, "keyToTxnId entry out of range of txnIds");
    return b;
}

}  // namespace

// RelationMultiMap.invert of every group: out = per group the Java int[] txnIdsToKeys (nv end offsets from nv, then
// the key indices of every TxnId in key order)
void rmm_invert(acc_ctx *ctx, const acc_rmm_batch *in, acc_csr_view *out)
{
    if (!out) fail(ACC_E_ARG, "null argument");
    Batch b = stage_batch(ctx, in, false);
    hipStream_t st = ctx->stream;
    uint64_t *slot = ctx->get<uint64_t>("inv_slot", b.NO);
    uint32_t *key = ctx->get<uint32_t>("inv_key", b.NO);
    uint32_t *cnt = ctx->get<uint32_t>("inv_cnt", b.NV + 1);
    uint32_t *start = ctx->get<uint32_t>("inv_start", b.NV + 1);
    ACC_HIP(hipMemsetAsync(cnt, 0, (b.NV + 1) * 4, st));
    const uint64_t total = b.NV + (b.NO - b.NK);
    int32_t *ints = ctx->get<int32_t>("inv_out", total + 1);
    uint64_t *off = ctx->get<uint64_t>("inv_off", (size_t)b.ng + 1);
    launch(ctx, "inv_off", k_inv_off, dim3(grid_for((size_t)b.ng + 1, BLOCK)), dim3(BLOCK), 0, b, off);
    if (b.NO) {
        launch(ctx, "inv_expand", k_inv_expand, dim3(grid_for(b.NO, BLOCK)), dim3(BLOCK), 0, b, slot, key, cnt);
        scan<uint32_t, OpAdd<uint32_t>>(ctx, cnt, start, b.NV + 1, true);
        Sorted s = radix_sort(ctx, "rs_inv", slot, key, b.NO, bits_for(b.NV));
        if (b.NV) launch(ctx, "inv_header", k_inv_header, dim3(grid_for(b.NV, BLOCK)), dim3(BLOCK), 0, b, (const uint32_t *)start,
                         (const uint32_t *)cnt, ints);
        const uint64_t nent = b.NO - b.NK;
        if (nent) launch(ctx, "inv_entries", k_inv_entries, dim3(grid_for(nent, BLOCK)), dim3(BLOCK), 0, b, nent,
                         (const uint64_t *)s.keys, (const uint32_t *)s.vals, ints);
    } else if (b.NV) {
        ACC_HIP(hipMemsetAsync(start, 0, (b.NV + 1) * 4, st));
        launch(ctx, "inv_header", k_inv_header, dim3(grid_for(b.NV, BLOCK)), dim3(BLOCK), 0, b, (const uint32_t *)start,
               (const uint32_t *)cnt, ints);
    }
    ctx->sync();
    *out = acc_csr_view{ b.ng, total, off, ints };
}

void rmm_slice(acc_ctx *ctx, const acc_rmm_batch *in, const acc_ranges_in *select, acc_slice_view *out)
{
    if (!out || !select) fail(ACC_E_ARG, "null argument");
    const bool is_range = in && in->key_b != nullptr;
    Batch b = stage_batch(ctx, in, is_range);
    hipStream_t st = ctx->stream;
    Sel sel{};
    sel.off = stage_in(ctx, "sl_sel_off", select->off, (size_t)b.ng + 1, in->mem);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, sel.off + b.ng, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t NS = ctx->pinned[0];
    sel.s = stage_in(ctx, "sl_sel_s", select->start, NS, in->mem);
    sel.e = stage_in(ctx, "sl_sel_e", select->end, NS, in->mem);
    sel.end_inclusive = select->end_inclusive;
    sel.is_range = is_range;
    uint32_t *flag = ctx->get<uint32_t>("sl_flag", b.NK + 1);
    uint64_t *elen = ctx->get<uint64_t>("sl_elen", b.NK + 1);
    uint32_t *sel_excl = ctx->get<uint32_t>("sl_sel_excl", b.NK + 1);
    uint64_t *ent_excl = ctx->get<uint64_t>("sl_ent_excl", b.NK + 1);
    ACC_HIP(hipMemsetAsync(flag + b.NK, 0, 4, st));
    ACC_HIP(hipMemsetAsync(elen + b.NK, 0, 8, st));
    if (b.NK) launch(ctx, "sl_select", k_sl_select, dim3(grid_for(b.NK, BLOCK)), dim3(BLOCK), 0, b, sel, flag, elen);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, flag, sel_excl, b.NK + 1, true);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, elen, ent_excl, b.NK + 1, true);
    SlG gx{};
    gx.sel_excl = sel_excl; gx.ent_excl = ent_excl;
    gx.mode = ctx->get<uint32_t>("sl_mode", b.ng + 1);
    gx.c_keys = ctx->get<uint64_t>("sl_c_keys", (size_t)b.ng + 1);
    gx.c_k2v = ctx->get<uint64_t>("sl_c_k2v", (size_t)b.ng + 1);
    if (b.ng) launch(ctx, "sl_group", k_sl_group, dim3(grid_for(b.ng, BLOCK)), dim3(BLOCK), 0, b, sel, gx);
    uint32_t *used = ctx->get<uint32_t>("sl_used", b.NV + 1);
    uint32_t *used_excl = ctx->get<uint32_t>("sl_used_excl", b.NV + 1);
    ACC_HIP(hipMemsetAsync(used + b.NV, 0, 4, st));
    if (b.NV) launch(ctx, "sl_used_all", k_sl_used_all, dim3(grid_for(b.NV, BLOCK)), dim3(BLOCK), 0, b, (const uint32_t *)gx.mode, used);
    if (b.NO) launch(ctx, "sl_used_entries", k_sl_used_entries, dim3(grid_for(b.NO, BLOCK)), dim3(BLOCK), 0, b,
                     (const uint32_t *)gx.mode, (const uint32_t *)flag, used);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, used, used_excl, b.NV + 1, true);
    // per-group value counts from the used scan at the group boundaries
    uint64_t *key_out = ctx->get<uint64_t>("sl_key_out", (size_t)b.ng + 1);
    uint64_t *val_out = ctx->get<uint64_t>("sl_val_out", (size_t)b.ng + 1);
    uint64_t *k2v_out = ctx->get<uint64_t>("sl_k2v_out", (size_t)b.ng + 1);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, gx.c_keys, key_out, b.ng, true, key_out + b.ng);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, gx.c_k2v, k2v_out, b.ng, true, k2v_out + b.ng);
    // val_out[g] = used_excl[val_off[g]] (kept TxnIds before the group)
    launch(ctx, "sl_val_out", k_gather_u32, dim3(grid_for((size_t)b.ng + 1, BLOCK)), dim3(BLOCK), 0, (size_t)b.ng + 1, b.val_off,
           (const uint32_t *)used_excl, val_out);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, key_out + b.ng, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, val_out + b.ng, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 2, k2v_out + b.ng, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t TK = ctx->pinned[0], TV = ctx->pinned[1], TO = ctx->pinned[2];
    SlOut o{};
    o.mode = gx.mode; o.flag = flag; o.sel_excl = sel_excl; o.used_excl = used_excl; o.ent_excl = ent_excl;
    o.key_out = key_out; o.val_out = val_out; o.k2v_out = k2v_out; o.is_range = is_range;
    o.key_idx = ctx->get<uint32_t>("sl_key_idx", TK + 1);
    o.val_idx = ctx->get<uint32_t>("sl_val_idx", TV + 1);
    o.k2v = ctx->get<int32_t>("sl_k2v", TO + 1);
    if (b.NK) launch(ctx, "sl_write_keys", k_sl_write_keys, dim3(grid_for(b.NK, BLOCK)), dim3(BLOCK), 0, b, o);
    if (b.NV) launch(ctx, "sl_write_vals", k_sl_write_vals, dim3(grid_for(b.NV, BLOCK)), dim3(BLOCK), 0, b, o);
    if (b.NO) launch(ctx, "sl_write_entries", k_sl_write_entries, dim3(grid_for(b.NO, BLOCK)), dim3(BLOCK), 0, b, o);
    ctx->sync();
    *out = acc_slice_view{ b.ng, TK, TV, TO, key_out, o.key_idx, val_out, o.val_idx, k2v_out, o.k2v };
}

void rangedeps_stab(acc_ctx *ctx, const acc_rmm_batch *rd, const acc_stab_in *q, acc_stab_view *out)
{
    if (!q || !out) fail(ACC_E_ARG, "null argument");
    if (!rd || !rd->key_b) fail(ACC_E_ARG, "stabbing needs RangeDeps (key_b = Range.end codes)");
    if (q->mem != ACC_MEM_HOST && q->mem != ACC_MEM_DEVICE) fail(ACC_E_ARG, "mem must be ACC_MEM_HOST or ACC_MEM_DEVICE");
    Batch b = stage_batch(ctx, rd, true);
    hipStream_t st = ctx->stream;
    Stab s{};
    s.nq = q->n_queries;
    s.end_inclusive = q->end_inclusive;
    s.grp = stage_in(ctx, "st_grp", q->grp, s.nq, q->mem);
    s.qs = stage_in(ctx, "st_qs", q->q_start, s.nq, q->mem);
    s.qe = q->q_end ? stage_in(ctx, "st_qe", q->q_end, s.nq, q->mem) : nullptr;
    // prefix max of ends per group (segmented by the group id in the high word of the scanned composite)
    const uint64_t *ew[1] = { b.key_b };
    DenseRank er = dense_rank(ctx, "st_edict", b.NK, 1, ew, nullptr, nullptr, true);
    uint64_t *pm_in = ctx->get<uint64_t>("st_pm_in", b.NK + 1);
    uint64_t *pm = ctx->get<uint64_t>("st_pm", b.NK + 1);
    uint64_t *pmax = ctx->get<uint64_t>("st_pmax", b.NK + 1);
    if (b.ng >= (1u << 30)) fail(ACC_E_CAP, "too many RangeDeps in one stabbing batch");
    if (b.NK) {
        launch(ctx, "st_pm_in", k_stab_pm_in, dim3(grid_for(b.NK, BLOCK)), dim3(BLOCK), 0, b, (const uint32_t *)er.rank, pm_in);
        scan<uint64_t, OpMax<uint64_t>>(ctx, pm_in, pm, b.NK, false);
        launch(ctx, "st_pm_out", k_stab_pm_out, dim3(grid_for(b.NK, BLOCK)), dim3(BLOCK), 0, b.NK, (const uint64_t *)pm,
               (const uint32_t *)er.first, b.key_b, pmax);
    }
    s.pmax = pmax;
    uint64_t *cnt = ctx->get<uint64_t>("st_cnt", (size_t)s.nq + 1);
    uint64_t *tcnt = ctx->get<uint64_t>("st_tcnt", (size_t)s.nq + 1);
    uint64_t *roff = ctx->get<uint64_t>("st_roff", (size_t)s.nq + 1);
    uint64_t *toff = ctx->get<uint64_t>("st_toff", (size_t)s.nq + 1);
    const unsigned gq = grid_for(s.nq, BLOCK);
    if (s.nq) launch(ctx, "st_count", k_stab<false>, dim3(gq), dim3(BLOCK), 0, b, s, cnt, (const uint64_t *)nullptr,
                     (uint32_t *)nullptr, tcnt);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, cnt, roff, s.nq, true, roff + s.nq);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, tcnt, toff, s.nq, true, toff + s.nq);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, roff + s.nq, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, toff + s.nq, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t TR = ctx->pinned[0], TT = ctx->pinned[1];
    uint32_t *ridx = ctx->get<uint32_t>("st_ridx", TR + 1);
    if (s.nq) launch(ctx, "st_emit", k_stab<true>, dim3(gq), dim3(BLOCK), 0, b, s, (uint64_t *)nullptr, (const uint64_t *)roff, ridx,
                     (uint64_t *)nullptr);
    acc_stab_view v{ s.nq, TR, 0, roff, ridx, nullptr, nullptr };
    if (q->want_txns) {
        // computeTxnIds: sorted unique TxnId indices of the hit ranges
        const int vb = std::max(1, bits_for(b.NV ? b.NV - 1 : 0));
        const int qb = bits_for(s.nq ? s.nq - 1 : 0);
        if (vb + qb > 64) fail(ACC_E_CAP, "stabbing batch too large for the TxnId composite");
        uint64_t *tk = ctx->get<uint64_t>("st_tkey", TT + 1);
        if (s.nq) launch(ctx, "st_txns", k_stab_txns, dim3(gq), dim3(BLOCK), 0, b, s, (const uint64_t *)roff, (const uint32_t *)ridx,
                         (const uint64_t *)toff, vb, tk);
        Sorted srt = radix_sort(ctx, "rs_st", tk, nullptr, TT, vb + qb);
        uint32_t *uf = ctx->get<uint32_t>("st_uflag", TT + 1);
        uint32_t *ui = ctx->get<uint32_t>("st_uincl", TT + 1);
        uint64_t *ucnt = ctx->get<uint64_t>("st_ucnt", (size_t)s.nq + 1);
        uint64_t *uoff = ctx->get<uint64_t>("st_uoff", (size_t)s.nq + 1);
        ACC_HIP(hipMemsetAsync(ucnt, 0, ((size_t)s.nq + 1) * 8, st));
        if (TT) launch(ctx, "st_uflag", k_stab_uflag, dim3(grid_for(TT, BLOCK)), dim3(BLOCK), 0, TT, (const uint64_t *)srt.keys, vb, uf, ucnt);
        scan<uint32_t, OpAdd<uint32_t>>(ctx, uf, ui, TT, false);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, ucnt, uoff, s.nq, true, uoff + s.nq);
        uint32_t *tidx = ctx->get<uint32_t>("st_tidx", TT + 1);
        if (TT) launch(ctx, "st_uwrite", k_stab_uwrite, dim3(grid_for(TT, BLOCK)), dim3(BLOCK), 0, TT, (const uint64_t *)srt.keys, vb,
                       (const uint32_t *)uf, (const uint32_t *)ui, tidx);
        ACC_HIP(hipMemcpyAsync(ctx->pinned, uoff + s.nq, 8, hipMemcpyDeviceToHost, st));
        ctx->sync();
        v.total_txns = ctx->pinned[0];
        v.txn_off = uoff;
        v.txn_idx = tidx;
    }
    ctx->sync();
    *out = v;
}

}  // namespace acc
