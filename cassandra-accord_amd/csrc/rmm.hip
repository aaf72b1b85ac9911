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

// ---------------------------------------------------------------- without (RelationMultiMap.remove)
// RelationMultiMap.remove (utils/RelationMultiMap.java:843-905) of every group: a value is removed when its TxnId is in
// the group's set a or set b (Deps::contains = KeyDeps.contains || RangeDeps.contains, primitives/Deps.java:107-110, each
// Arrays.binarySearch: Timestamp.compareTo == 0). The Java builds remapValue by counting the kept values in order
// (:855-860), then walks keysToValues once (:877-891); here both are exclusive scans of keep flags: over the values
// (the remap) and over the int positions (the new end offsets and entry slots), so every output is one thread's write.

namespace {

struct WoSet {
    const uint64_t *off, *m, *l;
    const int32_t *n;
};

struct Wo {
    uint32_t ng;
    const uint64_t *key_off, *val_off, *k2v_off;
    const int32_t *k2v;
    uint64_t NK, NV, NO;
    const uint64_t *tm, *tl;   // the half's TxnIds [NV]
    const int32_t *tn;
    WoSet a, b;
    uint32_t *keep, *ekeep;           // [NV + 1], [NO + 1]
    const uint32_t *keep_x, *ekeep_x; // their exclusive scans
    uint8_t *kind;
    uint64_t *c_keys, *c_vals, *c_k2v, *cnt;
    const uint64_t *key_out, *val_out, *k2v_out;
    uint32_t *key_idx, *val_idx;
    int32_t *out;
};

// Timestamp.compareTo (primitives/Timestamp.java:208-217): msb, then lsb & IDENTITY_LSB (lowHlc, identity flags), node
__device__ __forceinline__ int wo_cmp(uint64_t am, uint64_t al, int32_t an, uint64_t bm, uint64_t bl, int32_t bn)
{
    if (am != bm) return am < bm ? -1 : 1;
    const uint64_t a1 = al & 0xFFFFFFFFFFFF001EULL, b1 = bl & 0xFFFFFFFFFFFF001EULL;
    if (a1 != b1) return a1 < b1 ? -1 : 1;
    if (an != bn) return an < bn ? -1 : 1;
    return 0;
}

__device__ __forceinline__ bool wo_contains(const WoSet &s, uint64_t g, uint64_t m, uint64_t l, int32_t n)
{
    if (!s.off) return false;
    uint64_t lo = s.off[g], hi = s.off[g + 1];
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        const int c = wo_cmp(s.m[mid], s.l[mid], s.n[mid], m, l, n);
        if (c == 0) return true;
        if (c < 0) lo = mid + 1; else hi = mid;
    }
    return false;
}

// a set's offsets monotone and its TxnIds strictly ascending within each group (err bit 4)
__global__ __launch_bounds__(BLOCK) void k_wo_set_check(uint32_t ng, WoSet s, uint64_t ns, uint64_t *__restrict__ err)
{
    const uint64_t q = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    bool bad = false;
    if (q < ng && s.off[q + 1] < s.off[q]) bad = true;
    if (q < ns) {
        const uint64_t g = ub64(s.off, 0, (uint64_t)ng + 1, q) - 1;
        if (q > s.off[g] && wo_cmp(s.m[q - 1], s.l[q - 1], s.n[q - 1], s.m[q], s.l[q], s.n[q]) >= 0) bad = true;
    }
    if (__ballot(bad) && bad) atomicOr((unsigned long long *)err, 4ull);
}

// per value: kept unless in set a or b (the remove predicate, :855-860)
__global__ __launch_bounds__(BLOCK) void k_wo_keep(Wo w)
{
    const uint64_t s = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (s > w.NV) return;
    if (s == w.NV) { w.keep[s] = 0; return; }
    const uint64_t g = ub64(w.val_off, 0, (uint64_t)w.ng + 1, s) - 1;
    const uint64_t m = w.tm[s], l = w.tl[s];
    const int32_t n = w.tn[s];
    w.keep[s] = (wo_contains(w.a, g, m, l, n) || wo_contains(w.b, g, m, l, n)) ? 0u : 1u;
}

// per int position: 1 for an entry whose TxnId is kept (header slots 0)
__global__ __launch_bounds__(BLOCK) void k_wo_ekeep(Wo w)
{
    const uint64_t q = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (q > w.NO) return;
    if (q == w.NO) { w.ekeep[q] = 0; return; }
    const uint64_t g = ub64(w.k2v_off, 0, (uint64_t)w.ng + 1, q) - 1;
    const uint64_t nk = w.key_off[g + 1] - w.key_off[g], local = q - w.k2v_off[g];
    w.ekeep[q] = local >= nk ? w.keep[w.val_off[g] + (uint32_t)w.k2v[q]] : 0u;
}

// per group: the Java's three returns (:844-845 isEmpty -> from; :862-863 nothing removed -> from; :865-866 all removed
// -> none) and the output sizes
__global__ __launch_bounds__(BLOCK) void k_wo_group(Wo w)
{
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    uint32_t kd = 3;
    if (g < w.ng) {
        const uint64_t nk = w.key_off[g + 1] - w.key_off[g], nv = w.val_off[g + 1] - w.val_off[g];
        const uint64_t no = w.k2v_off[g + 1] - w.k2v_off[g];
        const uint64_t kept = w.keep_x[w.val_off[g + 1]] - w.keep_x[w.val_off[g]];
        const uint64_t kept_e = w.ekeep_x[w.k2v_off[g + 1]] - w.ekeep_x[w.k2v_off[g]];
        kd = (no == nk || kept == nv) ? ACC_WITHOUT_FROM : kept == 0 ? ACC_WITHOUT_NONE : ACC_WITHOUT_NEW;
        w.kind[g] = (uint8_t)kd;
        w.c_keys[g] = kd == ACC_WITHOUT_NONE ? 0 : nk;
        w.c_vals[g] = kd == ACC_WITHOUT_FROM ? nv : kd == ACC_WITHOUT_NONE ? 0 : kept;
        w.c_k2v[g] = kd == ACC_WITHOUT_FROM ? no : kd == ACC_WITHOUT_NONE ? 0 : nk + kept_e;
    }
    for (uint32_t k = 0; k < 3; ++k) {
        const uint64_t b = __ballot(kd == k);
        if (lane_id() == 0 && b) atomicAdd((unsigned long long *)&w.cnt[k], (unsigned long long)__popcll(b));
    }
}

__global__ __launch_bounds__(BLOCK) void k_wo_keys(Wo w)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= w.NK) return;
    const uint64_t g = ub64(w.key_off, 0, (uint64_t)w.ng + 1, i) - 1;
    if (w.kind[g] != ACC_WITHOUT_NONE) w.key_idx[w.key_out[g] + (i - w.key_off[g])] = (uint32_t)(i - w.key_off[g]);
}

__global__ __launch_bounds__(BLOCK) void k_wo_vals(Wo w)
{
    const uint64_t s = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (s >= w.NV) return;
    const uint64_t g = ub64(w.val_off, 0, (uint64_t)w.ng + 1, s) - 1;
    const uint32_t local = (uint32_t)(s - w.val_off[g]);
    const uint8_t kd = w.kind[g];
    if (kd == ACC_WITHOUT_FROM) w.val_idx[w.val_out[g] + local] = local;
    else if (kd == ACC_WITHOUT_NEW && w.keep[s]) w.val_idx[w.val_out[g] + (w.keep_x[s] - w.keep_x[w.val_off[g]])] = local;
}

// the new keysToValues (:874-894): end offset of key k = nk + kept entries before its old end; entry = remapValue
__global__ __launch_bounds__(BLOCK) void k_wo_ints(Wo w)
{
    const uint64_t q = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (q >= w.NO) return;
    const uint64_t g = ub64(w.k2v_off, 0, (uint64_t)w.ng + 1, q) - 1;
    const uint8_t kd = w.kind[g];
    if (kd == ACC_WITHOUT_NONE) return;
    const uint64_t o0 = w.k2v_off[g], local = q - o0, base = w.k2v_out[g];
    const int32_t x = w.k2v[q];
    if (kd == ACC_WITHOUT_FROM) { w.out[base + local] = x; return; }
    const uint64_t nk = w.key_off[g + 1] - w.key_off[g];
    if (local < nk) {
        w.out[base + local] = (int32_t)(nk + (w.ekeep_x[o0 + (uint32_t)x] - w.ekeep_x[o0]));
    } else if (w.ekeep[q]) {
        const uint64_t v0 = w.val_off[g];
        w.out[base + nk + (w.ekeep_x[q] - w.ekeep_x[o0])] = (int32_t)(w.keep_x[v0 + (uint32_t)x] - w.keep_x[v0]);
    }
}

}  // namespace

// the without of one half held in device memory (layout already valid; sets sorted); results in the context's "wo_*"
// buffers under the caller's namespace
void rmm_without_dev(acc_ctx *ctx, uint32_t ng, const acc_rmm_in &h, uint64_t NK, uint64_t NV, uint64_t NO,
                     const acc_txn_sets *sa, const acc_txn_sets *sb, acc_without_view *out)
{
    hipStream_t st = ctx->stream;
    if (NK >= 0xFFFFFFFFull || NV >= 0xFFFFFFFFull || NO >= 0xFFFFFFFFull) fail(ACC_E_CAP, "deps batch too large");
    Wo w{};
    w.ng = ng; w.key_off = h.key_off; w.val_off = h.val_off; w.k2v_off = h.k2v_off; w.k2v = h.k2v;
    w.NK = NK; w.NV = NV; w.NO = NO;
    w.tm = h.txn.msb; w.tl = h.txn.lsb; w.tn = h.txn.node;
    w.a = WoSet{ sa ? sa->off : nullptr, sa ? sa->txn.msb : nullptr, sa ? sa->txn.lsb : nullptr, sa ? sa->txn.node : nullptr };
    w.b = WoSet{ sb ? sb->off : nullptr, sb ? sb->txn.msb : nullptr, sb ? sb->txn.lsb : nullptr, sb ? sb->txn.node : nullptr };
    w.keep = ctx->get<uint32_t>("wo_keep", NV + 1);
    w.ekeep = ctx->get<uint32_t>("wo_ekeep", NO + 1);
    uint32_t *keep_x = ctx->get<uint32_t>("wo_keep_x", NV + 1), *ekeep_x = ctx->get<uint32_t>("wo_ekeep_x", NO + 1);
    w.keep_x = keep_x; w.ekeep_x = ekeep_x;
    w.kind = ctx->get<uint8_t>("wo_kind", (size_t)ng + 1);
    w.c_keys = ctx->get<uint64_t>("wo_c_keys", (size_t)ng + 1);
    w.c_vals = ctx->get<uint64_t>("wo_c_vals", (size_t)ng + 1);
    w.c_k2v = ctx->get<uint64_t>("wo_c_k2v", (size_t)ng + 1);
    w.cnt = ctx->get<uint64_t>("wo_cnt", 4);
    ACC_HIP(hipMemsetAsync(w.cnt, 0, 32, st));
    launch(ctx, "wo_keep", k_wo_keep, dim3(grid_for(NV + 1, BLOCK)), dim3(BLOCK), 0, w);
    launch(ctx, "wo_ekeep", k_wo_ekeep, dim3(grid_for(NO + 1, BLOCK)), dim3(BLOCK), 0, w);
    {
        const uint32_t *si[2] = { w.keep, w.ekeep };
        uint32_t *so[2] = { keep_x, ekeep_x };
        const size_t sn[2] = { NV + 1, NO + 1 };
        scan_multi<uint32_t, OpAdd<uint32_t>>(ctx, 2, si, so, sn, true, (uint32_t *const *)nullptr);
    }
    if (ng) launch(ctx, "wo_group", k_wo_group, dim3(grid_for(ng, BLOCK)), dim3(BLOCK), 0, w);
    uint64_t *key_out = ctx->get<uint64_t>("wo_key_out", (size_t)ng + 1);
    uint64_t *val_out = ctx->get<uint64_t>("wo_val_out", (size_t)ng + 1);
    uint64_t *k2v_out = ctx->get<uint64_t>("wo_k2v_out", (size_t)ng + 1);
    {
        const uint64_t *si[3] = { w.c_keys, w.c_vals, w.c_k2v };
        uint64_t *so[3] = { key_out, val_out, k2v_out }, *tot[3] = { key_out + ng, val_out + ng, k2v_out + ng };
        const size_t sn[3] = { ng, ng, ng };
        scan_multi<uint64_t, OpAdd<uint64_t>>(ctx, 3, si, so, sn, true, tot);
    }
    ACC_HIP(hipMemcpyAsync(ctx->pinned, key_out + ng, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, val_out + ng, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 2, k2v_out + ng, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 3, w.cnt, 24, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t TK = ctx->pinned[0], TV = ctx->pinned[1], TO = ctx->pinned[2];
    const uint64_t nf = ctx->pinned[3], nn = ctx->pinned[4], nw = ctx->pinned[5];
    w.key_out = key_out; w.val_out = val_out; w.k2v_out = k2v_out;
    w.key_idx = ctx->get<uint32_t>("wo_key_idx", TK + 1);
    w.val_idx = ctx->get<uint32_t>("wo_val_idx", TV + 1);
    w.out = ctx->get<int32_t>("wo_k2v", TO + 1);
    if (NK) launch(ctx, "wo_keys", k_wo_keys, dim3(grid_for(NK, BLOCK)), dim3(BLOCK), 0, w);
    if (NV) launch(ctx, "wo_vals", k_wo_vals, dim3(grid_for(NV, BLOCK)), dim3(BLOCK), 0, w);
    if (NO) launch(ctx, "wo_ints", k_wo_ints, dim3(grid_for(NO, BLOCK)), dim3(BLOCK), 0, w);
    ctx->sync();
    ctx->stat("without.from", nf);
    ctx->stat("without.none", nn);
    ctx->stat("without.new", nw);
    *out = acc_without_view{ acc_slice_view{ ng, TK, TV, TO, key_out, w.key_idx, val_out, w.val_idx, k2v_out, w.out },
                             w.kind, nf, nn, nw };
}

// The ABI form: one deps half per group from caller memory, validated (layout as acc_rmm_slice; sets sorted unique).
void rmm_without(acc_ctx *ctx, const acc_rmm_batch *in, const acc_ts_cols *txn, const acc_txn_sets *set_a,
                 const acc_txn_sets *set_b, acc_without_view *out)
{
    if (!out || !txn) fail(ACC_E_ARG, "null argument");
    Batch b = stage_batch(ctx, in, false);
    hipStream_t st = ctx->stream;
    acc_rmm_in h{};
    h.key_off = b.key_off; h.val_off = b.val_off; h.k2v_off = b.k2v_off; h.k2v = b.k2v;
    h.txn.msb = stage_in(ctx, "wo_tm", txn->msb, b.NV, in->mem);
    h.txn.lsb = stage_in(ctx, "wo_tl", txn->lsb, b.NV, in->mem);
    h.txn.node = stage_in(ctx, "wo_tn", txn->node, b.NV, in->mem);
    acc_txn_sets sets[2];
    const acc_txn_sets *src[2] = { set_a, set_b };
    uint64_t ns[2] = { 0, 0 };
    const char *nm[2][4] = { { "wo_a_off", "wo_a_m", "wo_a_l", "wo_a_n" }, { "wo_b_off", "wo_b_m", "wo_b_l", "wo_b_n" } };
    for (int k = 0; k < 2; ++k) {
        sets[k] = acc_txn_sets{};
        if (!src[k] || !src[k]->off) continue;
        sets[k].off = stage_in(ctx, nm[k][0], src[k]->off, (size_t)b.ng + 1, in->mem);
        ACC_HIP(hipMemcpyAsync(ctx->pinned + k, sets[k].off + b.ng, 8, hipMemcpyDeviceToHost, st));
    }
    ctx->sync();
    for (int k = 0; k < 2; ++k) if (sets[k].off) ns[k] = ctx->pinned[k];
    uint64_t *err = ctx->get<uint64_t>("wo_err", 1);
    ACC_HIP(hipMemsetAsync(err, 0, 8, st));
    for (int k = 0; k < 2; ++k) {
        if (!sets[k].off) continue;
        if (ns[k] >= 0xFFFFFFFFull) fail(ACC_E_CAP, "TxnId sets too large");
        sets[k].txn.msb = stage_in(ctx, nm[k][1], src[k]->txn.msb, ns[k], in->mem);
        sets[k].txn.lsb = stage_in(ctx, nm[k][2], src[k]->txn.lsb, ns[k], in->mem);
        sets[k].txn.node = stage_in(ctx, nm[k][3], src[k]->txn.node, ns[k], in->mem);
        const WoSet ws{ sets[k].off, sets[k].txn.msb, sets[k].txn.lsb, sets[k].txn.node };
        launch(ctx, "wo_set_check", k_wo_set_check, dim3(grid_for(std::max<uint64_t>(ns[k], b.ng), BLOCK)), dim3(BLOCK), 0,
               b.ng, ws, ns[k], err);
    }
    ACC_HIP(hipMemcpyAsync(ctx->pinned, err, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    if (ctx->pinned[0] & 4) fail(ACC_E_ARG, "without: a TxnId set is not sorted unique (Arrays.binarySearch needs sorted input)");
    rmm_without_dev(ctx, b.ng, h, b.NK, b.NV, b.NO, sets[0].off ? &sets[0] : nullptr, sets[1].off ? &sets[1] : nullptr, out);
}

}  // namespace acc
