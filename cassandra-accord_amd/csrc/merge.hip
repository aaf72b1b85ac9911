// merge.hip — batched KeyDeps.merge (primitives/KeyDeps.java:115-135) for many coordinated txns.
//
// The reference folds replies left to right with RelationMultiMap.linearUnion through a LinearMerger
// (utils/RelationMultiMap.java:284-406, 561-816), skipping empty replies (KeyDeps.isEmpty,
// KeyDeps.java:292-295: no entries). Its result is the canonical union (KeyDepsTest.testMergedProperty,
// KeyDepsTest.java:275-283): keys = sorted union of the non-empty replies' key arrays, txnIds = sorted
// union of their txnId arrays (unreferenced ids included), and per key the sorted union of referenced ids.
// Here every group (one coordinated txn) is merged at once:
//   1. expand: (group, key), (group, value) and (group, key, value) records of the non-empty replies,
//      written at their input offsets (header slots and empty replies become all-ones pads);
//   2. three stable radix sorts of compacted composite keys;
//   3. unique + per-group counts (scans) -> per-group CSR in Java layout; each (key, value) entry becomes
//      the index of the value in the group's txnId array (binary search within the group).
#include <algorithm>
#include <cstdio>

#include "dict.hpp"

namespace acc {

template <int NWV = WAVES>
__device__ __forceinline__ void block_or1(uint64_t v, uint64_t *dst)
{
    __shared__ uint64_t part[NWV];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v |= shfl_idx(v, (int)(lane_id() ^ d));
    if (lane_id() == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t x = 0;
        for (int q = 0; q < NWV; ++q) x |= part[q];
        if (x) atomicOr((unsigned long long *)dst, (unsigned long long)x);
    }
}

// per reply: group id, emptiness, input validation (KeyDeps ctor check, KeyDeps.java:184-185)
__global__ __launch_bounds__(BLOCK) void k_m_replies(uint32_t ng, const uint64_t *__restrict__ grp_off, uint32_t *__restrict__ grp_of)
{
    uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g >= ng) return;
    for (uint64_t r = grp_off[g]; r < grp_off[g + 1]; ++r) grp_of[r] = g;
}

// g[0] key-code varying bits, g[1] txn-rank varying bits, g[2] errors
__global__ __launch_bounds__(BLOCK) void k_m_prep(uint64_t R, const uint64_t *__restrict__ key_off, const uint64_t *__restrict__ key_code,
                                                  const uint64_t *__restrict__ val_off, const uint32_t *__restrict__ txn_rank,
                                                  const uint64_t *__restrict__ k2v_off, const int32_t *__restrict__ k2v,
                                                  uint64_t *__restrict__ g)
{
    uint64_t r = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    uint64_t km = 0, vm = 0, err = 0;
    if (r < R) {
        const uint64_t k0 = key_code[0], v0 = txn_rank[0];
        uint64_t ka = key_off[r], kb = key_off[r + 1], va = val_off[r], vb = val_off[r + 1];
        uint64_t oa = k2v_off[r], ob = k2v_off[r + 1];
        uint64_t nk = kb - ka, nv = vb - va, no = ob - oa;
        if (kb < ka || vb < va || ob < oa || no < nk) err |= 1;
        else {
            for (uint64_t i = ka; i < kb; ++i) {
                km |= key_code[i] ^ k0;
                if (i > ka && key_code[i - 1] >= key_code[i]) err |= 2;   // Keys sorted unique
            }
            for (uint64_t i = va; i < vb; ++i) {
                vm |= (uint64_t)txn_rank[i] ^ v0;
                if (i > va && txn_rank[i - 1] >= txn_rank[i]) err |= 4;   // txnIds sorted unique
            }
            if (nk && (uint64_t)(uint32_t)k2v[oa + nk - 1] != no) err |= 8;   // last offset == length
            if (!nk && no) err |= 8;                                           // entries without keys
            uint64_t prev_end = nk;
            for (uint64_t i = 0; i < nk && !(err & 8); ++i) {
                uint64_t end = (uint64_t)(uint32_t)k2v[oa + i];
                if (end < prev_end || end > no) { err |= 8; break; }
                for (uint64_t q = prev_end; q < end; ++q) {
                    int32_t x = k2v[oa + q];
                    if (x < 0 || (uint64_t)x >= nv) { err |= 16; break; }
                    if (q > prev_end && k2v[oa + q - 1] >= x) err |= 32;     // ascending unique per key
                }
                prev_end = end;
            }
        }
    }
    block_or1(km, &g[0]);
    block_or1(vm, &g[1]);
    block_or1(err, &g[2]);
}

struct MergePlan {
    Runs rk, rv;
    uint64_t pad_k, pad_v, pad_kv;       // all ones in each composite's sorted width: sorts after real records
    int gshift_k, gshift_v, gshift_kv;   // group field position in each composite
    int vshift_kv;                        // key field position in the (g, key, value) composite
};

// One thread per reply: expand its records at the input offsets. Empty replies and header slots: pads.
__global__ __launch_bounds__(BLOCK) void k_m_expand(uint64_t R, const uint32_t *__restrict__ grp_of,
                                                    const uint64_t *__restrict__ key_off, const uint64_t *__restrict__ key_code,
                                                    const uint64_t *__restrict__ val_off, const uint32_t *__restrict__ txn_rank,
                                                    const uint64_t *__restrict__ k2v_off, const int32_t *__restrict__ k2v,
                                                    MergePlan plan, uint64_t *__restrict__ sk, uint64_t *__restrict__ sv,
                                                    uint64_t *__restrict__ skv)
{
    uint64_t r = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (r >= R) return;
    const uint64_t g = grp_of[r];
    uint64_t ka = key_off[r], kb = key_off[r + 1], va = val_off[r], vb = val_off[r + 1];
    uint64_t oa = k2v_off[r], ob = k2v_off[r + 1];
    uint64_t nk = kb - ka;
    const bool empty = (ob - oa) == nk;
    for (uint64_t i = ka; i < kb; ++i)
        sk[i] = empty ? plan.pad_k : (g << plan.gshift_k) | pext_runs(key_code[i], plan.rk);
    for (uint64_t i = va; i < vb; ++i)
        sv[i] = empty ? plan.pad_v : (g << plan.gshift_v) | pext_runs(txn_rank[i], plan.rv);
    for (uint64_t i = 0; i < nk; ++i) skv[oa + i] = plan.pad_kv;
    uint64_t prev_end = nk;
    for (uint64_t i = 0; i < nk; ++i) {
        uint64_t end = (uint64_t)(uint32_t)k2v[oa + i];
        uint64_t kc = pext_runs(key_code[ka + i], plan.rk);
        for (uint64_t q = prev_end; q < end; ++q) {
            uint32_t v = txn_rank[va + (uint32_t)k2v[oa + q]];
            skv[oa + q] = (g << plan.gshift_kv) | (kc << plan.vshift_kv) | pext_runs(v, plan.rv);
        }
        prev_end = end;
    }
}

// unique flags: first of each distinct composite (pads excluded)
__global__ __launch_bounds__(BLOCK) void k_m_uniq(uint64_t n, const uint64_t *__restrict__ s, uint64_t pad,
                                                  uint64_t *__restrict__ flag)
{
    uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    flag[i] = s[i] != pad && (i == 0 || s[i] != s[i - 1]);
}

// per-group unique-record counts from the run boundaries of the sorted composites (records of a group are
// contiguous): the first record of group g stores its unique index, the last one the index past it
__global__ __launch_bounds__(BLOCK) void k_m_group_bounds(uint64_t n, const uint64_t *__restrict__ s, uint64_t pad,
                                                          const uint64_t *__restrict__ flag, const uint64_t *__restrict__ idx,
                                                          int gshift, uint64_t *__restrict__ gfirst, uint64_t *__restrict__ glast)
{
    uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n || s[i] == pad) return;
    uint64_t g = s[i] >> gshift;
    if (i == 0 || (s[i - 1] >> gshift) != g) gfirst[g] = idx[i];
    if (i + 1 == n || s[i + 1] == pad || (s[i + 1] >> gshift) != g) glast[g] = idx[i] + flag[i];
}

__global__ __launch_bounds__(BLOCK) void k_m_group_counts(uint32_t ng, const uint64_t *__restrict__ gfirst,
                                                          const uint64_t *__restrict__ glast, uint64_t *__restrict__ cnt)
{
    uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g < ng) cnt[g] = glast[g] - gfirst[g];
}

__global__ __launch_bounds__(BLOCK) void k_m_write_vals(uint64_t n, const uint64_t *__restrict__ flag, const uint64_t *__restrict__ idx,
                                                        const uint32_t *__restrict__ txn_rank, const uint32_t *__restrict__ src,
                                                        uint32_t *__restrict__ out_val)
{
    uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n || !flag[i]) return;
    out_val[idx[i]] = txn_rank[src[i]];
}

__global__ __launch_bounds__(BLOCK) void k_m_write_keys(uint64_t n, const uint64_t *__restrict__ flag, const uint64_t *__restrict__ idx,
                                                        const uint64_t *__restrict__ key_code, const uint32_t *__restrict__ src,
                                                        uint64_t *__restrict__ out_key)
{
    uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n || !flag[i]) return;
    out_key[idx[i]] = key_code[src[i]];
}

__device__ __forceinline__ uint64_t lb_u64(const uint64_t *a, uint64_t lo, uint64_t hi, uint64_t v)
{
    while (lo < hi) { uint64_t mid = (lo + hi) >> 1; if (a[mid] < v) lo = mid + 1; else hi = mid; }
    return lo;
}

// Entry part of keysToTxnIds: the index of the value in its group's txnIds. Header part: the record that
// closes a (group, key) run (duplicates included) writes that key's end offset and marks the key.
__global__ __launch_bounds__(BLOCK) void k_m_write_k2v(uint64_t n, const uint64_t *__restrict__ s, MergePlan plan,
                                                       const uint64_t *__restrict__ flag, const uint64_t *__restrict__ idx,
                                                       const uint64_t *__restrict__ kv_gstart, const uint64_t *__restrict__ k_gstart,
                                                       const uint64_t *__restrict__ v_gstart, const uint32_t *__restrict__ out_val,
                                                       const uint64_t *__restrict__ out_key, const uint32_t *__restrict__ txn_rank,
                                                       const uint32_t *__restrict__ src, const uint32_t *__restrict__ val_of_slot,
                                                       const uint32_t *__restrict__ key_of_slot, const uint64_t *__restrict__ key_code,
                                                       int32_t *__restrict__ out_k2v, uint8_t *__restrict__ has)
{
    uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint64_t x = s[i];
    if (x == plan.pad_kv) return;
    const uint64_t g = x >> plan.gshift_kv;
    const uint64_t k0 = k_gstart[g], nk = k_gstart[g + 1] - k0;
    const uint64_t obase = kv_gstart[g] + k0;      // entries + headers of earlier groups
    if (flag[i]) {
        const uint32_t v = txn_rank[val_of_slot[src[i]]];
        uint64_t lo = v_gstart[g], hi = v_gstart[g + 1];
        while (lo < hi) { uint64_t mid = (lo + hi) >> 1; if (out_val[mid] < v) lo = mid + 1; else hi = mid; }
        out_k2v[obase + nk + (idx[i] - kv_gstart[g])] = (int32_t)(lo - v_gstart[g]);
    }
    const bool last = i + 1 == n || s[i + 1] == plan.pad_kv || (s[i + 1] >> plan.vshift_kv) != (x >> plan.vshift_kv);
    if (last) {
        uint64_t a = lb_u64(out_key, k0, k0 + nk, key_code[key_of_slot[src[i]]]);
        out_k2v[obase + (a - k0)] = (int32_t)(nk + (idx[i] + flag[i] - kv_gstart[g]));
        has[a] = 1;
    }
}

// keys present only in key arrays (no union entries): end offset = previous key's end
__global__ __launch_bounds__(BLOCK) void k_m_fix_headers(uint32_t ng, const uint64_t *__restrict__ kv_gstart,
                                                         const uint64_t *__restrict__ k_gstart, int32_t *__restrict__ out_k2v,
                                                         const uint8_t *__restrict__ has, uint64_t *__restrict__ out_k2v_off)
{
    uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g > ng) return;
    out_k2v_off[g] = kv_gstart[g] + k_gstart[g];
    if (g == ng) return;
    const uint64_t k0 = k_gstart[g], nk = k_gstart[g + 1] - k0;
    const uint64_t obase = kv_gstart[g] + k0;
    int32_t prev = (int32_t)nk;
    for (uint64_t q = 0; q < nk; ++q) {
        if (!has[k0 + q]) out_k2v[obase + q] = prev;
        prev = out_k2v[obase + q];
    }
}

__global__ __launch_bounds__(BLOCK) void k_widen(uint64_t n, const uint32_t *__restrict__ in, uint64_t *__restrict__ out)
{
    uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) out[i] = in[i];
}

// key slot (index into key_code) of every k2v entry position, for the (g, key, value) records
__global__ __launch_bounds__(BLOCK) void k_m_key_of_slot(uint64_t R, const uint64_t *__restrict__ key_off,
                                                         const uint64_t *__restrict__ val_off,
                                                         const uint64_t *__restrict__ k2v_off, const int32_t *__restrict__ k2v,
                                                         uint32_t *__restrict__ key_of_slot, uint32_t *__restrict__ val_of_slot)
{
    uint64_t r = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (r >= R) return;
    uint64_t ka = key_off[r], nk = key_off[r + 1] - ka, oa = k2v_off[r], va = val_off[r];
    uint64_t prev_end = nk;
    for (uint64_t i = 0; i < nk; ++i) {
        uint64_t end = (uint64_t)(uint32_t)k2v[oa + i];
        for (uint64_t q = prev_end; q < end; ++q) {
            key_of_slot[oa + q] = (uint32_t)(ka + i);
            val_of_slot[oa + q] = (uint32_t)(va + (uint32_t)k2v[oa + q]);
        }
        prev_end = end;
    }
}

// ---------------------------------------------------------------- LDS tier: one workgroup per group
//
// A group whose replies fit (<= ML_REP replies, <= ML_KC key slots, <= ML_VC TxnId slots, <= ML_OC keysToTxnIds
// slots; config 5: 64 replies, 512 / ~2000 / ~2500) is merged entirely in LDS: its key, TxnId and (key, TxnId)
// records are loaded once with coalesced reads, merged (every reply's run is sorted) and de-duplicated in LDS, and the Java-layout result is
// written to scratch at the group's input offsets (the union is never larger than the input), then compacted. The
// per-reply validation of k_m_prep (KeyDeps ctor / checkValid) is done on the same loaded records.

constexpr int ML_REP = 256, ML_KC = 1024, ML_VC = 4096, ML_OC = 4096;
constexpr int ML_WB = 1024;   // TxnId bitmap words (rank spans up to 32768)
constexpr int ML_NT = 512;   // threads per group: more waves per CU for the LDS-latency-bound merge tree and searches

// per group: does it fit the LDS tier (offsets monotone, sizes within the caps)? g[3] |= 1 if some group does not
__global__ __launch_bounds__(BLOCK) void k_m_fit(uint32_t ng, const uint64_t *__restrict__ grp_off, const uint64_t *__restrict__ key_off,
                                                 const uint64_t *__restrict__ val_off, const uint64_t *__restrict__ k2v_off,
                                                 uint64_t *__restrict__ g, uint64_t *__restrict__ gmax)
{
    const uint32_t gi = blockIdx.x * BLOCK + threadIdx.x;
    bool bad = false;
    if (gi < ng) {
        const uint64_t r0 = grp_off[gi], r1 = grp_off[gi + 1];
        if (r1 < r0 || r1 - r0 > ML_REP) bad = true;
        else {
            for (uint64_t r = r0; r < r1 && !bad; ++r)
                if (key_off[r + 1] < key_off[r] || val_off[r + 1] < val_off[r] || k2v_off[r + 1] < k2v_off[r] ||
                    k2v_off[r + 1] - k2v_off[r] < key_off[r + 1] - key_off[r])
                    bad = true;
            if (!bad)
                bad = key_off[r1] - key_off[r0] > ML_KC || val_off[r1] - val_off[r0] > ML_VC ||
                      k2v_off[r1] - k2v_off[r0] > ML_OC;
        }
    }
    block_or1(bad ? 1ull : 0ull, &g[3]);
    uint64_t mx[4] = { 0, 0, 0, 0 };
    if (gi < ng && !bad) {
        const uint64_t r0 = grp_off[gi], r1 = grp_off[gi + 1];
        mx[0] = key_off[r1] - key_off[r0];
        mx[1] = val_off[r1] - val_off[r0];
        mx[2] = k2v_off[r1] - k2v_off[r0];
        mx[3] = (k2v_off[r1] - k2v_off[r0]) - (key_off[r1] - key_off[r0]);
    }
    // wave maxima first: four global atomics per wave instead of per group (they share one line)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint64_t x = mx[k];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) { const uint64_t y = shfl_idx(x, (int)(lane_id() ^ d)); x = y > x ? y : x; }
        if (lane_id() == 0 && x) atomicMax((unsigned long long *)&gmax[k], (unsigned long long)x);
    }
}

// Block-wide merge of NR sorted runs of src[0, N) (run r = [rs[r], rs[r + 1]), rs[NR] = N; rs is overwritten):
// ceil(log2 NR) levels, each merging run pairs with merge-path partitions of ceil(N / ML_NT) outputs per thread,
// ping-ponging between src and dst. Returns the buffer holding the sorted N elements. Every KeyDeps.merge input is
// already sorted per reply (keys, TxnIds, and (key, TxnId) entries once mapped through the monotone merged indices),
// so this replaces a bitonic network's O(log^2 N) barrier stages by O(log NR).
template <class T>
__device__ T *lds_merge_runs(T *src, T *dst, uint32_t *rs, uint32_t NR, uint32_t N)
{
    const uint32_t tid = threadIdx.x;
    const uint32_t CH = (N + ML_NT - 1) / ML_NT;
    while (NR > 1) {
        const uint32_t NP = (NR + 1) / 2;
        const uint32_t o0 = min(N, tid * CH), o1 = min(N, o0 + CH);
        if (o0 < o1) {
            uint32_t lo = 0, hi = NP;   // last pair starting at or before o0
            while (hi - lo > 1) { const uint32_t m = (lo + hi) >> 1; if (rs[2 * m] <= o0) lo = m; else hi = m; }
            uint32_t p = lo, q = o0;
            while (q < o1) {
                const uint32_t a0 = rs[2 * p], a1 = rs[min(2 * p + 1, NR)], b1 = rs[min(2 * p + 2, NR)];
                const uint32_t la = a1 - a0, lb = b1 - a1, end = min(o1, b1), d = q - a0;
                uint32_t i0 = d > lb ? d - lb : 0, i1 = min(d, la);
                while (i0 < i1) {
                    const uint32_t m = (i0 + i1) >> 1;
                    if (src[a0 + m] < src[a1 + d - 1 - m]) i0 = m + 1; else i1 = m;
                }
                uint32_t i = i0, j = d - i0;
                for (; q < end; ++q) {
                    const bool takeA = j >= lb || (i < la && src[a0 + i] < src[a1 + j]);
                    dst[q] = takeA ? src[a0 + i] : src[a1 + j];
                    i += takeA; j += !takeA;
                }
                ++p;
            }
        }
        __syncthreads();
        const uint32_t nv = tid < NP ? rs[2 * tid] : 0u;
        __syncthreads();
        if (tid < NP) rs[tid] = nv;
        if (tid == 0) rs[NP] = N;
        __syncthreads();
        NR = NP;
        T *sw = src; src = dst; dst = sw;
    }
    return src;
}

// pads s[N, up to a multiple of ML_NT) for lds_unique
template <class T>
__device__ __forceinline__ uint32_t lds_pad_block(T *s, uint32_t N, T pad)
{
    const uint32_t np = (N + ML_NT - 1) / ML_NT * ML_NT;
    for (uint32_t i = N + threadIdx.x; i < np; i += ML_NT) s[i] = pad;
    __syncthreads();
    return np;
}

// order-preserving in-place unique of the sorted s[0..np) (pads last); returns the count. np = ML_NT * per.
template <class T, int MAXI>
__device__ __forceinline__ uint32_t lds_unique(T *s, uint32_t np, T pad, uint32_t *scan_lds)
{
    const uint32_t per = np / ML_NT, base = threadIdx.x * per;
    T x[MAXI];
    uint32_t f = 0, c = 0;
#pragma unroll
    for (int q = 0; q < MAXI; ++q) {
        if ((uint32_t)q < per) {
            const uint32_t i = base + q;
            x[q] = s[i];
            const bool u = x[q] != pad && (i == 0 || s[i - 1] != x[q]);
            f |= (uint32_t)u << q;
            c += u;
        }
    }
    uint32_t total;
    uint32_t o = block_exclusive<uint32_t, OpAdd<uint32_t>, ML_NT / 64>(c, OpAdd<uint32_t>(), scan_lds, total);
#pragma unroll
    for (int q = 0; q < MAXI; ++q)
        if ((uint32_t)q < per && ((f >> q) & 1u)) s[o++] = x[q];
    __syncthreads();
    return total;
}

__device__ __forceinline__ uint32_t lds_ub(const uint32_t *a, uint32_t n, uint32_t v)   // first index with a[i] > v
{
    uint32_t lo = 0, hi = n;
    while (lo < hi) { uint32_t m = (lo + hi) >> 1; if (a[m] <= v) lo = m + 1; else hi = m; }
    return lo;
}

struct MlOut {
    uint64_t *s_key;
    uint32_t *s_val;
    int32_t *s_k2v;
    uint64_t *cnt_k, *cnt_v, *cnt_o;
    uint64_t *errs;
};

// LDS plan of k_m_lds (dynamic shared memory, sized by the largest group of the launch)
struct MlPlan {
    uint32_t kc, vc, oc;      // max key / TxnId / keysToTxnIds slots of a group
    uint32_t sp;              // sort area, u32 units: max(2 * pow2(kc), pow2(vc), pow2(oc - keys))
    uint32_t bytes;
};

#ifdef ACC_ML_PROF
// tuning build only: cycles per phase of k_m_lds summed over workgroups (thread 0's view)
__device__ unsigned long long *g_ml_prof;
#define ML_PH(k) do { if (threadIdx.x == 0) { const unsigned long long t_ = clock64(); atomicAdd(&g_ml_prof[k], t_ - ml_t); ml_t = t_; } } while (0)
#else
#define ML_PH(k) ((void)0)
#endif

__global__ __launch_bounds__(ML_NT) void k_m_lds(uint32_t ng, const uint64_t *__restrict__ grp_off, const uint64_t *__restrict__ key_off,
                                                 const uint64_t *__restrict__ key_code, const uint64_t *__restrict__ val_off,
                                                 const uint32_t *__restrict__ txn_rank, const uint64_t *__restrict__ k2v_off,
                                                 const int32_t *__restrict__ k2v, MlPlan pl, MlOut o)
{
    extern __shared__ uint64_t dsm[];
    // [rawk: kc u64][sort: 2 x sp u32 (merge ping-pong)][rawv: vc u32][rawo: oc u32][hdr: kc u32]
    uint64_t *rawk = dsm;
    uint32_t *sort32 = reinterpret_cast<uint32_t *>(dsm + pl.kc);
    uint32_t *sort32b = sort32 + pl.sp;
    uint64_t *sort64 = reinterpret_cast<uint64_t *>(sort32);
    uint64_t *sort64b = reinterpret_cast<uint64_t *>(sort32b);
    uint32_t *rawv = sort32 + 2 * pl.sp;
    uint32_t *rawo = rawv + pl.vc;
    uint32_t *hdr = rawo + pl.oc;
    __shared__ uint32_t rk[ML_REP + 1], rv[ML_REP + 1], ro[ML_REP + 1];
    __shared__ uint32_t scan_lds[ML_NT / 64];
    __shared__ uint32_t rsm[ML_REP + 1];   // run starts of the merge tree
    __shared__ uint32_t wpre[ML_WB];       // TxnId bitmap: set bits before each word
    const uint32_t gi = blockIdx.x;
    const uint32_t tid = threadIdx.x;
#ifdef ACC_ML_PROF
    unsigned long long ml_t = clock64();
#endif
    const uint64_t R0 = grp_off[gi];
    const uint32_t nrep = (uint32_t)(grp_off[gi + 1] - R0);
    const uint64_t KA = key_off[R0], VA = val_off[R0], OA = k2v_off[R0];
    for (uint32_t r = tid; r <= nrep; r += ML_NT) {
        rk[r] = (uint32_t)(key_off[R0 + r] - KA);
        rv[r] = (uint32_t)(val_off[R0 + r] - VA);
        ro[r] = (uint32_t)(k2v_off[R0 + r] - OA);
    }
    __syncthreads();
    const uint32_t NK = rk[nrep], NV = rv[nrep], NO = ro[nrep], NE = NO - NK;
    // per-slot loops run reply-major: TR threads per reply (a power of two, nrep * TR <= ML_NT), so a slot's reply is
    // the thread's own and a keysToTxnIds value's key is found by walking the reply's headers forward, not by binary
    // searches per slot
    uint32_t TR = ML_NT;
    while (TR > 1 && TR * nrep > (uint32_t)ML_NT) TR >>= 1;
    const uint32_t my_r = tid / TR, my_t = tid % TR;
    const bool has_r = my_r < nrep;
    // one coalesced pass over the group's three input ranges
    for (uint32_t i = tid; i < NK; i += ML_NT) rawk[i] = key_code[KA + i];
    for (uint32_t i = tid; i < NV; i += ML_NT) rawv[i] = txn_rank[VA + i];
    for (uint32_t i = tid; i < NO; i += ML_NT) rawo[i] = (uint32_t)k2v[OA + i];
    __syncthreads();
    uint64_t err = 0;
    const uint64_t PADK = ~0ull;
    const uint32_t PAD32 = 0xFFFFFFFFu;
    // ---- keys: sort, unique, write, map every key slot to its merged index
    if (has_r) {
        const uint32_t r = my_r;
        const bool live = ro[r + 1] - ro[r] != rk[r + 1] - rk[r];
        for (uint32_t i = rk[r] + my_t; i < rk[r + 1]; i += TR) {
            if (i > rk[r] && rawk[i - 1] >= rawk[i]) err |= 2;   // Keys sorted unique
            sort64[i] = live ? rawk[i] : PADK;
        }
    }
    __syncthreads();
    ML_PH(0);
    // the distinct keys of the replies with entries: a slot is a first occurrence unless an earlier slot holds the
    // same key (a group's replies repeat the same few keys, so duplicates stop at the first reply); compacted, then
    // each slot's merged index = the number of distinct keys below it (sorted output without a sort)
    uint64_t *dk = sort64b;
    uint32_t fmask = 0, nf = 0;
#pragma unroll
    for (int q = 0; q < ML_KC / ML_NT; ++q) {
        const uint32_t i = tid + q * ML_NT;
        if (i < NK) {
            const uint64_t x = sort64[i];
            bool first = x != PADK;
            for (uint32_t j = 0; first && j < i; ++j) first = sort64[j] != x;
            fmask |= (first ? 1u : 0u) << q;
            nf += first;
        }
    }
    uint32_t Kg;
    uint32_t fpos = block_exclusive<uint32_t, OpAdd<uint32_t>, ML_NT / 64>(nf, OpAdd<uint32_t>(), scan_lds, Kg);
#pragma unroll
    for (int q = 0; q < ML_KC / ML_NT; ++q)
        if ((fmask >> q) & 1u) dk[fpos++] = sort64[tid + q * ML_NT];
    __syncthreads();
    uint32_t kmap[ML_KC / ML_NT];
#pragma unroll
    for (int q = 0; q < ML_KC / ML_NT; ++q) {
        const uint32_t i = tid + q * ML_NT;
        if (i < NK) {
            const uint64_t kc = rawk[i];
            uint32_t below = 0;
            for (uint32_t j = 0; j < Kg; ++j) below += dk[j] < kc;
            kmap[q] = below;
            if ((fmask >> q) & 1u) o.s_key[KA + below] = kc;
        }
    }
    __syncthreads();
    uint32_t *kidx = reinterpret_cast<uint32_t *>(rawk);   // key slot -> merged key index
#pragma unroll
    for (int q = 0; q < ML_KC / ML_NT; ++q) {
        const uint32_t i = tid + q * ML_NT;
        if (i < NK) kidx[i] = kmap[q];
    }
    ML_PH(1);
    // ---- TxnIds: the union as a bitmap over the group's rank span when it fits (config 5: the batch's ranks), so
    // each TxnId's merged index is a word prefix + popcount; otherwise the merge tree + unique + binary searches
    uint32_t vlo = 0xFFFFFFFFu, vhi = 0;
    if (has_r) {
        const uint32_t r = my_r;
        const bool live = ro[r + 1] - ro[r] != rk[r + 1] - rk[r];
        for (uint32_t i = rv[r] + my_t; i < rv[r + 1]; i += TR) {
            if (i > rv[r] && rawv[i - 1] >= rawv[i]) err |= 4;   // txnIds sorted unique
            const uint32_t x = live ? rawv[i] : PAD32;
            if (x != PAD32) { vlo = min(vlo, x); vhi = max(vhi, x); }
            sort32b[i] = x;
        }
    }
    uint32_t ghi, glo_inv;
    (void)block_exclusive<uint32_t, OpMax<uint32_t>, ML_NT / 64>(vhi, OpMax<uint32_t>(), scan_lds, ghi);
    (void)block_exclusive<uint32_t, OpMax<uint32_t>, ML_NT / 64>(~vlo, OpMax<uint32_t>(), scan_lds, glo_inv);
    const uint32_t glo = ~glo_inv;
    const uint64_t span = glo <= ghi ? (uint64_t)ghi - glo + 1 : 0;
    const uint32_t W = (uint32_t)((span + 31) / 32);
    ML_PH(2);
    uint32_t Ug;
    if (W <= (uint32_t)ML_WB && W <= pl.sp) {   // block-uniform
        uint32_t *bm = sort32;
        for (uint32_t w = tid; w < W; w += ML_NT) bm[w] = 0;
        __syncthreads();
        for (uint32_t i = tid; i < NV; i += ML_NT) {
            const uint32_t x = sort32b[i];
            if (x != PAD32) atomicOr(&bm[(x - glo) >> 5], 1u << ((x - glo) & 31u));
        }
        __syncthreads();
        const uint32_t per = (W + ML_NT - 1) / ML_NT, w0 = min(W, tid * per), w1 = min(W, w0 + per);
        uint32_t cnt = 0;
        for (uint32_t w = w0; w < w1; ++w) cnt += (uint32_t)__popc(bm[w]);
        uint32_t run = block_exclusive<uint32_t, OpAdd<uint32_t>, ML_NT / 64>(cnt, OpAdd<uint32_t>(), scan_lds, Ug);
        for (uint32_t w = w0; w < w1; ++w) { wpre[w] = run; run += (uint32_t)__popc(bm[w]); }
        __syncthreads();
        for (uint32_t i = tid; i < NV; i += ML_NT) {
            const uint32_t x = sort32b[i];
            uint32_t idx = 0;   // replies without entries: their TxnIds are never referenced
            if (x != PAD32) {
                const uint32_t d = x - glo, w = d >> 5;
                idx = wpre[w] + (uint32_t)__popc(bm[w] & ((1u << (d & 31u)) - 1u));
            }
            rawv[i] = idx;
        }
        for (uint32_t w = tid; w < W; w += ML_NT) {
            uint32_t bits = bm[w], k = wpre[w];
            while (bits) {
                o.s_val[VA + k++] = glo + 32u * w + (uint32_t)__builtin_ctz(bits);
                bits &= bits - 1u;
            }
        }
        __syncthreads();
    } else {
        for (uint32_t r = tid; r <= nrep; r += ML_NT) rsm[r] = rv[r];
        __syncthreads();
        uint32_t *vs = lds_merge_runs(sort32b, sort32, rsm, nrep, NV);
        Ug = lds_unique<uint32_t, ML_VC / ML_NT>(vs, lds_pad_block(vs, NV, PAD32), PAD32, scan_lds);
        for (uint32_t i = tid; i < NV; i += ML_NT) {
            const uint32_t v = rawv[i];
            uint32_t a = 0, b = Ug;
            while (a < b) { uint32_t m = (a + b) >> 1; if (vs[m] < v) a = m + 1; else b = m; }
            rawv[i] = a;   // each thread rewrites only its own slots
        }
        for (uint32_t u = tid; u < Ug; u += ML_NT) o.s_val[VA + u] = vs[u];
        __syncthreads();
    }
    ML_PH(3);
    // ---- (key, TxnId) entries as (merged key << 16 | TxnId index), headers validated. When the group's Kg x Ug
    // (key, TxnId) grid fits, the entries set bits of a key-major bitmap: key k's TxnIds are then its row's set bits in
    // order, and every offset a word prefix (no merge, no unique)
    const uint32_t WU = (Ug + 31) / 32, WE = Kg * WU;
    const bool ebm = WE <= (uint32_t)ML_WB && WE <= pl.sp;   // block-uniform
    uint32_t *ebits = sort32b;
    if (ebm) {
        for (uint32_t w = tid; w < WE; w += ML_NT) ebits[w] = 0;
        __syncthreads();
    }
    if (has_r) {
        const uint32_t r = my_r;
        const uint32_t nk = rk[r + 1] - rk[r], nv = rv[r + 1] - rv[r], no = ro[r + 1] - ro[r];
        const uint32_t *h = rawo + ro[r];
        if (nk == 0 && no != 0) err |= 8;   // keysToTxnIds entries without keys
        uint32_t kw = 0;   // headers <= qq, advanced monotonically along this thread's slots
        for (uint32_t qq = my_t; nk != 0 && qq < no; qq += TR) {
            if (qq < nk) {
                const uint32_t e = h[qq], prev = qq == 0 ? nk : h[qq - 1];
                if (e < prev || e > no || (qq + 1 == nk && e != no)) err |= 8;
                continue;
            }
            while (kw < nk && h[kw] <= qq) ++kw;
            const uint32_t i = kw < nk ? kw : nk - 1;
            const uint32_t start = i == 0 ? nk : h[i - 1];
            const int32_t xv = (int32_t)h[qq];
            uint32_t x = PAD32;
            if (xv < 0 || (uint32_t)xv >= nv) err |= 16;
            else {
                if (qq > start && (int32_t)h[qq - 1] >= xv) err |= 32;
                if (no != nk) x = (kidx[rk[r] + i] << 16) | rawv[rv[r] + (uint32_t)xv];
            }
            if (!ebm) sort32[ro[r] + qq - rk[r + 1]] = x;
            else if (x != PAD32) {
                const uint32_t u = x & 0xFFFFu;
                atomicOr(&ebits[(x >> 16) * WU + (u >> 5)], 1u << (u & 31u));
            }
        }
    }
    if (ebm) {
        __syncthreads();
        const uint32_t per = (WE + ML_NT - 1) / ML_NT, w0 = min(WE, tid * per), w1 = min(WE, w0 + per);
        uint32_t cnt = 0;
        for (uint32_t w = w0; w < w1; ++w) cnt += (uint32_t)__popc(ebits[w]);
        uint32_t Eu;
        uint32_t run = block_exclusive<uint32_t, OpAdd<uint32_t>, ML_NT / 64>(cnt, OpAdd<uint32_t>(), scan_lds, Eu);
        for (uint32_t w = w0; w < w1; ++w) { wpre[w] = run; run += (uint32_t)__popc(ebits[w]); }
        __syncthreads();
        for (uint32_t k = tid; k < Kg; k += ML_NT)   // header: end offset of key k's TxnId indices
            o.s_k2v[OA + k] = (int32_t)(Kg + (k + 1 < Kg ? wpre[(k + 1) * WU] : Eu));
        for (uint32_t w = tid; w < WE; w += ML_NT) {
            uint32_t bits = ebits[w], c = Kg + wpre[w];
            const uint32_t ub = 32u * (w % WU);
            while (bits) {
                o.s_k2v[OA + c++] = (int32_t)(ub + (uint32_t)__builtin_ctz(bits));
                bits &= bits - 1u;
            }
        }
        if (tid == 0) {
            o.cnt_k[gi] = Kg;
            o.cnt_v[gi] = Ug;
            o.cnt_o[gi] = Kg + Eu;
        }
        ML_PH(6);
        block_or1<ML_NT / 64>(err, o.errs);
        return;
    }
    for (uint32_t k = tid; k < Kg; k += ML_NT) hdr[k] = 0;
    for (uint32_t r = tid; r <= nrep; r += ML_NT) rsm[r] = ro[r] - rk[r];   // reply r's entries start there
    __syncthreads();
    ML_PH(4);
    uint32_t *es = lds_merge_runs(sort32, sort32b, rsm, nrep, NE);
    const uint32_t Eu = lds_unique<uint32_t, ML_VC / ML_NT>(es, lds_pad_block(es, NE, PAD32), PAD32, scan_lds);
    ML_PH(5);
    for (uint32_t c = tid; c < Eu; c += ML_NT) {
        const uint32_t kk = es[c] >> 16;
        if (c + 1 == Eu || (es[c + 1] >> 16) != kk) hdr[kk] = Kg + c + 1;
        o.s_k2v[OA + Kg + c] = (int32_t)(es[c] & 0xFFFFu);
    }
    __syncthreads();
    // keys without entries: end offset = the previous key's (prefix max, starting at Kg)
    {
        const uint32_t per = (Kg + ML_NT - 1) / ML_NT, base = tid * per;
        uint32_t m = 0;
        for (uint32_t q = 0; q < per && base + q < Kg; ++q) m = max(m, hdr[base + q]);
        uint32_t total;
        uint32_t run = block_exclusive<uint32_t, OpMax<uint32_t>, ML_NT / 64>(m, OpMax<uint32_t>(), scan_lds, total);
        run = max(run, Kg);
        for (uint32_t q = 0; q < per && base + q < Kg; ++q) {
            run = max(run, hdr[base + q]);
            o.s_k2v[OA + base + q] = (int32_t)run;
        }
    }
    if (tid == 0) {
        o.cnt_k[gi] = Kg;
        o.cnt_v[gi] = Ug;
        o.cnt_o[gi] = Kg + Eu;
    }
    ML_PH(6);
    block_or1<ML_NT / 64>(err, o.errs);
}

// scratch (at input offsets) -> final CSR: one wave per group
__global__ __launch_bounds__(BLOCK) void k_m_lds_compact(uint32_t ng, const uint64_t *__restrict__ grp_off, const uint64_t *__restrict__ key_off,
                                                         const uint64_t *__restrict__ val_off, const uint64_t *__restrict__ k2v_off,
                                                         MlOut o, const uint64_t *__restrict__ ko, const uint64_t *__restrict__ vo,
                                                         const uint64_t *__restrict__ oo, uint64_t *__restrict__ out_key,
                                                         uint32_t *__restrict__ out_val, int32_t *__restrict__ out_k2v)
{
    const uint32_t gi = (blockIdx.x * BLOCK + threadIdx.x) >> 6, lane = lane_id();
    if (gi >= ng) return;
    const uint64_t R0 = grp_off[gi];
    const uint64_t KA = key_off[R0], VA = val_off[R0], OA = k2v_off[R0];
    const uint64_t nk = ko[gi + 1] - ko[gi], nv = vo[gi + 1] - vo[gi], no = oo[gi + 1] - oo[gi];
    for (uint64_t i = lane; i < nk; i += 64) out_key[ko[gi] + i] = o.s_key[KA + i];
    for (uint64_t i = lane; i < nv; i += 64) out_val[vo[gi] + i] = o.s_val[VA + i];
    for (uint64_t i = lane; i < no; i += 64) out_k2v[oo[gi] + i] = o.s_k2v[OA + i];
}

static void merge_checks(uint64_t err)
{
    if (err & 1) fail(ACC_E_ARG, "merge offsets must be non-decreasing and k2v hold a header per key");
    if (err & 2) fail(ACC_E_ARG, "Keys of a KeyDeps must be sorted and unique");
    if (err & 4) fail(ACC_E_ARG, "txnIds of a KeyDeps must be sorted and unique");
    if (err & 8) fail(ACC_E_ARG, "Last key in keyToTxnId does not point to the end of the array");
    if (err & 16) fail(ACC_E_ARG, "keyToTxnId entry out of range of txnIds");
    if (err & 32) fail(ACC_E_STATE, "Duplicate value found for key (RelationMultiMap.checkValid)");
}

void keydeps_merge(acc_ctx *ctx, const acc_merge_in *in, acc_merge_view *view)
{
    if (!in || !view) fail(ACC_E_ARG, "null argument");
    const uint32_t ng = in->n_groups;
    const uint64_t R = in->n_replies;
    hipStream_t st = ctx->stream;
    ctx->merge_valid = false;
    if (in->mem != ACC_MEM_HOST && in->mem != ACC_MEM_DEVICE) fail(ACC_E_ARG, "mem must be ACC_MEM_HOST or ACC_MEM_DEVICE");
    const uint64_t *grp_off = stage_in(ctx, "m_grp_off", in->grp_off, (size_t)ng + 1, in->mem);
    const uint64_t *key_off = stage_in(ctx, "m_key_off", in->key_off, R + 1, in->mem);
    const uint64_t *val_off = stage_in(ctx, "m_val_off", in->val_off, R + 1, in->mem);
    const uint64_t *k2v_off = stage_in(ctx, "m_k2v_off", in->k2v_off, R + 1, in->mem);
    // totals (last offsets) are needed on the host to size the arrays
    uint64_t tot[3] = { 0, 0, 0 };
    ACC_HIP(hipMemcpyAsync(ctx->pinned, key_off + R, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, val_off + R, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 2, k2v_off + R, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    memcpy(tot, ctx->pinned, sizeof tot);
    const uint64_t NK = tot[0], NV = tot[1], NO = tot[2];
    if (NK >= 0xFFFFFFFFull || NV >= 0xFFFFFFFFull || NO >= 0xFFFFFFFFull) fail(ACC_E_CAP, "merge input too large");
    const uint64_t *key_code = stage_in(ctx, "m_key_code", in->key_code, NK, in->mem);
    const uint32_t *txn_rank = stage_in(ctx, "m_txn_rank", in->txn_rank, NV, in->mem);
    const int32_t *k2v = stage_in(ctx, "m_k2v", in->k2v, NO, in->mem);

    uint64_t *g = ctx->get<uint64_t>("m_g", 4);
    ACC_HIP(hipMemsetAsync(g, 0, 4 * 8, st));
    if (ng && !(ctx->flags & ACC_OPT_FORCE_REPLAY)) {
        // ---- LDS tier when every group fits
        uint64_t *gmax = ctx->get<uint64_t>("m_gmax", 4);
        ACC_HIP(hipMemsetAsync(gmax, 0, 4 * 8, st));
        launch(ctx, "m_fit", k_m_fit, dim3(grid_for(ng, BLOCK)), dim3(BLOCK), 0, ng, grp_off, key_off, val_off, k2v_off, g, gmax);
        ACC_HIP(hipMemcpyAsync(ctx->pinned, g + 3, 8, hipMemcpyDeviceToHost, st));
        ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, gmax, 4 * 8, hipMemcpyDeviceToHost, st));
        ctx->sync();
        if (ctx->pinned[0] == 0) {
            auto rb = [](uint64_t n) { return std::max<uint64_t>(ML_NT, (n + ML_NT - 1) / ML_NT * ML_NT); };
            MlPlan pl;
            pl.kc = (uint32_t)ctx->pinned[1];
            pl.vc = (uint32_t)ctx->pinned[2];
            pl.oc = (uint32_t)ctx->pinned[3];
            pl.sp = (uint32_t)std::max({ 2 * rb(pl.kc), rb(pl.vc), rb(ctx->pinned[4]) });   // one merge buffer (u32)
            pl.kc = (pl.kc + 1) & ~1u;   // keep the u32 areas after rawk 8-byte aligned
            pl.bytes = 8 * pl.kc + 8 * pl.sp + 4 * pl.vc + 4 * pl.oc + 4 * pl.kc;
            MlOut mo;
            mo.s_key = ctx->get<uint64_t>("m_s_key", NK + 1);
            mo.s_val = ctx->get<uint32_t>("m_s_val", NV + 1);
            mo.s_k2v = ctx->get<int32_t>("m_s_k2v", NO + 1);
            mo.cnt_k = ctx->get<uint64_t>("m_cnt_k", ng);
            mo.cnt_v = ctx->get<uint64_t>("m_cnt_v", ng);
            mo.cnt_o = ctx->get<uint64_t>("m_cnt_o", ng);
            mo.errs = g + 2;
#ifdef ACC_ML_PROF
            unsigned long long *mlp = ctx->get<unsigned long long>("ml_prof", 8);
            ACC_HIP(hipMemsetAsync(mlp, 0, 64, st));
            ACC_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_ml_prof), &mlp, sizeof mlp, 0, hipMemcpyHostToDevice, st));
#endif
            launch(ctx, "m_lds", k_m_lds, dim3(ng), dim3(ML_NT), pl.bytes, ng, grp_off, key_off, key_code, val_off, txn_rank,
                   k2v_off, k2v, pl, mo);
#ifdef ACC_ML_PROF
            {
                unsigned long long h[8];
                ACC_HIP(hipMemcpyAsync(h, mlp, 64, hipMemcpyDeviceToHost, st));
                ACC_HIP(hipStreamSynchronize(st));
                fprintf(stderr, "[ml_prof] per group cycles: stage %.0f keys %.0f tx-prep %.0f tx %.0f ent-prep %.0f ent %.0f out %.0f\n",
                        h[0] / (double)ng, h[1] / (double)ng, h[2] / (double)ng, h[3] / (double)ng, h[4] / (double)ng,
                        h[5] / (double)ng, h[6] / (double)ng);
            }
#endif
            uint64_t *ko = ctx->get<uint64_t>("m_k_gstart", (size_t)ng + 1);
            uint64_t *vo = ctx->get<uint64_t>("m_v_gstart", (size_t)ng + 1);
            uint64_t *oo = ctx->get<uint64_t>("m_out_k2v_off", (size_t)ng + 1);
            scan<uint64_t, OpAdd<uint64_t>>(ctx, mo.cnt_k, ko, ng, true, ko + ng);
            scan<uint64_t, OpAdd<uint64_t>>(ctx, mo.cnt_v, vo, ng, true, vo + ng);
            scan<uint64_t, OpAdd<uint64_t>>(ctx, mo.cnt_o, oo, ng, true, oo + ng);
            ACC_HIP(hipMemcpyAsync(ctx->pinned, g + 2, 8, hipMemcpyDeviceToHost, st));
            ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, ko + ng, 8, hipMemcpyDeviceToHost, st));
            ACC_HIP(hipMemcpyAsync(ctx->pinned + 2, vo + ng, 8, hipMemcpyDeviceToHost, st));
            ACC_HIP(hipMemcpyAsync(ctx->pinned + 3, oo + ng, 8, hipMemcpyDeviceToHost, st));
            ctx->sync();
            merge_checks(ctx->pinned[0]);
            const uint64_t TK = ctx->pinned[1], TV = ctx->pinned[2], TO = ctx->pinned[3];
            uint64_t *out_key = ctx->get<uint64_t>("m_out_key", TK + 1);
            uint32_t *out_val = ctx->get<uint32_t>("m_out_val", TV + 1);
            int32_t *out_k2v = ctx->get<int32_t>("m_out_k2v", TO + 1);
            launch(ctx, "m_lds_compact", k_m_lds_compact, dim3(grid_for((size_t)ng * 64, BLOCK)), dim3(BLOCK), 0, ng, grp_off,
                   key_off, val_off, k2v_off, mo, (const uint64_t *)ko, (const uint64_t *)vo, (const uint64_t *)oo, out_key,
                   out_val, out_k2v);
            ctx->sync();
            ctx->stat("merge.lds_tier", 1);
            *view = acc_merge_view{ ng, TK, TV, TO, NO, ko, out_key, vo, out_val, oo, out_k2v };
            ctx->merge_view = *view;
            ctx->merge_valid = true;
            return;
        }
    }
    ctx->stat("merge.lds_tier", 0);
    uint32_t *grp_of = ctx->get<uint32_t>("m_grp_of", R);
    launch(ctx, "m_replies", k_m_replies, dim3(grid_for(ng, BLOCK)), dim3(BLOCK), 0, ng, grp_off, grp_of);
    launch(ctx, "m_prep", k_m_prep, dim3(grid_for(R, BLOCK)), dim3(BLOCK), 0, R, key_off, key_code, val_off, txn_rank,
           k2v_off, k2v, g);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, g, 3 * 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t kmask = ctx->pinned[0], vmask = ctx->pinned[1], err = ctx->pinned[2];
    merge_checks(err);

    MergePlan plan;
    plan.rk = make_runs(kmask);
    plan.rv = make_runs(vmask);
    const int gb = bits_for(ng ? ng - 1 : 0) + 1;   // +1: real records stay below the all-ones pad
    // Wide key codes (hashed keys use every bit) leave no room for the group field: sort on dense ranks of the codes
    // (and of the TxnId ranks) instead; the outputs still carry the caller's codes.
    const uint64_t *ekey = key_code;
    const uint32_t *eval = txn_rank;
    if (gb + plan.rk.bits + plan.rv.bits > 64) {
        const uint64_t *kw[1] = { key_code };
        DenseRank kd = dense_rank(ctx, "m_kdict", NK, 1, kw, nullptr, nullptr, false);
        uint64_t *kr64 = ctx->get<uint64_t>("m_kr64", NK);
        launch(ctx, "m_widen", k_widen, dim3(grid_for(NK, BLOCK)), dim3(BLOCK), 0, NK, (const uint32_t *)kd.rank, kr64);
        ACC_HIP(hipMemcpyAsync(ctx->pinned, kd.count_dev, 8, hipMemcpyDeviceToHost, st));
        uint64_t *vw64 = ctx->get<uint64_t>("m_vw64", NV);
        launch(ctx, "m_widen", k_widen, dim3(grid_for(NV, BLOCK)), dim3(BLOCK), 0, NV, txn_rank, vw64);
        const uint64_t *vw[1] = { vw64 };
        DenseRank vd = dense_rank(ctx, "m_vdict", NV, 1, vw, nullptr, nullptr, false);
        ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, vd.count_dev, 8, hipMemcpyDeviceToHost, st));
        ctx->sync();
        ekey = kr64;
        eval = vd.rank;
        plan.rk = make_runs(ctx->pinned[0] > 1 ? (1ull << bits_for(ctx->pinned[0] - 1)) - 1 : 0);
        plan.rv = make_runs(ctx->pinned[1] > 1 ? (1ull << bits_for(ctx->pinned[1] - 1)) - 1 : 0);
        ctx->stat("merge.dense_keys", 1);
    } else {
        ctx->stat("merge.dense_keys", 0);
    }
    const int kb = plan.rk.bits, vb = plan.rv.bits;
    if (gb + kb + vb > 64) fail(ACC_E_CAP, "merge composite key exceeds 64 bits (groups x distinct keys x distinct TxnIds)");
    plan.gshift_k = kb; plan.gshift_v = vb; plan.gshift_kv = kb + vb; plan.vshift_kv = vb;
    auto ones = [](int b) { return b >= 64 ? ~0ull : ((1ull << b) - 1); };
    plan.pad_k = ones(gb + kb); plan.pad_v = ones(gb + vb); plan.pad_kv = ones(gb + kb + vb);

    uint64_t *sk = ctx->get<uint64_t>("m_sk", NK);
    uint64_t *sv = ctx->get<uint64_t>("m_sv", NV);
    uint64_t *skv = ctx->get<uint64_t>("m_skv", NO);
    uint32_t *key_of_slot = ctx->get<uint32_t>("m_key_of_slot", NO);
    uint32_t *val_of_slot = ctx->get<uint32_t>("m_val_of_slot", NO);
    launch(ctx, "m_expand", k_m_expand, dim3(grid_for(R, BLOCK)), dim3(BLOCK), 0, R, (const uint32_t *)grp_of, key_off,
           ekey, val_off, eval, k2v_off, k2v, plan, sk, sv, skv);
    launch(ctx, "m_key_of_slot", k_m_key_of_slot, dim3(grid_for(R, BLOCK)), dim3(BLOCK), 0, R, key_off, val_off, k2v_off,
           k2v, key_of_slot, val_of_slot);
    Sorted ssk = radix_sort(ctx, "m_rs_k", sk, nullptr, NK, gb + kb);
    Sorted ssv = radix_sort(ctx, "m_rs_v", sv, nullptr, NV, gb + vb);
    Sorted sskv = radix_sort(ctx, "m_rs_kv", skv, nullptr, NO, gb + kb + vb);

    struct U { uint64_t *flag, *idx, *gstart; };
    auto uniq = [&](const char *tag, const Sorted &so, uint64_t n, int gshift, uint64_t pad) {
        char a[48], b2[48], c[48], d[48], e[48], f[48];
        snprintf(a, sizeof a, "%s_flag", tag); snprintf(b2, sizeof b2, "%s_idx", tag);
        snprintf(c, sizeof c, "%s_gstart", tag); snprintf(d, sizeof d, "%s_gfirst", tag);
        snprintf(e, sizeof e, "%s_glast", tag); snprintf(f, sizeof f, "%s_gcnt", tag);
        U u{ ctx->get<uint64_t>(a, n), ctx->get<uint64_t>(b2, n + 1), ctx->get<uint64_t>(c, (size_t)ng + 1) };
        uint64_t *gfirst = ctx->get<uint64_t>(d, ng), *glast = ctx->get<uint64_t>(e, ng), *gcnt = ctx->get<uint64_t>(f, ng);
        launch(ctx, "m_uniq", k_m_uniq, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint64_t *)so.keys, pad, u.flag);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, u.flag, u.idx, n, true, u.idx + n);
        ACC_HIP(hipMemsetAsync(gfirst, 0, (size_t)ng * 8, st));
        ACC_HIP(hipMemsetAsync(glast, 0, (size_t)ng * 8, st));
        launch(ctx, "m_group_bounds", k_m_group_bounds, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint64_t *)so.keys,
               pad, (const uint64_t *)u.flag, (const uint64_t *)u.idx, gshift, gfirst, glast);
        launch(ctx, "m_group_counts", k_m_group_counts, dim3(grid_for(ng, BLOCK)), dim3(BLOCK), 0, ng,
               (const uint64_t *)gfirst, (const uint64_t *)glast, gcnt);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, gcnt, u.gstart, ng, true, u.gstart + ng);
        return u;
    };
    U uk = uniq("m_k", ssk, NK, plan.gshift_k, plan.pad_k);
    U uv = uniq("m_v", ssv, NV, plan.gshift_v, plan.pad_v);
    U ukv = uniq("m_kv", sskv, NO, plan.gshift_kv, plan.pad_kv);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, uk.gstart + ng, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, uv.gstart + ng, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 2, ukv.gstart + ng, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t TK = ctx->pinned[0], TV = ctx->pinned[1], TKV = ctx->pinned[2];

    uint64_t *out_key = ctx->get<uint64_t>("m_out_key", TK);
    uint32_t *out_val = ctx->get<uint32_t>("m_out_val", TV);
    int32_t *out_k2v = ctx->get<int32_t>("m_out_k2v", TK + TKV);
    uint8_t *has = ctx->get<uint8_t>("m_has", TK);
    uint64_t *out_k2v_off = ctx->get<uint64_t>("m_out_k2v_off", (size_t)ng + 1);
    launch(ctx, "m_write_keys", k_m_write_keys, dim3(grid_for(NK, BLOCK)), dim3(BLOCK), 0, NK, (const uint64_t *)uk.flag,
           (const uint64_t *)uk.idx, key_code, (const uint32_t *)ssk.vals, out_key);
    launch(ctx, "m_write_vals", k_m_write_vals, dim3(grid_for(NV, BLOCK)), dim3(BLOCK), 0, NV, (const uint64_t *)uv.flag,
           (const uint64_t *)uv.idx, txn_rank, (const uint32_t *)ssv.vals, out_val);
    ACC_HIP(hipMemsetAsync(has, 0, TK ? TK : 1, st));
    launch(ctx, "m_write_k2v", k_m_write_k2v, dim3(grid_for(NO, BLOCK)), dim3(BLOCK), 0, NO, (const uint64_t *)sskv.keys, plan,
           (const uint64_t *)ukv.flag, (const uint64_t *)ukv.idx, (const uint64_t *)ukv.gstart, (const uint64_t *)uk.gstart,
           (const uint64_t *)uv.gstart, (const uint32_t *)out_val, (const uint64_t *)out_key, txn_rank,
           (const uint32_t *)sskv.vals, (const uint32_t *)val_of_slot, (const uint32_t *)key_of_slot, key_code, out_k2v, has);
    launch(ctx, "m_fix_headers", k_m_fix_headers, dim3(grid_for((size_t)ng + 1, BLOCK)), dim3(BLOCK), 0, ng,
           (const uint64_t *)ukv.gstart, (const uint64_t *)uk.gstart, out_k2v, (const uint8_t *)has, out_k2v_off);
    ctx->sync();
    *view = acc_merge_view{ ng, TK, TV, TK + TKV, NO, uk.gstart, out_key, uv.gstart, out_val, out_k2v_off, out_k2v };
    ctx->merge_view = *view;
    ctx->merge_valid = true;
}

}  // namespace acc
