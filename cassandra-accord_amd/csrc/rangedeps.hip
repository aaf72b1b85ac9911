// rangedeps.hip — RangeDeps of a mixed key/range batch on CDNA4 (SURVEY.md §8 rows A4, A8 range part, A18).
//
// For every txn T of one CommandStore snapshot, the range-command part of
// InMemorySafeStore.mapReduceActive (impl/InMemoryCommandStore.java:863-870 -> mapReduceRangesInternal :883-1016)
// under PreAccept.calculatePartialDeps (messages/PreAccept.java:245-265):
//   every range command C (range-domain txn, status not erased: INVALID_OR_TRUNCATED here) with
//   C.txnId < T.executeAt (STARTED_BEFORE), T.kind().witnesses(C.kind), C != p1, contributes (r, C) for each
//   of its ranges r that intersects T's keys (Range.contains) or T's ranges (start < that.end && end > that.start);
//   the TreeMap<Range, List> (Range::compare) then RangeDeps.Builder (utils/RelationMultiMap.java:88-260) give the
//   Java layout: ranges sorted unique, txnIds sorted unique, rangesToTxnIds = end-offset header + indices.
//
// Pipeline (one HIP stream):
//   1. prep + dictionary (shared with keydeps.hip): validation, dense order ranks of every TxnId/executeAt.
//   2. range-command entries: the ranges of non-erased range txns; stored-range dictionary (distinct (start, end)
//      in Range::compare order -> range id); entries re-sorted by (width class, start) where class c holds widths
//      in (4^(c-1), 4^c]: a range of class c containing / intersecting a query [lo, hi] starts in [lo - 4^c, hi].
//   3. stabbing: every query (a key of a key txn, or a range of a range txn) sorted by its low bound; a workgroup
//      of 256 consecutive queries streams, per class, the entries starting in its window through LDS (coalesced
//      tiles shared by the 256 queries) and tests each against its own query: count -> scan -> emit of
//      (range id << 32 | TxnId rank) per query, contiguous per txn.
//   4. build: per txn, sort (range id, TxnId rank) = TreeMap order, dedupe, TxnId union + index: one wave per txn
//      (<= 64 raw entries, register bitonic), one workgroup per txn (<= 8192, LDS bitonic), one workgroup on a
//      global scratch region beyond that. Two passes: sizes, then the Java-layout writes.
// Integer work only: HBM/latency bound, no MFMA.

#include "dict.hpp"

namespace acc {

namespace rd {

constexpr int NCLS = 33;          // width classes 0..32 (4^32 = 2^64 covers every u64 width)
constexpr int TILE = 1024;        // entries per LDS tile in the stabbing pass
constexpr uint32_t WAVE_E = 64;   // wave tier: raw entries per txn
constexpr uint32_t BLOCK_E = 8192;  // workgroup tier (LDS)

enum : uint64_t {
    ERR_DOMAIN = 1u << 8,
    ERR_RANGE_EMPTY = 1u << 9,
    ERR_RANGES_UNSORTED = 1u << 10,
    ERR_RNG_OFF = 1u << 11,
};

__device__ __forceinline__ uint32_t witnesses(uint32_t kind)
{
    // Kind.witnesses() (primitives/Txn.java:221-236) as a mask over Kind ordinals; LocalOnly is rejected in prep
    switch (kind) {
    case 0: case 2: return 1u << 1;
    case 1: case 3: return (1u << 0) | (1u << 1);
    case 4:         return (1u << 0) | (1u << 1) | (1u << 3) | (1u << 4);
    default:        return 0;
    }
}

__device__ __forceinline__ uint32_t width_class(uint64_t s, uint64_t e)
{
    const uint64_t w = e - s;                 // >= 1 after validation
    const uint32_t bits = w <= 1 ? 0u : 64u - (uint32_t)__builtin_clzll(w - 1);   // ceil(log2 w)
    return (bits + 1) >> 1;                   // w <= 4^class
}

__device__ __forceinline__ uint64_t class_width(uint32_t c) { return c >= 32 ? ~0ull : (1ull << (2 * c)); }

// ---------------------------------------------------------------- small helpers

__global__ __launch_bounds__(BLOCK) void k_permute_u64(size_t n, const uint32_t *__restrict__ perm, const uint64_t *__restrict__ in,
                                                       uint64_t *__restrict__ out)
{
    const size_t p = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p < n) out[p] = in[perm[p]];
}

__global__ __launch_bounds__(BLOCK) void k_pext_u64(size_t n, const uint64_t *__restrict__ in, Runs plan, uint64_t *__restrict__ out)
{
    const size_t p = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p < n) out[p] = pext_runs(in[p], plan);
}

__global__ __launch_bounds__(BLOCK) void k_widen_u32(size_t n, const uint32_t *__restrict__ in, uint64_t *__restrict__ out)
{
    const size_t p = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p < n) out[p] = in[p];
}

// ---------------------------------------------------------------- prep

// Per txn: domain consistency (TxnId.domain(), primitives/TxnId.java:134-157), Range start < end (Range.java ctor)
// and Ranges.ofSortedAndDeoverlapped (AbstractRanges.java:789-796); range owners; entry flags (non-erased range
// commands); OR-masks of the range bounds and the query low bounds (bit compaction plans).
// g: [0] start mask, [1] end mask, [2] query-lo mask (all relative to ref[]), [3] errors, [4] non-empty ranges.
__global__ __launch_bounds__(BLOCK) void k_rd_prep(uint32_t n, const uint64_t *__restrict__ tl, const uint8_t *__restrict__ status,
                                                   const uint32_t *__restrict__ key_off, const uint64_t *__restrict__ key_code,
                                                   const uint32_t *__restrict__ rng_off, const uint64_t *__restrict__ rs,
                                                   const uint64_t *__restrict__ re, uint64_t ref_s, uint64_t ref_e,
                                                   uint64_t ref_lo, uint32_t *__restrict__ rowner,
                                                   uint32_t *__restrict__ eflag, uint64_t *__restrict__ g)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    uint64_t ms = 0, me = 0, ml = 0, errs = 0;
    if (t < n) {
        const bool isr = (tl[t] & 1u) != 0;
        const uint32_t k0 = key_off[t], k1 = key_off[t + 1];
        const uint32_t r0 = rng_off[t], r1 = rng_off[t + 1];
        if (r1 < r0) errs |= ERR_RNG_OFF;
        else {
            if (isr && k1 != k0) errs |= ERR_DOMAIN;
            if (!isr && r1 != r0) errs |= ERR_DOMAIN;
            const uint32_t live = status[t] != 7;
            for (uint32_t j = r0; j < r1; ++j) {
                const uint64_t s = rs[j], e = re[j];
                if (s >= e) errs |= ERR_RANGE_EMPTY;
                if (j > r0 && re[j - 1] > s) errs |= ERR_RANGES_UNSORTED;
                rowner[j] = t;
                eflag[j] = live;
                ms |= s ^ ref_s;
                me |= e ^ ref_e;
                ml |= s ^ ref_lo;
            }
        }
        if (k1 >= k0)
            for (uint32_t j = k0; j < k1; ++j) ml |= key_code[j] ^ ref_lo;
    }
    __shared__ uint64_t part[WAVES][4];
    uint64_t v[4] = { ms, me, ml, errs };
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        uint64_t x = v[w];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) x |= shfl_xor(x, d);
        if (lane_id() == 0) part[threadIdx.x >> 6][w] = x;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        uint64_t x = 0;
#pragma unroll
        for (int q = 0; q < WAVES; ++q) x |= part[q][threadIdx.x];
        if (x) atomicOr((unsigned long long *)&g[threadIdx.x], (unsigned long long)x);
    }
}

// compacted entry columns (input order) + the (start, end) dictionary sort key
__global__ __launch_bounds__(BLOCK) void k_rd_entries(uint32_t R, uint32_t n, const uint32_t *__restrict__ eflag,
                                                      const uint32_t *__restrict__ eidx, const uint32_t *__restrict__ rowner,
                                                      const uint64_t *__restrict__ rs, const uint64_t *__restrict__ re,
                                                      const uint32_t *__restrict__ rank, const uint64_t *__restrict__ tl,
                                                      Runs rs_plan, Runs re_plan, int e_bits, int split,
                                                      uint64_t *__restrict__ e_s, uint64_t *__restrict__ e_e,
                                                      uint32_t *__restrict__ e_rank, uint8_t *__restrict__ e_kind,
                                                      uint64_t *__restrict__ dkey, uint64_t *__restrict__ ekey)
{
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= R || !eflag[j]) return;
    const uint32_t i = eidx[j], t = rowner[j];
    const uint64_t s = rs[j], e = re[j];
    e_s[i] = s;
    e_e[i] = e;
    e_rank[i] = rank[t];
    e_kind[i] = (uint8_t)((tl[t] >> 1) & 7u);
    const uint64_t sc = pext_runs(s, rs_plan), ec = pext_runs(e, re_plan);
    if (split) { dkey[i] = sc; ekey[i] = ec; }      // two-key LSD: end first, then start (stable)
    else dkey[i] = (sc << e_bits) | ec;
}

// rid per (start, end)-sorted position; dictionary arrays
__global__ __launch_bounds__(BLOCK) void k_rd_dict_flags(uint32_t ne, const uint32_t *__restrict__ perm,
                                                         const uint64_t *__restrict__ e_s, const uint64_t *__restrict__ e_e,
                                                         uint32_t *__restrict__ flag)
{
    const uint32_t p = blockIdx.x * BLOCK + threadIdx.x;
    if (p >= ne) return;
    uint32_t f = 1;
    if (p > 0) {
        const uint32_t a = perm[p], b = perm[p - 1];
        f = e_s[a] != e_s[b] || e_e[a] != e_e[b];
    }
    flag[p] = f;
}

__global__ __launch_bounds__(BLOCK) void k_rd_dict_write(uint32_t ne, const uint32_t *__restrict__ perm,
                                                         const uint32_t *__restrict__ flag, const uint32_t *__restrict__ incl,
                                                         const uint64_t *__restrict__ e_s, const uint64_t *__restrict__ e_e,
                                                         uint32_t *__restrict__ rid_of, uint64_t *__restrict__ dict_s,
                                                         uint64_t *__restrict__ dict_e, Runs rs_plan, int s_bits, int cls_only,
                                                         uint64_t *__restrict__ ckey, uint32_t *__restrict__ cls_hist)
{
    __shared__ uint32_t h[NCLS];
    if (threadIdx.x < NCLS) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t p = blockIdx.x * BLOCK + threadIdx.x;
    if (p < ne) {
        const uint32_t i = perm[p], rid = incl[p] - 1;
        rid_of[i] = rid;
        if (flag[p]) { dict_s[rid] = e_s[i]; dict_e[rid] = e_e[i]; }
        const uint32_t c = width_class(e_s[i], e_e[i]);
        ckey[i] = cls_only ? (uint64_t)c : (((uint64_t)c << s_bits) | pext_runs(e_s[i], rs_plan));
        atomicAdd(&h[c], 1u);   // LDS histogram; one global atomic per class and block (33 hot words otherwise)
    }
    __syncthreads();
    if (threadIdx.x < NCLS && h[threadIdx.x]) atomicAdd(&cls_hist[threadIdx.x], h[threadIdx.x]);
}

__global__ void k_rd_class_off(const uint32_t *__restrict__ hist, uint32_t *__restrict__ off)
{
    if (threadIdx.x != 0) return;
    uint32_t a = 0;
    for (int c = 0; c < NCLS; ++c) { off[c] = a; a += hist[c]; }
    off[NCLS] = a;
}

// class-sorted entry columns
__global__ __launch_bounds__(BLOCK) void k_rd_class_cols(uint32_t ne, const uint32_t *__restrict__ perm,
                                                         const uint64_t *__restrict__ e_s, const uint64_t *__restrict__ e_e,
                                                         const uint32_t *__restrict__ e_rank, const uint8_t *__restrict__ e_kind,
                                                         const uint32_t *__restrict__ rid_of, uint64_t *__restrict__ cs_s,
                                                         uint64_t *__restrict__ cs_e, uint2 *__restrict__ cs_info,
                                                         uint8_t *__restrict__ cs_kind)
{
    const uint32_t p = blockIdx.x * BLOCK + threadIdx.x;
    if (p >= ne) return;
    const uint32_t i = perm[p];
    cs_s[p] = e_s[i];
    cs_e[p] = e_e[i];
    cs_info[p] = make_uint2(rid_of[i], e_rank[i]);
    cs_kind[p] = e_kind[i];
}

// query low bounds (keys of key txns, starts of range txns' ranges), compacted, for the query sort
__global__ __launch_bounds__(BLOCK) void k_rd_query_keys(uint32_t P, uint32_t R, const uint64_t *__restrict__ key_code,
                                                         const uint64_t *__restrict__ rs, Runs plan,
                                                         uint64_t *__restrict__ qkey)
{
    const uint32_t q = blockIdx.x * BLOCK + threadIdx.x;
    if (q >= P + R) return;
    qkey[q] = pext_runs(q < P ? key_code[q] : rs[q - P], plan);
}

// ---------------------------------------------------------------- stabbing (count / emit)

struct View {
    uint32_t n, P, R, Q;
    int end_inclusive;
    const uint32_t *qperm;        // queries sorted by low bound
    const uint64_t *key_code;
    const uint32_t *owner;        // txn of key pair
    const uint64_t *rs, *re;
    const uint32_t *rowner;       // txn of range
    const uint32_t *rank;         // [2n]
    const uint64_t *tl;
    const uint64_t *cs_s, *cs_e;  // entries by (class, start)
    const uint2 *cs_info;         // (range id, TxnId rank)
    const uint8_t *cs_kind;
    const uint32_t *class_off;    // [NCLS + 1]
};

__device__ __forceinline__ uint32_t lower_bound_s(const uint64_t *a, uint32_t lo, uint32_t hi, uint64_t v)
{
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ uint32_t upper_bound_s(const uint64_t *a, uint32_t lo, uint32_t hi, uint64_t v)
{
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] <= v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

template <bool EMIT>
__global__ __launch_bounds__(BLOCK) void k_rd_stab(View v, uint32_t *__restrict__ cnt, const uint64_t *__restrict__ q_off,
                                                   uint64_t *__restrict__ ent)
{
    __shared__ uint64_t t_s[TILE], t_e[TILE];
    __shared__ uint2 t_info[TILE];
    __shared__ uint8_t t_kind[TILE];
    __shared__ uint64_t s_hi[WAVES];
    __shared__ uint64_t s_lo;
    __shared__ uint32_t s_b0, s_b1;
    const uint32_t tid = threadIdx.x;
    const uint32_t i = blockIdx.x * BLOCK + tid;
    const bool valid = i < v.Q;
    uint32_t q = 0, t = 0;
    uint64_t lo = 0, hi = 0;
    bool isr = false;
    if (valid) {
        q = v.qperm[i];
        if (q < v.P) { lo = hi = v.key_code[q]; t = v.owner[q]; }
        else { lo = v.rs[q - v.P]; hi = v.re[q - v.P]; t = v.rowner[q - v.P]; isr = true; }
    }
    const uint32_t exec_rank = valid ? v.rank[v.n + t] : 0u;
    const uint32_t txn_rank = valid ? v.rank[t] : 0u;
    const uint32_t wm = valid ? witnesses((uint32_t)(v.tl[t] >> 1) & 7u) : 0u;
    // block window: queries are sorted by lo, so thread 0 holds the smallest; hi needs a max
    uint64_t h = valid ? hi : 0;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) { uint64_t o = shfl_xor(h, d); h = o > h ? o : h; }
    if (lane_id() == 0) s_hi[tid >> 6] = h;
    if (tid == 0) s_lo = lo;
    __syncthreads();
    uint64_t hi_max = 0;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) hi_max = s_hi[w] > hi_max ? s_hi[w] : hi_max;
    const uint64_t lo_min = s_lo;

    uint32_t count = 0;
    uint64_t out = 0;
    if (EMIT && valid) out = q_off[q];
    for (uint32_t c = 0; c < (uint32_t)NCLS; ++c) {
        const uint32_t a0 = v.class_off[c], a1 = v.class_off[c + 1];
        if (a0 == a1) continue;
        const uint64_t W = class_width(c);
        if (tid == 0) {
            const uint64_t wlo = lo_min > W ? lo_min - W : 0;
            const uint32_t b0 = lower_bound_s(v.cs_s, a0, a1, wlo);
            s_b0 = b0;
            s_b1 = upper_bound_s(v.cs_s, b0, a1, hi_max);
        }
        __syncthreads();
        const uint32_t b0 = s_b0, b1 = s_b1;
        __syncthreads();
        const uint64_t qwlo = lo > W ? lo - W : 0;
        for (uint32_t base = b0; base < b1; base += TILE) {
            const uint32_t len = min((uint32_t)TILE, b1 - base);
            for (uint32_t k = tid; k < len; k += BLOCK) {
                t_s[k] = v.cs_s[base + k];
                t_e[k] = v.cs_e[base + k];
                t_info[k] = v.cs_info[base + k];
                t_kind[k] = v.cs_kind[base + k];
            }
            __syncthreads();
            if (valid) {
                // this query's own window inside the tile: starts in [lo - W, hi]
                uint32_t k = lower_bound_s(t_s, 0, len, qwlo);
                for (; k < len; ++k) {
                    const uint64_t s = t_s[k];
                    if (s > hi) break;
                    const uint64_t e = t_e[k];
                    bool hit;
                    if (isr) hit = s < hi && e > lo;                              // Range.compareIntersecting == 0
                    else if (v.end_inclusive) hit = s < lo && lo <= e;            // EndInclusive.contains (s, e]
                    else hit = s <= lo && lo < e;                                 // StartInclusive.contains [s, e)
                    if (!hit) continue;
                    const uint2 info = t_info[k];
                    if (info.y >= exec_rank || info.y == txn_rank) continue;     // STARTED_BEFORE; p1
                    if (!((wm >> t_kind[k]) & 1u)) continue;                     // testKind
                    if (EMIT) ent[out + count] = ((uint64_t)info.x << 32) | info.y;
                    ++count;
                }
            }
            __syncthreads();
        }
    }
    if (!EMIT && valid) cnt[q] = count;
}

// ---------------------------------------------------------------- per-txn build

struct Out {
    const uint32_t *key_off, *rng_off;
    uint32_t P;
    const uint64_t *q_off;        // [P + R + 1]
    const uint64_t *ent;
    const uint32_t *txn_of_rank;
    uint32_t *rd_cnt, *u_cnt;     // sizes pass
    uint64_t *a_cnt;
    const uint64_t *arena_off, *rd_off, *u_off;   // write pass
    int32_t *arena;
    uint32_t *range_id, *dep_txn;
    uint32_t *blk_list, *glb_list;
    const uint64_t *glb_off;      // scratch offsets of the global tier (u64 elements)
    uint64_t *scratch;
    uint64_t *gstat;              // [0] block-tier txns, [1] global-tier txns, [2] global scratch elements
};

__device__ __forceinline__ void txn_range(const Out &o, uint32_t t, uint64_t &e0, uint64_t &e1)
{
    const uint32_t k0 = o.key_off[t], k1 = o.key_off[t + 1];
    if (k1 > k0) { e0 = o.q_off[k0]; e1 = o.q_off[k1]; return; }
    const uint32_t r0 = o.rng_off[t], r1 = o.rng_off[t + 1];
    e0 = o.q_off[o.P + r0];
    e1 = o.q_off[o.P + r1];
}

// Wave tier: one wave per txn with <= 64 raw entries; also routes the larger txns (sizes pass).
template <bool WRITE>
__global__ __launch_bounds__(BLOCK) void k_rd_build_wave(uint32_t n, Out o)
{
    __shared__ uint32_t slot[WAVES][64];
    const uint32_t wave = threadIdx.x >> 6, lane = lane_id();
    const uint32_t t = blockIdx.x * WAVES + wave;
    if (t >= n) return;
    uint64_t e0, e1;
    txn_range(o, t, e0, e1);
    const uint64_t m = e1 - e0;
    if (m > WAVE_E) {
        if (!WRITE && lane == 0) {
            if (m <= BLOCK_E) o.blk_list[atomicAdd((unsigned long long *)&o.gstat[0], 1ull)] = t;
            else {
                o.glb_list[atomicAdd((unsigned long long *)&o.gstat[1], 1ull)] = t;
                uint64_t n2 = 1; while (n2 < m) n2 <<= 1;
                atomicAdd((unsigned long long *)&o.gstat[2], 2 * n2);
            }
        }
        return;
    }
    if (m == 0) {
        if (!WRITE && lane == 0) { o.rd_cnt[t] = 0; o.u_cnt[t] = 0; o.a_cnt[t] = 0; }
        return;
    }
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    uint64_t x = lane < m ? o.ent[e0 + lane] : ~0ull;
    x = bitonic_reg(x);
    const uint64_t prev = shfl_up(x, 1);
    const bool valid = lane < m && (lane == 0 || x != prev);          // dedupe identical (range, txn)
    const uint64_t vb = __ballot(valid);
    const uint32_t M = (uint32_t)__popcll(vb);
    const uint32_t pos = (uint32_t)__popcll(vb & lt);
    const uint32_t rid = (uint32_t)(x >> 32), rk = (uint32_t)x;
    // RangeDeps.txnIds: distinct ranks, ascending; each entry's index into them
    uint64_t y = valid ? (((uint64_t)rk << 6) | pos) : ~0ull;
    y = bitonic_reg(y);
    const uint64_t yprev = shfl_up(y, 1);
    const bool yin = lane < M;
    const bool ynew = yin && (lane == 0 || (y >> 6) != (yprev >> 6));
    const uint64_t nb = __ballot(ynew);
    const uint32_t U = (uint32_t)__popcll(nb);
    const uint32_t uidx = (uint32_t)__popcll(nb & lt) + (ynew ? 1u : 0u) - 1u;
    // ranges: a new group where the range id changes
    const bool rnew = valid && (lane == 0 || (uint32_t)(prev >> 32) != rid);
    const uint64_t rb = __ballot(rnew);
    const uint32_t Rd = (uint32_t)__popcll(rb);
    if (!WRITE) {
        if (lane == 0) { o.rd_cnt[t] = Rd; o.u_cnt[t] = U; o.a_cnt[t] = (uint64_t)Rd + M; }
        return;
    }
    if (yin) slot[wave][(uint32_t)(y & 63u)] = uidx;
    if (ynew) o.dep_txn[o.u_off[t] + uidx] = o.txn_of_rank[(uint32_t)(y >> 6)];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const uint64_t abase = o.arena_off[t];
    const uint32_t g = (uint32_t)__popcll(rb & lt) + (rnew ? 1u : 0u) - 1u;
    // rangesToTxnIds header: group g - 1 ends where group g starts; the last group ends at Rd + M
    if (valid) {
        o.arena[abase + Rd + pos] = (int32_t)slot[wave][pos];
        if (rnew) {
            o.range_id[o.rd_off[t] + g] = rid;
            if (g > 0) o.arena[abase + g - 1] = (int32_t)(Rd + pos);
        }
    }
    if (lane == 0) o.arena[abase + Rd - 1] = (int32_t)(Rd + M);
}

// block-wide exclusive scan of per-thread counts (256 threads)
__device__ __forceinline__ uint32_t block_excl(uint32_t v, uint32_t *lds, uint32_t &total)
{
    return block_exclusive(v, OpAdd<uint32_t>(), lds, total);
}

// One workgroup per txn over buffers A, B of n2 >= m elements (LDS for the block tier, global scratch beyond).
template <bool WRITE>
__device__ void build_block(const Out &o, uint32_t t, uint64_t e0, uint32_t m, uint64_t *A, uint64_t *B, uint32_t *red)
{
    const uint32_t tid = threadIdx.x;
    uint32_t n2 = 64;
    while (n2 < m) n2 <<= 1;
    for (uint32_t i = tid; i < n2; i += BLOCK) A[i] = i < m ? o.ent[e0 + i] : ~0ull;
    __syncthreads();
    block_bitonic(A, n2);
    // dedupe + compact into B; each thread owns a contiguous slice of n2 / BLOCK (or 1) elements
    const uint32_t per = (n2 + BLOCK - 1) / BLOCK;
    const uint32_t lo = tid * per, hi = min(lo + per, n2);
    uint32_t c = 0;
    for (uint32_t i = lo; i < hi; ++i) c += (i < m && (i == 0 || A[i] != A[i - 1])) ? 1u : 0u;
    uint32_t M;
    uint32_t p = block_excl(c, red, M);
    for (uint32_t i = lo; i < hi; ++i)
        if (i < m && (i == 0 || A[i] != A[i - 1])) B[p++] = A[i];
    __syncthreads();
    uint32_t n2m = 64;
    while (n2m < M) n2m <<= 1;
    for (uint32_t i = tid; i < n2m; i += BLOCK) A[i] = i < M ? (((uint64_t)(uint32_t)B[i] << 32) | i) : ~0ull;
    __syncthreads();
    block_bitonic(A, n2m);
    // distinct TxnId ranks -> index; B[e] becomes (range id << 32 | index)
    const uint32_t per2 = (n2m + BLOCK - 1) / BLOCK;
    const uint32_t lo2 = tid * per2, hi2 = min(lo2 + per2, n2m);
    c = 0;
    for (uint32_t i = lo2; i < hi2; ++i) c += (i < M && (i == 0 || (A[i] >> 32) != (A[i - 1] >> 32))) ? 1u : 0u;
    uint32_t U;
    uint32_t u = block_excl(c, red, U);
    if (WRITE) {
        const uint64_t ub = o.u_off[t];
        for (uint32_t i = lo2; i < hi2; ++i) {
            if (i >= M) break;
            const bool nw = i == 0 || (A[i] >> 32) != (A[i - 1] >> 32);
            if (nw) { o.dep_txn[ub + u] = o.txn_of_rank[(uint32_t)(A[i] >> 32)]; ++u; }
            const uint32_t e = (uint32_t)A[i];
            B[e] = (B[e] & 0xFFFFFFFF00000000ull) | (u - 1);
        }
    }
    __syncthreads();
    // range groups over B[0, M)
    const uint32_t per3 = (M + BLOCK - 1) / BLOCK;
    const uint32_t lo3 = min(tid * per3, M), hi3 = min(lo3 + per3, M);
    c = 0;
    for (uint32_t e = lo3; e < hi3; ++e) c += (e == 0 || (B[e] >> 32) != (B[e - 1] >> 32)) ? 1u : 0u;
    uint32_t Rd;
    uint32_t g = block_excl(c, red, Rd);
    if (!WRITE) {
        if (tid == 0) { o.rd_cnt[t] = Rd; o.u_cnt[t] = U; o.a_cnt[t] = (uint64_t)Rd + M; }
        return;
    }
    const uint64_t abase = o.arena_off[t], rbase = o.rd_off[t];
    for (uint32_t e = lo3; e < hi3; ++e) {
        const uint32_t rid = (uint32_t)(B[e] >> 32);
        const bool nw = e == 0 || (B[e - 1] >> 32) != rid;
        if (nw) { o.range_id[rbase + g] = rid; ++g; }
        o.arena[abase + Rd + e] = (int32_t)(uint32_t)B[e];
        const bool last = e + 1 == M || (uint32_t)(B[e + 1] >> 32) != rid;
        if (last) o.arena[abase + g - 1] = (int32_t)(Rd + e + 1);
    }
}

template <bool WRITE>
__global__ __launch_bounds__(BLOCK) void k_rd_build_block(Out o)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    const uint32_t t = o.blk_list[blockIdx.x];
    uint64_t e0, e1;
    txn_range(o, t, e0, e1);
    // all LDS dynamic (no static __shared__ ahead of it: the base stays 16-B aligned, Guideline 17)
    build_block<WRITE>(o, t, e0, (uint32_t)(e1 - e0), lds, lds + BLOCK_E, reinterpret_cast<uint32_t *>(lds + 2 * BLOCK_E));
}

template <bool WRITE>
__global__ __launch_bounds__(BLOCK) void k_rd_build_global(Out o)
{
    const uint32_t t = o.glb_list[blockIdx.x];
    uint64_t e0, e1;
    txn_range(o, t, e0, e1);
    uint64_t *A = o.scratch + o.glb_off[blockIdx.x];
    uint32_t n2 = 64;
    while (n2 < e1 - e0) n2 <<= 1;
    __shared__ uint32_t red[WAVES];
    build_block<WRITE>(o, t, e0, (uint32_t)(e1 - e0), A, A + n2, red);
}

__global__ __launch_bounds__(BLOCK) void k_rd_glb_sizes(uint32_t ng, const uint32_t *__restrict__ glb_list, Out o,
                                                        uint64_t *__restrict__ sz)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= ng) return;
    uint64_t e0, e1;
    txn_range(o, glb_list[i], e0, e1);
    uint64_t n2 = 64;
    while (n2 < e1 - e0) n2 <<= 1;
    sz[i] = 2 * n2;
}

}  // namespace rd

using namespace rd;

static void rd_check_errors(uint64_t errs)
{
    if (errs & ERR_DOMAIN) fail(ACC_E_ARG, "a range-domain txn lists keys or a key-domain txn lists ranges (TxnId.domain())");
    if (errs & ERR_RANGE_EMPTY) fail(ACC_E_ARG, "range start must be below its end (Range: start >= end)");
    if (errs & ERR_RANGES_UNSORTED) fail(ACC_E_ARG, "ranges of a txn must be sorted and deoverlapped (Ranges.ofSortedAndDeoverlapped)");
    if (errs & ERR_RNG_OFF) fail(ACC_E_ARG, "rng_off must be non-decreasing");
}

void rangedeps_batch(acc_ctx *ctx, const acc_range_batch_in *in, acc_rangedeps_view *view)
{
    if (!in || !view) fail(ACC_E_ARG, "null argument");
    if (in->mem != ACC_MEM_HOST && in->mem != ACC_MEM_DEVICE) fail(ACC_E_ARG, "mem must be ACC_MEM_HOST or ACC_MEM_DEVICE");
    if (in->end_inclusive > 1) fail(ACC_E_ARG, "end_inclusive must be 0 (StartInclusive) or 1 (EndInclusive)");
    const uint32_t n = in->n_txn;
    const size_t P = (size_t)in->n_pairs, R = (size_t)in->n_ranges;
    if (P + R >= 0xFFFFFFFFull) fail(ACC_E_ARG, "n_pairs + n_ranges must be < 2^32");
    hipStream_t st = ctx->stream;
    ctx->rd_valid = false;
    const uint32_t Q = (uint32_t)(P + R);

    uint64_t *arena_off = ctx->get<uint64_t>("rd_arena_off", (size_t)n + 1);
    uint64_t *rd_off = ctx->get<uint64_t>("rd_rd_off", (size_t)n + 1);
    uint64_t *u_off = ctx->get<uint64_t>("rd_u_off", (size_t)n + 1);
    auto empty_result = [&]() {
        ACC_HIP(hipMemsetAsync(arena_off, 0, ((size_t)n + 1) * 8, st));
        ACC_HIP(hipMemsetAsync(rd_off, 0, ((size_t)n + 1) * 8, st));
        ACC_HIP(hipMemsetAsync(u_off, 0, ((size_t)n + 1) * 8, st));
        *view = acc_rangedeps_view{ n, 0, 0, 0, 0, 0, ctx->get<uint64_t>("rd_dict_s", 1), ctx->get<uint64_t>("rd_dict_e", 1),
                                    arena_off, ctx->get<int32_t>("rd_arena", 1), rd_off, ctx->get<uint32_t>("rd_range_id", 1),
                                    u_off, ctx->get<uint32_t>("rd_dep_txn", 1) };
        ctx->rd_view = *view;
        ctx->rd_valid = true;
        ctx->sync();
    };
    if (n == 0) { empty_result(); return; }

    const uint32_t *key_off = stage_in(ctx, "in_key_off", in->key_off, (size_t)n + 1, in->mem);
    const uint32_t *rng_off = stage_in(ctx, "in_rng_off", in->rng_off, (size_t)n + 1, in->mem);
    const uint64_t *tm = stage_in(ctx, "in_tm", in->txn_id.msb, n, in->mem);
    const uint64_t *tl = stage_in(ctx, "in_tl", in->txn_id.lsb, n, in->mem);
    const int32_t *tn = stage_in(ctx, "in_tn", in->txn_id.node, n, in->mem);
    const uint64_t *em = stage_in(ctx, "in_em", in->execute_at.msb, n, in->mem);
    const uint64_t *el = stage_in(ctx, "in_el", in->execute_at.lsb, n, in->mem);
    const int32_t *en = stage_in(ctx, "in_en", in->execute_at.node, n, in->mem);
    const uint8_t *status = stage_in(ctx, "in_status", in->status, n, in->mem);
    const uint64_t *key_code = stage_in(ctx, "in_key_code", in->key_code, P, in->mem);
    const uint64_t *rs = stage_in(ctx, "in_rng_start", in->rng_start, R, in->mem);
    const uint64_t *re = stage_in(ctx, "in_rng_end", in->rng_end, R, in->mem);

    // ---- 1. prep + dictionary (also validates keys, statuses, kinds, TxnId order and uniqueness)
    uint64_t *g = ctx->get<uint64_t>("g", 8);
    uint32_t *owner = ctx->get<uint32_t>("owner", P);
    Dictionary dict;
    prep_dictionary(ctx, n, P, tm, tl, tn, em, el, en, status, key_off, key_code, owner, g, dict);

    // reference codes for the masks (first range bound / first query bound)
    uint64_t ref[2] = { 0, 0 };
    {
        uint32_t last_r = 0;
        ACC_HIP(hipMemcpyAsync(ctx->pinned + 8, rng_off + n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        if (R) {
            ACC_HIP(hipMemcpyAsync(ctx->pinned + 9, rs, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
            ACC_HIP(hipMemcpyAsync(ctx->pinned + 10, re, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        }
        if (P) ACC_HIP(hipMemcpyAsync(ctx->pinned + 11, key_code, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        ctx->sync();
        memcpy(&last_r, ctx->pinned + 8, sizeof(uint32_t));
        if (last_r != R) fail(ACC_E_ARG, "rng_off[n_txn] must equal n_ranges");
        ref[0] = R ? ctx->pinned[9] : 0;
        ref[1] = R ? ctx->pinned[10] : 0;
    }
    const uint64_t ref_lo = P ? ctx->pinned[11] : ref[0];
    uint64_t *rg = ctx->get<uint64_t>("rd_g", 8);
    ACC_HIP(hipMemsetAsync(rg, 0, 8 * sizeof(uint64_t), st));
    uint32_t *rowner = ctx->get<uint32_t>("rd_rowner", R);
    uint32_t *eflag = ctx->get<uint32_t>("rd_eflag", R);
    uint32_t *eidx = ctx->get<uint32_t>("rd_eidx", R + 1);
    launch(ctx, "rd_prep", k_rd_prep, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, tl, status, key_off, key_code, rng_off, rs,
           re, ref[0], ref[1], ref_lo, rowner, eflag, rg);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, eflag, eidx, R, true, eidx + R);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, rg, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    {
        uint32_t *pn = reinterpret_cast<uint32_t *>(ctx->pinned + 4);
        if (R) ACC_HIP(hipMemcpyAsync(pn, eidx + R, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        else *pn = 0;
    }
    ctx->sync();
    uint64_t hm[4];
    memcpy(hm, ctx->pinned, sizeof hm);
    rd_check_errors(hm[3]);
    const uint32_t NE = R ? *reinterpret_cast<uint32_t *>(ctx->pinned + 4) : 0;
    const uint32_t *rank = dict.rank;

    // ---- 2. range-command entries, stored-range dictionary, class order
    const Runs rs_plan = make_runs(hm[0]), re_plan = make_runs(hm[1]);
    uint64_t *e_s = ctx->get<uint64_t>("rd_e_s", NE), *e_e = ctx->get<uint64_t>("rd_e_e", NE);
    uint32_t *e_rank = ctx->get<uint32_t>("rd_e_rank", NE);
    uint8_t *e_kind = ctx->get<uint8_t>("rd_e_kind", NE);
    uint64_t *dkey = ctx->get<uint64_t>("rd_dkey", NE), *ekey = ctx->get<uint64_t>("rd_ekey", NE);
    const bool split = rs_plan.bits + re_plan.bits > 64;
    launch(ctx, "rd_entries", k_rd_entries, dim3(grid_for(R, BLOCK)), dim3(BLOCK), 0, (uint32_t)R, n, (const uint32_t *)eflag,
           (const uint32_t *)eidx, (const uint32_t *)rowner, rs, re, rank, tl, rs_plan, re_plan, re_plan.bits, split ? 1 : 0,
           e_s, e_e, e_rank, e_kind, dkey, ekey);
    Sorted ds;
    if (!split) {
        ds = radix_sort(ctx, "rs_rd_dict", dkey, nullptr, NE, rs_plan.bits + re_plan.bits);
    } else {
        // two-key LSD: stable sort by end, then by start
        Sorted by_e = radix_sort(ctx, "rs_rd_e", ekey, nullptr, NE, re_plan.bits);
        uint64_t *dk3 = ctx->get<uint64_t>("rd_dkey3", NE);
        launch(ctx, "rd_permute", k_permute_u64, dim3(grid_for(NE, BLOCK)), dim3(BLOCK), 0, (size_t)NE,
               (const uint32_t *)by_e.vals, (const uint64_t *)dkey, dk3);
        ds = radix_sort(ctx, "rs_rd_dict", dk3, by_e.vals, NE, rs_plan.bits);
    }
    uint32_t *dflag = ctx->get<uint32_t>("rd_dflag", NE), *dincl = ctx->get<uint32_t>("rd_dincl", NE + 1);
    launch(ctx, "rd_dict_flags", k_rd_dict_flags, dim3(grid_for(NE, BLOCK)), dim3(BLOCK), 0, NE, (const uint32_t *)ds.vals,
           (const uint64_t *)e_s, (const uint64_t *)e_e, dflag);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, dflag, dincl, NE, false, dincl + NE);
    uint32_t *rid_of = ctx->get<uint32_t>("rd_rid_of", NE);
    uint64_t *dict_s = ctx->get<uint64_t>("rd_dict_s", NE), *dict_e = ctx->get<uint64_t>("rd_dict_e", NE);
    uint64_t *ckey = ctx->get<uint64_t>("rd_ckey", NE);
    uint32_t *cls = ctx->get<uint32_t>("rd_cls", 2 * (NCLS + 1));
    uint32_t *cls_hist = cls, *class_off = cls + (NCLS + 1);
    ACC_HIP(hipMemsetAsync(cls_hist, 0, (NCLS + 1) * sizeof(uint32_t), st));
    const bool csplit = rs_plan.bits + 6 > 64;
    launch(ctx, "rd_dict_write", k_rd_dict_write, dim3(grid_for(NE, BLOCK)), dim3(BLOCK), 0, NE, (const uint32_t *)ds.vals,
           (const uint32_t *)dflag, (const uint32_t *)dincl, (const uint64_t *)e_s, (const uint64_t *)e_e, rid_of, dict_s,
           dict_e, rs_plan, rs_plan.bits, csplit ? 1 : 0, ckey, cls_hist);
    launch(ctx, "rd_class_off", k_rd_class_off, dim3(1), dim3(64), 0, (const uint32_t *)cls_hist, class_off);
    Sorted cs;
    if (!csplit) {
        cs = radix_sort(ctx, "rs_rd_cls", ckey, nullptr, NE, rs_plan.bits + 6);
    } else {
        // > 58 start bits: stable sort by start, then by class (the class key alone is in ckey's low bits)
        uint64_t *sk = ctx->get<uint64_t>("rd_skey", NE);
        launch(ctx, "rd_skey", k_pext_u64, dim3(grid_for(NE, BLOCK)), dim3(BLOCK), 0, (size_t)NE, (const uint64_t *)e_s,
               rs_plan, sk);
        Sorted by_s = radix_sort(ctx, "rs_rd_s", sk, nullptr, NE, rs_plan.bits);
        uint64_t *ck2 = ctx->get<uint64_t>("rd_ckey2", NE);
        launch(ctx, "rd_permute", k_permute_u64, dim3(grid_for(NE, BLOCK)), dim3(BLOCK), 0, (size_t)NE,
               (const uint32_t *)by_s.vals, (const uint64_t *)ckey, ck2);
        cs = radix_sort(ctx, "rs_rd_cls", ck2, by_s.vals, NE, 6);
    }
    uint64_t *cs_s = ctx->get<uint64_t>("rd_cs_s", NE), *cs_e = ctx->get<uint64_t>("rd_cs_e", NE);
    uint2 *cs_info = ctx->get<uint2>("rd_cs_info", NE);
    uint8_t *cs_kind = ctx->get<uint8_t>("rd_cs_kind", NE);
    launch(ctx, "rd_class_cols", k_rd_class_cols, dim3(grid_for(NE, BLOCK)), dim3(BLOCK), 0, NE, (const uint32_t *)cs.vals,
           (const uint64_t *)e_s, (const uint64_t *)e_e, (const uint32_t *)e_rank, (const uint8_t *)e_kind,
           (const uint32_t *)rid_of, cs_s, cs_e, cs_info, cs_kind);

    // ---- 3. queries sorted by low bound; stabbing count -> offsets -> emit
    const Runs q_plan = make_runs(hm[2]);
    uint64_t *qkey = ctx->get<uint64_t>("rd_qkey", Q);
    launch(ctx, "rd_query_keys", k_rd_query_keys, dim3(grid_for(Q, BLOCK)), dim3(BLOCK), 0, (uint32_t)P, (uint32_t)R, key_code,
           rs, q_plan, qkey);
    Sorted qs = radix_sort(ctx, "rs_rd_q", qkey, nullptr, Q, q_plan.bits);
    View v;
    v.n = n; v.P = (uint32_t)P; v.R = (uint32_t)R; v.Q = Q; v.end_inclusive = (int)in->end_inclusive;
    v.qperm = qs.vals; v.key_code = key_code; v.owner = owner; v.rs = rs; v.re = re; v.rowner = rowner; v.rank = rank;
    v.tl = tl; v.cs_s = cs_s; v.cs_e = cs_e; v.cs_info = cs_info; v.cs_kind = cs_kind; v.class_off = class_off;
    uint32_t *cnt = ctx->get<uint32_t>("rd_cnt", Q);
    uint64_t *cnt64 = ctx->get<uint64_t>("rd_cnt64", Q);
    uint64_t *q_off = ctx->get<uint64_t>("rd_q_off", (size_t)Q + 1);
    launch(ctx, "rd_stab_count", k_rd_stab<false>, dim3(grid_for(Q, BLOCK)), dim3(BLOCK), 0, v, cnt,
           (const uint64_t *)nullptr, (uint64_t *)nullptr);
    launch(ctx, "rd_widen", k_widen_u32, dim3(grid_for(Q, BLOCK)), dim3(BLOCK), 0, (size_t)Q, (const uint32_t *)cnt, cnt64);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, cnt64, q_off, Q, true, q_off + Q);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, q_off + Q, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t E = Q ? ctx->pinned[0] : 0;
    uint64_t *ent = ctx->get<uint64_t>("rd_ent", E);
    launch(ctx, "rd_stab_emit", k_rd_stab<true>, dim3(grid_for(Q, BLOCK)), dim3(BLOCK), 0, v, cnt, (const uint64_t *)q_off, ent);

    // ---- 4. per-txn RangeDeps: sizes, offsets, writes
    Out o{};
    o.key_off = key_off; o.rng_off = rng_off; o.P = (uint32_t)P; o.q_off = q_off; o.ent = ent;
    o.txn_of_rank = dict.txn_of_rank;
    o.rd_cnt = ctx->get<uint32_t>("rd_rd_cnt", n);
    o.u_cnt = ctx->get<uint32_t>("rd_u_cnt", n);
    o.a_cnt = ctx->get<uint64_t>("rd_a_cnt", n);
    o.blk_list = ctx->get<uint32_t>("rd_blk_list", n);
    o.glb_list = ctx->get<uint32_t>("rd_glb_list", n);
    o.gstat = ctx->get<uint64_t>("rd_gstat", 4);
    ACC_HIP(hipMemsetAsync(o.gstat, 0, 4 * sizeof(uint64_t), st));
    const unsigned gw = (n + WAVES - 1) / WAVES;
    launch(ctx, "rd_build_wave_sizes", k_rd_build_wave<false>, dim3(gw), dim3(BLOCK), 0, n, o);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, o.gstat, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t nblk = ctx->pinned[0], nglb = ctx->pinned[1], glb_elems = ctx->pinned[2];
    const size_t blk_lds = 2 * (size_t)BLOCK_E * sizeof(uint64_t) + 64;
    if (nblk) {
        ACC_HIP(hipFuncSetAttribute((const void *)k_rd_build_block<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)blk_lds));
        ACC_HIP(hipFuncSetAttribute((const void *)k_rd_build_block<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)blk_lds));
        launch(ctx, "rd_build_block_sizes", k_rd_build_block<false>, dim3((unsigned)nblk), dim3(BLOCK), blk_lds, o);
    }
    if (nglb) {
        uint64_t *gsz = ctx->get<uint64_t>("rd_glb_sz", nglb);
        uint64_t *goff = ctx->get<uint64_t>("rd_glb_off", nglb + 1);
        launch(ctx, "rd_glb_sizes", k_rd_glb_sizes, dim3(grid_for(nglb, BLOCK)), dim3(BLOCK), 0, (uint32_t)nglb,
               (const uint32_t *)o.glb_list, o, gsz);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, gsz, goff, nglb, true, goff + nglb);
        o.glb_off = goff;
        o.scratch = ctx->get<uint64_t>("rd_glb_scratch", glb_elems);
        launch(ctx, "rd_build_global_sizes", k_rd_build_global<false>, dim3((unsigned)nglb), dim3(BLOCK), 0, o);
    }
    uint64_t *rd_cnt64 = ctx->get<uint64_t>("rd_rd_cnt64", n), *u_cnt64 = ctx->get<uint64_t>("rd_u_cnt64", n);
    launch(ctx, "rd_widen", k_widen_u32, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, (size_t)n, (const uint32_t *)o.rd_cnt, rd_cnt64);
    launch(ctx, "rd_widen", k_widen_u32, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, (size_t)n, (const uint32_t *)o.u_cnt, u_cnt64);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, o.a_cnt, arena_off, n, true, arena_off + n);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, rd_cnt64, rd_off, n, true, rd_off + n);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, u_cnt64, u_off, n, true, u_off + n);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, arena_off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, rd_off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 2, u_off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 3, dincl + NE, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t tot_arena = ctx->pinned[0], tot_rd = ctx->pinned[1], tot_u = ctx->pinned[2];
    const uint32_t n_dict = NE ? *reinterpret_cast<uint32_t *>(ctx->pinned + 3) : 0;
    o.arena_off = arena_off; o.rd_off = rd_off; o.u_off = u_off;
    o.arena = ctx->get<int32_t>("rd_arena", tot_arena);
    o.range_id = ctx->get<uint32_t>("rd_range_id", tot_rd);
    o.dep_txn = ctx->get<uint32_t>("rd_dep_txn", tot_u);
    launch(ctx, "rd_build_wave", k_rd_build_wave<true>, dim3(gw), dim3(BLOCK), 0, n, o);
    if (nblk) launch(ctx, "rd_build_block", k_rd_build_block<true>, dim3((unsigned)nblk), dim3(BLOCK), blk_lds, o);
    if (nglb) launch(ctx, "rd_build_global", k_rd_build_global<true>, dim3((unsigned)nglb), dim3(BLOCK), 0, o);
    ctx->stat("rangedeps.entries", NE);
    ctx->stat("rangedeps.stored_ranges", n_dict);
    ctx->stat("rangedeps.queries", Q);
    ctx->stat("rangedeps.raw_entries", E);
    ctx->stat("rangedeps.block_txns", nblk);
    ctx->stat("rangedeps.global_txns", nglb);
    ctx->sync();
    *view = acc_rangedeps_view{ n, n_dict, tot_arena, tot_rd, tot_u, tot_arena - tot_rd, dict_s, dict_e, arena_off, o.arena,
                                rd_off, o.range_id, u_off, o.dep_txn };
    ctx->rd_view = *view;
    ctx->rd_valid = true;
}

}  // namespace acc
