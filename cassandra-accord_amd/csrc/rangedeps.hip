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

constexpr int RD_TS = 16;         // chunks of BLOCK txns per workgroup in the per-txn passes with global counters
constexpr int NCLS = 33;          // width classes 0..32 (4^32 = 2^64 covers every u64 width)
#ifndef ACC_RD_TILE
#define ACC_RD_TILE 256
#endif
constexpr int TILE = ACC_RD_TILE;   // entries per LDS tile in the stabbing pass (LDS per block sets the occupancy)
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
    uint64_t ms = 0, me = 0, ml = 0, errs = 0;
    // RD_TS chunks of BLOCK txns per workgroup: one OR per word and workgroup into g (its 4 words share one line)
    for (int r = 0; r < RD_TS; ++r) {
    const uint32_t t = (blockIdx.x * RD_TS + (uint32_t)r) * BLOCK + threadIdx.x;
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
            for (uint32_t jb = k0; jb < k1; jb += 8) {   // eight key loads in flight
                uint64_t kc[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) kc[u] = jb + u < k1 ? key_code[jb + u] ^ ref_lo : 0ull;
#pragma unroll
                for (int u = 0; u < 8; ++u) ml |= kc[u];
            }
    }
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
                                                      const uint4 *__restrict__ tinfo, const uint64_t *__restrict__ tl,
                                                      Runs rs_plan, Runs re_plan, int e_bits, int split, uint4 *__restrict__ erec,
                                                      uint64_t *__restrict__ dkey, uint64_t *__restrict__ ekey)
{
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= R || !eflag[j]) return;
    const uint32_t i = eidx[j], t = rowner[j];
    const uint64_t s = rs[j], e = re[j];
    // the entry's 32-B record: start, end | TxnId position, kind, range id (k_rd_dict_write) — the permuted reads of
    // the dictionary and class passes take one record per entry instead of a line per column
    erec[2 * (size_t)i] = make_uint4((uint32_t)s, (uint32_t)(s >> 32), (uint32_t)e, (uint32_t)(e >> 32));
    erec[2 * (size_t)i + 1] = make_uint4(tinfo[t].y, (uint32_t)((tl[t] >> 1) & 7u), 0u, 0u);
    const uint64_t sc = pext_runs(s, rs_plan), ec = pext_runs(e, re_plan);
    if (split) { dkey[i] = sc; ekey[i] = ec; }      // two-key LSD: end first, then start (stable)
    else dkey[i] = (sc << e_bits) | ec;
}

// rid per (start, end)-sorted position; dictionary arrays
__global__ __launch_bounds__(BLOCK) void k_rd_dict_flags(uint32_t ne, const uint32_t *__restrict__ perm,
                                                         const uint4 *__restrict__ erec, uint32_t *__restrict__ flag)
{
    const uint32_t p = blockIdx.x * BLOCK + threadIdx.x;
    if (p >= ne) return;
    uint32_t f = 1;
    if (p > 0) {
        const uint4 a = erec[2 * (size_t)perm[p]], b = erec[2 * (size_t)perm[p - 1]];
        f = a.x != b.x || a.y != b.y || a.z != b.z || a.w != b.w;
    }
    flag[p] = f;
}

__global__ __launch_bounds__(BLOCK) void k_rd_dict_write(uint32_t ne, const uint32_t *__restrict__ perm,
                                                         const uint32_t *__restrict__ flag, const uint32_t *__restrict__ incl,
                                                         uint4 *__restrict__ erec, uint64_t *__restrict__ dict_s,
                                                         uint64_t *__restrict__ dict_e, uint64_t *__restrict__ ckey,
                                                         uint32_t *__restrict__ cls_hist)
{
    __shared__ uint32_t h[NCLS];
    if (threadIdx.x < NCLS) h[threadIdx.x] = 0;
    __syncthreads();
    // RD_TS chunks of BLOCK entries per workgroup: one global add per class and workgroup (the 33 counters share two lines)
    for (int r = 0; r < RD_TS; ++r) {
    const uint32_t p = (blockIdx.x * RD_TS + (uint32_t)r) * BLOCK + threadIdx.x;
    uint32_t c = 0xFFu;
    if (p < ne) {
        const uint32_t i = perm[p], rid = incl[p] - 1;
        const uint4 a = erec[2 * (size_t)i];
        const uint64_t es = ((uint64_t)a.y << 32) | a.x, ee = ((uint64_t)a.w << 32) | a.z;
        reinterpret_cast<uint32_t *>(erec + 2 * (size_t)i + 1)[2] = rid;   // the entry's range id
        if (flag[p]) { dict_s[rid] = es; dict_e[rid] = ee; }
        c = width_class(es, ee);
        ckey[p] = c;   // in (start, end) order: one stable pass by class gives the (class, start) order
    }
    // LDS histogram, one add per distinct class of a wave (per-thread atomics on a few hot words serialise); one global
    // atomic per class and block
    {
        const uint32_t lane = lane_id();
        uint64_t rem = __ballot(c != 0xFFu);
        while (rem) {
            const uint32_t leader = (uint32_t)__builtin_ctzll(rem);
            const uint32_t c0 = (uint32_t)__shfl((int)c, (int)leader, 64);
            const uint64_t m = __ballot(c == c0) & rem;
            if (lane == leader) atomicAdd(&h[c0], (uint32_t)__popcll(m));
            rem &= ~m;
        }
    }
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
                                                         const uint4 *__restrict__ erec, uint64_t *__restrict__ cs_s,
                                                         uint64_t *__restrict__ cs_e, uint2 *__restrict__ cs_info,
                                                         uint8_t *__restrict__ cs_kind)
{
    const uint32_t p = blockIdx.x * BLOCK + threadIdx.x;
    if (p >= ne) return;
    const uint32_t i = perm[p];
    const uint4 a = erec[2 * (size_t)i], b = erec[2 * (size_t)i + 1];
    cs_s[p] = ((uint64_t)a.y << 32) | a.x;
    cs_e[p] = ((uint64_t)a.w << 32) | a.z;
    cs_info[p] = make_uint2(b.z, b.x);   // (range id, TxnId position)
    cs_kind[p] = (uint8_t)b.y;
}

// ---------------------------------------------------------------- txn columns

// isT[r] = 1 where r is the rank of a TxnId (the dictionary ranks every TxnId and executeAt of the batch)
__global__ __launch_bounds__(BLOCK) void k_rd_txnflag(uint32_t n, const uint32_t *__restrict__ rank, uint32_t *__restrict__ isT)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t < n) isT[rank[t]] = 1;
}

// Per txn {lim, tpos, witness mask, is range}: tpos = position of its TxnId among the batch's TxnIds (TxnId order),
// lim = number of TxnIds below its executeAt, so C.txnId < T.executeAt <=> tpos(C) < lim(T) (STARTED_BEFORE,
// InMemoryCommandStore.java:897-898). txn_of_tpos inverts tpos (identity for a batch given in TxnId order).
__global__ __launch_bounds__(BLOCK) void k_rd_txncols(uint32_t n, const uint32_t *__restrict__ rank, const uint32_t *__restrict__ tcnt,
                                                      const uint64_t *__restrict__ tl, uint4 *__restrict__ tinfo,
                                                      uint32_t *__restrict__ txn_of_tpos)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= n) return;
    const uint32_t tpos = tcnt[rank[t]], lim = tcnt[rank[n + t]];
    tinfo[t] = make_uint4(lim, tpos, witnesses((uint32_t)(tl[t] >> 1) & 7u), (uint32_t)(tl[t] & 1u));
    txn_of_tpos[tpos] = t;
}

// ---------------------------------------------------------------- queries

// query q: a key of a key txn (q < P) or a range of a range txn (q >= P); [lo, hi] its bounds
struct QRec {
    uint64_t lo, hi;
    uint32_t lim, tpos;
    uint32_t flags;   // witness mask | is-range << 8
    uint32_t q;
};

__global__ __launch_bounds__(BLOCK) void k_rd_qrec(uint32_t P, uint32_t R, const uint64_t *__restrict__ key_code,
                                                   const uint32_t *__restrict__ owner, const uint64_t *__restrict__ rs,
                                                   const uint64_t *__restrict__ re, const uint32_t *__restrict__ rowner,
                                                   const uint4 *__restrict__ tinfo, Runs plan, QRec *__restrict__ rec,
                                                   uint64_t *__restrict__ qkey, uint32_t rbit, int ibits, int qdrop)
{
    const uint32_t q = blockIdx.x * BLOCK + threadIdx.x;
    if (q >= P + R) return;
    QRec r;
    uint32_t t;
    if (q < P) { r.lo = r.hi = key_code[q]; t = owner[q]; }
    else { r.lo = rs[q - P]; r.hi = re[q - P]; t = rowner[q - P]; }
    const uint4 ti = tinfo[t];
    r.lim = ti.x; r.tpos = ti.y; r.flags = ti.z | (ti.w << 8); r.q = q;
    rec[q] = r;
    // range queries after the key queries (rbit < 64): a range query scans its whole span, so mixing the two in one
    // wave would leave the key lanes idle behind it
    // ibits > 0: the query index packed under the key (a keys-only sort, 8 B per element moved instead of 12)
    // rbit < 62: range queries also grouped by width (2 bits under the range bit: widths below 2^4, 2^8, 2^12, beyond),
    // so a block's lanes scan spans of similar length — a wave waits for its widest lane
    uint64_t k = pext_runs(r.lo, plan);
    if (q >= P && rbit < 64) {
        if (rbit < 62) {
            const uint64_t w = r.hi - r.lo;
            const uint32_t g = min(3u, (63u - (uint32_t)__builtin_clzll(w | 1)) / 4u);
            k |= (4ull | g) << rbit;
        } else {
            k |= 1ull << rbit;
        }
    }
    // qdrop: the low key bits the sort leaves out (the stabbing blocks need neighbouring queries, not an exact order)
    qkey[q] = ibits ? ((k >> qdrop) << ibits) | q : k >> qdrop;
}

// The sorted runs' bounds bnd[0..4]: key queries [0, bnd[0] = P), range queries of width group g at [bnd[g], bnd[g + 1])
// (the group in the top 3 sorted key bits: 4 | g). One thread per group boundary, a binary search over the sorted keys.
__global__ void k_rd_qgroups(const uint64_t *__restrict__ keys, uint32_t P, uint32_t Q, int top_shift, int groups,
                             uint32_t *__restrict__ bnd)
{
    const uint32_t g = threadIdx.x;
    if (g > 4) return;
    uint32_t b = g == 0 ? P : Q;
    if (groups && g >= 1 && g <= 3) {
        uint32_t lo = P, hi = Q;   // first sorted position whose group field is >= 4 | g
        while (lo < hi) {
            const uint32_t mid = lo + ((hi - lo) >> 1);
            if ((keys[mid] >> top_shift) < (4u | g)) lo = mid + 1; else hi = mid;
        }
        b = lo;
    }
    bnd[g] = b;
}

// sorted records, and per block of BLOCK sorted queries (the stabbing blocks) the largest high bound
// Each sorted run (the key queries, then each width group of range queries) starts at a block boundary: no block mixes
// two runs, so no block's window spans the key space between them. Run g of c_g queries at padded position base_g
// (base_0 = Pp = P rounded up to a block, base_{g+1} = base_g + c_g rounded up); the gaps hold PAD records.
constexpr uint32_t QPAD = 1u << 31;
// perm: the sorted query indices, or (perm null) the low bits (imask) of the sorted packed keys pk
__global__ __launch_bounds__(BLOCK) void k_rd_qsort(uint32_t Qp, uint32_t P, uint32_t Pp, const uint32_t *__restrict__ bnd,
                                                    const uint32_t *__restrict__ perm,
                                                    const uint64_t *__restrict__ pk, uint64_t imask,
                                                    const QRec *__restrict__ rec, QRec *__restrict__ srec,
                                                    uint64_t *__restrict__ blo, uint64_t *__restrict__ bhi)
{
    __shared__ uint64_t wh[WAVES], wl[WAVES];
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    uint64_t h = 0, l = ~0ull;
    if (i < Qp) {
        uint32_t j = 0xFFFFFFFFu;   // sorted position of padded position i (none: PAD)
        if (i < P) {
            j = i;
        } else {
            uint32_t base = Pp;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const uint32_t c = bnd[g + 1] - bnd[g];
                if (i >= base && i < base + c) j = bnd[g] + (i - base);
                base += (c + BLOCK - 1) / BLOCK * BLOCK;
            }
        }
        if (j == 0xFFFFFFFFu) {
            QRec r{};
            r.flags = QPAD;
            srec[i] = r;
        } else {
            const QRec r = rec[perm ? perm[j] : (uint32_t)(pk[j] & imask)];
            srec[i] = r; h = r.hi; l = r.lo;
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t o = shfl_xor(h, d), p = shfl_xor(l, d);
        h = o > h ? o : h;
        l = p < l ? p : l;
    }
    if (lane_id() == 0) { wh[threadIdx.x >> 6] = h; wl[threadIdx.x >> 6] = l; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t m = 0, n = ~0ull;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) { m = wh[w] > m ? wh[w] : m; n = wl[w] < n ? wl[w] : n; }
        bhi[blockIdx.x] = m;
        blo[blockIdx.x] = n;
    }
}

// ---------------------------------------------------------------- stabbing

struct View {
    uint32_t Q;
    int end_inclusive;
    const QRec *srec;             // queries sorted by low bound
    const uint64_t *cs_s, *cs_e;  // entries by (class, start)
    const uint2 *cs_info;         // (range id, TxnId position)
    const uint8_t *cs_kind;
    const uint32_t *class_off;    // [NCLS + 1]
    const uint32_t *win;          // per block: b0[NCLS], b1[NCLS] (k_rd_stab_win)
    const uint64_t *blo, *bhi;    // per block: lowest low bound, highest high bound of its queries
    uint64_t *cursor;             // global output cursor
    uint64_t cap;                 // capacity of ent
    uint64_t *ent;                // (range id << 32 | TxnId position) per emitted pair
    ulonglong2 *q_out;            // per query (original index): (first entry, entries), one 16-B store per query
};

__device__ __forceinline__ uint32_t lower_bound_s(const uint64_t *a, uint32_t lo, uint32_t hi, uint64_t v)
{
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ uint32_t lower_bound_u32(const uint32_t *a, uint32_t lo, uint32_t hi, uint32_t v)
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

// 64-ary search by one wave: first index in [lo, hi) whose value is >= v (upper = false) or > v (upper = true).
// Each round is one parallel probe of 64 positions, so a 1M-entry class takes 4 dependent loads, not 20.
__device__ __forceinline__ uint32_t wave_search(const uint64_t *a, uint32_t lo, uint32_t hi, uint64_t v, bool upper)
{
    const uint32_t lane = lane_id();
    while (hi - lo > 64) {
        const uint32_t step = (hi - lo + 63) / 64;
        const uint32_t p = lo + lane * step;
        const bool below = p < hi && (upper ? a[p] <= v : a[p] < v);
        const uint32_t c = (uint32_t)__popcll(__ballot(below));
        if (c == 0) return lo;
        const uint32_t base = lo + (c - 1) * step;   // a[base] is below v, the answer is in (base, base + step]
        lo = base + 1;
        hi = min(base + step + 1, hi);
    }
    const uint32_t p = lo + lane;
    const bool below = p < hi && (upper ? a[p] <= v : a[p] < v);
    return lo + (uint32_t)__popcll(__ballot(below));
}

struct StabTile {
    uint64_t s[TILE], e[TILE];
    uint32_t s32[TILE], e32[TILE];  // flat tile, rel: bounds - rbase (ends clamped to 2^32 - 1)
    uint2 info[TILE];
    uint8_t kind[TILE];
    uint64_t rbase;
    uint32_t rel;                  // flat tile: the block's window spans less than 2^32 - 1 above rbase
    uint32_t b0[NCLS], b1[NCLS];   // the block's window per width class
    uint32_t pre[NCLS + 1];        // flat tile: class c at [pre[c], pre[c + 1])
    uint32_t red[WAVES];
    uint64_t base;
};

// One pass over the block's windows: EMIT = false counts this query's pairs, EMIT = true writes them at out. The
// (class, tile) sequence is software-pipelined: the next tile's entries are loaded into registers while the current
// one is scanned from LDS, so a block pays one memory latency per pass instead of one per tile.
constexpr int ST_PT = TILE / BLOCK;   // tile entries per thread
static_assert(TILE >= BLOCK && TILE % BLOCK == 0, "a tile is whole rounds of the block");

struct StabRegs {
    uint64_t s[ST_PT], e[ST_PT];
    uint2 info[ST_PT];
    uint32_t kind[ST_PT];
};

__device__ __forceinline__ void stab_load(const View &v, StabRegs &g, uint32_t base, uint32_t len)
{
#pragma unroll
    for (int u = 0; u < ST_PT; ++u) {
        const uint32_t k = threadIdx.x + (uint32_t)u * BLOCK;
        if (k < len) {
            g.s[u] = v.cs_s[base + k];
            g.e[u] = v.cs_e[base + k];
            g.info[u] = v.cs_info[base + k];
            g.kind[u] = v.cs_kind[base + k];
        }
    }
}

// next non-empty (class, tile) after (c, base) (c = NCLS: none)
__device__ __forceinline__ void stab_next(const StabTile &T, uint32_t &c, uint32_t &base)
{
    base += TILE;
    if (c < (uint32_t)NCLS && base < T.b1[c]) return;
    for (++c; c < (uint32_t)NCLS; ++c)
        if (T.b0[c] < T.b1[c]) { base = T.b0[c]; return; }
}

// REL: the probes on 32-bit offsets above the block's rbase (as stab_flat_rel)
template <bool EMIT, bool REL>
__device__ __forceinline__ uint32_t stab_pass(const View &v, StabTile &T, bool valid, const QRec &r, uint64_t out,
                                              uint64_t *stage)
{
    const uint32_t tid = threadIdx.x;
    const bool isr = (r.flags >> 8) & 1u;
    const uint32_t wm = r.flags & 0xFFu;
    const uint64_t rb = REL ? T.rbase : 0;
    const uint32_t qlo = (uint32_t)(r.lo - rb), qhi = (uint32_t)(r.hi - rb);   // (REL)
    uint32_t count = 0;
    uint32_t c = 0, base = 0;
    while (c < (uint32_t)NCLS && T.b0[c] >= T.b1[c]) ++c;
    if (c < (uint32_t)NCLS) base = T.b0[c];
    StabRegs g;
    if (c < (uint32_t)NCLS) stab_load(v, g, base, min((uint32_t)TILE, T.b1[c] - base));
    while (c < (uint32_t)NCLS) {
        const uint32_t len = min((uint32_t)TILE, T.b1[c] - base);
#pragma unroll
        for (int u = 0; u < ST_PT; ++u) {
            const uint32_t k = tid + (uint32_t)u * BLOCK;
            if (k < len) {
                if (REL) {
                    T.s32[k] = (uint32_t)(g.s[u] - rb);
                    T.e32[k] = g.e[u] - rb < 0xFFFFFFFFull ? (uint32_t)(g.e[u] - rb) : 0xFFFFFFFFu;
                } else {
                    T.s[k] = g.s[u]; T.e[k] = g.e[u];
                }
                T.info[k] = g.info[u]; T.kind[k] = (uint8_t)g.kind[u];
            }
        }
        __syncthreads();
        uint32_t c2 = c, base2 = base;
        stab_next(T, c2, base2);
        if (c2 < (uint32_t)NCLS) stab_load(v, g, base2, min((uint32_t)TILE, T.b1[c2] - base2));
        if (valid) {
            const uint64_t W = class_width(c);
            // this query's own window inside the tile: starts in [lo - W, hi]
            uint32_t k;
            if (REL) k = lower_bound_u32(T.s32, 0, len, (uint64_t)qlo > W ? qlo - (uint32_t)W : 0u);
            else k = lower_bound_s(T.s, 0, len, r.lo > W ? r.lo - W : 0);
            for (; k < len; ++k) {
                bool hit;
                if (REL) {
                    const uint32_t s = T.s32[k];
                    if (s > qhi) break;
                    const uint32_t e = T.e32[k];
                    if (isr) hit = s < qhi && e > qlo;                         // Range.compareIntersecting == 0
                    else if (v.end_inclusive) hit = s < qlo && qlo <= e;       // EndInclusive.contains (s, e]
                    else hit = s <= qlo && qlo < e;                            // StartInclusive.contains [s, e)
                } else {
                    const uint64_t s = T.s[k];
                    if (s > r.hi) break;
                    const uint64_t e = T.e[k];
                    if (isr) hit = s < r.hi && e > r.lo;
                    else if (v.end_inclusive) hit = s < r.lo && r.lo <= e;
                    else hit = s <= r.lo && r.lo < e;
                }
                if (!hit) continue;
                const uint2 info = T.info[k];
                if (info.y >= r.lim || info.y == r.tpos) continue;            // STARTED_BEFORE; p1
                if (!((wm >> T.kind[k]) & 1u)) continue;                      // testKind
                if (EMIT) {
                    const uint64_t x = ((uint64_t)info.x << 32) | info.y;
                    if (stage) stage[out + count] = x; else v.ent[out + count] = x;
                }
                ++count;
            }
        }
        __syncthreads();
        c = c2; base = base2;
    }
    return count;
}

// The stabbing blocks' windows: one thread per (block, width class) and bound, a plain binary search over the class's
// starts (starts in [lo_min - 4^c, hi_max] for the block's sorted queries). Thousands of independent searches keep the
// loads in flight, where a search inside the stabbing block would stall it for every dependent round.
__global__ __launch_bounds__(BLOCK) void k_rd_stab_win(uint32_t nsb, const uint64_t *__restrict__ blo,
                                                       const uint64_t *__restrict__ bhi, View v, uint32_t *__restrict__ win)
{
    const uint64_t g = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (g >= (uint64_t)nsb * NCLS) return;
    const uint32_t blk = (uint32_t)(g / NCLS), c = (uint32_t)(g % NCLS);
    const uint32_t a0 = v.class_off[c], a1 = v.class_off[c + 1];
    uint32_t b0 = a0, b1 = a0;
    if (a1 > a0) {
        const uint64_t lo = blo[blk], hi = bhi[blk], W = class_width(c);
        b0 = lower_bound_s(v.cs_s, a0, a1, lo > W ? lo - W : 0);
        b1 = upper_bound_s(v.cs_s, b0, a1, hi);
    }
    win[(size_t)blk * 2 * NCLS + c] = b0;
    win[(size_t)blk * 2 * NCLS + NCLS + c] = b1;
}

// Every class's window of the block in one tile (when they fit TILE together): one load round for the block.
// Count pass (hv != null): the query's first STAB_RH hits are kept in registers. Emit pass: hits to ent at out.
// REL: bounds as 32-bit offsets above the block's rbase (half the LDS bytes per probe and per candidate: the pass is
// bound by LDS reads); a candidate's TxnId position and kind are read only when its bounds hit.
constexpr int STAB_RH = 16;   // hits a query keeps in registers through the count pass (flat blocks)

template <bool EMIT>
__device__ __forceinline__ uint32_t stab_flat_rel(const View &v, StabTile &T, bool valid, const QRec &r, uint64_t out,
                                                  uint64_t (*hv)[STAB_RH])
{
    uint32_t count = 0;
    if (!valid) return 0;
    const bool isr = (r.flags >> 8) & 1u;
    const uint32_t wm = r.flags & 0xFFu;
    const uint32_t qlo = (uint32_t)(r.lo - T.rbase), qhi = (uint32_t)(r.hi - T.rbase);
    for (uint32_t c = 0; c < (uint32_t)NCLS; ++c) {
        const uint32_t p0 = T.pre[c], p1 = T.pre[c + 1];
        if (p0 == p1) continue;
        const uint64_t W = class_width(c);
        const uint32_t qwlo = (uint64_t)qlo > W ? qlo - (uint32_t)W : 0u;
        for (uint32_t k = lower_bound_u32(T.s32, p0, p1, qwlo); k < p1; ++k) {
            const uint32_t s = T.s32[k];
            if (s > qhi) break;
            const uint32_t e = T.e32[k];
            bool hit;
            if (isr) hit = s < qhi && e > qlo;                             // Range.compareIntersecting == 0
            else if (v.end_inclusive) hit = s < qlo && qlo <= e;           // EndInclusive.contains (s, e]
            else hit = s <= qlo && qlo < e;                                // StartInclusive.contains [s, e)
            if (hit) {
                const uint2 info = T.info[k];
                hit = info.y < r.lim && info.y != r.tpos                   // STARTED_BEFORE; p1
                      && ((wm >> T.kind[k]) & 1u);                         // testKind
                if (hit) {
                    const uint64_t x = ((uint64_t)info.x << 32) | info.y;
                    if (EMIT) {
                        v.ent[out + count] = x;
                    } else if (hv) {
#pragma unroll
                        for (int u = 0; u < STAB_RH; ++u)
                            if ((uint32_t)u == count) (*hv)[u] = x;
                    }
                    ++count;
                }
            }
        }
    }
    return count;
}

template <bool EMIT>
__device__ __forceinline__ uint32_t stab_flat(const View &v, StabTile &T, bool valid, const QRec &r, uint64_t out,
                                              uint64_t (*hv)[STAB_RH])
{
    uint32_t count = 0;
    if (!valid) return 0;
    const bool isr = (r.flags >> 8) & 1u;
    const uint32_t wm = r.flags & 0xFFu;
    for (uint32_t c = 0; c < (uint32_t)NCLS; ++c) {
        const uint32_t p0 = T.pre[c], p1 = T.pre[c + 1];
        if (p0 == p1) continue;
        const uint64_t W = class_width(c);
        const uint64_t qwlo = r.lo > W ? r.lo - W : 0;
        for (uint32_t k = lower_bound_s(T.s, p0, p1, qwlo); k < p1; ++k) {
            const uint64_t s = T.s[k];
            if (s > r.hi) break;
            const uint64_t e = T.e[k];
            bool hit;
            if (isr) hit = s < r.hi && e > r.lo;                           // Range.compareIntersecting == 0
            else if (v.end_inclusive) hit = s < r.lo && r.lo <= e;         // EndInclusive.contains (s, e]
            else hit = s <= r.lo && r.lo < e;                              // StartInclusive.contains [s, e)
            const uint2 info = T.info[k];
            hit = hit && info.y < r.lim && info.y != r.tpos                // STARTED_BEFORE; p1
                  && ((wm >> T.kind[k]) & 1u);                             // testKind
            const uint64_t x = ((uint64_t)info.x << 32) | info.y;
            if (EMIT) {
                if (hit) v.ent[out + count] = x;
            } else if (hv) {
#pragma unroll
                for (int u = 0; u < STAB_RH; ++u)
                    if (hit && (uint32_t)u == count) (*hv)[u] = x;
            }
            count += hit ? 1u : 0u;
        }
    }
    return count;
}

#ifdef ACC_PHASE_PROF
// tuning build only: per-block phase cycles of k_rd_stab (thread 0, each phase closed by a barrier and a full waitcnt)
__device__ unsigned long long *g_stab_prof;
#define SB_PH(i) do { __syncthreads(); __builtin_amdgcn_s_waitcnt(0); ph[i] = clock64(); } while (0)
#else
#define SB_PH(i) ((void)0)
#endif

// A workgroup of BLOCK consecutive (sorted) queries over its precomputed windows: count every query's pairs, take the
// block's output slice with one atomic, write them. When the windows fit one tile they are loaded once and each query
// keeps its first STAB_RH hits in registers through the count pass: a query with no more than that writes them from
// there, a query with more scans the tile again. Otherwise the (class, tile) sequence is scanned again to emit.
// (A config-4 key block holds ~1,400 hits: an LDS pool of them would cost the occupancy, a per-hit slot claim the
// count pass's time.)
__global__ __launch_bounds__(BLOCK) void k_rd_stab(View v)
{
#ifdef ACC_PHASE_PROF
    uint64_t ph[6];
#endif
    SB_PH(0);
    __shared__ StabTile T;
    const uint32_t tid = threadIdx.x;
    const uint32_t i = blockIdx.x * BLOCK + tid;
    QRec r{};
    if (i < v.Q) r = v.srec[i];
    const bool valid = i < v.Q && !(r.flags & QPAD);
    if (tid < (uint32_t)NCLS) {
        T.b0[tid] = v.win[(size_t)blockIdx.x * 2 * NCLS + tid];
        T.b1[tid] = v.win[(size_t)blockIdx.x * 2 * NCLS + NCLS + tid];
    }
    __syncthreads();
    if (tid < 64) {   // wave 0: the classes' tile offsets by one wave scan (a serial loop over 33 classes cost ~3K cycles)
        const uint32_t len = tid < (uint32_t)NCLS ? T.b1[tid] - T.b0[tid] : 0u;
        const uint32_t incl = wave_inclusive(len, OpAdd<uint32_t>());
        if (tid < (uint32_t)NCLS) T.pre[tid] = incl - len;
        if (tid == (uint32_t)NCLS - 1) T.pre[NCLS] = incl;
        const uint64_t ne = __ballot(len != 0);
        if (tid == 0) {
            const uint32_t cmax = ne ? 63u - (uint32_t)__builtin_clzll(ne) : 0u;
            // every windowed start is at least the block's lowest bound less its widest class; the highest probe
            // bound is bhi
            const uint64_t W = class_width(cmax), lo = v.blo[blockIdx.x], hi = v.bhi[blockIdx.x];
            T.rbase = lo > W ? lo - W : 0;
            T.rel = hi >= T.rbase && hi - T.rbase < 0xFFFFFFFFull;
        }
    }
    __syncthreads();
    SB_PH(1);
    const uint32_t wtot = T.pre[NCLS];
    const bool flat = wtot <= (uint32_t)TILE;
    uint32_t count;
    uint64_t hv[STAB_RH];
    if (flat) {
        for (uint32_t k = tid; k < wtot; k += BLOCK) {
            uint32_t lo = 0, hi = NCLS;   // the class holding flat position k: last c with pre[c] <= k
            while (hi - lo > 1) { const uint32_t md = (lo + hi) >> 1; if (T.pre[md] <= k) lo = md; else hi = md; }
            const uint32_t src = T.b0[lo] + (k - T.pre[lo]);
            const uint64_t cs = v.cs_s[src], ce = v.cs_e[src];
            T.s[k] = cs; T.e[k] = ce; T.info[k] = v.cs_info[src]; T.kind[k] = v.cs_kind[src];
            T.s32[k] = (uint32_t)(cs - T.rbase);
            T.e32[k] = ce - T.rbase < 0xFFFFFFFFull ? (uint32_t)(ce - T.rbase) : 0xFFFFFFFFu;
        }
        __syncthreads();
        SB_PH(2);
        count = T.rel ? stab_flat_rel<false>(v, T, valid, r, 0, &hv) : stab_flat<false>(v, T, valid, r, 0, &hv);
    } else {
        SB_PH(2);
        count = T.rel ? stab_pass<false, true>(v, T, valid, r, 0, nullptr) : stab_pass<false, false>(v, T, valid, r, 0, nullptr);
    }
    SB_PH(3);
    uint32_t total;
    const uint32_t mine = block_exclusive(count, OpAdd<uint32_t>(), T.red, total);
    if (tid == 0) T.base = atomicAdd((unsigned long long *)v.cursor, (unsigned long long)total);
    __syncthreads();
    SB_PH(4);
    const uint64_t base = T.base;
    if (valid) v.q_out[r.q] = make_ulonglong2(base + mine, count);
    if (base + total > v.cap) return;   // uniform: the host re-runs with a larger capacity
    if (flat && count <= (uint32_t)STAB_RH) {
#pragma unroll
        for (int u = 0; u < STAB_RH; ++u)
            if ((uint32_t)u < count) v.ent[base + mine + u] = hv[u];
    } else if (flat) {
        if (T.rel) stab_flat_rel<true>(v, T, valid, r, base + mine, nullptr);
        else stab_flat<true>(v, T, valid, r, base + mine, nullptr);
    } else {
        if (T.rel) stab_pass<true, true>(v, T, valid, r, base + mine, nullptr);
        else stab_pass<true, false>(v, T, valid, r, base + mine, nullptr);
    }
#ifdef ACC_PHASE_PROF
    SB_PH(5);
    if (tid == 0) {
        unsigned long long *row = g_stab_prof + 8 * (size_t)blockIdx.x;
        for (int k = 0; k < 5; ++k) row[k] = ph[k + 1] - ph[k];
        row[6] = flat ? 1 : 2;
        row[5] = total;
        row[7] = 1;
    }
#endif
}

// ---------------------------------------------------------------- per-txn build

struct Out {
    uint32_t n, P;
    const uint32_t *key_off, *rng_off;
    const ulonglong2 *q_out;      // (first entry, entries) per query
    const uint64_t *ent;
    const uint32_t *txn_of_tpos;  // null: batch in TxnId order (tpos = batch index)
    const uint64_t *raw_off;      // [n + 1] raw entries per txn (scratch placement)
    uint32_t *s_arena, *s_rid, *s_dep;   // scratch at 2 raw_off / raw_off / raw_off
    uint32_t *rd_cnt, *u_cnt;
    uint64_t *a_cnt;
    const uint32_t *list;         // txns of the tier (build kernels)
    const uint64_t *glb_off;      // scratch offsets of the global tier (u64 elements)
    uint64_t *gscratch;
    // compaction
    const uint64_t *arena_off, *rd_off, *u_off;
    int32_t *arena;
    uint32_t *range_id, *dep_txn;
};

__device__ __forceinline__ void txn_queries(const Out &o, uint32_t t, uint32_t &q0, uint32_t &q1)
{
    const uint32_t k0 = o.key_off[t], k1 = o.key_off[t + 1];
    if (k1 > k0) { q0 = k0; q1 = k1; return; }
    q0 = o.P + o.rng_off[t];
    q1 = o.P + o.rng_off[t + 1];
}

__device__ __forceinline__ uint32_t dep_of(const Out &o, uint32_t tpos) { return o.txn_of_tpos ? o.txn_of_tpos[tpos] : tpos; }

// per txn: raw entry count and tier; the tier counts of the batch (hist, zeroed before): one ballot per tier value and
// wave, summed over RD_TS chunks of BLOCK txns per workgroup, one global add per tier and workgroup (the 12 counters
// share one line: per-256-txn adds serialised there, and per-thread LDS atomics on 12 words before that)
constexpr int RD_TIERS = 12;
__global__ __launch_bounds__(BLOCK) void k_rd_tsize(uint32_t n, Out o, uint64_t *__restrict__ m_raw, uint32_t *__restrict__ tier,
                                                    uint32_t *__restrict__ hist)
{
    __shared__ uint32_t h[WAVES][RD_TIERS];
    const uint32_t w = threadIdx.x >> 6, lane = lane_id();
    uint32_t acc[RD_TIERS] = {};   // this wave's counts (lane 0)
    for (int r = 0; r < RD_TS; ++r) {
        const uint32_t t = (blockIdx.x * RD_TS + (uint32_t)r) * BLOCK + threadIdx.x;
        uint32_t tr = 0xFFu;
        if (t < n) {
            uint32_t q0, q1;
            txn_queries(o, t, q0, q1);
            uint64_t m = 0;
            for (uint32_t qb = q0; qb < q1; qb += 8) {   // eight count loads in flight, not one dependent add per load
                uint32_t c[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) c[u] = qb + u < q1 ? (uint32_t)o.q_out[qb + u].y : 0u;
#pragma unroll
                for (int u = 0; u < 8; ++u) m += c[u];
            }
            m_raw[t] = m;
            // tiers: 0 none, 1 <= 16 (16-lane groups), 11 <= 32 (half waves), 2 <= 64 (wave), 3..9 LDS workgroups of
            // 128..8192, 10 global
            if (m == 0) tr = 0;
            else if (m <= 16) tr = 1;
            else if (m <= 32) tr = 11;
            else if (m <= 64) tr = 2;
            else if (m <= BLOCK_E) { uint32_t n2 = 128, b = 3; while (n2 < m) { n2 <<= 1; ++b; } tr = b; }
            else tr = 10;
            tier[t] = tr;
            if (m == 0) { o.rd_cnt[t] = 0; o.u_cnt[t] = 0; o.a_cnt[t] = 0; }
        }
#pragma unroll
        for (int v = 0; v < RD_TIERS; ++v) acc[v] += (uint32_t)__popcll(__ballot(tr == (uint32_t)v));
    }
    if (lane == 0)
#pragma unroll
        for (int v = 0; v < RD_TIERS; ++v) h[w][v] = acc[v];
    __syncthreads();
    if (threadIdx.x < RD_TIERS) {
        uint32_t c = 0;
        for (int q = 0; q < WAVES; ++q) c += h[q][threadIdx.x];
        if (c) atomicAdd(&hist[threadIdx.x], c);
    }
}


// bitonic sort within lane groups of S (lane-aligned: the xor partners stay inside), ascending; partners through DPP /
// permlane swaps (xor_lanes: the whole wave active, as at every call below)
template <int S, class T>
__device__ __forceinline__ T group_sort(T x, uint32_t lane)
{
#pragma unroll
    for (uint32_t k = 2; k <= (uint32_t)S; k <<= 1) {
#pragma unroll
        for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
            const T y = xor_lanes(x, (int)jj);
            const bool up = k == (uint32_t)S || (lane & k) == 0, lower = (lane & jj) == 0;
            const T mn = x < y ? x : y, mx = x < y ? y : x;
            x = (lower == up) ? mn : mx;
        }
    }
    return x;
}

// One chunk of S queries [qc, min(qc + S, q1)) of a txn whose (first entry, entries) records the group's lanes hold
// in qv: an inclusive count scan, a shuffle search for the query holding entry `sub` of the txn (after the m entries
// of earlier chunks), and that entry's load (issued here, waited for by the first use).
template <int S>
__device__ __forceinline__ void seg_chunk(const Out &o, ulonglong2 qv, uint32_t sub, int gb, uint64_t &m, uint64_t &x)
{
    const uint32_t c = (uint32_t)qv.y;
    const uint64_t qo = qv.x;
    uint32_t incl = c;
#pragma unroll
    for (int d = 1; d < S; d <<= 1) {
        const uint32_t u = __shfl_up(incl, d, 64);
        if (sub >= (uint32_t)d) incl += u;
    }
    const uint32_t total = __shfl(incl, gb + S - 1, 64);
    uint32_t j = 0;   // lanes whose queries end at or before entry sub
#pragma unroll
    for (int step = S / 2; step >= 1; step >>= 1) {
        const uint32_t end = (uint32_t)m + __shfl(incl, gb + (int)j + step - 1, 64);
        if (end <= sub) j += step;
    }
    j = min(j, (uint32_t)S - 1);
    const uint64_t qoj = shfl_idx(qo, gb + (int)j);
    const uint32_t startj = (uint32_t)m + __shfl(incl - c, gb + (int)j, 64);
    if (sub >= m && sub < m + total) x = o.ent[qoj + (sub - startj)];
    m += total;
}

// Groups of S lanes (S = 16, 32 or 64), K txns each in turn: load, sort (range id, TxnId position), dedupe, TxnId
// union and index, range groups; results to the scratch regions of the txn.
// The K txns' loads are issued together — list entries, then their offsets, then their first S query records, then
// their entries — so a group waits for four dependent memory latencies per K txns, not per txn (the tier is
// latency-bound: each of those loads costs ~2.5K cycles under the build's load, the sorts ~1K).
// NARROW (range ids and TxnId positions below 2^26): both sorts on 32-bit keys, half the cross-lane traffic of the
// 64-bit network. The first sorts (range id << 6 | lane) and each lane then takes its key's entry; when some range id is
// held by entries of different TxnIds (commands with identical ranges: rare) the (range id, lane) order may separate
// duplicates or misorder TxnIds, so that wave sorts the 64-bit entries instead.
#ifdef ACC_PHASE_PROF
// tuning build only (tools/build_prof.sh): per-wave phase cycles of k_rd_build_seg, one row of 8 per wave, each phase
// closed by a full s_waitcnt so a phase owns its loads' latency
__device__ unsigned long long *g_rd_prof;
#define RD_PH(i) do { __builtin_amdgcn_s_waitcnt(0); ph[i] = clock64(); } while (0)
#else
#define RD_PH(i) ((void)0)
#endif
#ifndef ACC_RD_SEGK
#define ACC_RD_SEGK 4
#endif
constexpr int RD_SEGK = ACC_RD_SEGK;   // txns per lane group

template <int S, bool NARROW, int K>
__global__ __launch_bounds__(BLOCK) void k_rd_build_seg(uint32_t cnt, Out o)
{
#ifdef ACC_PHASE_PROF
    uint64_t ph[6];
#endif
    RD_PH(0);
    __shared__ uint32_t slot[WAVES][64];
    constexpr int G = 64 / S;
    const uint32_t wave = threadIdx.x >> 6, lane = lane_id();
    const uint32_t grp = lane / S, sub = lane & (S - 1);
    const uint32_t li0 = ((blockIdx.x * WAVES + wave) * G + grp) * K;
    const uint64_t gmask = S == 64 ? ~0ull : (((1ull << (S & 63)) - 1) << (grp * S));
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const int gb = (int)(grp * S);
    const uint32_t g0 = grp * S;
    uint32_t t[K], q0[K], q1[K];
    uint64_t ra[K], m[K], x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) t[k] = li0 + k < cnt ? o.list[li0 + k] : 0u;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        // both the key and the range bounds (txn_queries' choice made after the loads, not between them)
        q0[k] = q1[k] = 0; ra[k] = 0;
        if (li0 + k < cnt) {
            const uint32_t k0 = o.key_off[t[k]], k1 = o.key_off[t[k] + 1];
            const uint32_t r0 = o.rng_off[t[k]], r1 = o.rng_off[t[k] + 1];
            ra[k] = o.raw_off[t[k]];
            if (k1 > k0) { q0[k] = k0; q1[k] = k1; } else { q0[k] = o.P + r0; q1[k] = o.P + r1; }
        }
    }
    RD_PH(1);
    ulonglong2 qv[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t q = q0[k] + sub;
        qv[k] = make_ulonglong2(0, 0);
        if (q < q1[k]) qv[k] = o.q_out[q];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        m[k] = 0; x[k] = ~0ull;
        seg_chunk<S>(o, qv[k], sub, gb, m[k], x[k]);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        for (uint32_t qc = q0[k] + S; qc < q1[k]; qc += S) {   // group-uniform: txns of more than S queries
            const uint32_t q = qc + sub;
            ulonglong2 v = make_ulonglong2(0, 0);
            if (q < q1[k]) v = o.q_out[q];
            seg_chunk<S>(o, v, sub, gb, m[k], x[k]);
        }
    }
    RD_PH(2);
#ifdef ACC_PHASE_PROF
    uint64_t sort_cy = 0, write_cy = 0;
    bool wlive = false;
#endif
#pragma unroll
    for (int k = 0; k < K; ++k) {
#ifdef ACC_PHASE_PROF
        RD_PH(3);
#endif
        const bool live = li0 + k < cnt;
        uint64_t xk = x[k];
        const uint64_t mk = m[k];
        if (NARROW) {
            uint32_t k1 = (live && sub < mk) ? ((uint32_t)(xk >> 32) << 6) | sub : 0xFFFFFFFFu;
            k1 = group_sort<S>(k1, lane);
            const uint64_t xs = shfl_idx(xk, (int)(grp * S + (k1 & 63u)));
            xk = k1 == 0xFFFFFFFFu ? ~0ull : xs;
            const uint64_t pv = shfl_up(xk, 1);
            const bool mixed = live && sub > 0 && sub < mk && (uint32_t)(pv >> 32) == (uint32_t)(xk >> 32) && (uint32_t)pv != (uint32_t)xk;
            if (__ballot(mixed)) xk = group_sort<S>(xk, lane);   // wave-uniform; sorted groups stay as they are
        } else {
            xk = group_sort<S>(xk, lane);
        }
        const uint64_t prev = shfl_up(xk, 1);
        const bool valid = live && sub < mk && (sub == 0 || xk != prev);       // dedupe identical (range, txn)
        const uint64_t vb = __ballot(valid) & gmask;
        const uint32_t M = (uint32_t)__popcll(vb);
        const uint32_t pos = (uint32_t)__popcll(vb & lt);
        const uint32_t rid = (uint32_t)(xk >> 32), tp = (uint32_t)xk;
        // (TxnId position, entry) sorted: the TxnId union and each entry's index
        uint32_t ytp, ypos;
        if (NARROW) {
            const uint32_t y = group_sort<S>(valid ? (tp << 6) | pos : 0xFFFFFFFFu, lane);
            ytp = y >> 6; ypos = y & 63u;
        } else {
            const uint64_t y = group_sort<S>(valid ? (((uint64_t)tp << 8) | pos) : ~0ull, lane);
            ytp = (uint32_t)(y >> 8); ypos = (uint32_t)y & 0xFFu;
        }
        const uint32_t yprev = __shfl_up(ytp, 1, 64);
        const bool ynew = live && sub < M && (sub == 0 || ytp != yprev);
        const uint64_t nb = __ballot(ynew) & gmask;
        const uint32_t U = (uint32_t)__popcll(nb);
        const bool yin = live && sub < M;
        const uint32_t uidx = (uint32_t)__popcll(nb & lt) + (ynew ? 1u : 0u) - 1u;   // index of this entry's TxnId
        const bool rnew = valid && (sub == 0 || (uint32_t)(prev >> 32) != rid);
        const uint64_t rb = __ballot(rnew) & gmask;
        const uint32_t Rd = (uint32_t)__popcll(rb);
#ifdef ACC_PHASE_PROF
        RD_PH(4);
        sort_cy += ph[4] - ph[3];
        wlive = wlive || __ballot(live && mk != 0) != 0;
#endif
        __builtin_amdgcn_wave_barrier();   // the previous txn's reads of slot are done
        if (yin) slot[wave][g0 + ypos] = uidx;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        if (live && mk != 0) {
            uint32_t *sa = o.s_arena + 2 * ra[k], *sr = o.s_rid + ra[k], *sd = o.s_dep + ra[k];
            if (ynew) sd[uidx] = dep_of(o, ytp);
            const uint32_t g = (uint32_t)__popcll(rb & lt);
            if (valid) {
                sa[Rd + pos] = slot[wave][g0 + pos];
                if (rnew) {
                    sr[g] = rid;
                    if (g > 0) sa[g - 1] = Rd + pos;
                }
            }
            if (sub == 0) {
                sa[Rd - 1] = Rd + M;
                o.rd_cnt[t[k]] = Rd; o.u_cnt[t[k]] = U; o.a_cnt[t[k]] = (uint64_t)Rd + M;
            }
        }
#ifdef ACC_PHASE_PROF
        RD_PH(5);
        write_cy += ph[5] - ph[4];
#endif
    }
#ifdef ACC_PHASE_PROF
    if (lane == 0 && wlive) {
        unsigned long long *row = g_rd_prof + 8 * ((size_t)blockIdx.x * WAVES + wave);
        row[0] = ph[1] - ph[0]; row[1] = ph[2] - ph[1]; row[2] = sort_cy; row[3] = write_cy;
        row[7] = 1;
    }
#endif
}

// One workgroup per txn over buffers A, B of n2 >= m elements (LDS sized to the tier, or global scratch)
// qs / qo: LDS of BLOCK + 1 / BLOCK entries (query starts in the txn's raw list, query offsets in ent)
__device__ void build_block(const Out &o, uint32_t t, uint64_t *A, uint64_t *B, uint32_t *red, uint32_t *qs, uint64_t *qo)
{
    const uint32_t tid = threadIdx.x;
    uint32_t q0, q1;
    txn_queries(o, t, q0, q1);
    uint32_t m = 0;
    const uint32_t nq = q1 - q0;
    if (nq <= (uint32_t)BLOCK) {
        // every query's count and offset in one load round, then the raw entries four loads per thread at a time
        uint32_t c = 0;
        uint64_t off = 0;
        if (tid < nq) { const ulonglong2 qv = o.q_out[q0 + tid]; c = (uint32_t)qv.y; off = qv.x; }
        const uint32_t st = block_exclusive(c, OpAdd<uint32_t>(), red, m);
        if (tid < nq) { qs[tid] = st; qo[tid] = off; }
        __syncthreads();
        for (uint32_t k0 = tid; k0 < m; k0 += 4 * BLOCK) {
            uint64_t x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t k = k0 + (uint32_t)u * BLOCK;
                x[u] = 0;
                if (k < m) {
                    uint32_t lo = 0, hi = nq;   // last query starting at or before k
                    while (hi - lo > 1) { const uint32_t md = (lo + hi) >> 1; if (qs[md] <= k) lo = md; else hi = md; }
                    x[u] = o.ent[qo[lo] + (k - qs[lo])];
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) if (k0 + (uint32_t)u * BLOCK < m) A[k0 + (uint32_t)u * BLOCK] = x[u];
        }
    } else {
        for (uint32_t q = q0; q < q1; ++q) {
            const ulonglong2 qv = o.q_out[q];
            const uint32_t c = (uint32_t)qv.y;
            const uint64_t off = qv.x;
            for (uint32_t k = tid; k < c; k += BLOCK) A[m + k] = o.ent[off + k];
            m += c;
        }
    }
    uint32_t n2 = 64;
    while (n2 < m) n2 <<= 1;
    for (uint32_t i = m + tid; i < n2; i += BLOCK) A[i] = ~0ull;
    __syncthreads();
    block_bitonic(A, n2);
    // dedupe + compact into B; each thread owns a contiguous slice
    const uint32_t per = (n2 + BLOCK - 1) / BLOCK;
    const uint32_t lo = tid * per, hi = min(lo + per, n2);
    uint32_t c = 0;
    for (uint32_t i = lo; i < hi; ++i) c += (i < m && (i == 0 || A[i] != A[i - 1])) ? 1u : 0u;
    uint32_t M;
    uint32_t p = block_exclusive(c, OpAdd<uint32_t>(), red, M);
    for (uint32_t i = lo; i < hi; ++i)
        if (i < m && (i == 0 || A[i] != A[i - 1])) B[p++] = A[i];
    __syncthreads();
    uint32_t n2m = 64;
    while (n2m < M) n2m <<= 1;
    for (uint32_t i = tid; i < n2m; i += BLOCK) A[i] = i < M ? (((uint64_t)(uint32_t)B[i] << 32) | i) : ~0ull;
    __syncthreads();
    block_bitonic(A, n2m);
    // distinct TxnId positions -> index; B[e] becomes (range id << 32 | index)
    const uint64_t ra = o.raw_off[t];
    uint32_t *sa = o.s_arena + 2 * ra, *sr = o.s_rid + ra, *sd = o.s_dep + ra;
    const uint32_t per2 = (n2m + BLOCK - 1) / BLOCK;
    const uint32_t lo2 = tid * per2, hi2 = min(lo2 + per2, n2m);
    c = 0;
    for (uint32_t i = lo2; i < hi2; ++i) c += (i < M && (i == 0 || (A[i] >> 32) != (A[i - 1] >> 32))) ? 1u : 0u;
    uint32_t U;
    uint32_t u = block_exclusive(c, OpAdd<uint32_t>(), red, U);
    for (uint32_t i = lo2; i < hi2; ++i) {
        if (i >= M) break;
        const bool nw = i == 0 || (A[i] >> 32) != (A[i - 1] >> 32);
        if (nw) { sd[u] = dep_of(o, (uint32_t)(A[i] >> 32)); ++u; }
        const uint32_t e = (uint32_t)A[i];
        B[e] = (B[e] & 0xFFFFFFFF00000000ull) | (u - 1);
    }
    __syncthreads();
    // range groups over B[0, M)
    const uint32_t per3 = (M + BLOCK - 1) / BLOCK;
    const uint32_t lo3 = min(tid * per3, M), hi3 = min(lo3 + per3, M);
    c = 0;
    for (uint32_t e = lo3; e < hi3; ++e) c += (e == 0 || (B[e] >> 32) != (B[e - 1] >> 32)) ? 1u : 0u;
    uint32_t Rd;
    uint32_t g = block_exclusive(c, OpAdd<uint32_t>(), red, Rd);
    for (uint32_t e = lo3; e < hi3; ++e) {
        const uint32_t rid = (uint32_t)(B[e] >> 32);
        const bool nw = e == 0 || (B[e - 1] >> 32) != rid;
        if (nw) { sr[g] = rid; ++g; }
        sa[Rd + e] = (uint32_t)B[e];
        const bool last = e + 1 == M || (uint32_t)(B[e + 1] >> 32) != rid;
        if (last) sa[g - 1] = Rd + e + 1;
    }
    if (tid == 0) { o.rd_cnt[t] = Rd; o.u_cnt[t] = U; o.a_cnt[t] = (uint64_t)Rd + M; }
}

__global__ __launch_bounds__(BLOCK) void k_rd_build_block(Out o, uint32_t n2)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    // all LDS dynamic (no static __shared__ ahead of it: the base stays 16-B aligned, Guideline 17):
    // [A: n2 u64][B: n2 u64][qo: BLOCK u64][red: 16 u32][qs: BLOCK + 1 u32]
    uint64_t *qo = lds + 2 * n2;
    uint32_t *red = reinterpret_cast<uint32_t *>(qo + BLOCK);
    build_block(o, o.list[blockIdx.x], lds, lds + n2, red, red + 16, qo);
}

__global__ __launch_bounds__(BLOCK) void k_rd_build_global(Out o)
{
    __shared__ uint32_t red[WAVES];
    __shared__ uint32_t qs[BLOCK + 1];
    __shared__ uint64_t qo[BLOCK];
    const uint32_t t = o.list[blockIdx.x];
    uint64_t *A = o.gscratch + o.glb_off[blockIdx.x];
    const uint64_t m = o.raw_off[t + 1] - o.raw_off[t];
    uint64_t n2 = 64;
    while (n2 < m) n2 <<= 1;
    build_block(o, t, A, A + n2, red, qs, qo);
}

__global__ __launch_bounds__(BLOCK) void k_rd_glb_sizes(uint32_t ng, Out o, uint64_t *__restrict__ sz)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= ng) return;
    const uint32_t t = o.list[i];
    const uint64_t m = o.raw_off[t + 1] - o.raw_off[t];
    uint64_t n2 = 64;
    while (n2 < m) n2 <<= 1;
    sz[i] = 2 * n2;
}

// scratch -> Java-layout CSR. A workgroup owns BLOCK consecutive txns, whose output runs are one contiguous range of
// each output array, copied in chunks of CP_CHUNK elements: each txn whose run starts inside the chunk marks its start
// in an LDS owner map (LDS max: of the txns starting at one position the last, the only non-empty one, wins), a block
// max-scan spreads the owners over the chunk (CP_PT consecutive positions per thread, written back to the map), and the
// block copies the chunk element-interleaved from the txns' scratch: every store instruction writes whole lines and no
// element searches for its txn.
constexpr int CP_PT = 8;
constexpr int CP_CHUNK = CP_PT * BLOCK;

__device__ __forceinline__ void compact_array(uint32_t nt, const uint64_t *off, const uint64_t *src_base,
                                              const uint32_t *__restrict__ src, uint32_t *__restrict__ dst,
                                              uint32_t *own, uint32_t *red)
{
    const uint32_t tid = threadIdx.x;
    const uint64_t j1 = off[nt];
    uint32_t carry = 0;
    for (uint64_t c0 = off[0]; c0 < j1; c0 += CP_CHUNK) {
        chunk_owners<CP_PT>(nt, off, c0, own, red, carry);
        // copies interleaved across the block (element u * BLOCK + tid): each store instruction writes whole lines
        uint32_t x[CP_PT];
#pragma unroll
        for (int u = 0; u < CP_PT; ++u) {
            const uint32_t p = (uint32_t)u * BLOCK + tid;
            const uint64_t j = c0 + p;
            const uint32_t k = own[p];
            x[u] = j < j1 ? src[src_base[k] + (j - off[k])] : 0u;
        }
#pragma unroll
        for (int u = 0; u < CP_PT; ++u) {
            const uint64_t j = c0 + (uint64_t)u * BLOCK + tid;
            if (j < j1) dst[j] = x[u];
        }
    }
}

__global__ __launch_bounds__(BLOCK) void k_rd_compact(uint32_t n, Out o)
{
    __shared__ uint64_t ao[BLOCK + 1], ro[BLOCK + 1], uo[BLOCK + 1], sa[BLOCK], sr[BLOCK];
    __shared__ uint32_t own[CP_CHUNK], red[WAVES];
    const uint32_t t0 = blockIdx.x * BLOCK, nt = min((uint32_t)BLOCK, n - t0), tid = threadIdx.x;
    if (tid < nt) {
        const uint32_t t = t0 + tid;
        ao[tid] = o.arena_off[t]; ro[tid] = o.rd_off[t]; uo[tid] = o.u_off[t];
        const uint64_t ra = o.raw_off[t];
        sa[tid] = 2 * ra; sr[tid] = ra;
    }
    if (tid == 0) { ao[nt] = o.arena_off[t0 + nt]; ro[nt] = o.rd_off[t0 + nt]; uo[nt] = o.u_off[t0 + nt]; }   // the block's ends
    __syncthreads();
    compact_array(nt, ao, sa, o.s_arena, reinterpret_cast<uint32_t *>(o.arena), own, red);
    compact_array(nt, ro, sr, o.s_rid, o.range_id, own, red);
    compact_array(nt, uo, sr, o.s_dep, o.dep_txn, own, red);
}

}  // namespace rd

using namespace rd;

#ifdef ACC_PHASE_PROF
// tuning build: rows for one k_rd_build_seg launch of `blocks` workgroups; rd_prof_print after it (serialises the tier)
static unsigned long long *rd_prof_arm(acc_ctx *ctx, uint32_t blocks)
{
    const size_t rows = (size_t)blocks * WAVES;
    unsigned long long *buf = ctx->get<unsigned long long>("rd_prof", 8 * rows);
    ACC_HIP(hipMemsetAsync(buf, 0, 8 * rows * sizeof(unsigned long long), ctx->stream));
    ACC_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_rd_prof), &buf, sizeof buf, 0, hipMemcpyHostToDevice, ctx->stream));
    return buf;
}
static void rd_prof_print(acc_ctx *ctx, const char *tier, unsigned long long *buf, uint32_t blocks)
{
    const size_t rows = (size_t)blocks * WAVES;
    std::vector<unsigned long long> h(8 * rows);
    ACC_HIP(hipMemcpyAsync(h.data(), buf, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, ctx->stream));
    ACC_HIP(hipStreamSynchronize(ctx->stream));
    double sum[4] = {};
    size_t w = 0;
    for (size_t r = 0; r < rows; ++r) {
        if (!h[8 * r + 7]) continue;
        ++w;
        for (int i = 0; i < 4; ++i) sum[i] += (double)h[8 * r + i];
    }
    const double d = w ? (double)w : 1.0;
    fprintf(stderr, "[rd_phase] %s waves=%zu avg cycles: head %.0f gather %.0f sort %.0f write %.0f\n", tier, w, sum[0] / d,
            sum[1] / d, sum[2] / d, sum[3] / d);
}
#endif

static void rd_check_errors(uint64_t errs)
{
    if (errs & ERR_DOMAIN) fail(ACC_E_ARG, "a range-domain txn lists keys or a key-domain txn lists ranges (TxnId.domain())");
    if (errs & ERR_RANGE_EMPTY) fail(ACC_E_ARG, "range start must be below its end (Range: start >= end)");
    if (errs & ERR_RANGES_UNSORTED) fail(ACC_E_ARG, "ranges of a txn must be sorted and deoverlapped (Ranges.ofSortedAndDeoverlapped)");
    if (errs & ERR_RNG_OFF) fail(ACC_E_ARG, "rng_off must be non-decreasing");
}

void rangedeps_batch(acc_ctx *ctx, const acc_range_batch_in *in, acc_rangedeps_view *view, const SharedDict *shared)
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
    if (n == 0) {
        ACC_HIP(hipMemsetAsync(arena_off, 0, 8, st));
        ACC_HIP(hipMemsetAsync(rd_off, 0, 8, st));
        ACC_HIP(hipMemsetAsync(u_off, 0, 8, st));
        *view = acc_rangedeps_view{ n, 0, 0, 0, 0, 0, ctx->get<uint64_t>("rd_dict_s", 1), ctx->get<uint64_t>("rd_dict_e", 1),
                                    arena_off, ctx->get<int32_t>("rd_arena", 1), rd_off, ctx->get<uint32_t>("rd_range_id", 1),
                                    u_off, ctx->get<uint32_t>("rd_dep_txn", 1) };
        ctx->rd_view = *view;
        ctx->rd_valid = true;
        ctx->sync();
        return;
    }

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
    // (acc_partial_deps_batch: the KeyDeps half already built it over the same batch)
    const uint32_t *owner;
    Dictionary dict;
    if (shared && shared->valid) {
        dict = shared->dict;
        owner = shared->owner;
        ctx->stat("rangedeps.shared_dictionary", 1);
    } else {
        uint64_t *g = ctx->get<uint64_t>("g", PREP_G_WORDS);
        uint32_t *own = ctx->get<uint32_t>("owner", P);
        prep_dictionary(ctx, n, P, tm, tl, tn, em, el, en, status, key_off, key_code, own, g, dict);
        owner = own;
        ctx->stat("rangedeps.shared_dictionary", 0);
    }
    // TxnId positions and STARTED_BEFORE limits
    const size_t m2 = 2 * (size_t)n;
    uint32_t *isT = ctx->get<uint32_t>("rd_isT", m2);
    uint32_t *tcnt = ctx->get<uint32_t>("rd_tcnt", m2 + 1);
    ACC_HIP(hipMemsetAsync(isT, 0, m2 * sizeof(uint32_t), st));
    launch(ctx, "rd_txnflag", k_rd_txnflag, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint32_t *)dict.rank, isT);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, isT, tcnt, m2, true, tcnt + m2);
    uint4 *tinfo = ctx->get<uint4>("rd_tinfo", n);
    uint32_t *txn_of_tpos = ctx->get<uint32_t>("rd_txn_of_tpos", n);
    launch(ctx, "rd_txncols", k_rd_txncols, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint32_t *)dict.rank,
           (const uint32_t *)tcnt, tl, tinfo, txn_of_tpos);

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
    launch(ctx, "rd_prep", k_rd_prep, dim3(grid_for(n, (size_t)BLOCK * RD_TS)), dim3(BLOCK), 0, n, tl, status, key_off, key_code, rng_off, rs,
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

    // ---- 2. range-command entries, stored-range dictionary, class order
    const Runs rs_plan = make_runs(hm[0]), re_plan = make_runs(hm[1]);
    uint4 *erec = ctx->get<uint4>("rd_erec", 2 * (size_t)NE);
    uint64_t *dkey = ctx->get<uint64_t>("rd_dkey", NE), *ekey = ctx->get<uint64_t>("rd_ekey", NE);
    const bool split = rs_plan.bits + re_plan.bits > 64;
    launch(ctx, "rd_entries", k_rd_entries, dim3(grid_for(R, BLOCK)), dim3(BLOCK), 0, (uint32_t)R, n, (const uint32_t *)eflag,
           (const uint32_t *)eidx, (const uint32_t *)rowner, rs, re, (const uint4 *)tinfo, tl, rs_plan, re_plan, re_plan.bits,
           split ? 1 : 0, erec, dkey, ekey);
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
           (const uint4 *)erec, dflag);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, dflag, dincl, NE, false, dincl + NE);
    uint64_t *dict_s = ctx->get<uint64_t>("rd_dict_s", NE), *dict_e = ctx->get<uint64_t>("rd_dict_e", NE);
    uint64_t *ckey = ctx->get<uint64_t>("rd_ckey", NE);
    uint32_t *cls = ctx->get<uint32_t>("rd_cls", 2 * (NCLS + 1));
    uint32_t *cls_hist = cls, *class_off = cls + (NCLS + 1);
    ACC_HIP(hipMemsetAsync(cls_hist, 0, (NCLS + 1) * sizeof(uint32_t), st));
    launch(ctx, "rd_dict_write", k_rd_dict_write, dim3(grid_for(NE, (size_t)BLOCK * RD_TS)), dim3(BLOCK), 0, NE, (const uint32_t *)ds.vals,
           (const uint32_t *)dflag, (const uint32_t *)dincl, erec, dict_s, dict_e, ckey, cls_hist);
    launch(ctx, "rd_class_off", k_rd_class_off, dim3(1), dim3(64), 0, (const uint32_t *)cls_hist, class_off);
    // (class, start) order: the (start, end)-sorted entries partitioned stably by class, one 8-bit pass
    const Sorted cs = radix_sort(ctx, "rs_rd_cls", ckey, ds.vals, NE, 6);
    uint64_t *cs_s = ctx->get<uint64_t>("rd_cs_s", NE), *cs_e = ctx->get<uint64_t>("rd_cs_e", NE);
    uint2 *cs_info = ctx->get<uint2>("rd_cs_info", NE);
    uint8_t *cs_kind = ctx->get<uint8_t>("rd_cs_kind", NE);
    launch(ctx, "rd_class_cols", k_rd_class_cols, dim3(grid_for(NE, BLOCK)), dim3(BLOCK), 0, NE, (const uint32_t *)cs.vals,
           (const uint4 *)erec, cs_s, cs_e, cs_info, cs_kind);

    // ---- 3. query records sorted by low bound; stabbing (one pass, block-sliced output)
    const Runs q_plan = make_runs(hm[2]);
    QRec *rec = ctx->get<QRec>("rd_qrec", Q), *srec = nullptr;
    uint64_t *qkey = ctx->get<uint64_t>("rd_qkey", Q);
    const int qbits_full = q_plan.bits < 62 ? q_plan.bits + 3 : q_plan.bits < 64 ? q_plan.bits + 1 : 64;
    // Only the high bits of the low bound are sorted: a stabbing block needs BLOCK queries with neighbouring low bounds
    // (its windows span their lowest to highest bound), and each query's scan is independent of its place in the block.
    // 2^(bits_for(Q) - 2) buckets hold ~4 queries each on spread keys, so a block spans ~64 buckets — about the span of
    // an exact sort — in whole 8-bit passes (config 4: 3 passes instead of 5).
    const int qsort_bits = std::min(qbits_full, std::max(8, (bits_for(Q) - 2 + 7) / 8 * 8));
    const int qdrop = qbits_full - qsort_bits;
    const int qbits = qsort_bits;
    const int ibits = qbits + bits_for(Q) <= 64 && Q < OS_VAL ? std::max(1, bits_for(Q)) : 0;
    launch(ctx, "rd_qrec", k_rd_qrec, dim3(grid_for(Q, BLOCK)), dim3(BLOCK), 0, (uint32_t)P, (uint32_t)R, key_code,
           (const uint32_t *)owner, rs, re, (const uint32_t *)rowner, (const uint4 *)tinfo, q_plan, rec, qkey,
           (uint32_t)q_plan.bits, ibits, qdrop);
    Sorted qs{ nullptr, nullptr };
    const uint64_t *qpk = nullptr;
    if (ibits) qpk = radix_sort_keys(ctx, "rs_rd_q", qkey, Q, ibits, qbits);
    else qs = radix_sort(ctx, "rs_rd_q", qkey, nullptr, Q, qbits);
    const uint32_t Pp = q_plan.bits < 64 && P && R ? (uint32_t)((P + BLOCK - 1) / BLOCK * BLOCK) : (uint32_t)P;
    // the range queries' width groups (q_plan.bits < 62) each from a block boundary: their sizes stay on the device, so
    // the padded length is bounded (three more gaps of under a block)
    const int wgroups = q_plan.bits < 62 && R ? 1 : 0;
    const uint32_t Qp = Q + (Pp - (uint32_t)P) + (wgroups ? 3u * BLOCK : 0u);
    uint32_t *qbnd = ctx->get<uint32_t>("rd_qbnd", 8);
    launch(ctx, "rd_qgroups", k_rd_qgroups, dim3(1), dim3(64), 0, ibits ? qpk : (const uint64_t *)qs.keys, (uint32_t)P, Q,
           ibits + qbits - 3, wgroups, qbnd);
    const uint32_t nsb = (uint32_t)grid_for(Qp, BLOCK);
    uint64_t *bhi = ctx->get<uint64_t>("rd_bhi", nsb), *blo = ctx->get<uint64_t>("rd_blo", nsb);
    srec = ctx->get<QRec>("rd_qrec_sorted", Qp);
    launch(ctx, "rd_qsort", k_rd_qsort, dim3(nsb), dim3(BLOCK), 0, Qp, (uint32_t)P, Pp, (const uint32_t *)qbnd,
           (const uint32_t *)qs.vals, qpk,
           ibits ? (1ull << ibits) - 1 : 0ull, (const QRec *)rec, srec, blo, bhi);
    View v{};
    v.Q = Qp; v.end_inclusive = (int)in->end_inclusive; v.srec = srec;
    v.cs_s = cs_s; v.cs_e = cs_e; v.cs_info = cs_info; v.cs_kind = cs_kind; v.class_off = class_off;
    v.q_out = ctx->get<ulonglong2>("rd_q_out", Q);
    v.cursor = ctx->get<uint64_t>("rd_cursor", 1);
    uint32_t *win = ctx->get<uint32_t>("rd_win", (size_t)nsb * 2 * NCLS);
    v.win = win;
    v.blo = blo; v.bhi = bhi;
    uint64_t E = 0;
    if (Q) {
        launch(ctx, "rd_stab_win", k_rd_stab_win, dim3(grid_for((uint64_t)nsb * NCLS, BLOCK)), dim3(BLOCK), 0, nsb,
               (const uint64_t *)blo, (const uint64_t *)bhi, v, win);
        for (int attempt = 0; attempt < 2; ++attempt) {
            // capacity: the last batch's need on this context, at least 16 per query
            const uint64_t want = std::max<uint64_t>(ctx->rd_ent_hint, 16ull * Q + 1024);
            v.ent = ctx->get<uint64_t>("rd_ent", want);
            v.cap = ctx->bufs["rd_ent"].bytes / sizeof(uint64_t);
            ACC_HIP(hipMemsetAsync(v.cursor, 0, 8, st));
#ifdef ACC_PHASE_PROF
            unsigned long long *sbp = ctx->get<unsigned long long>("stab_prof", 8 * (size_t)nsb);
            ACC_HIP(hipMemsetAsync(sbp, 0, 8 * (size_t)nsb * sizeof(unsigned long long), st));
            ACC_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_stab_prof), &sbp, sizeof sbp, 0, hipMemcpyHostToDevice, st));
#endif
            launch(ctx, "rd_stab", k_rd_stab, dim3(nsb), dim3(BLOCK), 0, v);
#ifdef ACC_PHASE_PROF
            {
                std::vector<unsigned long long> h(8 * (size_t)nsb);
                ACC_HIP(hipMemcpyAsync(h.data(), sbp, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
                ACC_HIP(hipStreamSynchronize(st));
                for (int f = 1; f <= 2; ++f) {
                    double sum[6] = {};
                    size_t nb = 0;
                    for (size_t b = 0; b < nsb; ++b) {
                        if (!h[8 * b + 7] || h[8 * b + 6] != (unsigned long long)f) continue;
                        ++nb;
                        for (int k = 0; k < 6; ++k) sum[k] += (double)h[8 * b + k];
                    }
                    const double d = nb ? (double)nb : 1.0;
                    fprintf(stderr, "[stab_phase] %s blocks=%zu avg cycles: head %.0f tile %.0f count %.0f scan+claim %.0f write %.0f | hits %.0f\n",
                            f == 1 ? "flat" : "tiled", nb, sum[0] / d, sum[1] / d, sum[2] / d, sum[3] / d, sum[4] / d, sum[5] / d);
                }
            }
#endif
            ACC_HIP(hipMemcpyAsync(ctx->pinned, v.cursor, 8, hipMemcpyDeviceToHost, st));
            ctx->sync();
            E = ctx->pinned[0];
            ctx->rd_ent_hint = std::max(ctx->rd_ent_hint, E);
            if (E <= v.cap) break;
            if (attempt == 1) fail(ACC_E_STATE, "internal: range-deps output grew between passes");
        }
    } else {
        v.ent = ctx->get<uint64_t>("rd_ent", 0);
    }

    // ---- 4. per-txn RangeDeps: raw sizes and tiers, build into scratch, offsets, compaction
    Out o{};
    o.n = n; o.P = (uint32_t)P; o.key_off = key_off; o.rng_off = rng_off; o.q_out = v.q_out;
    o.ent = v.ent;
    o.txn_of_tpos = dict.batch_sorted ? nullptr : txn_of_tpos;
    o.rd_cnt = ctx->get<uint32_t>("rd_rd_cnt", n);
    o.u_cnt = ctx->get<uint32_t>("rd_u_cnt", n);
    o.a_cnt = ctx->get<uint64_t>("rd_a_cnt", n);
    uint64_t *m_raw = ctx->get<uint64_t>("rd_m_raw", n);
    uint32_t *tier = ctx->get<uint32_t>("rd_tier", n);
    uint64_t *raw_off = ctx->get<uint64_t>("rd_raw_off", (size_t)n + 1);
    uint32_t *thist = ctx->get<uint32_t>("rd_thist", 16);
    ACC_HIP(hipMemsetAsync(thist, 0, 16 * sizeof(uint32_t), st));
    launch(ctx, "rd_tsize", k_rd_tsize, dim3(grid_for(n, (size_t)BLOCK * RD_TS)), dim3(BLOCK), 0, n, o, m_raw, tier, thist);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, m_raw, raw_off, n, true, raw_off + n);
    o.raw_off = raw_off;
    // txns grouped by tier: one 8-bit radix pass (stable)
    uint64_t *tkey = ctx->get<uint64_t>("rd_tkey", n);
    launch(ctx, "rd_widen", k_widen_u32, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, (size_t)n, (const uint32_t *)tier, tkey);
    Sorted ts = radix_sort(ctx, "rs_rd_tier", tkey, nullptr, n, 4);
    uint32_t hh[16];
    ACC_HIP(hipMemcpyAsync(ctx->pinned, thist, 16 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    ctx->sync();
    memcpy(hh, ctx->pinned, sizeof hh);
    uint32_t toff[17];
    toff[0] = 0;
    for (int i = 0; i < 16; ++i) toff[i + 1] = toff[i] + hh[i];
    o.s_arena = ctx->get<uint32_t>("rd_s_arena", 2 * E);
    o.s_rid = ctx->get<uint32_t>("rd_s_rid", E);
    o.s_dep = ctx->get<uint32_t>("rd_s_dep", E);
    const uint32_t *tl_sorted = ts.vals;
    // 32-bit sort keys in the lane-group tiers: range ids (< NE) and TxnId positions (< n) within 26 bits
    const bool narrow = NE < (1u << 26) && n < (1u << 26) && !(ctx->flags & ACC_OPT_RD_WIDE_SORT);   // (testing: 64-bit sorts throughout)
    ctx->stat("rangedeps.narrow_sorts", narrow ? 1 : 0);
    // tiers own disjoint txns (disjoint scratch): LDS workgroup tiers on side stream 1, 16-lane groups on side
    // stream 0, waves on the main stream, all concurrently
    ctx->fork(2);
    if (hh[1]) {
        ctx->launch_stream = ctx->aux[0];
        o.list = tl_sorted + toff[1];
#ifdef ACC_PHASE_PROF
        const uint32_t pb16 = (hh[1] + RD_SEGK * 4 * WAVES - 1) / (RD_SEGK * 4 * WAVES);
        ctx->launch_stream = nullptr;
        unsigned long long *pf16 = rd_prof_arm(ctx, pb16);
#endif
        if (narrow)
            launch(ctx, "rd_build_s16", k_rd_build_seg<16, true, RD_SEGK>, dim3((hh[1] + RD_SEGK * 4 * WAVES - 1) / (RD_SEGK * 4 * WAVES)), dim3(BLOCK), 0, hh[1], o);
        else
            launch(ctx, "rd_build_s16", k_rd_build_seg<16, false, RD_SEGK>, dim3((hh[1] + RD_SEGK * 4 * WAVES - 1) / (RD_SEGK * 4 * WAVES)), dim3(BLOCK), 0, hh[1], o);
#ifdef ACC_PHASE_PROF
        rd_prof_print(ctx, "s16", pf16, pb16);
#endif
    }
    if (hh[11]) {
        ctx->launch_stream = ctx->aux[0];
        o.list = tl_sorted + toff[11];
#ifdef ACC_PHASE_PROF
        const uint32_t pb32 = (hh[11] + RD_SEGK * 2 * WAVES - 1) / (RD_SEGK * 2 * WAVES);
        ctx->launch_stream = nullptr;
        unsigned long long *pf32 = rd_prof_arm(ctx, pb32);
#endif
        if (narrow)
            launch(ctx, "rd_build_s32", k_rd_build_seg<32, true, RD_SEGK>, dim3((hh[11] + RD_SEGK * 2 * WAVES - 1) / (RD_SEGK * 2 * WAVES)), dim3(BLOCK), 0, hh[11], o);
        else
            launch(ctx, "rd_build_s32", k_rd_build_seg<32, false, RD_SEGK>, dim3((hh[11] + RD_SEGK * 2 * WAVES - 1) / (RD_SEGK * 2 * WAVES)), dim3(BLOCK), 0, hh[11], o);
#ifdef ACC_PHASE_PROF
        rd_prof_print(ctx, "s32", pf32, pb32);
#endif
    }
    uint64_t nblk = 0;
    ctx->launch_stream = ctx->aux[1];
    for (int b = 9; b >= 3; --b) {
        if (!hh[b]) continue;
        const uint32_t n2 = 128u << (b - 3);
        const size_t lds = 2 * (size_t)n2 * sizeof(uint64_t) + BLOCK * 8 + 64 + (BLOCK + 1) * 4;
        if (lds > 64 * 1024)
            ACC_HIP(hipFuncSetAttribute((const void *)k_rd_build_block, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        o.list = tl_sorted + toff[b];
        launch(ctx, "rd_build_block", k_rd_build_block, dim3(hh[b]), dim3(BLOCK), lds, o, n2);
        nblk += hh[b];
    }
    ctx->launch_stream = nullptr;
    if (hh[2]) {
        o.list = tl_sorted + toff[2];
#ifdef ACC_PHASE_PROF
        const uint32_t pb64 = (hh[2] + RD_SEGK * WAVES - 1) / (RD_SEGK * WAVES);
        ctx->launch_stream = nullptr;
        unsigned long long *pf64 = rd_prof_arm(ctx, pb64);
#endif
        if (narrow)
            launch(ctx, "rd_build_s64", k_rd_build_seg<64, true, RD_SEGK>, dim3((hh[2] + RD_SEGK * WAVES - 1) / (RD_SEGK * WAVES)), dim3(BLOCK), 0, hh[2], o);
        else
            launch(ctx, "rd_build_s64", k_rd_build_seg<64, false, RD_SEGK>, dim3((hh[2] + RD_SEGK * WAVES - 1) / (RD_SEGK * WAVES)), dim3(BLOCK), 0, hh[2], o);
#ifdef ACC_PHASE_PROF
        rd_prof_print(ctx, "s64", pf64, pb64);
#endif
    }
    ctx->join(2);
    const uint32_t nglb = hh[10];
    if (nglb) {
        o.list = tl_sorted + toff[10];
        uint64_t *gsz = ctx->get<uint64_t>("rd_glb_sz", nglb);
        uint64_t *goff = ctx->get<uint64_t>("rd_glb_off", (size_t)nglb + 1);
        launch(ctx, "rd_glb_sizes", k_rd_glb_sizes, dim3(grid_for(nglb, BLOCK)), dim3(BLOCK), 0, nglb, o, gsz);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, gsz, goff, nglb, true, goff + nglb);
        ACC_HIP(hipMemcpyAsync(ctx->pinned, goff + nglb, 8, hipMemcpyDeviceToHost, st));
        ctx->sync();
        o.glb_off = goff;
        o.gscratch = ctx->get<uint64_t>("rd_glb_scratch", ctx->pinned[0]);
        launch(ctx, "rd_build_global", k_rd_build_global, dim3(nglb), dim3(BLOCK), 0, o);
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
    if (n) launch(ctx, "rd_compact", k_rd_compact, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, o);
    ctx->stat("rangedeps.entries", NE);
    ctx->stat("rangedeps.stored_ranges", n_dict);
    ctx->stat("rangedeps.queries", Q);
    ctx->stat("rangedeps.raw_entries", E);
    ctx->stat("rangedeps.s16_txns", hh[1]);
    ctx->stat("rangedeps.s32_txns", hh[11]);
    ctx->stat("rangedeps.s64_txns", hh[2]);
    ctx->stat("rangedeps.block_txns", nblk);
    ctx->stat("rangedeps.global_txns", nglb);
    ctx->sync();
    *view = acc_rangedeps_view{ n, n_dict, tot_arena, tot_rd, tot_u, tot_arena - tot_rd, dict_s, dict_e, arena_off, o.arena,
                                rd_off, o.range_id, u_off, o.dep_txn };
    ctx->rd_view = *view;
    ctx->rd_valid = true;
}

}  // namespace acc
