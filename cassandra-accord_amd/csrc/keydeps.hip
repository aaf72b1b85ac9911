// keydeps.hip — batched PreAccept.calculatePartialDeps on CDNA4.
//
// For every txn T of a batch (one CommandsForKey snapshot), for every key k of T:
//   deps(T,k) = CommandsForKey.mapReduceActive(startedBefore = T.executeAt, T.kind().witnesses())
//               (local/CommandsForKey.java:614-650) minus p1 (messages/PreAccept.java:253-259),
// then the KeyDeps.Builder result (utils/RelationMultiMap.java:88-260) in Java layout.
//
// Pipeline (all on one HIP stream, three host syncs for sizes):
//   1. prep        validate, OR-reduce varying bits of TxnId/executeAt/key words, sortedness.
//   2. dictionary  compact the 148-bit Timestamp order key (Timestamp.compareTo :208-217) to its varying
//                  bits, radix-sort the 2N timestamps, dense order ranks (equal <=> Timestamp.equals).
//   3. CFK build   radix-sort (key, txnRank) pairs -> one segment per key = CommandsForKey.txns;
//                  committed[] per segment sorted by (executeAt rank, txn order) (ctor :459-469);
//                  lastWrite index, per-segment prefix-max of committed executeAt, uncommitted list.
//   4. scan        count -> exclusive scan -> emit. Each (T,k) query finds maxCommittedBefore with the
//                  reference's FAST bisection (SortedArrays.java:992-1027, replayed on ranks, so ties
//                  resolve identically), then only touches [scanStart, insertPos) plus the
//                  uncommitted entries before scanStart instead of the whole O(prefix).
//   5. build       per-T union of the per-key lists, indices into it, Java keysToTxnIds layout.
#include "dict.hpp"

#include <vector>

namespace acc {

// Timestamp words: w0 = msb (unsigned), w1 = lsb & IDENTITY_LSB (lowHlc then identity flags, unsigned
// compare is exact because lowHlc < 2^48), w2 = node ^ 0x80000000 (signed -> unsigned order).
constexpr uint64_t IDENTITY_LSB = 0xFFFFFFFFFFFF001EULL;

__device__ __forceinline__ uint64_t ts_w1(uint64_t lsb) { return lsb & IDENTITY_LSB; }
__device__ __forceinline__ uint64_t ts_w2(int32_t node) { return (uint64_t)((uint32_t)node ^ 0x80000000u); }

__device__ __forceinline__ int ts_cmp(uint64_t am, uint64_t al, int32_t an, uint64_t bm, uint64_t bl, int32_t bn)
{
    if (am != bm) return am < bm ? -1 : 1;
    uint64_t a1 = ts_w1(al), b1 = ts_w1(bl);
    if (a1 != b1) return a1 < b1 ? -1 : 1;
    if (an != bn) return an < bn ? -1 : 1;
    return 0;
}

// Kind.witnesses() as a bitmask over Kind ordinals (primitives/Txn.java:221-236); 0 = throws.
__device__ __forceinline__ uint32_t witnesses(uint32_t kind)
{
    switch (kind) {
    case 0: case 2: return 1u << 1;                                   // Read, EphemeralRead -> Ws
    case 1: case 3: return (1u << 0) | (1u << 1);                     // Write, SyncPoint -> RsOrWs
    case 4:         return (1u << 0) | (1u << 1) | (1u << 3) | (1u << 4);  // ESP -> AnyGloballyVisible
    default:        return 0;
    }
}

struct TsPlan {
    Runs r0, r1, r2;
    int b0, b1, b2;
};

enum : uint32_t {
    ERR_BAD_STATUS = 1u << 0,
    ERR_BAD_KIND = 1u << 1,
    ERR_LOCAL_ONLY = 1u << 2,
    ERR_KEYS_UNSORTED = 1u << 3,
    ERR_DUP_TXNID = 1u << 4,
    ERR_KEY_OFF = 1u << 5,
    ERR_KEY_TOTAL = 1u << 6,   // key_off[n] != n_pairs
};

// g[0..2] ts word masks, g[3] key mask, g[4] error bits, g[5] batch-not-in-TxnId-order flag.
// Block-level OR (wave shuffles, then LDS across waves) and ONE atomic per block and word: same-address
// atomics from every wave serialise at the L2 (1.4 ms for 8M pairs in the first build).
template <int NW>
__device__ __forceinline__ void block_or_n(uint64_t (&v)[NW], uint64_t *dst)
{
    __shared__ uint64_t part[WAVES][NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        uint64_t x = v[w];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) x |= shfl_idx(x, (int)(lane_id() ^ d));
        if (lane_id() == 0) part[threadIdx.x >> 6][w] = x;
    }
    __syncthreads();
    if (threadIdx.x < NW) {
        uint64_t x = 0;
#pragma unroll
        for (int q = 0; q < WAVES; ++q) x |= part[q][threadIdx.x];
        if (x) atomicOr((unsigned long long *)&dst[threadIdx.x], (unsigned long long)x);
    }
}

// Per txn: executeAt != TxnId flags, varying-bit masks, status / kind checks, TxnId order; per pair (a chunk's txns'
// pairs are one contiguous range, walked coalesced with each pair's txn found in the chunk's key offsets in LDS):
// owner[], key order within a txn (Keys.ofSortedUnique), the key-code varying-bit mask. Pair indices are bounded by P
// (a malformed key_off is reported, never followed out of bounds). One chunk of BLOCK txns per block (full occupancy:
// a few resident blocks per CU left every chunk's HBM round trips exposed, 0.11 ms for config 2); each block folds its
// words into one of PREP_SLOTS slot rows of g (same-address atomics serialise at the L2) and the host ORs the rows.
constexpr uint32_t PREP_SLOTS = 64;   // 64 x 8 words = ctx->pinned's slot area

__global__ __launch_bounds__(BLOCK) void k_prep_txn(uint32_t n, size_t P, const uint64_t *__restrict__ tm, const uint64_t *__restrict__ tl,
                                                    const int32_t *__restrict__ tn, const uint64_t *__restrict__ em,
                                                    const uint64_t *__restrict__ el, const int32_t *__restrict__ en,
                                                    const uint8_t *__restrict__ status, const uint32_t *__restrict__ key_off,
                                                    const uint64_t *__restrict__ key_code, uint32_t *__restrict__ owner,
                                                    uint32_t *__restrict__ bflag, uint64_t *__restrict__ g)
{
    __shared__ uint32_t ko[BLOCK + 1];
    const uint32_t tid = threadIdx.x;
    uint64_t m0 = 0, m1 = 0, m2 = 0, km = 0, errs = 0, unsorted = 0, ornk = 0;
    uint32_t differs = 0;
    const uint64_t r0 = tm[0], r1 = ts_w1(tl[0]), r2 = ts_w2(tn[0]);
    const uint64_t kref = P ? key_code[0] : 0;
    if (blockIdx.x == 0 && tid == 0 && key_off[n] != P) errs |= ERR_KEY_TOTAL;
    for (uint32_t t0 = blockIdx.x * BLOCK; t0 < n; t0 += gridDim.x * BLOCK) {
        const uint32_t t = t0 + tid;
        const uint32_t tcnt = min((uint32_t)BLOCK, n - t0);
        __syncthreads();   // the previous chunk's ko[] readers are done
        if (tid < tcnt) ko[tid] = key_off[t];
        if (tid == 0) ko[tcnt] = key_off[t0 + tcnt];
        if (t < n) {
            // executeAt != txnId (Timestamp.equals): these are the only executeAts the sorted-batch
            // dictionary has to sort
            const bool d = tm[t] != em[t] || ts_w1(tl[t]) != ts_w1(el[t]) || tn[t] != en[t];
            differs += d;
            bflag[t] = (uint32_t)d;
            m0 |= (tm[t] ^ r0) | (em[t] ^ r0);
            m1 |= (ts_w1(tl[t]) ^ r1) | (ts_w1(el[t]) ^ r1);
            m2 |= (ts_w2(tn[t]) ^ r2) | (ts_w2(en[t]) ^ r2);
            if (status[t] > 7) errs |= ERR_BAD_STATUS;
            uint32_t kind = (uint32_t)(tl[t] >> 1) & 7u;
            if (kind >= 6) errs |= ERR_BAD_KIND;
            else if (kind == 5) errs |= ERR_LOCAL_ONLY;
            if (t + 1 < n && ts_cmp(tm[t], tl[t], tn[t], tm[t + 1], tl[t + 1], tn[t + 1]) >= 0) unsorted = 1;
        }
        __syncthreads();
        const bool bad = tid < tcnt && ko[tid + 1] < ko[tid];
        if (bad) errs |= ERR_KEY_OFF;
        else if (tid < tcnt) ornk |= ko[tid + 1] - ko[tid];   // bounds the keys per txn (pair packing)
        if (!__syncthreads_or(bad ? 1 : 0) && P) {
            const uint32_t a = (uint32_t)min((size_t)ko[0], P), b = (uint32_t)min((size_t)ko[tcnt], P);
            for (uint32_t j = a + tid; j < b; j += BLOCK) {
                uint32_t lo = 0, hi = tcnt;   // last txn i with ko[i] <= j (empty txns share their offset with the next)
                while (hi - lo > 1) { const uint32_t m = (lo + hi) >> 1; if (ko[m] <= j) lo = m; else hi = m; }
                owner[j] = t0 + lo;
                const uint64_t kc = key_code[j];
                km |= kc ^ kref;
                if (j > ko[lo] && key_code[j - 1] >= kc) errs |= ERR_KEYS_UNSORTED;
            }
        }
    }
    uint64_t *gs = g + 8 * (blockIdx.x % PREP_SLOTS);
    uint64_t v[7] = { m0, m1, m2, km, errs, unsorted, ornk };
    block_or_n<7>(v, gs);
    __shared__ uint32_t s_nd;
    if (tid == 0) s_nd = 0;
    __syncthreads();
    if (differs) atomicAdd(&s_nd, differs);
    __syncthreads();
    if (tid == 0 && s_nd) atomicAdd((unsigned long long *)&gs[7], (unsigned long long)s_nd);
}

// ---- sorted-batch dictionary: TxnIds are already in order; only the differing executeAts (B) are sorted.
// rank(txnId_t) = t + |{b in B : b < txnId_t}|, rank(b_k) = k + |{txnIds < b_k}|; exact dense ranks when no
// executeAt equals another timestamp (checked here; otherwise the general sort recomputes them).
__global__ __launch_bounds__(BLOCK) void k_b_compact(uint32_t n, const uint32_t *__restrict__ bflag, const uint32_t *__restrict__ bidx,
                                                     const uint64_t *__restrict__ em, const uint64_t *__restrict__ el,
                                                     const int32_t *__restrict__ en, const uint64_t *__restrict__ tm,
                                                     const uint64_t *__restrict__ tl, const int32_t *__restrict__ tn,
                                                     TsPlan plan, uint64_t *__restrict__ bkey, uint32_t *__restrict__ bsrc,
                                                     uint64_t *__restrict__ tkey)
{
    uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= n) return;
    uint64_t c0 = pext_runs(tm[t], plan.r0), c1 = pext_runs(ts_w1(tl[t]), plan.r1), c2 = pext_runs(ts_w2(tn[t]), plan.r2);
    tkey[t] = (plan.b0 ? (c0 << (plan.b1 + plan.b2)) : 0) | (plan.b1 ? (c1 << plan.b2) : 0) | c2;
    if (bflag[t]) {
        c0 = pext_runs(em[t], plan.r0); c1 = pext_runs(ts_w1(el[t]), plan.r1); c2 = pext_runs(ts_w2(en[t]), plan.r2);
        uint32_t b = bidx[t];
        bkey[b] = (plan.b0 ? (c0 << (plan.b1 + plan.b2)) : 0) | (plan.b1 ? (c1 << plan.b2) : 0) | c2;
        bsrc[b] = t;
    }
}

__device__ __forceinline__ uint32_t lower_bound_u64(const uint64_t *a, uint32_t lo, uint32_t hi, uint64_t v)
{
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(BLOCK) void k_rank_txn_sorted(uint32_t n, uint32_t nb, const uint64_t *__restrict__ tkey,
                                                           const uint64_t *__restrict__ sb, const uint32_t *__restrict__ bflag,
                                                           uint32_t *__restrict__ rank, uint32_t *__restrict__ txn_of_rank,
                                                           uint64_t *__restrict__ g)
{
    uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    uint64_t tie = 0;
    if (t < n) {
        uint32_t lb = lower_bound_u64(sb, 0, nb, tkey[t]);
        if (lb < nb && sb[lb] == tkey[t]) tie = 1;
        uint32_t r = t + lb;
        rank[t] = r;
        txn_of_rank[r] = t;
        if (!bflag[t]) rank[n + t] = r;
    }
    uint64_t v[1] = { tie };
    block_or_n<1>(v, g + 6);
}

__global__ __launch_bounds__(BLOCK) void k_rank_b_sorted(uint32_t n, uint32_t nb, const uint64_t *__restrict__ tkey,
                                                         const uint64_t *__restrict__ sb, const uint32_t *__restrict__ sperm,
                                                         const uint32_t *__restrict__ bsrc, uint32_t *__restrict__ rank,
                                                         uint64_t *__restrict__ g)
{
    uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    uint64_t tie = 0;
    if (k < nb) {
        if (k > 0 && sb[k] == sb[k - 1]) tie = 1;
        uint32_t t = bsrc[sperm[k]];
        rank[n + t] = k + lower_bound_u64(tkey, 0, n, sb[k]);
    }
    uint64_t v[1] = { tie };
    block_or_n<1>(v, g + 6);
}

// ---------------------------------------------------------------- dictionary (order ranks)

// i < N: TxnId of txn i; i >= N: executeAt of txn i-N. word_sel < 0: whole compacted key (fits 64 bits);
// else the compaction of that single word.
__global__ __launch_bounds__(BLOCK) void k_ts_compact(uint32_t n, const uint64_t *__restrict__ tm, const uint64_t *__restrict__ tl,
                                                      const int32_t *__restrict__ tn, const uint64_t *__restrict__ em,
                                                      const uint64_t *__restrict__ el, const int32_t *__restrict__ en,
                                                      TsPlan plan, int word_sel, const uint32_t *__restrict__ perm,
                                                      uint64_t *__restrict__ out)
{
    size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= 2 * (size_t)n) return;
    size_t src = perm ? perm[i] : i;
    uint32_t t = (uint32_t)(src < n ? src : src - n);
    bool is_exec = src >= n;
    uint64_t w0 = is_exec ? em[t] : tm[t];
    uint64_t w1 = ts_w1(is_exec ? el[t] : tl[t]);
    uint64_t w2 = ts_w2(is_exec ? en[t] : tn[t]);
    uint64_t c0 = pext_runs(w0, plan.r0), c1 = pext_runs(w1, plan.r1), c2 = pext_runs(w2, plan.r2);
    uint64_t k;
    if (word_sel < 0) k = (plan.b0 ? (c0 << (plan.b1 + plan.b2)) : 0) | (plan.b1 ? (c1 << plan.b2) : 0) | c2;
    else k = word_sel == 0 ? c0 : word_sel == 1 ? c1 : c2;
    out[i] = k;
}

// flag[i] = sorted key i differs from key i-1 (all compacted words compared).
__global__ __launch_bounds__(BLOCK) void k_rank_flags(size_t m, const uint32_t *__restrict__ perm, const uint64_t *__restrict__ c0,
                                                      const uint64_t *__restrict__ c1, const uint64_t *__restrict__ c2,
                                                      const uint64_t *__restrict__ sorted_single, uint32_t *__restrict__ flag)
{
    size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= m) return;
    uint32_t f = 1;
    if (i > 0) {
        if (sorted_single) f = sorted_single[i] != sorted_single[i - 1];
        else {
            uint32_t a = perm[i], b = perm[i - 1];
            f = (c0[a] != c0[b]) || (c1[a] != c1[b]) || (c2[a] != c2[b]);
        }
    }
    flag[i] = f;
}

// rank[src] = inclusive(flag) - 1 (equal Timestamps share a rank); txn_of_rank for TxnId entries.
__global__ __launch_bounds__(BLOCK) void k_rank_scatter(size_t m, uint32_t n, const uint32_t *__restrict__ perm,
                                                        const uint32_t *__restrict__ incl, uint32_t *__restrict__ rank,
                                                        uint32_t *__restrict__ txn_of_rank)
{
    size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= m) return;
    uint32_t src = perm[i];
    uint32_t r = incl[i] - 1;
    rank[src] = r;
    if (src < n) txn_of_rank[r] = src;
}

// Count TxnId entries per rank to detect duplicate TxnIds (CommandsForKey txns are sorted unique).
__global__ __launch_bounds__(BLOCK) void k_dup_txn(uint32_t n, const uint32_t *__restrict__ rank, uint32_t *__restrict__ seen,
                                                   uint64_t *__restrict__ g)
{
    uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    uint64_t err = 0;
    if (t < n) {
        if (atomicAdd(&seen[rank[t]], 1u) != 0) err = ERR_DUP_TXNID;
    }
    uint64_t v[1] = { err };
    block_or_n<1>(v, g + 4);
}

// g[6] != 0: some executeAt compares equal to another txn's TxnId or executeAt. Only then can two
// committed entries of one key tie on executeAt, where the FAST bisection's pick (CommandsForKey.java:619)
// is order-dependent; such batches take the exact replay path (v1).
__global__ __launch_bounds__(BLOCK) void k_exec_ties(uint32_t n, const uint32_t *__restrict__ rank, uint32_t *__restrict__ seen,
                                                     uint64_t *__restrict__ g)
{
    uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    uint64_t tie = 0;
    if (t < n && rank[n + t] != rank[t]) {
        if (atomicAdd(&seen[rank[n + t]], 1u) != 0) tie = 1;
    }
    uint64_t v[1] = { tie };
    block_or_n<1>(v, g + 6);
}

// ---------------------------------------------------------------- CFK build

struct PairPlan {
    Runs rk;       // key code compaction
    int rbits;     // txn-rank bits in the composite (0 when the batch is already in TxnId order)
    int mode;      // 0: key only (sorted batch), 1: (key << rbits) | rank, 2: key only after a rank pre-sort,
                   // 3: (key << 32) | pair index, keys-only sort (sorted batch, key within 32 bits);
                   // 4: (key << 32) | owner << sb | slot (mode 3 with the pair's txn packed: the CFK columns gather the
                   //    16-MB txn records directly instead of a 16-B per-pair copy)
    int sb;        // mode 4: bits of the key slot within its txn
};

// the per-txn record k_txn_info writes, done by k_pair_keys' first n threads when tinfo is set (one launch fewer)
struct TxnInfoArgs {
    uint32_t n = 0;
    const uint8_t *status = nullptr;
    const uint64_t *tl = nullptr;
    uint4 *tinfo = nullptr;
    uint32_t *bigflag = nullptr;
};

__device__ __forceinline__ void txn_info_one(uint32_t t, uint32_t n, const uint32_t *rank, const uint8_t *status,
                                             const uint64_t *tl, const uint32_t *key_off, uint4 *tinfo, uint32_t *bigflag)
{
    if (bigflag) bigflag[t] = 0;
    const uint32_t kind = (uint32_t)(tl[t] >> 1) & 7u;
    tinfo[t] = make_uint4(rank[t], rank[n + t], (uint32_t)status[t] | (kind << 3), key_off[t]);
}

__global__ __launch_bounds__(BLOCK) void k_pair_keys(size_t P, const uint64_t *__restrict__ key_code,
                                                     const uint32_t *__restrict__ owner, const uint32_t *__restrict__ key_off,
                                                     const uint32_t *__restrict__ rank,
                                                     const uint32_t *__restrict__ perm, PairPlan plan,
                                                     int rank_only, uint64_t *__restrict__ out, TxnInfoArgs ti)
{
    size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (ti.tinfo && i < ti.n) txn_info_one((uint32_t)i, ti.n, rank, ti.status, ti.tl, key_off, ti.tinfo, ti.bigflag);
    if (i >= P) return;
    size_t j = perm ? perm[i] : i;
    if (rank_only) { out[i] = rank[owner[j]]; return; }
    uint64_t kc = pext_runs(key_code[j], plan.rk);
    if (plan.mode == 4) {
        const uint32_t t = owner[j];
        out[i] = (kc << 32) | ((uint64_t)t << plan.sb) | (uint64_t)(j - key_off[t]);
        return;
    }
    out[i] = plan.mode == 1 ? ((kc << plan.rbits) | rank[owner[j]]) : plan.mode == 3 ? ((kc << 32) | i) : kc;
}

// packed (key << 32 | pair index) sort output: segment-start flags and the permutation
// sb >= 0 (mode 4): the low word is owner << sb | slot; the pair index is key_off[owner] + slot, the owner goes to pown
__global__ __launch_bounds__(BLOCK) void k_seg_flags_packed(size_t P, const uint64_t *__restrict__ sp, uint32_t *__restrict__ flag,
                                                            uint32_t *__restrict__ perm, int sb, const uint32_t *__restrict__ key_off,
                                                            uint32_t *__restrict__ pown)
{
    size_t p = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p >= P) return;
    const uint64_t x = sp[p];
    flag[p] = p == 0 || (x >> 32) != (sp[p - 1] >> 32);
    if (sb < 0) { perm[p] = (uint32_t)x; return; }
    const uint32_t t = (uint32_t)x >> sb, slot = (uint32_t)x & ((1u << sb) - 1u);
    perm[p] = key_off[t] + slot;
    pown[p] = t;
}

__global__ __launch_bounds__(BLOCK) void k_seg_flags(size_t P, const uint64_t *__restrict__ skeys, int key_shift,
                                                     uint32_t *__restrict__ flag)
{
    size_t p = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p >= P) return;
    flag[p] = p == 0 || (skeys[p] >> key_shift) != (skeys[p - 1] >> key_shift);
}

// Gather per-position CFK columns; fill seg_start; classify committed (C) / uncommitted (U).
// per-txn record for the CFK gather: one 16-B random read per pair instead of four
// .w = key_off[t] (the CFK gather turns (owner, slot) into the pair index from the same 16-B read)
// also zeroes the count pass's big-txn flags (no memset launch)
__global__ __launch_bounds__(BLOCK) void k_txn_info(uint32_t n, const uint32_t *__restrict__ rank, const uint8_t *__restrict__ status,
                                                    const uint64_t *__restrict__ tl, const uint32_t *__restrict__ key_off,
                                                    uint4 *__restrict__ tinfo, uint32_t *__restrict__ bigflag)
{
    uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t < n) txn_info_one(t, n, rank, status, tl, key_off, tinfo, bigflag);
}

// per-pair copy of its txn's record, written in pair order (owner[] is monotone, so both reads stream): the CFK
// gather then does ONE random 16-B read per pair instead of the dependent owner[j] -> tinfo[owner[j]] pair
__global__ __launch_bounds__(BLOCK) void k_pair_tinfo(size_t P, const uint32_t *__restrict__ owner, const uint4 *__restrict__ tinfo,
                                                      uint4 *__restrict__ ptinfo)
{
    size_t j = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (j < P) ptinfo[j] = tinfo[owner[j]];
}

// inverse of the CFK permutation, only for the consumers that address pairs by index (exact replay, the global
// write tier, the range-domain KeyDeps): a random 4-B scatter per pair the common path does not pay
__global__ __launch_bounds__(BLOCK) void k_pair_pos(size_t P, const uint32_t *__restrict__ perm, uint32_t *__restrict__ pair_pos)
{
    size_t p = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p < P) pair_pos[perm[p]] = (uint32_t)p;
}

// v1 only: committed / uncommitted flags and the segmented prefix-max input
// multi_seg (non-null): committed[] lists only for segments of two or more entries (the mixed path answers
// single-entry segments without them, k_mx_pcount)
__global__ __launch_bounds__(BLOCK) void k_v1_flags(size_t P, const uint8_t *__restrict__ s_info, const uint32_t *__restrict__ s_exec,
                                                    const uint32_t *__restrict__ seg_incl, const uint32_t *__restrict__ multi_seg,
                                                    uint32_t *__restrict__ cflag, uint32_t *__restrict__ uflag,
                                                    uint64_t *__restrict__ pmax_in)
{
    size_t p = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p >= P) return;
    uint32_t st = s_info[p] & 7u;
    bool c = st >= 4 && st <= 6;
    if (multi_seg) {
        const uint32_t sg = seg_incl[p] - 1;
        cflag[p] = c && multi_seg[sg + 1] - multi_seg[sg] >= 2;
    } else {
        cflag[p] = c;
    }
    uflag[p] = st >= 1 && st <= 3;
    // segmented prefix-max via a segment-id prefix: max over (seg << 32 | exec+1) never crosses segments
    pmax_in[p] = ((uint64_t)(seg_incl[p] - 1) << 32) | (c ? (uint64_t)s_exec[p] + 1 : 0);
}

__global__ __launch_bounds__(BLOCK) void k_low32(size_t P, const uint64_t *__restrict__ in, uint32_t *__restrict__ out)
{
    size_t p = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p < P) out[p] = (uint32_t)in[p];
}
__global__ __launch_bounds__(BLOCK) void k_low32x2(size_t P, const uint64_t *__restrict__ a, uint32_t *__restrict__ a32,
                                                   const uint64_t *__restrict__ b, uint32_t *__restrict__ b32)
{
    size_t p = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p < P) { a32[p] = (uint32_t)a[p]; b32[p] = (uint32_t)b[p]; }
}

// Committed entries -> (seg << ebits | execRank) composite for the stable (seg, executeAt) sort; pads
// (all ones in `bits`) fill [NC, P) so the sort runs on the host-known size P.
__global__ __launch_bounds__(BLOCK) void k_committed_keys(size_t P, const uint32_t *__restrict__ cflag, const uint32_t *__restrict__ cum_c,
                                                          const uint32_t *__restrict__ seg_incl, const uint32_t *__restrict__ s_exec,
                                                          const uint32_t *__restrict__ uflag, const uint32_t *__restrict__ cum_u,
                                                          int ebits, int bits, uint64_t *__restrict__ ckey,
                                                          uint32_t *__restrict__ cpos, uint32_t *__restrict__ u_pos, int pads)
{
    size_t p = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p >= P) return;
    uint32_t nc = cum_c[P];
    if (cflag[p]) {
        uint32_t c = cum_c[p];
        ckey[c] = ((uint64_t)(seg_incl[p] - 1) << ebits) | s_exec[p];
        cpos[c] = (uint32_t)p;
    }
    if (pads && p >= nc) {
        ckey[p] = bits >= 64 ? ~0ull : ((1ull << bits) - 1);
        cpos[p] = 0xFFFFFFFFu;
    }
    if (uflag[p]) u_pos[cum_u[p]] = (uint32_t)p;
}

// cl_exec / lastWrite input / cl_start per segment.
__global__ __launch_bounds__(BLOCK) void k_committed_cols(size_t P, const uint32_t *__restrict__ cpos_sorted,
                                                          const uint32_t *__restrict__ s_exec, const uint8_t *__restrict__ s_info,
                                                          const uint32_t *__restrict__ cum_c, uint32_t *__restrict__ cl_exec,
                                                          uint32_t *__restrict__ lastw_in)
{
    size_t c = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (c >= P) return;
    uint32_t nc = cum_c[P];
    if (c >= nc) { lastw_in[c] = 0; return; }
    uint32_t p = cpos_sorted[c];
    cl_exec[c] = s_exec[p];
    // committed[i].kind().isWrite(): kind of the TxnId (CommandsForKey.java:623)
    lastw_in[c] = ((s_info[p] >> 3) == 1) ? (uint32_t)c + 1 : 0;
}

__global__ __launch_bounds__(BLOCK) void k_seg_committed_start(size_t P, const uint32_t *__restrict__ seg_incl,
                                                               const uint32_t *__restrict__ seg_start, const uint32_t *__restrict__ cum_c,
                                                               uint32_t *__restrict__ cl_start)
{
    size_t s = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    uint32_t nseg = seg_incl[P - 1];
    if (s > nseg) return;
    cl_start[s] = s == nseg ? cum_c[P] : cum_c[seg_start[s]];
}

// ---------------------------------------------------------------- the conflict scan

struct CfkView {
    const uint32_t *seg_start, *s_rank, *s_exec, *seg_incl, *pair_pos, *owner, *rank;
    const uint8_t *s_info;
    const uint32_t *cl_start, *cl_exec, *lastw;   // lastw = inclusive max-scan of (isWrite ? c+1 : 0)
    const uint32_t *pmax;                          // low 32 bits of the segmented prefix max (exec+1)
    const uint32_t *cum_u, *u_pos;
    const uint64_t *tl;
    uint32_t n;
    const uint32_t *vseg;   // non-null: query j is (owner[j], segment vseg[j]) (range-domain txns, no CFK member)
};

struct Query {
    uint32_t s0, pos, scan_start, ub, ue, trank, wk;
    bool p1, has_m;
    uint32_t m;
};

__device__ __forceinline__ uint32_t lower_bound_u32(const uint32_t *a, uint32_t lo, uint32_t hi, uint32_t v)
{
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ Query make_query_ts(const CfkView &v, uint32_t t, uint32_t seg);

// first i in [lo, hi) with (uint32_t)a[i] >= v, the low words ascending over the range (one segment's prefix maxima)
__device__ __forceinline__ uint32_t lower_bound_lo32(const uint64_t *a, uint32_t lo, uint32_t hi, uint32_t v)
{
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if ((uint32_t)a[m] < v) lo = m + 1; else hi = m;
    }
    return lo;
}

__device__ __forceinline__ Query make_query(const CfkView &v, uint32_t j)
{
    return make_query_ts(v, v.owner[j], v.vseg ? v.vseg[j] : v.seg_incl[v.pair_pos[j]] - 1);
}

// the query of txn t against CFK segment seg
__device__ __forceinline__ Query make_query_ts(const CfkView &v, uint32_t t, uint32_t seg)
{
    Query q;
    uint32_t s0 = v.seg_start[seg], s1 = v.seg_start[seg + 1];
    uint32_t S = v.rank[v.n + t];          // startedBefore = T.executeAt
    q.trank = v.rank[t];
    q.p1 = S != q.trank;                   // p1 = executeAt.equals(txnId) ? null : txnId
    q.wk = witnesses((uint32_t)(v.tl[t] >> 1) & 7u);
    q.s0 = s0;
    // insertPos(0, startedBefore): first txn with TxnId >= S (CommandsForKey.java:1698-1703)
    q.pos = lower_bound_u32(v.s_rank, s0, s1, S);
    // maxCommittedBefore (CommandsForKey.java:618-625): FAST bisection of S over committed[] by executeAt
    uint32_t c0 = v.cl_start[seg], c1 = v.cl_start[seg + 1];
    uint32_t from = c0, to = c1;
    long i = -1;
    bool found = false;
    while (from < to) {
        uint32_t mid = (from + to) >> 1;
        uint32_t e = v.cl_exec[mid];
        if (S < e) to = mid;
        else if (S > e) from = mid + 1;
        else { i = (long)mid - 1; found = true; break; }
    }
    if (!found) i = (long)to - 1;
    q.has_m = false;
    q.m = 0;
    if (i >= (long)c0) {
        uint32_t w = v.lastw[i];           // greatest Write index <= i, +1 (0: none anywhere before)
        if (w != 0 && w - 1 >= c0) { q.has_m = true; q.m = v.cl_exec[w - 1]; }
    }
    // Committed entries below scanStart all have executeAt < M (prefix max < M): pruned
    q.scan_start = q.has_m ? lower_bound_u32(v.pmax, s0, q.pos, q.m + 1) : s0;
    q.ub = v.cum_u[s0];
    q.ue = v.cum_u[q.scan_start];
    return q;
}

// EMIT: every entry to out[0..c); FIRST (count pass): only the first entry, to out[0]
template <bool EMIT, bool FIRST = false>
__device__ __forceinline__ uint32_t run_query(const CfkView &v, const Query &q, uint32_t *__restrict__ out)
{
    uint32_t c = 0;
    // uncommitted (HISTORICAL / PREACCEPTED / ACCEPTED) entries below scanStart: always witnessed
    for (uint32_t u = q.ub; u < q.ue; ++u) {
        uint32_t p = v.u_pos[u];
        uint32_t kind = v.s_info[p] >> 3;
        if (!((q.wk >> kind) & 1u)) continue;
        uint32_t r = v.s_rank[p];
        if (q.p1 && r == q.trank) continue;
        if (EMIT) out[c] = r;
        else if (FIRST && c == 0) out[0] = r;
        ++c;
    }
    // [scanStart, insertPos): the reference's per-entry switch (CommandsForKey.java:628-647)
    for (uint32_t p = q.scan_start; p < q.pos; ++p) {
        uint32_t info = v.s_info[p];
        uint32_t st = info & 7u, kind = info >> 3;
        if (!((q.wk >> kind) & 1u)) continue;
        if (st == 0 || st == 7) continue;                                    // TRANSITIVELY_KNOWN, INVALID
        if (st >= 4 && st <= 6 && q.has_m && v.s_exec[p] < q.m) continue;   // pruned committed
        uint32_t r = v.s_rank[p];
        if (q.p1 && r == q.trank) continue;
        if (EMIT) out[c] = r;
        else if (FIRST && c == 0) out[0] = r;
        ++c;
    }
    return c;
}

__global__ __launch_bounds__(BLOCK) void k_query_count(size_t P, CfkView v, uint64_t *__restrict__ cnt)
{
    size_t j = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (j >= P) return;
    Query q = make_query(v, (uint32_t)j);
    cnt[j] = run_query<false>(v, q, nullptr);
}

__global__ __launch_bounds__(BLOCK) void k_query_emit(size_t P, CfkView v, const uint64_t *__restrict__ dep_off,
                                                      uint32_t *__restrict__ deps, uint32_t *__restrict__ list_of)
{
    size_t j = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (j >= P) return;
    Query q = make_query(v, (uint32_t)j);
    uint64_t o = dep_off[j];
    uint32_t c = run_query<true>(v, q, deps + o);
    for (uint32_t k = 0; k < c; ++k) list_of[o + k] = (uint32_t)j;
}

// ---------------------------------------------------------------- KeyDeps assembly

__device__ __forceinline__ bool contains_u32(const uint32_t *a, uint64_t lo, uint64_t hi, uint32_t v)
{
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        uint32_t x = a[mid];
        if (x < v) lo = mid + 1;
        else if (x > v) hi = mid;
        else return true;
    }
    return false;
}

__device__ __forceinline__ uint64_t lower_bound_u32_64(const uint32_t *a, uint64_t lo, uint64_t hi, uint32_t v)
{
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// first[e] = dep is not in an earlier key's list of the same txn (the union keeps one copy).
__global__ __launch_bounds__(BLOCK) void k_first(uint64_t E, const uint32_t *__restrict__ deps, const uint32_t *__restrict__ list_of,
                                                 const uint32_t *__restrict__ owner, const uint32_t *__restrict__ key_off,
                                                 const uint64_t *__restrict__ dep_off, uint32_t *__restrict__ first)
{
    uint64_t e = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e >= E) return;
    uint32_t j = list_of[e];
    uint32_t t = owner[j];
    uint32_t d = deps[e];
    uint32_t f = 1;
    for (uint32_t jj = key_off[t]; jj < j; ++jj)
        if (contains_u32(deps, dep_off[jj], dep_off[jj + 1], d)) { f = 0; break; }
    first[e] = f;
}

__global__ __launch_bounds__(BLOCK) void k_nonempty(size_t P, const uint64_t *__restrict__ cnt, uint32_t *__restrict__ nz)
{
    size_t j = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (j < P) nz[j] = cnt[j] != 0;
}

__global__ __launch_bounds__(BLOCK) void k_txn_sizes(uint32_t n, const uint32_t *__restrict__ key_off, const uint64_t *__restrict__ dep_off,
                                                     const uint32_t *__restrict__ cnz, const uint32_t *__restrict__ cumf,
                                                     uint64_t *__restrict__ kd_cnt, uint64_t *__restrict__ u_cnt,
                                                     uint64_t *__restrict__ a_cnt)
{
    uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= n) return;
    uint32_t j0 = key_off[t], j1 = key_off[t + 1];
    uint64_t e0 = dep_off[j0], e1 = dep_off[j1];
    uint64_t kd = cnz[j1] - cnz[j0];
    kd_cnt[t] = kd;
    u_cnt[t] = cumf[e1] - cumf[e0];
    a_cnt[t] = kd + (e1 - e0);
}

// arena indices (KeyDeps.keysToTxnIds value part) and KeyDeps.txnIds (as batch indices)
__global__ __launch_bounds__(BLOCK) void k_write_entries(uint64_t E, const uint32_t *__restrict__ deps, const uint32_t *__restrict__ list_of,
                                                         const uint32_t *__restrict__ owner, const uint32_t *__restrict__ key_off,
                                                         const uint64_t *__restrict__ dep_off, const uint32_t *__restrict__ cumf,
                                                         const uint32_t *__restrict__ first, const uint32_t *__restrict__ cnz,
                                                         const uint64_t *__restrict__ arena_off, const uint64_t *__restrict__ u_off,
                                                         const uint32_t *__restrict__ txn_of_rank, int32_t *__restrict__ arena,
                                                         uint32_t *__restrict__ dep_txn)
{
    uint64_t e = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e >= E) return;
    uint32_t j = list_of[e];
    uint32_t t = owner[j];
    uint32_t d = deps[e];
    uint32_t j0 = key_off[t], j1 = key_off[t + 1];
    // index of d in the sorted union = number of distinct deps of T smaller than d
    uint32_t idx = 0;
    for (uint32_t jj = j0; jj < j1; ++jj) {
        uint64_t a = dep_off[jj], b = dep_off[jj + 1];
        if (a == b) continue;
        uint64_t lb = jj == j ? e : lower_bound_u32_64(deps, a, b, d);
        idx += cumf[lb] - cumf[a];
    }
    uint32_t kd = cnz[j1] - cnz[j0];
    uint64_t base = dep_off[j0];
    arena[arena_off[t] + kd + (e - base)] = (int32_t)idx;
    if (first[e]) dep_txn[u_off[t] + idx] = txn_of_rank[d];
}

// per non-empty (T,k): KeyDeps.keys entry and the end-offset header int (KeyDeps.java:150-172)
__global__ __launch_bounds__(BLOCK) void k_write_keys(size_t P, const uint64_t *__restrict__ cnt, const uint32_t *__restrict__ owner,
                                                      const uint32_t *__restrict__ key_off, const uint64_t *__restrict__ dep_off,
                                                      const uint32_t *__restrict__ cnz, const uint64_t *__restrict__ kd_off,
                                                      const uint64_t *__restrict__ arena_off, uint32_t *__restrict__ key_idx,
                                                      int32_t *__restrict__ arena)
{
    size_t j = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (j >= P || cnt[j] == 0) return;
    uint32_t t = owner[j];
    uint32_t j0 = key_off[t], j1 = key_off[t + 1];
    uint32_t slot = cnz[j] - cnz[j0];
    uint32_t kd = cnz[j1] - cnz[j0];
    key_idx[kd_off[t] + slot] = (uint32_t)j - j0;
    arena[arena_off[t] + slot] = (int32_t)(kd + (dep_off[j + 1] - dep_off[j0]));
}

// ---------------------------------------------------------------- v2: run-based conflict scan
//
// Without executeAt ties (k_exec_ties), the reference scan of (T, k) equals the union of three kinds of
// sorted runs over the CFK segment (positions [s0, s1) in TxnId order), with S = T.executeAt,
// pos = insertPos(S), M = maxCommittedBefore and posM = first position with TxnId >= M:
//   R1[c]: uncommitted (HISTORICAL/PREACCEPTED/ACCEPTED) entries of kind class c in [s0, pos)
//   R2[c]: committed entries of kind class c in [posM, pos)   (TxnId >= M  =>  executeAt >= M)
//   R3   : committed entries before posM with executeAt >= M  (only "bumped" ones, executeAt != TxnId)
// for every class c witnessed by T.kind, minus T itself (p1). Runs are ranges of per-class position
// lists, so counts are O(1) prefix differences. M = max(last unbumped committed Write before pos
// [segmented prefix max], predecessor of S among bumped committed Writes [small sorted list]).

constexpr int NLIST = 6;   // U_R, U_W, U_S, C_R, C_W, C_S
constexpr int NCNT = 9;    // 6 list counts, bumped-committed count, last-unbumped-committed-write max, segment starts
constexpr int NRD = 8;     // the rank directory's columns (all but the segment count)
__device__ __forceinline__ bool cnt_is_max(int q) { return q == 7; }

// Kind class for the Kinds predicates (Txn.java:140-152): Read 0, Write 1, SyncPoint/ExclusiveSyncPoint 2;
// EphemeralRead and LocalOnly are witnessed by no predicate (3 = none).
__device__ __forceinline__ uint32_t kind_class(uint32_t kind)
{
    return kind == 0 ? 0u : kind == 1 ? 1u : (kind == 3 || kind == 4) ? 2u : 3u;
}
// witness mask over kinds -> mask over classes
__device__ __forceinline__ uint32_t wk_classes(uint32_t wk)
{
    return (wk & 1u) | (((wk >> 1) & 1u) << 1) | (((wk >> 3) & 1u) << 2);
}

// per-position code: bits 0-2 list id (7 = none), bit 3 bumped committed (class < 3), bit 4 unbumped committed Write
__device__ __forceinline__ uint32_t v2_code(uint32_t rank, uint32_t exec, uint32_t info)
{
    uint32_t st = info & 7u, kind = info >> 3, cls = kind_class(kind);
    bool u = st >= 1 && st <= 3, c = st >= 4 && st <= 6;
    uint32_t list = cls < 3 ? (u ? cls : c ? 3 + cls : 7u) : 7u;
    uint32_t bc = (c && cls < 3 && exec != rank) ? 1u : 0u;
    uint32_t ucw = (c && kind == 1 && exec == rank) ? 1u : 0u;
    return list | (bc << 3) | (ucw << 4);
}

constexpr int V2_ITEMS = 4;               // consecutive positions per thread: one 16-B load per column
constexpr int V2_TILE = BLOCK * V2_ITEMS;

// 4 consecutive positions' codes (s_rank / s_exec / s_info are allocated with 4 entries of padding)
// bqm: bit i set when position base + i is a bumped query (executeAt != TxnId)
__device__ __forceinline__ void v2_codes4(size_t P, size_t base, const uint32_t *__restrict__ s_rank, const uint32_t *__restrict__ s_exec,
                                          const uint8_t *__restrict__ s_info, uint32_t (&code)[V2_ITEMS], uint32_t (&rk)[V2_ITEMS],
                                          uint32_t &bqm)
{
    uint4 r = *reinterpret_cast<const uint4 *>(s_rank + base);
    uint4 e = *reinterpret_cast<const uint4 *>(s_exec + base);
    uint32_t inf = *reinterpret_cast<const uint32_t *>(s_info + base);
    rk[0] = r.x; rk[1] = r.y; rk[2] = r.z; rk[3] = r.w;
    const uint32_t ex[4] = { e.x, e.y, e.z, e.w };
    bqm = 0;
#pragma unroll
    for (int i = 0; i < V2_ITEMS; ++i) {
        code[i] = base + i < P ? v2_code(rk[i], ex[i], (inf >> (8 * i)) & 0xFFu) : 7u;
        bqm |= (base + i < P && ex[i] != rk[i] ? 1u : 0u) << i;
    }
}

// The CFK columns of four consecutive positions per thread (s_rank / s_exec / s_info from the per-pair txn records, the
// segment starts, optionally pair_pos) and the per-tile counts of the class lists (the multi-scan's reduce step) over
// the same 1024-position tile that k_v2_apply scans.
// pown (mode 4): each position's owner txn, its record read from tinfo (16 B per txn) instead of ptinfo (per pair)
// sp (mode 4, sb >= 0): the sorted packed pair keys (key << 32 | owner << sb | slot) are unpacked here: the segment
// flags and the pair index perm = key_off[owner] + slot are written, key_off[owner] coming with the owner's record
// (tinfo[t].w), so each pair costs one random 16-B read. Otherwise perm / seg_flag are inputs and the record is
// ptinfo[perm].
__global__ __launch_bounds__(BLOCK) void k_cfk_gather4(size_t P, uint32_t *__restrict__ perm, const uint4 *__restrict__ ptinfo,
                                                       const uint64_t *__restrict__ sp, int sb, const uint4 *__restrict__ tinfo,
                                                       uint32_t *__restrict__ seg_flag, uint32_t *__restrict__ s_rank,
                                                       uint32_t *__restrict__ s_exec, uint8_t *__restrict__ s_info,
                                                       uint32_t *__restrict__ pair_pos, uint32_t *__restrict__ tile_sums,
                                                       uint32_t ntiles)
{
    __shared__ uint32_t lds[WAVES];
    const size_t base = (size_t)blockIdx.x * V2_TILE + (size_t)threadIdx.x * V2_ITEMS;
    uint32_t c[NCNT] = {};
    if (base < P) {
        uint32_t j[V2_ITEMS], fl[V2_ITEMS];
        uint4 ti[V2_ITEMS];
        if (sp) {
            uint64_t x[V2_ITEMS];
            const uint64_t xp = base > 0 ? sp[base - 1] : 0;
#pragma unroll
            for (int i = 0; i < V2_ITEMS; ++i) x[i] = base + i < P ? sp[base + i] : 0;
            const uint32_t smask = (1u << sb) - 1u;
#pragma unroll
            for (int i = 0; i < V2_ITEMS; ++i) {
                const bool in = base + i < P;
                const uint64_t prev = i == 0 ? xp : x[i - 1];
                fl[i] = in && (base + i == 0 || (x[i] >> 32) != (prev >> 32)) ? 1u : 0u;
                ti[i] = in ? tinfo[(uint32_t)x[i] >> sb] : make_uint4(0u, 0u, 0u, 0u);
            }
#pragma unroll
            for (int i = 0; i < V2_ITEMS; ++i) j[i] = ti[i].w + ((uint32_t)x[i] & smask);
            if (base + V2_ITEMS <= P) {
                *reinterpret_cast<uint4 *>(seg_flag + base) = make_uint4(fl[0], fl[1], fl[2], fl[3]);
                *reinterpret_cast<uint4 *>(perm + base) = make_uint4(j[0], j[1], j[2], j[3]);
            } else {
#pragma unroll
                for (int i = 0; i < V2_ITEMS; ++i)
                    if (base + i < P) { seg_flag[base + i] = fl[i]; perm[base + i] = j[i]; }
            }
        } else {
#pragma unroll
            for (int i = 0; i < V2_ITEMS; ++i) {
                const bool in = base + i < P;
                j[i] = in ? perm[base + i] : 0u;
                fl[i] = in ? seg_flag[base + i] : 0u;
            }
#pragma unroll
            for (int i = 0; i < V2_ITEMS; ++i) ti[i] = base + i < P ? ptinfo[j[i]] : make_uint4(0u, 0u, 0u, 0u);
        }
        uint32_t inf = 0;
#pragma unroll
        for (int i = 0; i < V2_ITEMS; ++i) {
            const size_t p = base + i;
            if (p >= P) break;
            if (pair_pos) pair_pos[j[i]] = (uint32_t)p;
            c[8] += fl[i] != 0;
            inf |= (ti[i].z & 0xFFu) << (8 * i);
            const uint32_t code = v2_code(ti[i].x, ti[i].y, ti[i].z & 0xFFu);
            const uint32_t l = code & 7u;
#pragma unroll
            for (int q = 0; q < NLIST; ++q) c[q] += l == (uint32_t)q;
            c[6] += (code >> 3) & 1u;
            if ((code >> 4) & 1u) c[7] = (uint32_t)p + 1;
        }
        // the column arrays carry V2_ITEMS entries of padding: whole 16-B / 4-B stores
        *reinterpret_cast<uint4 *>(s_rank + base) = make_uint4(ti[0].x, ti[1].x, ti[2].x, ti[3].x);
        *reinterpret_cast<uint4 *>(s_exec + base) = make_uint4(ti[0].y, ti[1].y, ti[2].y, ti[3].y);
        *reinterpret_cast<uint32_t *>(s_info + base) = inf;
    }
#pragma unroll
    for (int q = 0; q < NCNT; ++q) {
        uint32_t total;
        if (!cnt_is_max(q)) block_exclusive(c[q], OpAdd<uint32_t>(), lds, total);
        else block_exclusive(c[q], OpMax<uint32_t>(), lds, total);
        if (threadIdx.x == 0) tile_sums[(size_t)q * ntiles + blockIdx.x] = total;
    }
}

// The per-position prefix columns as a rank directory: one 64-B chunk per RD_W = 32 CFK positions, = one HBM line
// (16 MB at config 2's 8M positions, instead of a 32-B row per position): words 0-7 = the 8 running values at the
// chunk's first position (exclusive prefix counts of the 6 class lists, the bumped-committed count, the last unbumped
// committed Write as pos+1: prefix max), words 8-15 = one bit plane per column over the chunk's positions (list
// membership, bumped committed, unbumped committed Write). A query's "row" at p is the chunk's running values plus the
// popcounts of the planes below p (the last set bit for the Write column): one line read and a few ALU ops.
constexpr int RW_CBC = 6, RW_LUCW = 7;
constexpr uint32_t RD_W = 32;

struct V2Cols {
    uint4 *rdir;          // [P / RD_W + 1] chunks of 16 u32, as 4 x uint4
    uint32_t *list_rank;  // class lists (TxnId ranks), list l at bases[l]
    uint32_t *bc_rank, *bc_exec;  // bumped committed, position order
    uint8_t *bc_kind;
    uint64_t *bc_pm_in;   // (seg << 32) | exec+1, for the segmented prefix max
    uint64_t *bc_key;     // (seg << rbits) | exec, for the (seg, executeAt) sort
};

__global__ __launch_bounds__(BLOCK) void k_v2_apply(size_t P, const uint32_t *__restrict__ s_rank, const uint32_t *__restrict__ s_exec,
                                                    const uint8_t *__restrict__ s_info, const uint32_t *__restrict__ seg_flag,
                                                    const uint32_t *__restrict__ tile_pref, const uint32_t *__restrict__ totals,
                                                    uint32_t ntiles, int rbits, V2Cols o, uint32_t *__restrict__ seg_incl,
                                                    uint32_t *__restrict__ seg_start, const uint32_t *__restrict__ perm,
                                                    const uint64_t *__restrict__ key_code, uint64_t *__restrict__ seg_key,
                                                    const uint64_t *__restrict__ sp, Runs krun, uint64_t rk_mask,
                                                    uint32_t *__restrict__ bases, uint64_t *__restrict__ z0, uint32_t nz0,
                                                    uint64_t *__restrict__ z1, uint32_t nz1, const uint64_t *__restrict__ g,
                                                    uint64_t *__restrict__ stage)
{
    __shared__ uint32_t lds[WAVES];
    if (blockIdx.x == 0) {
        // the list bases for the count pass (list l at [bases[l], bases[l] + totals[l]) of the class-list arrays), the
        // count / mark passes' accumulators zeroed, the dictionary's error / tie words staged beside the totals
        if (threadIdx.x == 0) {
            uint32_t b = 0;
            for (int l = 0; l < NLIST; ++l) { bases[l] = b; b += totals[l]; }
            bases[NLIST] = b;
        }
        for (uint32_t i = threadIdx.x; i < nz0; i += BLOCK) z0[i] = 0;
        for (uint32_t i = threadIdx.x; i < nz1; i += BLOCK) z1[i] = 0;
        if (threadIdx.x < 3) stage[threadIdx.x] = g[4 + threadIdx.x];
    }
    const size_t base = (size_t)blockIdx.x * V2_TILE + (size_t)threadIdx.x * V2_ITEMS;
    uint32_t code[V2_ITEMS] = { 7u, 7u, 7u, 7u }, rk[V2_ITEMS] = {};
    uint32_t c[NCNT] = {};
    uint32_t fl[V2_ITEMS] = {};
    uint64_t kc[V2_ITEMS] = {};
    uint32_t bqm = 0;
    if (base < P) {
        v2_codes4(P, base, s_rank, s_exec, s_info, code, rk, bqm);
#pragma unroll
        for (int i = 0; i < V2_ITEMS; ++i) {
            uint32_t l = code[i] & 7u;
#pragma unroll
            for (int q = 0; q < NLIST; ++q) c[q] += l == (uint32_t)q;
            c[6] += (code[i] >> 3) & 1u;
            if ((code[i] >> 4) & 1u) c[7] = (uint32_t)(base + i) + 1;
            fl[i] = base + i < P ? seg_flag[base + i] : 0u;
            c[8] += fl[i] != 0;
        }
        if (seg_key && sp) {
            // mode 4: the key code from the sorted pair key itself (its compacted bits deposited back over key_code[0]'s
            // constant bits; the varying bits all lie in the runs), a sequential read instead of a gather
            const uint64_t kconst = key_code[0] & ~rk_mask;
#pragma unroll
            for (int i = 0; i < V2_ITEMS; ++i)
                if (fl[i]) {
                    const uint64_t c = sp[base + i] >> 32;
                    uint64_t w = kconst;
                    for (int r = 0; r < krun.n; ++r) {
                        const uint64_t m = krun.len[r] >= 64 ? ~0ull : ((1ull << krun.len[r]) - 1);
                        w |= ((c >> krun.dst[r]) & m) << krun.lo[r];
                    }
                    kc[i] = w;
                }
        } else if (seg_key) {   // segment starts' key codes: the gathers issued here, their latency hidden by the block scans
            uint32_t pi[V2_ITEMS] = {};
            if (base + V2_ITEMS <= P) {
                const uint4 pv = *reinterpret_cast<const uint4 *>(perm + base);
                pi[0] = pv.x; pi[1] = pv.y; pi[2] = pv.z; pi[3] = pv.w;
            } else {
                for (int i = 0; i < V2_ITEMS; ++i) if (base + i < P) pi[i] = perm[base + i];
            }
#pragma unroll
            for (int i = 0; i < V2_ITEMS; ++i) if (fl[i]) kc[i] = key_code[pi[i]];
        }
    }
    uint32_t run[NCNT];
#pragma unroll
    for (int q = 0; q < NCNT; ++q) {
        uint32_t total;
        uint32_t pre = tile_pref[(size_t)q * ntiles + blockIdx.x];
        if (!cnt_is_max(q)) run[q] = pre + block_exclusive(c[q], OpAdd<uint32_t>(), lds, total);
        else { uint32_t e = block_exclusive(c[q], OpMax<uint32_t>(), lds, total); run[q] = e > pre ? e : pre; }
    }
    // rank directory: the chunk's running values from its first thread (RD_W / V2_ITEMS = 8 threads per chunk), the bit
    // planes OR-reduced over those 8 threads (threads past P contribute nothing)
    static_assert(RD_W == 8 * V2_ITEMS, "eight threads per directory chunk");
    {
        uint32_t pl[NRD] = {};
#pragma unroll
        for (int i = 0; i < V2_ITEMS; ++i) {
            const uint32_t l = code[i] & 7u;
#pragma unroll
            for (int q = 0; q < NLIST; ++q) pl[q] |= (l == (uint32_t)q ? 1u : 0u) << i;
            pl[6] |= ((code[i] >> 3) & 1u) << i;
            pl[7] |= ((code[i] >> 4) & 1u) << i;
        }
        const uint32_t sh = V2_ITEMS * (threadIdx.x & 7u);
#pragma unroll
        for (int q = 0; q < NRD; ++q) {
            uint32_t x = pl[q] << sh;
            x |= __shfl_xor(x, 1, 64);
            x |= __shfl_xor(x, 2, 64);
            x |= __shfl_xor(x, 4, 64);
            pl[q] = x;
        }
        if ((threadIdx.x & 7u) == 0 && base < P) {
            uint4 *ch = o.rdir + 4 * (base / RD_W);
            ch[0] = make_uint4(run[0], run[1], run[2], run[3]);
            ch[1] = make_uint4(run[4], run[5], run[6], run[7]);
            ch[2] = make_uint4(pl[0], pl[1], pl[2], pl[3]);
            ch[3] = make_uint4(pl[4], pl[5], pl[6], pl[7]);
        }
    }
    if (base >= P) return;
    uint32_t lb[NLIST];
    {
        uint32_t b = 0;
#pragma unroll
        for (int l = 0; l < NLIST; ++l) { lb[l] = b; b += totals[l]; }
    }
    uint32_t segi[V2_ITEMS];
#pragma unroll
    for (int i = 0; i < V2_ITEMS; ++i) {   // segment numbers (seg_incl = inclusive count of segment starts) and starts
        const size_t p = base + i;
        if (p >= P) break;
        if (fl[i]) {
            seg_start[run[8]] = (uint32_t)p;
            if (seg_key) seg_key[run[8]] = kc[i];   // the segment's key code (range-domain queries)
        }
        run[8] += fl[i] != 0;
        segi[i] = run[8];
        if (p == P - 1) seg_start[run[8]] = (uint32_t)P;
    }
    if (base + V2_ITEMS <= P) *reinterpret_cast<uint4 *>(seg_incl + base) = make_uint4(segi[0], segi[1], segi[2], segi[3]);
    else for (int i = 0; i < V2_ITEMS; ++i) if (base + i < P) seg_incl[base + i] = segi[i];
#pragma unroll
    for (int i = 0; i < V2_ITEMS; ++i) {
        size_t p = base + i;
        if (p >= P) break;
        uint32_t l = code[i] & 7u;
        uint32_t r = rk[i];
        if (l < NLIST) {
            uint32_t idx = 0;
#pragma unroll
            for (int q = 0; q < NLIST; ++q) if ((uint32_t)q == l) idx = lb[q] + run[q];
            o.list_rank[idx] = r;
#pragma unroll
            for (int q = 0; q < NLIST; ++q) run[q] += (uint32_t)q == l;
        }
        if ((code[i] >> 3) & 1u) {
            uint32_t b = run[6]++;
            uint32_t seg = segi[i] - 1, e = s_exec[p];
            o.bc_rank[b] = r;
            o.bc_exec[b] = e;
            o.bc_kind[b] = (uint8_t)(s_info[p] >> 3);
            o.bc_pm_in[b] = ((uint64_t)seg << 32) | ((uint64_t)e + 1);
            o.bc_key[b] = ((uint64_t)seg << rbits) | e;
        }
        if ((code[i] >> 4) & 1u) run[7] = (uint32_t)p + 1;
        if (p == P - 1 && P % RD_W == 0) {
            // position P opens a chunk of its own: its running values and empty planes
            uint4 *ch = o.rdir + 4 * (P / RD_W);
            ch[0] = make_uint4(run[0], run[1], run[2], run[3]);
            ch[1] = make_uint4(run[4], run[5], run[6], run[7]);
            ch[2] = make_uint4(0u, 0u, 0u, 0u);
            ch[3] = make_uint4(0u, 0u, 0u, 0u);
        }
    }
}

// bumped committed sorted by (segment, executeAt): exec column and nearest-Write index (+1) per entry
__global__ __launch_bounds__(BLOCK) void k_v2_bcs_cols(uint32_t nbc, const uint64_t *__restrict__ skeys, const uint32_t *__restrict__ svals,
                                                       const uint8_t *__restrict__ bc_kind, uint64_t rmask,
                                                       uint32_t *__restrict__ bcs_exec, uint64_t *__restrict__ lastw_in)
{
    uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= nbc) return;
    bcs_exec[i] = (uint32_t)(skeys[i] & rmask);
    lastw_in[i] = bc_kind[svals[i]] == 1 ? i + 1 : 0;
}

__device__ __forceinline__ uint32_t rd_cbc(const uint4 *rdir, uint32_t p);   // the rank directory, below

// The eight per-tile column scans of the multi-scan (7 counts: exclusive sums; the last-unbumped-committed-Write
// column: exclusive max) in ONE launch, one workgroup per column, carrying the running value across chunks.
constexpr int V2TS_ITEMS = 32;
__global__ __launch_bounds__(BLOCK) void k_v2_tile_scans(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, uint32_t nt,
                                                         uint32_t *__restrict__ totals)
{
    __shared__ uint32_t red[WAVES];
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    const bool mx = q == 7;
    const uint32_t *a = in + (size_t)q * nt;
    uint32_t *o = out + (size_t)q * nt;
    uint32_t carry = 0;
    for (uint32_t base = 0; base < nt; base += BLOCK * V2TS_ITEMS) {
        uint32_t v[V2TS_ITEMS];
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < V2TS_ITEMS; ++i) {
            const uint32_t idx = base + tid * V2TS_ITEMS + i;
            v[i] = idx < nt ? a[idx] : 0u;
            acc = mx ? max(acc, v[i]) : acc + v[i];
        }
        uint32_t tot;
        const uint32_t pre = mx ? block_exclusive(acc, OpMax<uint32_t>(), red, tot) : block_exclusive(acc, OpAdd<uint32_t>(), red, tot);
        uint32_t run = mx ? max(carry, pre) : carry + pre;
#pragma unroll
        for (int i = 0; i < V2TS_ITEMS; ++i) {
            const uint32_t idx = base + tid * V2TS_ITEMS + i;
            if (idx < nt) o[idx] = run;
            run = mx ? max(run, v[i]) : run + v[i];
        }
        carry = mx ? max(carry, tot) : carry + tot;
    }
    if (tid == 0) totals[q] = carry;
}

struct V2View {
    const uint32_t *perm, *pair_pos, *seg_incl, *seg_start, *s_rank, *s_exec;
    const uint8_t *s_info;
    const uint4 *rdir;
    const uint32_t *list_rank, *bases;
    const uint32_t *bc_rank, *bc_exec;
    const uint64_t *bc_pm;    // (segment << 32 | executeAt + 1) prefix maxima: the low word within a segment
    const uint8_t *bc_kind;
    const uint32_t *bcs_exec;
    const uint64_t *bcs_lastw;   // nearest Write index + 1 (prefix maximum, the low word)
    const uint4 *tinfo;   // per txn: rank, executeAt rank, status | kind << 3
    const uint32_t *irec32;  // the count pass's inline records as u32 (IREC_W words per pair; word 7 = E | flag)
    const uint4 *rec;        // the count pass's 64-B records (runs; inline entries beyond IREC_N)
};

struct Row { uint32_t c[8]; };

// the 8 running values at CFK position p from its rank-directory chunk
__device__ __forceinline__ Row ld_row(const V2View &v, uint32_t p)
{
    const uint4 *ch = v.rdir + 4 * (size_t)(p / RD_W);
    const uint4 a = ch[0], b = ch[1], c = ch[2], d = ch[3];
    const uint32_t r = p % RD_W, mask = (1u << r) - 1u;
    Row o;
    o.c[0] = a.x + __popc(c.x & mask); o.c[1] = a.y + __popc(c.y & mask);
    o.c[2] = a.z + __popc(c.z & mask); o.c[3] = a.w + __popc(c.w & mask);
    o.c[4] = b.x + __popc(d.x & mask); o.c[5] = b.y + __popc(d.y & mask);
    o.c[6] = b.z + __popc(d.z & mask);
    const uint32_t w = d.w & mask;
    o.c[7] = w ? (p - r) + (31u - (uint32_t)__clz(w)) + 1u : b.w;
    return o;
}
// the bumped-committed count below position p (column RW_CBC only)
__device__ __forceinline__ uint32_t rd_cbc(const uint4 *rdir, uint32_t p)
{
    const uint32_t *ch = reinterpret_cast<const uint32_t *>(rdir) + 16 * (size_t)(p / RD_W);
    const uint32_t r = p % RD_W;
    return ch[RW_CBC] + __popc(ch[8 + RW_CBC] & ((1u << r) - 1u));
}
__device__ __forceinline__ uint32_t ld_cbc(const V2View &v, uint32_t p) { return rd_cbc(v.rdir, p); }

struct V2Query {
    uint32_t trank, info, wk, wc, s0, pos, posm, m, bstart, bend;
    bool bq, has_m;
    Row r0, rp, rm;   // rows at s0, pos, posM
};

// The query of the pair at CFK position p (pair order (key, TxnId)): every per-txn input comes from the
// position-ordered columns, so neighbouring lanes read neighbouring rows. The loads are ordered for a short dependency
// chain: the pair's own row and columns; then its segment's bounds; then, together, the segment start's row, the
// bumped-committed count at the segment end, and -- speculatively, assuming M is the last unbumped committed Write
// before the pair (it is unless the segment holds bumped committed entries or the query's executeAt is bumped, ~1.5% of
// pairs, recomputed below) -- that Write's TxnId and its row.
__device__ __forceinline__ V2Query v2_query(const V2View &v, uint32_t p)
{
    V2Query q;
    const Row rpp = ld_row(v, p);
    const uint32_t seg = v.seg_incl[p] - 1;
    q.trank = v.s_rank[p];
    const uint32_t S = v.s_exec[p];
    q.info = v.s_info[p];
    q.s0 = v.seg_start[seg];
    const uint32_t s1 = v.seg_start[seg + 1];
    q.wk = witnesses(q.info >> 3);
    q.wc = wk_classes(q.wk);
    q.bq = S != q.trank;
    // level 3: issued together
    const uint32_t lu0 = rpp.c[RW_LUCW];
    const bool spec = !q.bq && lu0 > q.s0;   // the last unbumped committed Write before p lies in p's segment
    q.r0 = ld_row(v, q.s0);
    const uint32_t b1 = ld_cbc(v, s1);
    uint32_t mu = 0;
    Row rms = q.r0;
    if (spec) { mu = v.s_rank[lu0 - 1]; rms = ld_row(v, lu0 - 1); }
    const uint32_t b0 = q.r0.c[RW_CBC];
    if (!q.bq && b1 == b0) {
        // common path: no bumped committed entry in the segment, executeAt == TxnId
        q.pos = p;
        q.rp = rpp;
        q.has_m = spec;
        q.m = mu;
        q.posm = spec ? lu0 - 1 : q.s0;
        q.rm = rms;
        q.bend = q.rm.c[RW_CBC];
        q.bstart = q.bend;   // no bumped committed entry before posM in this segment (b1 == b0)
        return q;
    }
    q.pos = q.bq ? lower_bound_u32(v.s_rank, p + 1, s1, S) : p;
    q.rp = q.bq ? ld_row(v, q.pos) : rpp;
    // M from the last unbumped committed Write before pos
    const uint32_t lu = q.rp.c[RW_LUCW];
    const bool has_mu = lu > q.s0;
    if (q.bq) mu = has_mu ? v.s_rank[lu - 1] : 0;
    // M from bumped committed Writes of this segment: predecessor of S by executeAt, then nearest Write
    bool has_mb = false;
    uint32_t mb = 0;
    if (b1 > b0) {
        uint32_t i = lower_bound_u32(v.bcs_exec, b0, b1, S);
        if (i > b0) {
            uint32_t w = (uint32_t)v.bcs_lastw[i - 1];
            if (w > b0) { has_mb = true; mb = v.bcs_exec[w - 1]; }
        }
    }
    q.has_m = has_mu || has_mb;
    q.m = (has_mb && (!has_mu || mb > mu)) ? mb : mu;
    if (!q.has_m) q.posm = q.s0;
    else if (has_mu && q.m == mu) q.posm = lu - 1;
    else q.posm = lower_bound_u32(v.s_rank, q.s0, q.pos, q.m);
    q.rm = q.posm == q.s0 ? q.r0 : (spec && q.posm == lu0 - 1) ? rms : ld_row(v, q.posm);
    q.bend = q.rm.c[RW_CBC];
    q.bstart = q.has_m ? lower_bound_lo32(v.bc_pm, b0, q.bend, q.m + 1) : q.bend;
    return q;
}

// per-pair results for the write pass, stored by pair index j (the write pass reads a txn's pairs contiguously):
//   irec[j] (32 B, every pair): word 7 = E, | REC_INLINE_FLAG for an inline record (the mark pass reads this word;
//           a separate 4-B E word per pair measured slower: the count pass's extra scattered store costs more than
//           the mark pass saves, config 3 +1.2 ms vs -0.1 ms);
//           inline (E <= REC_INLINE): the pair's dependency entries themselves (TxnId ranks, T and filtered R3 entries
//           already dropped), the first IREC_N in words 0-6, the rest (E > IREC_N) in words 0-7 of rec[j]. Gathered
//           here in CFK position order, where neighbouring pairs of a segment read the same class-list lines, instead
//           of by the write pass in txn order;
//   rec[j]  (64 B, run pairs, E > REC_INLINE): starts a[6] and lengths l[6] of R1/R2 per class (witnessed classes only),
//           R3 = [bs, bs + bl) filtered by executeAt >= M; word 15 = E.
// An inline entry is addressed as 16 * j + off (inl_entry).
constexpr uint32_t NO_M = 0xFFFFFFFFu;
constexpr uint32_t INLINE_M = 0xFFFFFFFEu;   // RunsT::m marker of an inline record
constexpr uint32_t REC_INLINE = 15;
constexpr uint32_t IREC_W = 8;               // u32 words per 32-B record
constexpr uint32_t IREC_N = 7;               // inline entries held by the 32-B record
constexpr uint32_t REC_INLINE_FLAG = 0x80000000u;

// inline entry off of pair j (idx = 16 * j + off)
__device__ __forceinline__ uint32_t inl_entry(const uint32_t *irec32, const uint4 *rec, uint32_t idx)
{
    const uint32_t j = idx >> 4, off = idx & 15u;
    return off < IREC_N ? irec32[IREC_W * (size_t)j + off] : reinterpret_cast<const uint32_t *>(rec)[16 * (size_t)j + off - IREC_N];
}

__device__ __forceinline__ void inl_put(uint32_t (&buf)[16], uint32_t &n, uint32_t x)
{
#pragma unroll
    for (uint32_t s = 0; s < REC_INLINE; ++s) if (s == n) buf[s] = x;   // static register indices (no scratch)
    ++n;
}

struct RecOut {
    uint4 *rec;         // run records, 4 x uint4 per pair
    uint4 *irec;        // inline records / E words, 2 x uint4 per pair
};

#ifdef ACC_PHASE_PROF
// tuning build only: per wave of k_v2_count, cycles of (query, R3 count, inline gather + record write) and lane counts
// (bumped query, segment with bumped committed entries, posM by search, sum of R3 candidates, run records)
__device__ unsigned long long *g_ct_prof;
#define CT_PH(i) ct_ph[i] = clock64()
#else
#define CT_PH(i) ((void)0)
#endif

#ifndef ACC_R3U
#define ACC_R3U 4   // R3 candidates loaded per round of the count pass's per-lane loops
#endif
#ifndef ACC_R3_COOP
#define ACC_R3_COOP 8   // a wave walks the R3 candidates cooperatively when one of its lanes has more
#endif
__device__ __forceinline__ uint64_t v2_count_one(const V2View &v, uint32_t p, const uint32_t *__restrict__ owner,
                                                  const RecOut &ro, uint32_t *__restrict__ bigflag)
{
#ifdef ACC_PHASE_PROF
    unsigned long long ct_ph[4];
#endif
    CT_PH(0);
    const uint32_t j = v.perm[p];   // independent of the query chain: issued first
    V2Query q = v2_query(v, p);
    CT_PH(1);
    uint32_t a[6] = {}, l[6] = {};
    uint64_t e = 0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        if (!((q.wc >> c) & 1u)) continue;
        a[2 * c] = v.bases[c] + q.r0.c[c];
        l[2 * c] = q.rp.c[c] - q.r0.c[c];
        a[2 * c + 1] = v.bases[3 + c] + q.rm.c[3 + c];
        l[2 * c + 1] = q.rp.c[3 + c] - q.rm.c[3 + c];
        e += l[2 * c] + l[2 * c + 1];
    }
    // the class runs' entries of a record that may be inline (L6 <= 16: e <= 15 needs it) are loaded before the R3
    // candidates are counted, so both sets of loads are in flight together (static slots, predicated)
    uint32_t pre[6], L6 = 0;
#pragma unroll
    for (int q2 = 0; q2 < 6; ++q2) { pre[q2] = L6; L6 += l[q2]; }
    uint32_t xs[REC_INLINE + 1];
    const bool may_inline = L6 <= REC_INLINE + 1;
#pragma unroll
    for (uint32_t s = 0; s <= REC_INLINE; ++s) {
        uint32_t idx = a[0] + s;
#pragma unroll
        for (int q2 = 1; q2 < 6; ++q2)
            if (s >= pre[q2]) idx = a[q2] + (s - pre[q2]);   // empty runs are overridden by the next one
        xs[s] = (may_inline && s < L6) ? v.list_rank[idx] : 0u;
    }
    // R3 candidates [bstart, bend): one lane walks its own (ACC_R3U loads in flight), or, when some lane of the wave has
    // more than ACC_R3_COOP (the lanes of a hot segment share nearly the same range), the wave loads the union of the
    // ranges 64 candidates at a time (coalesced) and every lane tests each candidate broadcast from its lane
    // (v_readlane): one memory round trip per 64 candidates instead of one per ACC_R3U
    const uint32_t nc = q.bend > q.bstart ? q.bend - q.bstart : 0u;
    uint32_t wmax = nc, clo = nc ? q.bstart : 0xFFFFFFFFu, chi = nc ? q.bend : 0u;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, d, 64));
        clo = min(clo, (uint32_t)__shfl_xor((int)clo, d, 64));
        chi = max(chi, (uint32_t)__shfl_xor((int)chi, d, 64));
    }
    const bool coop = wmax > (uint32_t)ACC_R3_COOP && chi - clo <= 64u * 64u;   // wave-uniform
    if (coop) {
        for (uint32_t c = clo; c < chi; c += 64) {
            const uint32_t i = c + lane_id();
            const uint32_t exl = i < chi ? v.bc_exec[i] : 0u, kdl = i < chi ? (uint32_t)v.bc_kind[i] : 0u;
            const uint32_t cnt = min(64u, chi - c);
            for (uint32_t u = 0; u < cnt; ++u) {
                const uint32_t exu = (uint32_t)__builtin_amdgcn_readlane((int)exl, (int)u);
                const uint32_t kdu = (uint32_t)__builtin_amdgcn_readlane((int)kdl, (int)u);
                const uint32_t iu = c + u;
                e += (iu >= q.bstart && iu < q.bend && exu >= q.m && ((q.wk >> kdu) & 1u)) ? 1u : 0u;
            }
        }
    } else {
        for (uint32_t i = q.bstart; i < q.bend; i += ACC_R3U) {
            uint32_t ex[ACC_R3U], kd[ACC_R3U];
#pragma unroll
            for (uint32_t u = 0; u < ACC_R3U; ++u) {
                ex[u] = i + u < q.bend ? v.bc_exec[i + u] : 0u;
                kd[u] = i + u < q.bend ? (uint32_t)v.bc_kind[i + u] : 0u;
            }
#pragma unroll
            for (uint32_t u = 0; u < ACC_R3U; ++u) e += (i + u < q.bend && ex[u] >= q.m && ((q.wk >> kd[u]) & 1u)) ? 1u : 0u;
        }
    }
    if (q.bq) {
        uint32_t st = q.info & 7u, kind = q.info >> 3;
        if (((q.wk >> kind) & 1u) && st != 0 && st != 7) --e;
    }
    CT_PH(2);
    const bool inl = e <= REC_INLINE;
    // an inline record: the class entries without T (L6 <= e + 1 <= 16: T itself is dropped at most once, so xs holds
    // every class entry), then the kept R3 entries
    uint32_t d = L6;   // position of T among them (at most one)
#pragma unroll
    for (uint32_t s = 0; s <= REC_INLINE; ++s)
        if (q.bq && s < L6 && xs[s] == q.trank) d = s;
    uint32_t buf[16] = {};
#pragma unroll
    for (uint32_t s = 0; s < REC_INLINE; ++s) buf[s] = s < d ? xs[s] : xs[s + 1];
    uint32_t n = L6 - (d < L6 ? 1u : 0u);
    if (coop) {
        const bool want = inl && q.has_m && nc;
        if (__ballot(want))
            for (uint32_t c = clo; c < chi; c += 64) {
                const uint32_t i = c + lane_id();
                const uint32_t exl = i < chi ? v.bc_exec[i] : 0u, kdl = i < chi ? (uint32_t)v.bc_kind[i] : 0u;
                const uint32_t xrl = i < chi ? v.bc_rank[i] : 0u;
                const uint32_t cnt = min(64u, chi - c);
                for (uint32_t u = 0; u < cnt; ++u) {
                    const uint32_t exu = (uint32_t)__builtin_amdgcn_readlane((int)exl, (int)u);
                    const uint32_t kdu = (uint32_t)__builtin_amdgcn_readlane((int)kdl, (int)u);
                    const uint32_t xru = (uint32_t)__builtin_amdgcn_readlane((int)xrl, (int)u);
                    const uint32_t iu = c + u;
                    if (want && iu >= q.bstart && iu < q.bend && exu >= q.m && ((q.wk >> kdu) & 1u) &&
                        !(q.bq && xru == q.trank))
                        inl_put(buf, n, xru);
                }
            }
    } else if (inl && q.has_m) {
        for (uint32_t i = q.bstart; i < q.bend; i += ACC_R3U) {   // R3 candidates, ACC_R3U at a time
            uint32_t ex[ACC_R3U], kd[ACC_R3U], xr[ACC_R3U];
#pragma unroll
            for (uint32_t u = 0; u < ACC_R3U; ++u) {
                const bool in = i + u < q.bend;
                ex[u] = in ? v.bc_exec[i + u] : 0u;
                kd[u] = in ? (uint32_t)v.bc_kind[i + u] : 0u;
                xr[u] = in ? v.bc_rank[i + u] : 0u;
            }
#pragma unroll
            for (uint32_t u = 0; u < ACC_R3U; ++u)
                if (i + u < q.bend && ex[u] >= q.m && ((q.wk >> kd[u]) & 1u) && !(q.bq && xr[u] == q.trank))
                    inl_put(buf, n, xr[u]);
        }
    }
    if (inl) {
        uint4 *r = ro.irec + 2 * (size_t)j;
        r[0] = make_uint4(buf[0], buf[1], buf[2], buf[3]);
        r[1] = make_uint4(buf[4], buf[5], buf[6], REC_INLINE_FLAG | (uint32_t)e);
        if (e > IREC_N) {
            uint4 *r2 = ro.rec + 4 * (size_t)j;
            r2[0] = make_uint4(buf[7], buf[8], buf[9], buf[10]);
            r2[1] = make_uint4(buf[11], buf[12], buf[13], buf[14]);
        }
    } else {
        uint4 *ir = ro.irec + 2 * (size_t)j;
        ir[0] = make_uint4(0u, 0u, 0u, 0u);
        ir[1] = make_uint4(0u, 0u, 0u, (uint32_t)e);
        uint4 *r = ro.rec + 4 * (size_t)j;
        r[0] = make_uint4(a[0], a[1], a[2], a[3]);
        r[1] = make_uint4(a[4], a[5], l[0], l[1]);
        r[2] = make_uint4(l[2], l[3], l[4], l[5]);
        r[3] = make_uint4(q.bstart, q.has_m ? q.bend - q.bstart : 0u, q.has_m ? q.m : NO_M, (uint32_t)e);
        bigflag[owner[j]] = 1u;
    }
#ifdef ACC_PHASE_PROF
    CT_PH(3);
    {
        const uint32_t s1 = v.seg_start[v.seg_incl[p]];
        const bool mb = ld_cbc(v, s1) > q.r0.c[RW_CBC];
        const bool psearch = q.has_m && q.posm != q.s0 && !(q.rp.c[RW_LUCW] > q.s0 && q.m == v.s_rank[q.rp.c[RW_LUCW] - 1]);
        uint32_t r3 = q.bend - q.bstart;
        for (int d = 1; d < 64; d <<= 1) r3 += __shfl_xor(r3, d, 64);
        if (lane_id() == 0) {
            unsigned long long *row = g_ct_prof + 8 * (size_t)((blockIdx.x * BLOCK + threadIdx.x) >> 6);
            row[0] = ct_ph[1] - ct_ph[0]; row[1] = ct_ph[2] - ct_ph[1]; row[2] = ct_ph[3] - ct_ph[2];
            row[3] = (unsigned long long)__popcll(__ballot(q.bq));
            row[4] = (unsigned long long)__popcll(__ballot(mb));
            row[5] = (unsigned long long)__popcll(__ballot(psearch));
            row[6] = r3;
            row[7] = (unsigned long long)__popcll(__ballot(e > REC_INLINE)) | (1ull << 32);
        }
    }
#endif
    return e;
}

// Also: bigflag[T] = 1 for txns with a run record (they take the v2 tiers, the rest the stream pass) and per-block
// entry totals (blk_e) for the batch's E.
__global__ __launch_bounds__(BLOCK) void k_v2_count(size_t P, V2View v, const uint32_t *__restrict__ owner,
                                                    RecOut ro, uint32_t *__restrict__ bigflag,
                                                    uint64_t *__restrict__ blk_e)
{
    __shared__ uint64_t lds[WAVES];
    const size_t p = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    uint64_t e = 0;
    if (p < P) e = v2_count_one(v, (uint32_t)p, owner, ro, bigflag);
    uint64_t total;
    block_exclusive(e, OpAdd<uint64_t>(), lds, total);
    if (threadIdx.x == 0) blk_e[blockIdx.x] = total;
}

// ---- write pass, three tiers by E_T (dependency entries of the txn; 98.7% of config-2 txns have <= 64):
//   small  (E <= 64,  <= 32 keys): one wave per txn, registers + 512 B of LDS staging, high occupancy
//   medium (E <= 1024, <= 64 keys): one wave per txn, bitonic sort of (value << 16 | key) in LDS
//   big    (E <= 8192, <= 64 keys): one block per txn, bitonic sort in 64 KiB of LDS
//   fallback (otherwise, rare):      global gather + two radix sorts
// Every tier: lane k derives the 7 runs of key k (R1/R2 per kind class, R3) from the count-pass record,
// the runs are gathered flattened by all lanes, T itself and non-qualifying R3 entries are dropped.

constexpr int NRUN = 7;
constexpr int MED_E = 1024, MED_K = 64;
constexpr int BIG_K = 64;
constexpr int BIG_E = 8192;                 // raw entries per block in LDS (32 KiB of u32 records)
constexpr int HUGE_E = 16384;               // second big launch (64 KiB + a 64 KiB merge buffer)

struct V2Out {
    const uint32_t *key_off;
    const uint64_t *dep_off, *arena_off;
    const uint32_t *cnz, *txn_of_rank;
    const uint4 *rec;        // run records, 4 x uint4 per pair (k_v2_count)
    const uint32_t *irec32;  // inline records, IREC_W words per pair (word 7 = E | REC_INLINE_FLAG)
    int32_t *arena;
    uint32_t *dep_scratch;   // at dep_off[j0] + idx, compacted later
    uint64_t *u_cnt;
    uint32_t *med_list, *big_list, *fb_list, *huge_list;
    uint64_t *gstat;         // [0] medium, [1] big, [2] count mismatches, [3] fallback txns, [4] fallback entries,
                             // [5] small, [6] huge (second big launch), [7] / [8] window tier (<= 8 / <= 16 keys)
};
constexpr int GSTAT_N = 12;

template <int MAXK>
struct RunsT {
    uint32_t start[MAXK][NRUN];
    uint32_t pre[MAXK][NRUN + 1];
    uint32_t kbase[MAXK + 1];
    uint32_t m[MAXK];
    uint32_t kc[MAXK];
    uint32_t total;
};

struct TxnCtx {
    uint32_t t, j0, j1, nk, E, trank, wk, wc;
    uint64_t e0;
    bool bq;
};

__device__ __forceinline__ TxnCtx txn_ctx(const V2View &v, const V2Out &o, uint32_t t)
{
    TxnCtx c;
    c.t = t;
    c.j0 = o.key_off[t]; c.j1 = o.key_off[t + 1]; c.nk = c.j1 - c.j0;
    c.e0 = o.dep_off[c.j0];
    c.E = (uint32_t)(o.dep_off[c.j1] - c.e0);
    uint4 ti = v.tinfo[t];
    c.trank = ti.x;
    c.bq = ti.y != c.trank;
    c.wk = witnesses(ti.z >> 3);
    c.wc = wk_classes(c.wk);
    return c;
}

// Key k's runs from its record (pair index jk); an inline record is one run of its own entries (m = INLINE_M,
// start = the pair index). Returns the key's raw length.
template <int MAXK>
__device__ __forceinline__ uint32_t load_record(RunsT<MAXK> &R, const uint4 *rec, const uint32_t *irec32, uint32_t jk, uint32_t k)
{
    const uint32_t w = irec32[IREC_W * (size_t)jk + 7];
    if (w & REC_INLINE_FLAG) {
        const uint32_t e = w & ~REC_INLINE_FLAG;
        R.start[k][0] = jk;
        R.pre[k][0] = 0;
#pragma unroll
        for (int q = 1; q <= NRUN; ++q) R.pre[k][q] = e;
        R.m[k] = INLINE_M;
        return e;
    }
    const uint4 *r = rec + 4 * (size_t)jk;
    const uint4 r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3];
    const uint32_t a[6] = { r0.x, r0.y, r0.z, r0.w, r1.x, r1.y };
    const uint32_t l[6] = { r1.z, r1.w, r2.x, r2.y, r2.z, r2.w };
    uint32_t acc = 0;
#pragma unroll
    for (int q = 0; q < 6; ++q) { R.start[k][q] = a[q]; R.pre[k][q] = acc; acc += l[q]; }
    R.start[k][6] = r3.x; R.pre[k][6] = acc; acc += r3.y;
    R.pre[k][7] = acc;
    R.m[k] = r3.z;
    return acc;
}

// Called by ONE wave: lane k < nk fills the runs of key k from its 64-B record. Returns the flattened raw length.
template <int MAXK>
__device__ uint32_t compute_runs(RunsT<MAXK> &R, const V2View &v, const V2Out &o, const uint64_t *cnt, const TxnCtx &c)
{
    const uint32_t lane = lane_id();
    uint32_t ktot = 0;
    if (lane < c.nk && cnt[c.j0 + lane] != 0) {
        ktot = load_record(R, o.rec, o.irec32, c.j0 + lane, lane);
    } else if (lane < c.nk) {
        for (int q = 0; q <= NRUN; ++q) R.pre[lane][q] = 0;
        R.m[lane] = NO_M;
    }
    if (lane < (uint32_t)MAXK) R.kc[lane] = 0;
    uint32_t incl = wave_inclusive(ktot, OpAdd<uint32_t>());
    if (lane < c.nk) R.kbase[lane] = incl - ktot;
    uint32_t total = shfl_idx(incl, 63);
    if (lane == 0) { R.kbase[c.nk] = total; R.total = total; }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    return total;
}

// Element e of the flattened runs: value x, key k; returns whether it is an entry of the txn's deps.
template <int MAXK>
__device__ __forceinline__ bool fetch_elem(const RunsT<MAXK> &R, const V2View &v, const TxnCtx &c, uint32_t e,
                                           uint32_t &x, uint32_t &k)
{
    uint32_t lo = 0, hi = c.nk;
    while (hi - lo > 1) { uint32_t mid = (lo + hi) >> 1; if (R.kbase[mid] <= e) lo = mid; else hi = mid; }
    k = lo;
    uint32_t off = e - R.kbase[k];
    if (R.m[k] == INLINE_M) {   // inline record: the entry itself (filters applied by the count pass)
        x = inl_entry(v.irec32, v.rec, 16 * R.start[k][0] + off);
        return true;
    }
    uint32_t r = 0;
    while (r + 1 < NRUN && R.pre[k][r + 1] <= off) ++r;
    uint32_t idx = R.start[k][r] + (off - R.pre[k][r]);
    bool keep;
    if (r < 6) {
        x = v.list_rank[idx];
        keep = true;
    } else {
        x = v.bc_rank[idx];
        keep = v.bc_exec[idx] >= R.m[k] && ((c.wk >> v.bc_kind[idx]) & 1u);
    }
    return keep && !(c.bq && x == c.trank);
}

// Gather the flattened runs into buf (compacted, at most cap entries). Returns the kept count.
template <int MAXK>
__device__ uint32_t gather_to(uint64_t *buf, uint32_t cap, const RunsT<MAXK> &R, const V2View &v, const TxnCtx &c,
                              uint32_t total)
{
    const uint32_t lane = lane_id();
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    uint32_t cursor = 0;
    for (uint32_t c0 = 0; c0 < total; c0 += 64) {
        uint32_t e = c0 + lane;
        bool keep = false;
        uint32_t x = 0, k = 0;
        if (e < total) keep = fetch_elem(R, v, c, e, x, k);
        uint64_t bal = __ballot(keep);
        if (keep) {
            uint32_t slot = cursor + (uint32_t)__popcll(bal & lt);
            if (slot < cap) buf[slot] = ((uint64_t)x << 16) | k;
        }
        cursor += (uint32_t)__popcll(bal);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    return cursor;
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m)
{
    uint32_t lo = __shfl_xor((uint32_t)v, m, 64), hi = __shfl_xor((uint32_t)(v >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}

// in-LDS bitonic sort of n2 (power of two, >= 128) u64 entries by one wave
__device__ __forceinline__ void wave_bitonic_lds(uint64_t *buf, uint32_t n2)
{
    const uint32_t lane = lane_id();
    for (uint32_t k = 2; k <= n2; k <<= 1) {
        for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
            for (uint32_t i = lane; i < n2; i += 64) {
                uint32_t l = i ^ jj;
                if (l > i) {
                    uint64_t a = buf[i], b = buf[l];
                    bool up = (i & k) == 0;
                    if ((a > b) == up) { buf[i] = b; buf[l] = a; }
                }
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        }
    }
}

// register bitonic across the 64 lanes (ascending by lane)
__device__ __forceinline__ uint64_t wave_bitonic_reg(uint64_t x)
{
    const uint32_t lane = lane_id();
#pragma unroll
    for (uint32_t k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
            uint64_t y = shfl_xor64(x, (int)jj);
            bool up = (lane & k) == 0, lower = (lane & jj) == 0;
            uint64_t lo = x < y ? x : y, hi = x < y ? y : x;
            x = (lower == up) ? lo : hi;
        }
    }
    return x;
}

// Emit one chunk of up to 64 sorted entries (lane holds x). Returns the updated distinct count.
// TRANSLATE = false: the TxnId rank is written and the caller maps the txn's ranks to TxnIds in one bulk pass (a
// dependent global load per chunk would otherwise serialise the chunks)
template <bool TRANSLATE = true>
__device__ __forceinline__ uint32_t emit_chunk(uint64_t x, bool in, uint64_t prev, bool has_prev, uint32_t distinct,
                                               uint32_t *kc, const V2Out &o, const TxnCtx &c, uint64_t abase)
{
    const uint32_t lane = lane_id();
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    uint32_t val = (uint32_t)(x >> 16), kj = (uint32_t)(x & 0xFFFFu);
    bool nw = in && (!has_prev || (uint32_t)(prev >> 16) != val);
    uint64_t bal = __ballot(nw);
    uint32_t idx = distinct + (uint32_t)__popcll(bal & lt) + (nw ? 1u : 0u) - 1u;
    uint64_t peers = __ballot(in);
#pragma unroll
    for (int b = 0; b < 6; ++b) {
        uint64_t bb = __ballot((kj >> b) & 1u);
        peers &= ((kj >> b) & 1u) ? bb : ~bb;
    }
    uint32_t before = (uint32_t)__popcll(peers & lt);
    if (in) {
        uint32_t slot = kc[kj] + before;
        uint64_t kbase = o.dep_off[c.j0 + kj] - c.e0;
        o.arena[abase + kbase + slot] = (int32_t)idx;
        if (nw) o.dep_scratch[c.e0 + idx] = TRANSLATE ? o.txn_of_rank[val] : val;
    }
    __builtin_amdgcn_wave_barrier();
    if (in && before == 0) kc[kj] += (uint32_t)__popcll(peers);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    return distinct + (uint32_t)__popcll(bal);
}

// Persistent over the routed list (count on the device: the v3 routing runs after the last host sync).
__global__ __launch_bounds__(BLOCK) void k_v2_write_medium(const uint64_t *__restrict__ cnt_dev, const uint32_t *__restrict__ list,
                                                           V2View v, const uint64_t *__restrict__ cnt, V2Out o)
{
    __shared__ uint64_t sbuf[WAVES][MED_E];
    __shared__ RunsT<MED_K> sruns[WAVES];
    const uint32_t wave = threadIdx.x >> 6, lane = lane_id();
    const uint32_t cnt_list = (uint32_t)*cnt_dev;
    RunsT<MED_K> &R = sruns[wave];
    uint64_t *buf = sbuf[wave];
    for (uint32_t i = blockIdx.x * WAVES + wave; i < cnt_list; i += gridDim.x * WAVES) {
        const uint32_t t = list[i];
        TxnCtx c = txn_ctx(v, o, t);
        uint32_t total = compute_runs(R, v, o, cnt, c);
        uint32_t got = gather_to(buf, MED_E, R, v, c, total);
        if (got != c.E) { if (lane == 0) atomicAdd((unsigned long long *)&o.gstat[2], 1ull); continue; }
        const uint64_t abase = o.arena_off[t] + (o.cnz[c.j1] - o.cnz[c.j0]);
        uint32_t n2 = 128;
        while (n2 < c.E) n2 <<= 1;
        for (uint32_t q = c.E + lane; q < n2; q += 64) buf[q] = ~0ull;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        wave_bitonic_lds(buf, n2);
        uint32_t distinct = 0;
        for (uint32_t q0 = 0; q0 < c.E; q0 += 64) {
            uint32_t q = q0 + lane;
            bool in = q < c.E;
            uint64_t x = in ? buf[q] : 0;
            uint64_t prev = q > 0 ? buf[q - 1] : 0;
            distinct = emit_chunk(x, in, prev, q > 0, distinct, R.kc, o, c, abase);
        }
        if (lane == 0) o.u_cnt[t] = distinct;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
}

// Locate element e of the flattened runs (LDS only): source index, key, R3 flag.
template <int MAXK>
__device__ __forceinline__ void locate_elem(const RunsT<MAXK> &R, uint32_t nk, uint32_t e, uint32_t &idx, uint32_t &k, bool &r3,
                                            bool &inl)
{
    uint32_t lo = 0, hi = nk;
    while (hi - lo > 1) { uint32_t mid = (lo + hi) >> 1; if (R.kbase[mid] <= e) lo = mid; else hi = mid; }
    k = lo;
    uint32_t off = e - R.kbase[k];
    inl = R.m[k] == INLINE_M;
    if (inl) { idx = 16 * R.start[k][0] + off; r3 = false; return; }
    uint32_t r = 0;
    while (r + 1 < NRUN && R.pre[k][r + 1] <= off) ++r;
    idx = R.start[k][r] + (off - R.pre[k][r]);
    r3 = r == 6;
}

// Big tier: one block per txn (raw run length <= BIG_E). All four waves gather (dropped entries become
// all-ones sentinels that sort last), the block bitonic-sorts (value << 16 | key), then each wave emits a
// quarter of the sorted entries with per-key / distinct-value bases from a per-wave count pass.
constexpr int BIG_GU = 4;   // independent loads in flight per thread during the gather

// Sort records are u32 (TxnId rank << 6 | key index): half the LDS of u64 records, twice the blocks per CU. The
// host takes these tiers only when ranks fit 25 bits (2N <= 2^25). CAP = raw run elements per block: MED_CAP (routed
// by k_v3_route), BIG_E (the txns beyond MED_CAP, routed or passed on by the first launch via gstat[1]), HUGE_E
// (txns the BIG_E launch passes on via gstat[6] / huge_list); beyond that the global path.
// MED_CAP / BIG_E sort by merging: a key's entries are at most NRUN runs that are each sorted by TxnId rank (CFK
// position order within a class list; inline records are sorted by one thread), so after compacting the kept
// entries a merge tree over the non-empty runs (log2 of the run count levels, merge-path partitions per thread)
// sorts them in a few LDS passes instead of the O(n log^2 n) of a bitonic network. HUGE_E keeps the bitonic sort
// in place (no room for a second buffer).
constexpr int MED_CAP = 1024;
constexpr int RUN_SLOTS = NRUN * BIG_K;

template <int CAP>
constexpr bool big_merges() { return CAP <= HUGE_E; }

template <int CAP, int NT>
struct BigLds {
    uint32_t buf[CAP];
    uint32_t tmp[big_merges<CAP>() ? CAP : 1];
    uint32_t rs[big_merges<CAP>() ? RUN_SLOTS + 1 : 1];
    uint32_t ss[big_merges<CAP>() ? RUN_SLOTS : 1];   // compacted start of each (key, run) slot
    RunsT<BIG_K> R;
    uint32_t s_kept, s_nr;
    uint32_t wk_cnt[NT / 64][BIG_K];
    uint32_t wdist[NT / 64];
};

// Sorts the kept entries of buf[0, total) (dropped = all-ones) into ascending order; returns the array holding the
// E sorted entries (buf or tmp). Block-wide; R = the txn's runs (raw layout: key-major, runs in slot order).
template <int CAP, int NT>
__device__ uint32_t *big_merge_sort(BigLds<CAP, NT> &L, uint32_t nk, uint32_t total, uint32_t E)
{
    uint32_t *buf = L.buf, *tmp = L.tmp, *rs = L.rs;
    const RunsT<BIG_K> &R = L.R;
    const uint32_t tid = threadIdx.x;
    __shared__ uint32_t lds[NT / 64];
    // ---- compaction (order kept): tmp[kept index] = entry; buf[raw e] = kept entries before e
    const uint32_t CHR = (total + NT - 1) / NT;
    const uint32_t r0 = min(total, tid * CHR), r1 = min(total, r0 + CHR);
    uint32_t cnt = 0;
    for (uint32_t e = r0; e < r1; ++e) cnt += buf[e] != 0xFFFFFFFFu;
    uint32_t tot;
    uint32_t pos = block_exclusive<uint32_t, OpAdd<uint32_t>, NT / 64>(cnt, OpAdd<uint32_t>(), lds, tot);
    for (uint32_t e = r0; e < r1; ++e) {
        const uint32_t x = buf[e];
        buf[e] = pos;
        if (x != 0xFFFFFFFFu) tmp[pos++] = x;
    }
    __syncthreads();
    // ---- run slots (key k, run q) -> compacted starts; inline keys (one unsorted slot of <= REC_INLINE) sorted here
    for (uint32_t k = tid; k < nk; k += NT) {
        const uint32_t kb = R.kbase[k];
        uint32_t st[NRUN + 1];
#pragma unroll
        for (int q = 0; q <= NRUN; ++q) {
            const uint32_t raw = kb + R.pre[k][q];
            st[q] = raw >= total ? E : buf[raw];
        }
        if (R.m[k] == INLINE_M) {
            for (uint32_t i = st[0] + 1; i < st[NRUN]; ++i) {   // insertion sort
                const uint32_t x = tmp[i];
                uint32_t j = i;
                while (j > st[0] && tmp[j - 1] > x) { tmp[j] = tmp[j - 1]; --j; }
                tmp[j] = x;
            }
        }
        // slot starts; a slot's end is the next slot's start (raw layout is key-major, slot-ordered)
#pragma unroll
        for (int q = 0; q < NRUN; ++q) L.ss[k * NRUN + q] = st[q];
    }
    __syncthreads();
    // ---- non-empty runs -> rs[0, NR), rs[NR] = E (one wave; slots in order)
    if (tid < 64) {
        const uint32_t lane = lane_id();
        const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
        const uint32_t ns = nk * NRUN;
        uint32_t nr = 0;
        for (uint32_t s0 = 0; s0 < ns; s0 += 64) {
            const uint32_t sl = s0 + lane;
            uint32_t a = 0, b = 0;
            if (sl < ns) {
                a = L.ss[sl];
                b = sl + 1 < ns ? L.ss[sl + 1] : E;
            }
            const bool ne = sl < ns && b > a;
            const uint64_t bal = __ballot(ne);
            if (ne) rs[nr + (uint32_t)__popcll(bal & lt)] = a;
            nr += (uint32_t)__popcll(bal);
        }
        if (lane == 0) { rs[nr] = E; L.s_nr = nr; }
    }
    __syncthreads();
    uint32_t NR = L.s_nr;
    uint32_t *src = tmp, *dst = buf;
    const uint32_t CH = (E + NT - 1) / NT;
    while (NR > 1) {
        const uint32_t NP = (NR + 1) / 2;
        const uint32_t o0 = min(E, tid * CH), o1 = min(E, o0 + CH);
        if (o0 < o1) {
            uint32_t lo = 0, hi = NP;   // last pair with start <= o0
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
        uint32_t nv = 0;
        if (tid < NP) nv = rs[2 * tid];
        __syncthreads();
        if (tid < NP) rs[tid] = nv;
        if (tid == 0) rs[NP] = E;
        __syncthreads();
        NR = NP;
        uint32_t *sw = src; src = dst; dst = sw;
    }
    return src;
}

template <int CAP, int NT>
__device__ void big_one(BigLds<CAP, NT> &L, uint32_t t, const V2View &v, const uint64_t *__restrict__ cnt, const V2Out &o)
{
    uint32_t *buf = L.buf;
    RunsT<BIG_K> &R = L.R;
    constexpr int NW = NT / 64;
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = lane_id();
    TxnCtx c = txn_ctx(v, o, t);
    bool oversize = c.nk > BIG_K || c.E > CAP;
    if (!oversize) {
        if (tid < 64) compute_runs(R, v, o, cnt, c);
        if (tid < BIG_K)
            for (int w = 0; w < NW; ++w) L.wk_cnt[w][tid] = 0;
        if (tid == 0) L.s_kept = 0;
        __syncthreads();
        oversize = R.total > CAP;
    }
    if (oversize) {
        if (tid == 0) {
            if (CAP == MED_CAP && c.nk <= BIG_K) {
                uint32_t f = (uint32_t)atomicAdd((unsigned long long *)&o.gstat[1], 1ull);
                o.big_list[f] = t;
            } else if (CAP == BIG_E && c.nk <= BIG_K) {
                uint32_t f = (uint32_t)atomicAdd((unsigned long long *)&o.gstat[6], 1ull);
                o.huge_list[f] = t;
            } else {
                uint32_t f = (uint32_t)atomicAdd((unsigned long long *)&o.gstat[3], 1ull);
                atomicAdd((unsigned long long *)&o.gstat[4], (unsigned long long)c.E);
                o.fb_list[f] = t;
            }
        }
        return;
    }
    const uint32_t total = R.total;
    uint32_t n2 = 128;
    while (n2 < total) n2 <<= 1;
    // ---- gather: raw element e -> buf[e] (all-ones sentinel when dropped)
    uint32_t kept = 0;
    for (uint32_t e0 = tid; e0 < n2; e0 += BIG_GU * NT) {
        uint32_t idx[BIG_GU], kk[BIG_GU], x[BIG_GU];
        bool r3[BIG_GU], in[BIG_GU], il[BIG_GU];
#pragma unroll
        for (int u = 0; u < BIG_GU; ++u) {
            const uint32_t e = e0 + u * NT;
            in[u] = e < total;
            idx[u] = 0; kk[u] = 0; r3[u] = false; il[u] = false;
            if (in[u]) locate_elem(R, c.nk, e, idx[u], kk[u], r3[u], il[u]);
        }
#pragma unroll
        for (int u = 0; u < BIG_GU; ++u)
            x[u] = in[u] ? (il[u] ? inl_entry(v.irec32, v.rec, idx[u]) : r3[u] ? v.bc_rank[idx[u]] : v.list_rank[idx[u]]) : 0u;
#pragma unroll
        for (int u = 0; u < BIG_GU; ++u) {
            const uint32_t e = e0 + u * NT;
            bool keep = in[u] && (il[u] || !(c.bq && x[u] == c.trank));
            if (keep && r3[u]) keep = v.bc_exec[idx[u]] >= R.m[kk[u]] && ((c.wk >> v.bc_kind[idx[u]]) & 1u);
            kept += keep;
            if (e < n2) buf[e] = keep ? ((x[u] << 6) | kk[u]) : 0xFFFFFFFFu;
        }
    }
    kept = wave_inclusive(kept, OpAdd<uint32_t>());
    if (lane == 63) atomicAdd(&L.s_kept, kept);
    __syncthreads();
    if (L.s_kept != c.E) {
        if (tid == 0) atomicAdd((unsigned long long *)&o.gstat[2], 1ull);
        return;
    }
    if constexpr (big_merges<CAP>()) {
        buf = big_merge_sort<CAP, NT>(L, c.nk, total, c.E);
    } else {
        // ---- bitonic sort over n2 (one compare-exchange per pair index)
        for (uint32_t k = 2; k <= n2; k <<= 1) {
            for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
                for (uint32_t pi = tid; pi < (n2 >> 1); pi += NT) {
                    const uint32_t i = ((pi & ~(jj - 1)) << 1) | (pi & (jj - 1));
                    const uint32_t l = i | jj;
                    const uint32_t xa = buf[i], ya = buf[l];
                    const bool up = (i & k) == 0;
                    if ((xa > ya) == up) { buf[i] = ya; buf[l] = xa; }
                }
                __syncthreads();
            }
        }
    }
    // ---- emit: wave w owns sorted positions [w*Q, (w+1)*Q), Q a multiple of 64
    const uint32_t E = c.E;
    const uint32_t Q = ((E + NW * 64 - 1) / (NW * 64)) * 64;
    const uint32_t q_lo = min(E, wave * Q), q_hi = min(E, q_lo + Q);
    uint32_t nd = 0;
    for (uint32_t q0 = q_lo; q0 < q_hi; q0 += 64) {
        const uint32_t q = q0 + lane;
        const bool in = q < q_hi;
        const uint32_t xq = in ? buf[q] : 0;
        const bool nw = in && (q == 0 || (buf[q - 1] >> 6) != (xq >> 6));
        nd += (uint32_t)__popcll(__ballot(nw));
        if (in) atomicAdd(&L.wk_cnt[wave][xq & 63u], 1u);
    }
    if (lane == 0) L.wdist[wave] = nd;
    __syncthreads();
    if (tid < BIG_K) {   // exclusive prefix over waves, per key
        uint32_t run = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) { uint32_t x = L.wk_cnt[w][tid]; L.wk_cnt[w][tid] = run; run += x; }
    }
    __syncthreads();
    uint32_t distinct = 0;
    for (int w = 0; w < (int)wave; ++w) distinct += L.wdist[w];
    const uint64_t abase = o.arena_off[t] + (o.cnz[c.j1] - o.cnz[c.j0]);
    auto widen = [](uint32_t r) { return ((uint64_t)(r >> 6) << 16) | (r & 63u); };
    for (uint32_t q0 = q_lo; q0 < q_hi; q0 += 64) {
        const uint32_t q = q0 + lane;
        const bool in = q < q_hi;
        const uint64_t xq = in ? widen(buf[q]) : 0;
        const uint64_t prev = (in && q > 0) ? widen(buf[q - 1]) : 0;
        distinct = emit_chunk<false>(xq, in, prev, q > 0, distinct, L.wk_cnt[wave], o, c, abase);
    }
    if (wave == NW - 1 && lane == 0) o.u_cnt[t] = distinct;
    __syncthreads();   // the block's rank writes are visible to the block
    // ranks -> TxnIds over the txn's distinct entries, four independent load chains per thread
    uint32_t U = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) U += L.wdist[w];
    uint32_t *dsc = o.dep_scratch + c.e0;
    for (uint32_t i0 = tid; i0 < U; i0 += 4 * NT) {
        uint32_t r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) r[u] = i0 + (uint32_t)u * NT < U ? dsc[i0 + (uint32_t)u * NT] : 0u;
#pragma unroll
        for (int u = 0; u < 4; ++u) if (i0 + (uint32_t)u * NT < U) r[u] = o.txn_of_rank[r[u]];
#pragma unroll
        for (int u = 0; u < 4; ++u) if (i0 + (uint32_t)u * NT < U) dsc[i0 + (uint32_t)u * NT] = r[u];
    }
}

// Persistent over the routed list: blocks loop (a grid of one block per listed txn made the 128-KiB launch pay a
// block launch + exit per big txn). CAP = MED_CAP reads its count from gstat[0], BIG_E from gstat[1], HUGE_E from
// gstat[6].
template <int CAP, int NT>
__global__ __launch_bounds__(NT) void k_v2_write_big(const uint32_t *__restrict__ list, V2View v,
                                                     const uint64_t *__restrict__ cnt, V2Out o)
{
    __shared__ BigLds<CAP, NT> L;
    const uint32_t cnt_list = (uint32_t)o.gstat[CAP > BIG_E ? 6 : CAP == MED_CAP ? 0 : 1];
    for (uint32_t b = blockIdx.x; b < cnt_list; b += gridDim.x) {
        big_one<CAP, NT>(L, list[b], v, cnt, o);
        __syncthreads();
    }
}

// ---- window tier: the KeyDeps of a big txn through per-key bitmaps over its rank span, no sorting.
//
// A big txn (config 2 / 3: the uncommitted window's txns on hot keys, 10^3-10^4 entries) takes its dependency entries
// from ranks below its executeAt S. Every entry of key k at rank x in [base, S), base = S - WIN_W * 32, sets bit
// x - base of key k's bitmap; the union's bitmap is the OR of the keys' bitmaps. A key's entries are distinct TxnIds
// (its runs are disjoint classes), so the builder's per-key ascending index lists (RelationMultiMap.java:245-257) are
// the key's set bits in order and each entry's index into the sorted unique TxnIds (:201-226) is a prefix popcount of
// the union: O(E + keys * span / 32) work instead of a merge sort. Entries below base (a cold key's last committed
// Write far back) go to a short sorted list that precedes the bitmap span. A txn whose list overflows is passed on to
// the sorting tier (k_v2_write_big<BIG_E>).
// One wave sorts buf[0, 64 R) ascending with R entries per lane in registers (element r * 64 + lane; positions >=
// n_valid read as all-ones pads): partners closer than 64 are lanes (shuffles), the others registers of the same lane.
template <int R>
__device__ __forceinline__ void wave_reg_sort_u32(uint32_t *buf, uint32_t n_valid)
{
    const uint32_t lane = lane_id();
    uint32_t v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i = (uint32_t)r * 64 + lane;
        v[r] = i < n_valid ? buf[i] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (uint32_t k = 2; k <= 64u * R; k <<= 1) {
#pragma unroll
        for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
            if (jj >= 64) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int r2 = r ^ (int)(jj / 64);
                    if (r2 > r) {
                        const bool up = (((uint32_t)r * 64 + lane) & k) == 0;
                        const uint32_t a = v[r], b = v[r2];
                        if ((a > b) == up) { v[r] = b; v[r2] = a; }
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t y = xor_lanes(v[r], (int)jj);
                    const bool up = (((uint32_t)r * 64 + lane) & k) == 0, lower = (lane & jj) == 0;
                    const uint32_t lo = min(v[r], y), hi = max(v[r], y);
                    v[r] = (lower == up) ? lo : hi;
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i = (uint32_t)r * 64 + lane;
        if (i < n_valid) buf[i] = v[r];
    }
}

constexpr uint32_t WIN_W = 512;      // bitmap words per key: 16384 ranks below S
constexpr uint32_t WIN_OUT = 1024;   // entries below the span

template <int WK>
struct WinLds {
    uint32_t bm[WK][WIN_W];
    uint32_t un[WIN_W];
    uint16_t pre[WK + 1][WIN_W];   // exclusive prefix popcounts per series (series WK... = the union, index nk)
    uint32_t out[WIN_OUT];         // (rank << 6 | key) of the entries below the span
    RunsT<WK> R;
    uint32_t kc[WK], out_k[WK], ser_tot[WK + 1];
    uint32_t n_out, kept, d_out, bad, minr;
};

#ifdef ACC_PHASE_PROF
// tuning build only: per workgroup of the window tier, summed over its txns: cycles in runs + span low end, bitmap gather,
// below-span sort, prefix popcounts, the span's writes, rank -> TxnId; then txns, entries, span words, entries below
__device__ unsigned long long *g_win_prof;
#define WN_PH(k) do { if (tid == 0) { const unsigned long long t_ = clock64(); wp[k] += t_ - wq; wq = t_; } } while (0)
#else
#define WN_PH(k) ((void)0)
#endif
template <int WK>
__global__ __launch_bounds__(BLOCK) void k_v2_write_win(const uint32_t *__restrict__ list, const uint64_t *__restrict__ cnt_dev,
                                                       V2View v, const uint64_t *__restrict__ cnt, V2Out o)
{
    __shared__ WinLds<WK> L;
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = lane_id();
    const uint32_t n_list = (uint32_t)*cnt_dev;
    RunsT<WK> &R = L.R;
#ifdef ACC_PHASE_PROF
    unsigned long long wp[10] = {}, wq = clock64();
#endif
    for (uint32_t b = blockIdx.x; b < n_list; b += gridDim.x) {
        WN_PH(9);
        const uint32_t t = list[b];
        const TxnCtx c = txn_ctx(v, o, t);
        const uint32_t S = v.tinfo[t].y;
        if (tid < 64) compute_runs(R, v, o, cnt, c);
        if (tid < (uint32_t)WK) { L.kc[tid] = 0; L.out_k[tid] = 0; }
        if (tid == 0) { L.n_out = 0; L.kept = 0; L.bad = 0; L.minr = 0xFFFFFFFFu; }
        __syncthreads();
        // the span's low end: the smallest rank an entry can have (a class run's first entry, an inline record's first
        // entry, any entry of a short R3 run), so the bitmaps cover only [min, S) instead of 16,384 ranks below S
        if (tid < c.nk) {
            const uint32_t k = tid;
            uint32_t mn = 0xFFFFFFFFu;
            if (R.m[k] == INLINE_M) {
                if (R.pre[k][1] > 0) mn = v.irec32[IREC_W * (size_t)R.start[k][0]];
            } else {
#pragma unroll
                for (int q = 0; q < 6; ++q)
                    if (R.pre[k][q + 1] > R.pre[k][q]) mn = min(mn, v.list_rank[R.start[k][q]]);
                if (R.pre[k][7] - R.pre[k][6] > 256) mn = 0u;   // (a long R3 run: from 0; a short one: below)
            }
            atomicMin(&L.minr, mn);
        }
        // the short R3 runs' smallest ranks, the block's threads side by side (one thread walking a run serially waits on
        // one load at a time)
        for (uint32_t k = 0; k < c.nk; ++k) {
            if (R.m[k] == INLINE_M) continue;
            const uint32_t l3 = R.pre[k][7] - R.pre[k][6];
            if (l3 > 256 || tid >= l3) continue;
            atomicMin(&L.minr, v.bc_rank[R.start[k][6] + tid]);
        }
        __syncthreads();
        const uint32_t lo_span = S > WIN_W * 32 ? S - WIN_W * 32 : 0u;
        uint32_t base = max(lo_span, min(L.minr, S));
        uint32_t nw = (S - base + 31) / 32;
        // a sparse span (fewer than one entry per 16 ranks: deps on old commands far below S) is all overhead, the
        // (nk + 1) bitmaps zeroed, scanned and walked word by word: every entry goes to the sorted list instead
        if (c.E <= WIN_OUT && (uint64_t)nw * 32 > 16ull * c.E) { base = S; nw = 0; }
        WN_PH(0);
        for (uint32_t i = tid; i < c.nk * nw; i += BLOCK) L.bm[i / nw][i % nw] = 0;
        __syncthreads();
        const uint32_t total = R.total;
        // ---- gather: bits of the span, the entries below it to the list
        uint32_t kept = 0;
        for (uint32_t e0 = tid; e0 < total; e0 += BIG_GU * BLOCK) {
            uint32_t idx[BIG_GU], kk[BIG_GU], x[BIG_GU];
            bool r3[BIG_GU], in[BIG_GU], il[BIG_GU];
#pragma unroll
            for (int u = 0; u < BIG_GU; ++u) {
                const uint32_t e = e0 + u * BLOCK;
                in[u] = e < total;
                idx[u] = 0; kk[u] = 0; r3[u] = false; il[u] = false;
                if (in[u]) locate_elem(R, c.nk, e, idx[u], kk[u], r3[u], il[u]);
            }
#pragma unroll
            for (int u = 0; u < BIG_GU; ++u)
                x[u] = in[u] ? (il[u] ? inl_entry(v.irec32, v.rec, idx[u]) : r3[u] ? v.bc_rank[idx[u]] : v.list_rank[idx[u]]) : 0u;
#pragma unroll
            for (int u = 0; u < BIG_GU; ++u) {
                bool keep = in[u] && (il[u] || !(c.bq && x[u] == c.trank));
                if (keep && r3[u]) keep = v.bc_exec[idx[u]] >= R.m[kk[u]] && ((c.wk >> v.bc_kind[idx[u]]) & 1u);
                if (!keep) continue;
                ++kept;
                if (x[u] >= base) {
                    const uint32_t d = x[u] - base;
                    if (d < nw * 32) atomicOr(&L.bm[kk[u]][d >> 5], 1u << (d & 31));
                    else L.bad = 1;   // an entry at or above S: impossible for a scan below S
                } else {
                    const uint32_t i = atomicAdd(&L.n_out, 1u);
                    if (i < WIN_OUT) L.out[i] = (x[u] << 6) | kk[u];
                    atomicAdd(&L.out_k[kk[u]], 1u);
                }
            }
        }
        kept = wave_inclusive(kept, OpAdd<uint32_t>());
        if (lane == 63) atomicAdd(&L.kept, kept);
        __syncthreads();
        if (L.kept != c.E || L.bad) {
            if (tid == 0) atomicAdd((unsigned long long *)&o.gstat[2], 1ull);
            __syncthreads();
            continue;
        }
        const uint32_t n_out = L.n_out;
        WN_PH(1);
#ifdef ACC_PHASE_PROF
        if (tid == 0) { wp[6] += 1; wp[7] += c.E; wp[8] += (uint64_t)nw << 32 | min(n_out, 0xFFFFFFFFu); }
#endif
        if (n_out > WIN_OUT) {   // too many entries below the span: the sorting tier
            if (tid == 0) {
                const uint32_t f = (uint32_t)atomicAdd((unsigned long long *)&o.gstat[1], 1ull);
                o.big_list[f] = t;
            }
            __syncthreads();
            continue;
        }
        // ---- union words
        for (uint32_t w = tid; w < nw; w += BLOCK) {
            uint32_t u = 0;
            for (uint32_t k = 0; k < c.nk; ++k) u |= L.bm[k][w];
            L.un[w] = u;
        }
        // ---- the entries below the span, sorted (rank, key): one wave in registers up to 512 (no block barriers), the
        // block's LDS bitonic beyond
        if (n_out > 1) {
            if (n_out <= 128) { if (wave == 0) wave_reg_sort_u32<2>(L.out, n_out); }
            else if (n_out <= 512) { if (wave == 0) wave_reg_sort_u32<8>(L.out, n_out); }
            else {
                uint32_t n2 = 64;
                while (n2 < n_out) n2 <<= 1;
                for (uint32_t q = n_out + tid; q < n2; q += BLOCK) L.out[q] = 0xFFFFFFFFu;
                __syncthreads();
                block_bitonic<uint32_t, BLOCK>(L.out, n2);
            }
        }
        __syncthreads();
        WN_PH(2);
        // ---- exclusive prefix popcounts of every series (keys 0..nk-1, union = nk): a wave per series, 8 words a lane
        for (uint32_t s = wave; s <= c.nk; s += WAVES) {
            const uint32_t *words = s < c.nk ? L.bm[s] : L.un;
            uint32_t run = 0;
            for (uint32_t w0 = 0; w0 < nw; w0 += 512) {
                const uint32_t wl = w0 + lane * 8;
                uint32_t pc[8], sum = 0;
#pragma unroll
                for (int i = 0; i < 8; ++i) { pc[i] = wl + i < nw ? (uint32_t)__popc(words[wl + i]) : 0u; sum += pc[i]; }
                const uint32_t incl = wave_inclusive(sum, OpAdd<uint32_t>());
                uint32_t r = run + incl - sum;
#pragma unroll
                for (int i = 0; i < 8; ++i) if (wl + i < nw) { L.pre[s][wl + i] = (uint16_t)r; r += pc[i]; }
                run += shfl_idx(incl, 63);
            }
            if (lane == 0) L.ser_tot[s] = run;
        }
        WN_PH(3);
        const uint64_t abase = o.arena_off[t] + (o.cnz[c.j1] - o.cnz[c.j0]);
        uint32_t *dsc = o.dep_scratch + c.e0;
        // ---- the sorted entries below the span (one wave): distinct TxnIds first in the union, each key's first slots
        if (wave == 0 && n_out) {
            const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
            uint32_t distinct = 0;
            for (uint32_t q0 = 0; q0 < n_out; q0 += 64) {
                const uint32_t q = q0 + lane;
                const bool in = q < n_out;
                const uint32_t xq = in ? L.out[q] : 0u;
                const uint32_t kj = xq & 63u;
                const bool nw_ = in && (q == 0 || (L.out[q - 1] >> 6) != (xq >> 6));
                const uint64_t bal = __ballot(nw_);
                const uint32_t idx = distinct + (uint32_t)__popcll(bal & lt) + (nw_ ? 1u : 0u) - 1u;
                uint64_t peers = __ballot(in);
#pragma unroll
                for (int bb = 0; bb < 6; ++bb) {
                    const uint64_t m = __ballot((kj >> bb) & 1u);
                    peers &= ((kj >> bb) & 1u) ? m : ~m;
                }
                const uint32_t before = (uint32_t)__popcll(peers & lt);
                if (in) {
                    o.arena[abase + (o.dep_off[c.j0 + kj] - c.e0) + L.kc[kj] + before] = (int32_t)idx;
                    if (nw_) dsc[idx] = o.txn_of_rank[xq >> 6];
                }
                __builtin_amdgcn_wave_barrier();
                if (in && before == 0) L.kc[kj] += (uint32_t)__popcll(peers);
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                distinct += (uint32_t)__popcll(bal);
            }
            if (lane == 0) L.d_out = distinct;
        } else if (tid == 0) {
            L.d_out = 0;
        }
        __syncthreads();
        // ---- the span: item (series, word); a key's words give its keysToTxnIds indices (union index = word prefix +
        // popcount), the union's words its TxnId ranks, mapped to TxnIds below with independent loads in flight
        const uint32_t d_out = L.d_out, nu = L.ser_tot[c.nk];
        const uint32_t items = (c.nk + 1) * nw;
        for (uint32_t i = tid; i < items; i += BLOCK) {
            const uint32_t s = i / nw, w = i - s * nw;
            const uint32_t ubase = d_out + L.pre[c.nk][w];
            if (s == c.nk) {
                uint32_t bits = L.un[w], j = 0;
                while (bits) {
                    dsc[ubase + j] = base + 32 * w + (uint32_t)__builtin_ctz(bits);
                    bits &= bits - 1;
                    ++j;
                }
            } else {
                uint32_t bits = L.bm[s][w];
                if (!bits) continue;
                const uint32_t uw = L.un[w];
                int32_t *dst = o.arena + abase + (o.dep_off[c.j0 + s] - c.e0) + L.out_k[s] + L.pre[s][w];
                uint32_t j = 0;
                while (bits) {
                    const uint32_t b2 = (uint32_t)__builtin_ctz(bits);
                    dst[j] = (int32_t)(ubase + (uint32_t)__popc(uw & ((1u << b2) - 1u)));
                    bits &= bits - 1;
                    ++j;
                }
            }
        }
        __syncthreads();   // the block's rank writes are visible to the block
        WN_PH(4);
        for (uint32_t i0 = d_out + tid; i0 < d_out + nu; i0 += 4 * BLOCK) {
            uint32_t r[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) r[u] = i0 + (uint32_t)u * BLOCK < d_out + nu ? dsc[i0 + (uint32_t)u * BLOCK] : 0u;
#pragma unroll
            for (int u = 0; u < 4; ++u) if (i0 + (uint32_t)u * BLOCK < d_out + nu) r[u] = o.txn_of_rank[r[u]];
#pragma unroll
            for (int u = 0; u < 4; ++u) if (i0 + (uint32_t)u * BLOCK < d_out + nu) dsc[i0 + (uint32_t)u * BLOCK] = r[u];
        }
        if (tid == 0) o.u_cnt[t] = d_out + nu;
        __syncthreads();
        WN_PH(5);
    }
#ifdef ACC_PHASE_PROF
    if (tid == 0)
        for (int k = 0; k < 10; ++k) atomicAdd(&g_win_prof[k], wp[k]);
#endif
}
#undef WN_PH

// ---- global path for txns beyond the wave path: gather to global, two radix sorts

__global__ __launch_bounds__(BLOCK) void k_v2_big_gather(uint32_t nbig, const uint32_t *__restrict__ big_list,
                                                         const uint64_t *__restrict__ big_off, V2View v,
                                                         const uint64_t *__restrict__ cnt, const uint32_t *__restrict__ key_off,
                                                         int rbits, int kbits, uint64_t *__restrict__ gkey)
{
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t b = blockIdx.x * WAVES + wave;
    if (b >= nbig) return;
    const uint32_t t = big_list[b];
    uint64_t *out = gkey + big_off[b];
    // reuse the wave appenders with an unbounded global buffer: WCAP guard off via a large cursor window
    const uint32_t lane = lane_id();
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const uint64_t tb = (uint64_t)b << (rbits + kbits);
    uint32_t cursor = 0;
    const uint32_t j0 = key_off[t], j1 = key_off[t + 1];
    for (uint32_t j = j0; j < j1; ++j) {
        if (cnt[j] == 0) continue;
        V2Query q = v2_query(v, v.pair_pos[j]);
        uint32_t kj = j - j0;
        for (int r = 0; r < 7; ++r) {
            const uint32_t *src;
            uint32_t a, e;
            bool r3 = r == 6;
            if (r3) {
                if (!q.has_m) continue;
                a = q.bstart; e = q.bend; src = v.bc_rank;
            } else {
                int c = r >> 1;
                if (!((q.wc >> c) & 1u)) continue;
                const int col = (r & 1) ? 3 + c : c;
                a = (r & 1) ? q.rm.c[col] : q.r0.c[col];
                e = q.rp.c[col];
                src = v.list_rank + v.bases[(r & 1) ? 3 + c : c];
            }
            for (uint32_t c = a; c < e; c += 64) {
                uint32_t i = c + lane;
                bool keep = false;
                uint32_t x = 0;
                if (i < e) {
                    x = src[i];
                    keep = !(q.bq && x == q.trank);
                    if (r3) keep = keep && v.bc_exec[i] >= q.m && ((q.wk >> v.bc_kind[i]) & 1u);
                }
                uint64_t bal = __ballot(keep);
                if (keep) out[cursor + (uint32_t)__popcll(bal & lt)] = tb | ((uint64_t)x << kbits) | kj;
                cursor += (uint32_t)__popcll(bal);
            }
        }
    }
}

// sorted by (txn, value, key): dense rank of value within txn; TxnId array for first occurrences
__global__ __launch_bounds__(BLOCK) void k_v2_big_newflag(uint64_t m, const uint64_t *__restrict__ skey, int kbits,
                                                          uint32_t *__restrict__ flag)
{
    uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= m) return;
    flag[i] = i == 0 || (skey[i] >> kbits) != (skey[i - 1] >> kbits);
}

__global__ __launch_bounds__(BLOCK) void k_v2_big_rank(uint64_t m, const uint64_t *__restrict__ skey, const uint32_t *__restrict__ incl,
                                                       const uint32_t *__restrict__ big_list, const uint64_t *__restrict__ big_off,
                                                       int rbits, int kbits, const uint32_t *__restrict__ key_off,
                                                       const uint64_t *__restrict__ dep_off, const uint32_t *__restrict__ txn_of_rank,
                                                       uint32_t *__restrict__ dep_scratch, uint64_t *__restrict__ u_cnt,
                                                       uint32_t *__restrict__ idx_by_pos1, uint64_t *__restrict__ key2)
{
    uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= m) return;
    uint64_t x = skey[i];
    uint32_t b = (uint32_t)(x >> (rbits + kbits));
    uint32_t val = (uint32_t)((x >> kbits) & ((1ull << rbits) - 1));
    uint32_t kj = (uint32_t)(x & ((1ull << kbits) - 1));
    uint64_t start = big_off[b];
    uint32_t base_incl = start == 0 ? 0 : incl[start - 1];
    uint32_t idx = incl[i] - base_incl - 1;
    uint32_t t = big_list[b];
    bool nw = i == start || (skey[i] >> kbits) != (skey[i - 1] >> kbits);
    if (nw) dep_scratch[dep_off[key_off[t]] + idx] = txn_of_rank[val];
    if (i + 1 == big_off[b + 1]) u_cnt[t] = idx + 1;
    idx_by_pos1[i] = idx;
    // arena order of the txn: (key, value); value of the second sort = this position
    key2[i] = ((uint64_t)b << (kbits + rbits)) | ((uint64_t)kj << rbits) | val;
}

__global__ __launch_bounds__(BLOCK) void k_v2_big_arena(uint64_t m, const uint32_t *__restrict__ sval2, const uint64_t *__restrict__ skey2,
                                                        const uint32_t *__restrict__ idx_by_pos1, const uint32_t *__restrict__ big_list,
                                                        const uint64_t *__restrict__ big_off, int rbits, int kbits,
                                                        const uint32_t *__restrict__ key_off, const uint32_t *__restrict__ cnz,
                                                        const uint64_t *__restrict__ arena_off, int32_t *__restrict__ arena)
{
    uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= m) return;
    uint32_t b = (uint32_t)(skey2[i] >> (kbits + rbits));
    uint32_t t = big_list[b];
    uint32_t kd = cnz[key_off[t + 1]] - cnz[key_off[t]];
    arena[arena_off[t] + kd + (i - big_off[b])] = (int32_t)idx_by_pos1[sval2[i]];
}

// per fallback txn: raw entry count; maxk[0] = the largest key count of a fallback txn (width of the key field of the
// global-tier sort keys: a txn may list any number of keys, Keys has no cap)
__global__ __launch_bounds__(BLOCK) void k_fb_sizes(uint32_t nfb, const uint32_t *__restrict__ fb_list,
                                                    const uint32_t *__restrict__ key_off, const uint64_t *__restrict__ dep_off,
                                                    uint64_t *__restrict__ fb_e, uint64_t *__restrict__ maxk)
{
    uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    uint64_t nk = 0;
    if (i < nfb) {
        uint32_t t = fb_list[i];
        fb_e[i] = dep_off[key_off[t + 1]] - dep_off[key_off[t]];
        nk = key_off[t + 1] - key_off[t];
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) nk = max(nk, shfl_xor(nk, d));
    if (lane_id() == 0 && nk) atomicMax((unsigned long long *)maxk, (unsigned long long)nk);
}



// ---------------------------------------------------------------- v3: streaming write pass
//
// A txn with at most ST_G keys, at most ST_N2 dependency entries and at most ST_RAW raw run elements (config 2: ~99% of
// txns) is finished by one kernel, k_v3_stream: a tile of txns per block, one lane per key, takes the
// inline entries of its count-pass records and gathers the entries of its run records, sorts the (rank, key) entries
// in LDS, counts the distinct TxnIds, takes the tile's output offsets (arena, keys, TxnIds) from a decoupled look-back
// over the previous tiles' sizes and writes the final KeyDeps arrays (arena_off / kd_off / u_off, arena, key_idx,
// dep_txn) directly: one read of 64 B of record per pair, writes of the outputs only.
// The other ("big") txns take the v2 tiers into scratch arrays addressed by prefix sums over the big txns in txn
// order (k_v3_bigfill gives them per-pair offsets, so the tiers' indexing is unchanged), report their sizes to the
// stream pass; their KeyDeps headers, key indices and entries go straight to the final arrays.

constexpr int ST_G = 16;                      // lanes per txn of the stream pass (one key per lane)
constexpr int ST_N2 = 128;                    // its dependency entries (LDS sort buffer, power of two)
constexpr int ST_SLOT = ST_N2;                // TxnId scratch slot per stream txn (t * ST_SLOT)
constexpr uint32_t ST_RAW = 1024;             // raw run elements of a stream txn
constexpr int MK_G = 8;                       // lanes per txn of the mark pass

// Per txn, MK_G lanes: its KeyDeps sizes A = Kd + E (arena ints) and K = Kd (keys with >= 1 dependency) from the
// count-pass records' word 7 (the exclusive scans of A and K are the txns' arena / key offsets, so the stream pass needs
// no look-back), and the classification: a stream txn has <= ST_G keys and <= ST_N2 entries (and, with run records:
// bigflag = 1 from the count pass, <= ST_RAW raw run elements), else it is big (bigflag = 1: the v2 tiers). (8 lanes per
// txn measured faster than 16 for the 8-key txns of configs 2 / 3; a 16-lane stream pass with 8 lanes per txn lost:
// its sort and gather sizes are wave-uniform maxima over twice the txns.)
__global__ __launch_bounds__(BLOCK) void k_v3_mark(uint32_t n, const uint32_t *__restrict__ key_off,
                                                   const uint32_t *__restrict__ irec32, const uint4 *__restrict__ rec,
                                                   uint32_t *__restrict__ psz, uint32_t raw_cap,
                                                   uint32_t *__restrict__ bigflag, uint64_t *__restrict__ szA,
                                                   uint64_t *__restrict__ szK, uint64_t *__restrict__ any16,
                                                   uint64_t *__restrict__ eb, uint32_t *__restrict__ runflag)
{
    const uint32_t t = (blockIdx.x * BLOCK + threadIdx.x) / MK_G, sub = threadIdx.x & (MK_G - 1);
    if (t >= n) return;   // group-uniform: shuffles stay inside the group
    const uint32_t j0 = key_off[t], nk = key_off[t + 1] - j0;
    const bool run_rec = bigflag[t] != 0;
    // could be big: a run record, more than ST_G keys, or more than 8 keys (8 inline records hold at most 8 * 15 <= ST_N2
    // entries; more may sum past ST_N2)
    const bool maybe_big = run_rec || nk > 8u;
    uint32_t e = 0, kd = 0, raw = 0;
    for (uint32_t c0 = 0; c0 < nk; c0 += MK_G) {
        if (c0 + sub < nk) {
            const uint32_t w = irec32[IREC_W * (size_t)(j0 + c0 + sub) + 7];
            const uint32_t ej = w & ~REC_INLINE_FLAG;
            e += ej;
            kd += ej != 0;
            if (run_rec && !(w & REC_INLINE_FLAG)) {
                const uint4 *r = rec + 4 * (size_t)(j0 + c0 + sub);
                const uint4 r1 = r[1], r2 = r[2], r3 = r[3];
                raw += r1.z + r1.w + r2.x + r2.y + r2.z + r2.w + r3.y;
            }
            if (maybe_big) psz[j0 + c0 + sub] = ej;   // the big txns' per-pair entry counts (k_v3_bigfill)
        }
    }
#pragma unroll
    for (int d = 1; d < MK_G; d <<= 1) {
        e += __shfl_xor(e, d, 64);
        kd += __shfl_xor(kd, d, 64);
        raw += __shfl_xor(raw, d, 64);
    }
    // (an all-inline txn of 9-16 keys can hold up to 240 entries: beyond ST_N2 it is big)
    const bool big = nk > (uint32_t)ST_G || e > (uint32_t)ST_N2 || (run_rec && raw > raw_cap);
    if (sub == 0) {
        bigflag[t] = big ? 1u : 0u;
        runflag[t] = run_rec && !big ? 1u : 0u;   // a stream txn with a run record: the RUNS stream pass
        szA[t] = (uint64_t)kd + e;
        szK[t] = kd;
        eb[t] = big ? e : 0u;   // the big txns' entries: their TxnId scratch bases by the same multi-scan
        // a big txn of 9-16 keys with entries: the 16-key window tier has work (read at the host sync after the scans)
        if (big && e && nk > 8 && nk <= 16 && !*any16) atomicOr((unsigned long long *)any16, 1ull);
    }
}


// per big txn (one wave each, list order): dependency entries E from the per-pair counts of the mark pass
__global__ __launch_bounds__(BLOCK) void k_v3_compact(uint32_t n, const uint32_t *__restrict__ bigflag,
                                                      const uint32_t *__restrict__ bpos, uint32_t *__restrict__ blist)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t < n && bigflag[t]) blist[bpos[t]] = t;
}
// tier routing of the big txns (thread per list entry, one atomic per list per block). With ranks within 25 bits: the
// window tier (<= 8 or <= 16 keys; gstat[7] / gstat[8]), else medium (E <= MED_E, <= MED_K keys) or the u32-record
// block tier; with wider ranks: the u64 wave tier (E <= MED_E, <= MED_K keys) or the global path.
__global__ __launch_bounds__(BLOCK) void k_v3_route(uint32_t nbig, const uint32_t *__restrict__ blist,
                                                    const uint32_t *__restrict__ key_off, const uint64_t *__restrict__ eb,
                                                    int big_ok, int win_ok, uint32_t *__restrict__ med_list,
                                                    uint32_t *__restrict__ big_list, uint32_t *__restrict__ fb_list,
                                                    uint32_t *__restrict__ w8_list, uint32_t *__restrict__ w16_list,
                                                    uint64_t *__restrict__ gstat)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    bool med = false, bg = false, fb = false, w8 = false, w16 = false;
    uint32_t t = 0;
    uint64_t E = 0;
    if (i < nbig) {
        t = blist[i];
        E = eb[t];
        const uint32_t nk = key_off[t + 1] - key_off[t];
        const bool win = E > 0 && big_ok && win_ok && nk <= 16;
        w8 = win && nk <= 8;
        w16 = win && nk > 8;
        med = E > 0 && !win && E <= (uint64_t)MED_E && nk <= (uint32_t)MED_K;
        bg = E > 0 && !win && !med && big_ok;
        fb = E > 0 && !win && !med && !big_ok;
    }
    __shared__ uint64_t lds[WAVES];
    __shared__ uint64_t base[5];
    const uint64_t packed = (med ? 1ull : 0ull) | (bg ? 1ull << 12 : 0ull) | (fb ? 1ull << 24 : 0ull) |
                            (w8 ? 1ull << 36 : 0ull) | (w16 ? 1ull << 48 : 0ull);
    uint64_t total;
    const uint64_t pre = block_exclusive(packed, OpAdd<uint64_t>(), lds, total);
    uint64_t efb = fb ? E : 0;
    uint64_t efb_tot;
    __syncthreads();
    block_exclusive(efb, OpAdd<uint64_t>(), lds, efb_tot);
    if (threadIdx.x < 5) {
        const int slot[5] = { 0, 1, 3, 7, 8 };
        const uint64_t cnt = (total >> (12 * threadIdx.x)) & 4095u;
        base[threadIdx.x] = cnt ? atomicAdd((unsigned long long *)&gstat[slot[threadIdx.x]], (unsigned long long)cnt) : 0ull;
    }
    if (threadIdx.x == 0 && efb_tot) atomicAdd((unsigned long long *)&gstat[4], (unsigned long long)efb_tot);
    __syncthreads();
    if (med) med_list[base[0] + (pre & 4095u)] = t;
    if (bg) big_list[base[1] + ((pre >> 12) & 4095u)] = t;
    if (fb) fb_list[base[2] + ((pre >> 24) & 4095u)] = t;
    if (w8) w8_list[base[3] + ((pre >> 36) & 4095u)] = t;
    if (w16) w16_list[base[4] + ((pre >> 48) & 4095u)] = t;
}

struct V3Big {
    const uint32_t *blist, *key_off;
    const uint32_t *psz;                      // per pair of a big txn: its entry count (k_v3_mark)
    const uint64_t *dB;                       // per txn: exclusive prefix of the big txns' E (TxnId scratch bases)
    const uint64_t *arena_off, *kd_off;       // the batch's final offsets (from the mark pass's scans)
    uint64_t *vdep_off, *vcnt;                // per pair of a big txn (dep_off / cnt of the v2 tiers)
    uint32_t *vcnz;                           // per pair of a big txn (cnz)
    uint64_t *u_cnt;                          // per txn (big txns only)
    int32_t *arena;
    uint32_t *key_idx;
};

// per big txn (one wave): the v2 tiers' per-pair offsets, and the KeyDeps header and key indices straight into the
// final arena / key_idx (the tiers then write the entries at arena_off[t] too: no copy into place afterwards)
__global__ __launch_bounds__(BLOCK) void k_v3_bigfill(uint32_t nbig, V3Big b)
{
    const uint32_t lane = lane_id();
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    for (uint32_t i = blockIdx.x * WAVES + (threadIdx.x >> 6); i < nbig; i += gridDim.x * WAVES) {
        const uint32_t t = b.blist[i], j0 = b.key_off[t], j1 = b.key_off[t + 1], nk = j1 - j0;
        const uint64_t dbase = b.dB[t], kbase = b.kd_off[t], abase = b.arena_off[t];
        const uint64_t E = b.dB[t + 1] - dbase, Kd = b.kd_off[t + 1] - kbase;
        uint64_t ecur = 0, kcur = 0;
        for (uint32_t c0 = 0; c0 < nk; c0 += 64) {
            const uint32_t j = j0 + c0 + lane;
            const bool in = c0 + lane < nk;
            const uint32_t e = in ? b.psz[j] : 0u;
            const uint64_t einc = wave_inclusive((uint64_t)e, OpAdd<uint64_t>());
            const uint64_t nzb = __ballot(e != 0);
            const uint32_t kb = (uint32_t)__popcll(nzb & lt);
            if (in) {
                const uint64_t eoff = ecur + einc - e;
                b.vdep_off[j] = dbase + eoff;
                b.vcnt[j] = e;
                b.vcnz[j] = (uint32_t)(kbase + kcur + kb);
                if (e) {
                    b.arena[abase + kcur + kb] = (int32_t)(Kd + eoff + e);
                    b.key_idx[kbase + kcur + kb] = c0 + lane;
                }
            }
            ecur += shfl_idx(einc, 63);
            kcur += (uint64_t)__popcll(nzb);
        }
        if (lane == 0) {
            b.vdep_off[j1] = dbase + E;
            b.vcnz[j1] = (uint32_t)(kbase + Kd);
            b.u_cnt[t] = 0;
        }
    }
}

struct V3Stream {
    V2View v;
    const uint32_t *key_off, *bigflag, *txn_of_rank;
    const uint32_t *list;                     // LIST: the txns of the pass (else every txn, the stream ones taken)
    const uint4 *rec, *irec;
    const uint64_t *arena_off, *kd_off;       // from the size scans
    uint64_t *u_cnt_out;
    int32_t *arena;
    uint32_t *key_idx, *dep_scr;              // dep_scr: TxnIds at the txn's slot t * ST_SLOT, compacted by k_v3_ucompact
    uint64_t *err;                            // gather count mismatches
    uint32_t n, ntiles;
};

// inclusive prefix over the G lanes of a group
template <int G>
__device__ __forceinline__ uint32_t group_inclusive(uint32_t x, uint32_t sub)
{
#pragma unroll
    for (uint32_t d = 1; d < (uint32_t)G; d <<= 1) {
        const uint32_t u = __shfl_up(x, d, 64);
        if (sub >= d) x += u;
    }
    return x;
}

template <class T>
__device__ __forceinline__ T gshfl_xor(T v, int m)
{
    return xor_lanes(v, m);   // (group_reg_sort runs in the whole wave: no lane of k_v3_stream returns early)
}
// Sorts buf[0, G * R) of a G-lane group ascending (positions >= n_valid read as all-ones pads) with R entries per lane
// in registers, element i = r * G + sub: partners at distance < G are lanes of the group (shuffles), the others registers
// of the same lane. Writes the sorted entries back.
template <class EntT, int G, int R>
__device__ __forceinline__ void group_reg_sort(EntT *buf, uint32_t sub, uint32_t n_valid)
{
    EntT v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i = r * G + sub;
        v[r] = i < n_valid ? buf[i] : ~(EntT)0;
    }
#pragma unroll
    for (uint32_t k = 2; k <= (uint32_t)(G * R); k <<= 1) {
#pragma unroll
        for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
            if (jj >= (uint32_t)G) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int r2 = r ^ (int)(jj / G);
                    if (r2 > r) {
                        const bool up = (((uint32_t)r * G + sub) & k) == 0;
                        const EntT a = v[r], b = v[r2];
                        if ((a > b) == up) { v[r] = b; v[r2] = a; }
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const EntT y = gshfl_xor(v[r], (int)jj);
                    const bool up = (((uint32_t)r * G + sub) & k) == 0, lower = (sub & jj) == 0;
                    const EntT lo = v[r] < y ? v[r] : y, hi = v[r] < y ? y : v[r];
                    v[r] = (lower == up) ? lo : hi;
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) buf[r * G + sub] = v[r];
}

#ifdef ACC_PHASE_PROF
// tuning build only (tools/build_prof.sh): per-phase wave cycles of k_v3_stream, one row of 8 per wave (no atomics)
__device__ unsigned long long *g_st_prof;
#define ST_PH(i) ph[i] = clock64()
#else
#define ST_PH(i) ((void)0)
#endif

// EntT: u32 (rank << 4 | key) when ranks fit 28 bits, else u64
#ifndef ACC_ST_WAVES
#define ACC_ST_WAVES 24   // resident waves per CU the stream pass is compiled for (32: a 64-VGPR budget that spills)
#endif
// G lanes per txn (one key each), N2 entries per txn at most. LIST = false: every txn (the stream ones taken); true: the
// txns of s.list[0, s.n).
template <class EntT, int NT, int G, int N2, bool LIST, bool RUNS>
__global__ __launch_bounds__(NT, ACC_ST_WAVES * 64 / NT) void k_v3_stream(V3Stream s)
{
    constexpr int TT = NT / G;   // txns per tile
    constexpr uint32_t KB = G <= 8 ? 3 : 4;   // key bits under the rank in an entry
    static_assert(G <= 16, "entries keep the key index in 4 bits");
#ifdef ACC_PHASE_PROF
    uint64_t ph[8];
#endif
    ST_PH(0);
    __shared__ EntT ent[TT][N2];
    __shared__ uint32_t kc[TT][G];
    __shared__ uint32_t kbase[TT][G];
    __shared__ uint16_t stA[TT][G + N2];
    const uint32_t tid = threadIdx.x, lane = lane_id(), sub = lane & (G - 1), grp = tid / G, g0 = lane & (64 - G);
    const uint64_t gmask = ((1ull << G) - 1) << g0;
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    // no block barriers: every wave is independent (its txns' arena / key offsets come from the size scans)
    const uint32_t tile = blockIdx.x * (NT / 64) + (tid >> 6);   // wave tile: 64 / G txns
    const uint32_t slot = tile * (64 / G) + lane / G;
    const bool valid = slot < s.n;
    const uint32_t t = LIST ? (valid ? s.list[slot] : 0u) : slot;
    TxnCtx c{};
    bool big = false;
    uint64_t aoff = 0, koff = 0;
    if (valid) {
        c.t = t;
        // independent loads issued together (the txn record is read even for big txns, which ignore it)
        c.j0 = s.key_off[t]; c.j1 = s.key_off[t + 1];
        const uint32_t bf = s.bigflag[t];
        const uint4 ti = s.v.tinfo[t];
        aoff = s.arena_off[t]; koff = s.kd_off[t];
        c.nk = c.j1 - c.j0;
        big = bf != 0;
        c.trank = ti.x;
        c.bq = ti.y != c.trank;
        c.wk = witnesses(ti.z >> 3);
    }
    const bool sm = valid && !big;
    EntT *buf = ent[grp];
    ST_PH(1);
    // ---- records: inline entries straight to LDS; a run record's runs stay in its lane's registers (RUNS only: the
    // lean pass leaves a txn with a run record to the RUNS pass, which the mark pass listed it for)
    uint32_t e = 0, rawk = 0;
    bool run = false;
    uint4 r0 = {}, r1 = {}, r2 = {}, r3 = {};
    if (sm && sub < c.nk) {
        const uint4 *ir = s.irec + 2 * (size_t)(c.j0 + sub);
        r0 = ir[0]; r1 = ir[1];
        const uint32_t w = r1.w;
        if (w & REC_INLINE_FLAG) {
            e = w & ~REC_INLINE_FLAG;
            if (e > IREC_N) {   // entries 7.. in the first half of the 64-B slot
                const uint4 *r = s.rec + 4 * (size_t)(c.j0 + sub);
                r2 = r[0]; r3 = r[1];
            }
        } else {
            run = true;
            e = w;
            if constexpr (RUNS) {
                const uint4 *r = s.rec + 4 * (size_t)(c.j0 + sub);
                r0 = r[0]; r1 = r[1]; r2 = r[2]; r3 = r[3];
                rawk = r1.z + r1.w + r2.x + r2.y + r2.z + r2.w + r3.y;
            }
        }
    }
    const uint32_t ein = run ? 0u : e;
    const uint32_t e_incl = group_inclusive<G>(e, sub), in_incl = group_inclusive<G>(ein, sub);
    const uint32_t E = __shfl(e_incl, (int)(g0 + G - 1), 64);
    const uint32_t E_in = __shfl(in_incl, (int)(g0 + G - 1), 64);
    const uint64_t nzb = __ballot(e != 0) & gmask;
    const uint32_t Kd = (uint32_t)__popcll(nzb);
    const uint64_t A = sm ? (uint64_t)Kd + E : 0;
    kbase[grp][sub] = e_incl - e;
    kc[grp][sub] = 0;
    if (sm && !run) {
        const uint32_t w[REC_INLINE] = { r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r2.x, r2.y, r2.z, r2.w, r3.x, r3.y, r3.z, r3.w };
        const uint32_t b0 = in_incl - ein;
#pragma unroll
        for (uint32_t q = 0; q < REC_INLINE; ++q)
            if (q < e) buf[b0 + q] = ((EntT)w[q] << KB) | (EntT)sub;
    }
    ST_PH(2);
    // ---- run records, one key at a time (its runs broadcast from the owning lane): the group gathers the flattened
    // runs R1/R2 per class and R3, dropping T itself and R3 entries below M or of unwitnessed kinds, after the inline
    // entries
    const uint64_t runmask = __ballot(sm && run) & gmask;
    uint32_t wnrun = RUNS ? (uint32_t)__popcll(runmask) : 0u;
#pragma unroll
    for (int d = G; d < 64; d <<= 1) wnrun = max(wnrun, xor_lanes(wnrun, d));
    uint32_t cursor = E_in;
    uint64_t rem = runmask;
    for (uint32_t ri = 0; ri < wnrun; ++ri) {
        const bool has = rem != 0;
        const int src = has ? (int)__builtin_ctzll(rem) : (int)lane;
        rem &= rem - 1;
        uint32_t st[NRUN], len[NRUN];
        st[0] = __shfl(r0.x, src, 64); st[1] = __shfl(r0.y, src, 64); st[2] = __shfl(r0.z, src, 64);
        st[3] = __shfl(r0.w, src, 64); st[4] = __shfl(r1.x, src, 64); st[5] = __shfl(r1.y, src, 64);
        st[6] = __shfl(r3.x, src, 64);
        len[0] = __shfl(r1.z, src, 64); len[1] = __shfl(r1.w, src, 64); len[2] = __shfl(r2.x, src, 64);
        len[3] = __shfl(r2.y, src, 64); len[4] = __shfl(r2.z, src, 64); len[5] = __shfl(r2.w, src, 64);
        len[6] = __shfl(r3.y, src, 64);
        const uint32_t mk = __shfl(r3.z, src, 64);
        const uint32_t raw = has ? __shfl(rawk, src, 64) : 0u;
        const uint32_t kj = (uint32_t)(src - (int)g0);
        uint32_t wr = raw;
#pragma unroll
        for (int d = G; d < 64; d <<= 1) wr = max(wr, xor_lanes(wr, d));
        for (uint32_t c0 = 0; c0 < wr; c0 += G) {
            const uint32_t off = c0 + sub;
            bool keep = false;
            uint32_t x = 0;
            if (off < raw) {
                uint32_t idx = 0, acc = 0;
                bool r3run = false, found = false;
#pragma unroll
                for (int q = 0; q < NRUN; ++q) {
                    if (!found && off < acc + len[q]) { found = true; idx = st[q] + (off - acc); r3run = q == 6; }
                    acc += len[q];
                }
                if (r3run) {
                    x = s.v.bc_rank[idx];
                    keep = s.v.bc_exec[idx] >= mk && ((c.wk >> s.v.bc_kind[idx]) & 1u);
                } else {
                    x = s.v.list_rank[idx];
                    keep = true;
                }
                keep = keep && !(c.bq && x == c.trank);
            }
            const uint64_t bal = __ballot(keep) & gmask;
            if (keep) {
                const uint32_t at = cursor + (uint32_t)__popcll(bal & lt);
                if (at < (uint32_t)N2) buf[at] = ((EntT)x << KB) | (EntT)kj;
            }
            cursor += (uint32_t)__popcll(bal);
        }
    }
    ST_PH(3);
    bool ok = sm && (RUNS || !runmask);   // (the lean pass skips a txn with a run record: the RUNS pass takes it)
    if (ok && cursor != E) {
        if (sub == 0) atomicAdd((unsigned long long *)s.err, 1ull);
        ok = false;
    }
    uint32_t wE = ok ? E : 0;
#pragma unroll
    for (int d = G; d < 64; d <<= 1) wE = max(wE, xor_lanes(wE, d));
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    // ---- sort each group's entries: registers + shuffles up to 4 per lane (wave-uniform choice), LDS bitonic beyond
    if (wE <= (uint32_t)G) group_reg_sort<EntT, G, 1>(buf, sub, ok ? E : 0);
    else if (wE <= 2u * G) group_reg_sort<EntT, G, 2>(buf, sub, ok ? E : 0);
    else if (wE <= 4u * G) group_reg_sort<EntT, G, 4>(buf, sub, ok ? E : 0);
    else {
        uint32_t n2 = G;
        while (n2 < E) n2 <<= 1;
        if (!ok) n2 = 0;
        for (uint32_t q = E + sub; q < n2; q += G) buf[q] = ~(EntT)0;
        uint32_t wn2 = n2;
#pragma unroll
        for (int d = G; d < 64; d <<= 1) wn2 = max(wn2, xor_lanes(wn2, d));
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        for (uint32_t k = 2; k <= wn2; k <<= 1) {
            for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
                if (k <= n2) {
                    for (uint32_t pi = sub; pi < (n2 >> 1); pi += G) {
                        const uint32_t i = ((pi & ~(jj - 1)) << 1) | (pi & (jj - 1));
                        const uint32_t l = i | jj;
                        const EntT xa = buf[i], ya = buf[l];
                        const bool up = (i & k) == 0;
                        if ((xa > ya) == up) { buf[i] = ya; buf[l] = xa; }
                    }
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    ST_PH(4);
    // ---- KeyDeps in LDS: the arena (header ints and per-key TxnId indices) staged as u16; the distinct TxnIds go
    // straight to the txn's fixed scratch slot t * ST_SLOT
    uint32_t distinct = 0;
    if (ok && e != 0) stA[grp][(uint32_t)__popcll(nzb & lt)] = (uint16_t)(Kd + e_incl);
    for (uint32_t q0 = 0; q0 < wE; q0 += G) {
        const uint32_t q = q0 + sub;
        const bool in = ok && q < E;
        const EntT x = in ? buf[q] : (EntT)0;
        const EntT pv = (in && q > 0) ? buf[q - 1] : (EntT)0;
        const uint32_t kj = (uint32_t)(x & ((1u << KB) - 1u));
        const bool nw = in && (q == 0 || (x >> KB) != (pv >> KB));
        const uint64_t bal = __ballot(nw) & gmask;
        const uint32_t idx = distinct + (uint32_t)__popcll(bal & lt) + (nw ? 1u : 0u) - 1u;
        uint64_t peers = __ballot(in) & gmask;
#pragma unroll
        for (uint32_t bb = 0; bb < KB; ++bb) {
            const uint64_t m = __ballot((kj >> bb) & 1u);
            peers &= ((kj >> bb) & 1u) ? m : ~m;
        }
        const uint32_t before = (uint32_t)__popcll(peers & lt);
        if (in) {
            stA[grp][Kd + kbase[grp][kj] + kc[grp][kj] + before] = (uint16_t)idx;
            if (nw) s.dep_scr[(size_t)t * ST_SLOT + idx] = s.txn_of_rank[(uint32_t)(x >> KB)];
        }
        __builtin_amdgcn_wave_barrier();
        if (in && before == 0) kc[grp][kj] += (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        distinct += (uint32_t)__popcll(bal);
    }
    if (ok && sub == 0) s.u_cnt_out[t] = distinct;
    ST_PH(5);
    // ---- the staged arena and key indices to their places
    if (!valid) return;
    if (ok) {
        for (uint32_t q = sub; q < (uint32_t)A; q += G) s.arena[aoff + q] = (int32_t)stA[grp][q];
        if (e != 0) s.key_idx[koff + (uint32_t)__popcll(nzb & lt)] = sub;
    }
#ifdef ACC_PHASE_PROF
    ST_PH(6);
    if (lane == 0 && !LIST) {
        unsigned long long *row = g_st_prof + 8 * (size_t)tile;
        for (int i = 0; i < 6; ++i) row[i] = ph[i + 1] - ph[i];
        row[7] = 1;
    }
#endif
}

// Sparse batches (a mixed batch's range txns have no KeyDeps of their own here): the txns with TxnIds, compacted with
// their u_off, so k_v3_ucompact's chunks span a few txns each instead of long runs of empty ones.
__global__ __launch_bounds__(BLOCK) void k_v3_neflag(uint32_t n, const uint64_t *__restrict__ u_cnt, uint32_t *__restrict__ flag)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t < n) flag[t] = u_cnt[t] != 0;
}

__global__ __launch_bounds__(BLOCK) void k_v3_nelist(uint32_t n, const uint32_t *__restrict__ flag, const uint32_t *__restrict__ pos,
                                                     const uint32_t *__restrict__ cnt, const uint64_t *__restrict__ u_off,
                                                     uint32_t *__restrict__ ne_t, uint64_t *__restrict__ ne_uoff)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t < n && flag[t]) { ne_t[pos[t]] = t; ne_uoff[pos[t]] = u_off[t]; }
    if (t == 0) ne_uoff[*cnt] = u_off[n];
}

// KeyDeps.txnIds: each txn's distinct TxnIds from its scratch (stream txns: at its slot t * ST_SLOT of dep_scr; big
// txns: at vdep_off of its first pair in dep_big) to dep_txn[u_off[t] ...). A block takes a fixed chunk
// of UC_CHUNK outputs (the uncommitted window's txns are consecutive and hold most TxnIds: partitioning by txns left a
// few blocks with most of the work), finds the txns spanning it by binary search over u_off, and strides over the
// chunk in windows of BLOCK txns (u_off / source bases in LDS, each output's txn by binary search there).
constexpr uint32_t UC_CHUNK = 4096;

__device__ __forceinline__ uint32_t last_le(const uint64_t *a, uint32_t n, uint64_t x)   // largest i < n with a[i] <= x
{
    uint32_t lo = 0, hi = n;
    while (hi - lo > 1) { const uint32_t m = (lo + hi) >> 1; if (a[m] <= x) lo = m; else hi = m; }
    return lo;
}

// tmap (optional): the txns are tmap[0, *n_dev) with offsets u_off[0, *n_dev] (the non-empty txns of a sparse batch,
// k_v3_nelist), else 0..n-1 over the batch's u_off.
__global__ __launch_bounds__(BLOCK) void k_v3_ucompact(uint32_t n, const uint64_t *__restrict__ u_off,
                                                       const uint64_t *__restrict__ arena_off, const uint64_t *__restrict__ kd_off,
                                                       const uint32_t *__restrict__ bigflag, const uint32_t *__restrict__ key_off,
                                                       const uint64_t *__restrict__ vdep_off, const uint32_t *__restrict__ dep_scr,
                                                       const uint32_t *__restrict__ dep_big,
                                                       const uint32_t *__restrict__ tmap, const uint32_t *__restrict__ n_dev,
                                                       uint32_t *__restrict__ dep_txn, const uint64_t *__restrict__ u_all,
                                                       uint64_t *__restrict__ totals)
{
    __shared__ uint64_t uo[BLOCK + 1];
    __shared__ uint64_t src[BLOCK];
    __shared__ uint32_t s_t[2];
    const uint32_t tid = threadIdx.x;
    if (tid == 0 && blockIdx.x == gridDim.x - 1) {   // the batch totals beside the status words: one host copy
        totals[0] = arena_off[n]; totals[1] = kd_off[n]; totals[2] = u_all[n];
    }
    if (tmap) n = *n_dev;
    const uint64_t total = u_off[n];
    const uint64_t c0 = (uint64_t)blockIdx.x * UC_CHUNK;
    if (c0 >= total) return;
    const uint64_t c1 = min(total, c0 + UC_CHUNK);
    if (tid == 0) { s_t[0] = last_le(u_off, n, c0); s_t[1] = last_le(u_off, n, c1 - 1); }
    __syncthreads();
    const uint32_t tlo = s_t[0], thi = s_t[1];
    auto source = [&](uint32_t j) {
        const uint32_t t = tmap ? tmap[j] : j;
        return bigflag[t] ? (vdep_off[key_off[t]] | (1ull << 63)) : (uint64_t)t * ST_SLOT;
    };
    if (thi - tlo >= 8 * BLOCK) {
        // sparse chunk (long runs of txns without TxnIds, e.g. the range txns of a mixed batch): every output finds its
        // txn by a binary search of u_off over the chunk's txn span
        for (uint64_t i = c0 + tid; i < c1; i += BLOCK) {
            uint32_t lo = tlo, hi = thi + 1;
            while (hi - lo > 1) { const uint32_t m = (lo + hi) >> 1; if (u_off[m] <= i) lo = m; else hi = m; }
            const uint64_t sb = source(lo), off = i - u_off[lo];
            dep_txn[i] = (sb >> 63) ? dep_big[(sb & ~(1ull << 63)) + off] : dep_scr[sb + off];
        }
        return;
    }
    // dense chunk: windows of BLOCK txns, offsets and sources staged in LDS
    for (uint32_t tw = tlo; tw <= thi; tw += BLOCK) {
        const uint32_t nt = min((uint32_t)BLOCK, thi + 1 - tw);
        __syncthreads();
        if (tid < nt) {
            uo[tid] = u_off[tw + tid];
            src[tid] = source(tw + tid);
        }
        if (tid == 0) uo[nt] = u_off[tw + nt];
        __syncthreads();
        const uint64_t lo = max(c0, uo[0]), hi = min(c1, uo[nt]);
        constexpr int U = 4;   // outputs per thread whose scratch and TxnId loads are in flight together
        for (uint64_t i0 = lo + tid; i0 < hi; i0 += U * BLOCK) {
            uint32_t x[U];
            bool big[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t i = i0 + (uint64_t)u * BLOCK;
                x[u] = 0; big[u] = false;
                if (i < hi) {
                    const uint32_t a = last_le(uo, nt, i);
                    const uint64_t sb = src[a], off = i - uo[a];
                    big[u] = (sb >> 63) != 0;
                    x[u] = big[u] ? dep_big[(sb & ~(1ull << 63)) + off] : dep_scr[sb + off];
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (i0 + (uint64_t)u * BLOCK < hi) dep_txn[i0 + (uint64_t)u * BLOCK] = x[u];
        }
    }
}

// ---------------------------------------------------------------- host orchestration

static void check_errors(uint64_t errs)
{
    if (errs & ERR_KEY_TOTAL) fail(ACC_E_ARG, "key_off[n_txn] must equal n_pairs");
    if (errs & ERR_BAD_STATUS) fail(ACC_E_ARG, "invalid InternalStatus ordinal (> INVALID_OR_TRUNCATED)");
    if (errs & ERR_BAD_KIND) fail(ACC_E_ARG, "Kind.ofOrdinal: invalid kind ordinal in TxnId flags");
    if (errs & ERR_KEY_OFF) fail(ACC_E_ARG, "key_off must be non-decreasing");
    if (errs & ERR_KEYS_UNSORTED) fail(ACC_E_ARG, "keys of a txn must be sorted and unique (Keys.ofSortedUnique)");
    if (errs & ERR_DUP_TXNID) fail(ACC_E_ARG, "TxnIds of a batch must be distinct (CommandsForKey txns are sorted unique)");
    if (errs & ERR_LOCAL_ONLY) fail(ACC_E_STATE, "Kind.witnesses(): unhandled kind LocalOnly (AssertionError)");
}

// Exact replay path (v1): committed[] per segment sorted by (executeAt, txn order) and the reference's
// FAST bisection per query; per-(T,k) lists emitted in order, then the per-T union by binary search.
// Used when executeAt ties exist (or ACC_OPT_FORCE_REPLAY).
// CommandsForKey state of a built batch, kept for the range-domain queries of acc_keydeps_mixed
struct KdState {
    bool cfk = false;                 // a CFK exists (P > 0)
    uint32_t n = 0;
    size_t P = 0;
    int rbits = 0;
    const uint32_t *rank = nullptr, *txn_of_rank = nullptr, *key_off = nullptr, *owner = nullptr;
    const uint32_t *seg_incl = nullptr, *seg_start = nullptr, *s_rank = nullptr, *s_exec = nullptr;
    const uint32_t *pair_pos = nullptr, *perm = nullptr;
    const uint8_t *s_info = nullptr;
    const uint64_t *tl = nullptr, *key_code = nullptr;
    const uint64_t *tm = nullptr, *em = nullptr, *el = nullptr;
    const int32_t *tn = nullptr, *en = nullptr;
    uint64_t *g = nullptr;
    bool have_dict = false;
    Dictionary dict;
    bool sparse = false;              // the batch has many txns without keys (a mixed batch's range txns)
    const uint64_t *seg_key = nullptr;   // per segment its key code (written by k_v2_apply)
    bool v1 = false;                  // the exact-replay columns below are built
    CfkView v1view{};
};

// Exact-replay CFK columns: uncommitted/committed flags and counts, segmented executeAt prefix max, committed[] per
// segment sorted by executeAt (CommandsForKey.java:462-469) with the nearest-Write scan
// multi_only: committed[] lists of the segments with two or more entries only, sorted at their exact size (one host
// sync): the mixed path's single-entry segments never read them
static CfkView build_v1_cfk(acc_ctx *ctx, uint32_t n, size_t P, int rbits, const uint64_t *tl, const uint32_t *owner,
                            const uint32_t *rank, const uint32_t *seg_incl, const uint32_t *seg_start,
                            const uint32_t *s_rank, const uint32_t *s_exec, const uint8_t *s_info, const uint32_t *pair_pos,
                            bool multi_only = false)
{
    const unsigned gP = grid_for(P, BLOCK);
    uint32_t *cflag = ctx->get<uint32_t>("cflag", P);
    uint32_t *uflag = ctx->get<uint32_t>("uflag", P);
    uint64_t *pmax_in = ctx->get<uint64_t>("pmax_in", P);
    launch(ctx, "v1_flags", k_v1_flags, dim3(gP), dim3(BLOCK), 0, P, s_info, s_exec, seg_incl,
           multi_only ? seg_start : (const uint32_t *)nullptr, cflag, uflag, pmax_in);
    uint32_t *cum_c = ctx->get<uint32_t>("cum_c", P + 1);
    uint32_t *cum_u = ctx->get<uint32_t>("cum_u", P + 1);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, cflag, cum_c, P, true, cum_c + P);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, uflag, cum_u, P, true, cum_u + P);
    uint64_t *pmax64 = ctx->get<uint64_t>("pmax64", P);
    scan<uint64_t, OpMax<uint64_t>>(ctx, pmax_in, pmax64, P, false);
    uint32_t *pmax = ctx->get<uint32_t>("pmax", P);
    launch(ctx, "low32", k_low32, dim3(gP), dim3(BLOCK), 0, P, (const uint64_t *)pmax64, pmax);

    // committed[] per segment: stable sort of (segment, executeAt rank)
    const int segbits = bits_for(P);
    const int cbits = segbits + rbits;
    if (cbits > 64) fail(ACC_E_ARG, "batch too large for the committed-list composite key");
    uint64_t *ckey = ctx->get<uint64_t>("ckey", P);
    uint32_t *cpos = ctx->get<uint32_t>("cpos", P);
    uint32_t *u_pos = ctx->get<uint32_t>("u_pos", P);
    launch(ctx, "committed_keys", k_committed_keys, dim3(gP), dim3(BLOCK), 0, P, (const uint32_t *)cflag,
           (const uint32_t *)cum_c, (const uint32_t *)seg_incl, (const uint32_t *)s_exec, (const uint32_t *)uflag,
           (const uint32_t *)cum_u, rbits, cbits, ckey, cpos, u_pos, multi_only ? 0 : 1);
    size_t NC = P;
    if (multi_only) {
        ACC_HIP(hipMemcpyAsync(ctx->pinned, cum_c + P, sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
        ctx->sync();
        NC = (size_t)(ctx->pinned[0] & 0xFFFFFFFFu);
        ctx->stat("keydeps.v1_committed_sorted", NC);
    }
    Sorted cs = radix_sort(ctx, "rs_cl", ckey, cpos, NC, cbits);
    uint32_t *cl_exec = ctx->get<uint32_t>("cl_exec", P);
    uint32_t *lastw_in = ctx->get<uint32_t>("lastw_in", P);
    uint32_t *lastw = ctx->get<uint32_t>("lastw", P);
    launch(ctx, "committed_cols", k_committed_cols, dim3(gP), dim3(BLOCK), 0, P, (const uint32_t *)cs.vals,
           (const uint32_t *)s_exec, (const uint8_t *)s_info, (const uint32_t *)cum_c, cl_exec, lastw_in);
    scan<uint32_t, OpMax<uint32_t>>(ctx, lastw_in, lastw, P, false);
    uint32_t *cl_start = ctx->get<uint32_t>("cl_start", P + 1);
    launch(ctx, "seg_committed_start", k_seg_committed_start, dim3(grid_for(P + 1, BLOCK)), dim3(BLOCK), 0, P,
           (const uint32_t *)seg_incl, (const uint32_t *)seg_start, (const uint32_t *)cum_c, cl_start);
    CfkView v;
    v.seg_start = seg_start; v.s_rank = s_rank; v.s_exec = s_exec; v.seg_incl = seg_incl; v.pair_pos = pair_pos;
    v.owner = owner; v.rank = rank; v.s_info = s_info; v.cl_start = cl_start; v.cl_exec = cl_exec; v.lastw = lastw;
    v.pmax = pmax; v.cum_u = cum_u; v.u_pos = u_pos; v.tl = tl; v.n = n; v.vseg = nullptr;
    return v;
}

static void keydeps_v1_tail(acc_ctx *ctx, acc_keydeps_view *view, uint32_t n, size_t P, int rbits,
                            const uint64_t *tl, const uint32_t *key_off, const uint32_t *owner,
                            const uint32_t *rank, const uint32_t *txn_of_rank, uint64_t *g, const uint32_t *seg_incl,
                            const uint32_t *seg_start, const uint32_t *s_rank, const uint32_t *s_exec, const uint8_t *s_info,
                            const uint32_t *pair_pos, KdState *ks)
{
    hipStream_t st = ctx->stream;
    const unsigned gP = grid_for(P, BLOCK);
    // ---- 4. conflict scan: count, scan, emit
    CfkView v = build_v1_cfk(ctx, n, P, rbits, tl, owner, rank, seg_incl, seg_start, s_rank, s_exec, s_info, pair_pos);
    if (ks) { ks->v1 = true; ks->v1view = v; }
    uint64_t *cnt = ctx->get<uint64_t>("cnt", P);
    uint64_t *dep_off = ctx->get<uint64_t>("dep_off", P + 1);
    launch(ctx, "query_count", k_query_count, dim3(gP), dim3(BLOCK), 0, P, v, cnt);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, cnt, dep_off, P, true, dep_off + P);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, dep_off + P, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, g + 4, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t E = ctx->pinned[0];
    check_errors(ctx->pinned[1]);
    if (E >= 0xFFFFFFFFull) fail(ACC_E_CAP, "more than 2^32-1 dependency entries in one batch");

    uint32_t *deps = ctx->get<uint32_t>("deps", E);
    uint32_t *list_of = ctx->get<uint32_t>("list_of", E);
    launch(ctx, "query_emit", k_query_emit, dim3(gP), dim3(BLOCK), 0, P, v, (const uint64_t *)dep_off, deps, list_of);

    // ---- 5. KeyDeps assembly
    const unsigned gE = grid_for(E, BLOCK);
    uint32_t *first = ctx->get<uint32_t>("first", E);
    uint32_t *cumf = ctx->get<uint32_t>("cumf", E + 1);
    launch(ctx, "first", k_first, dim3(gE), dim3(BLOCK), 0, E, (const uint32_t *)deps, (const uint32_t *)list_of,
           (const uint32_t *)owner, key_off, (const uint64_t *)dep_off, first);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, first, cumf, E, true, cumf + E);
    uint32_t *nz = ctx->get<uint32_t>("nz", P);
    uint32_t *cnz = ctx->get<uint32_t>("cnz", P + 1);
    launch(ctx, "nonempty", k_nonempty, dim3(gP), dim3(BLOCK), 0, P, (const uint64_t *)cnt, nz);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, nz, cnz, P, true, cnz + P);
    uint64_t *kd_cnt = ctx->get<uint64_t>("kd_cnt", n);
    uint64_t *u_cnt = ctx->get<uint64_t>("u_cnt", n);
    uint64_t *a_cnt = ctx->get<uint64_t>("a_cnt", n);
    launch(ctx, "txn_sizes", k_txn_sizes, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, key_off, (const uint64_t *)dep_off,
           (const uint32_t *)cnz, (const uint32_t *)cumf, kd_cnt, u_cnt, a_cnt);
    uint64_t *kd_off = ctx->get<uint64_t>("kd_off", (size_t)n + 1);
    uint64_t *u_off = ctx->get<uint64_t>("u_off", (size_t)n + 1);
    uint64_t *arena_off = ctx->get<uint64_t>("arena_off", (size_t)n + 1);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, kd_cnt, kd_off, n, true, kd_off + n);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, u_cnt, u_off, n, true, u_off + n);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, a_cnt, arena_off, n, true, arena_off + n);
    // upper bounds: ΣKd <= P, ΣU <= E, Σ(Kd+E) <= P + E
    int32_t *arena = ctx->get<int32_t>("arena", P + E);
    uint32_t *key_idx = ctx->get<uint32_t>("key_idx", P);
    uint32_t *dep_txn = ctx->get<uint32_t>("dep_txn", E);
    launch(ctx, "write_entries", k_write_entries, dim3(gE), dim3(BLOCK), 0, E, (const uint32_t *)deps,
           (const uint32_t *)list_of, (const uint32_t *)owner, key_off, (const uint64_t *)dep_off, (const uint32_t *)cumf,
           (const uint32_t *)first, (const uint32_t *)cnz, (const uint64_t *)arena_off, (const uint64_t *)u_off,
           (const uint32_t *)txn_of_rank, arena, dep_txn);
    launch(ctx, "write_keys", k_write_keys, dim3(gP), dim3(BLOCK), 0, P, (const uint64_t *)cnt, (const uint32_t *)owner,
           key_off, (const uint64_t *)dep_off, (const uint32_t *)cnz, (const uint64_t *)kd_off,
           (const uint64_t *)arena_off, key_idx, arena);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, arena_off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, kd_off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 2, u_off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    ctx->sync();
    *view = acc_keydeps_view{ n, ctx->pinned[0], ctx->pinned[1], ctx->pinned[2], E, arena_off, arena, kd_off,
                              key_idx, u_off, dep_txn };
    ctx->kd_view = *view;
    ctx->kd_valid = true;
}

// The general dictionary: a compacted LSD radix sort of all 2N timestamps (multi-word beyond 64 varying bits), dense
// ranks by a flag scan, duplicate-TxnId and executeAt-tie checks (g[4], g[6]).
static void general_ranks(acc_ctx *ctx, uint32_t n, const uint64_t *tm, const uint64_t *tl, const int32_t *tn,
                          const uint64_t *em, const uint64_t *el, const int32_t *en, const TsPlan &plan, uint64_t *g,
                          uint32_t *rank, uint32_t *txn_of_rank)
{
    hipStream_t st = ctx->stream;
    const size_t m = 2 * (size_t)n;
    uint32_t *flag = ctx->get<uint32_t>("rank_flag", m);
    uint32_t *incl = ctx->get<uint32_t>("rank_incl", m);
    const unsigned gm = grid_for(m, BLOCK);
    Sorted ts_sorted;
    if (plan.b0 + plan.b1 + plan.b2 <= 64) {
        uint64_t *ck = ctx->get<uint64_t>("ts_ckey", m);
        launch(ctx, "ts_compact", k_ts_compact, dim3(gm), dim3(BLOCK), 0, n, tm, tl, tn, em, el, en, plan, -1,
               (const uint32_t *)nullptr, ck);
        ts_sorted = radix_sort(ctx, "rs_ts", ck, nullptr, m, plan.b0 + plan.b1 + plan.b2);
        launch(ctx, "rank_flags", k_rank_flags, dim3(gm), dim3(BLOCK), 0, m, (const uint32_t *)ts_sorted.vals,
               (const uint64_t *)nullptr, (const uint64_t *)nullptr, (const uint64_t *)nullptr,
               (const uint64_t *)ts_sorted.keys, flag);
    } else {
        // multi-word LSD: node word, then lsb word, then msb word (each only over its varying bits)
        uint64_t *c[3] = { ctx->get<uint64_t>("ts_c0", m), ctx->get<uint64_t>("ts_c1", m), ctx->get<uint64_t>("ts_c2", m) };
        for (int w = 0; w < 3; ++w)
            launch(ctx, "ts_compact", k_ts_compact, dim3(gm), dim3(BLOCK), 0, n, tm, tl, tn, em, el, en, plan, w,
                   (const uint32_t *)nullptr, c[w]);
        uint64_t *tmpk = ctx->get<uint64_t>("ts_tmpk", m);
        uint32_t *permb = ctx->get<uint32_t>("ts_perm", m);
        const uint32_t *perm = nullptr;
        const int wbits[3] = { plan.b0, plan.b1, plan.b2 };
        for (int w = 2; w >= 0; --w) {
            const uint64_t *keys = c[w];
            if (perm) {
                launch(ctx, "ts_compact", k_ts_compact, dim3(gm), dim3(BLOCK), 0, n, tm, tl, tn, em, el, en, plan, w,
                       perm, tmpk);
                keys = tmpk;
            }
            Sorted s = radix_sort(ctx, "rs_ts", keys, perm, m, wbits[w]);
            ACC_HIP(hipMemcpyAsync(permb, s.vals, m * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
            perm = permb;
        }
        ts_sorted = { nullptr, permb };
        launch(ctx, "rank_flags", k_rank_flags, dim3(gm), dim3(BLOCK), 0, m, (const uint32_t *)permb,
               (const uint64_t *)c[0], (const uint64_t *)c[1], (const uint64_t *)c[2], (const uint64_t *)nullptr, flag);
    }
    scan<uint32_t, OpAdd<uint32_t>>(ctx, flag, incl, m, false);
    launch(ctx, "rank_scatter", k_rank_scatter, dim3(gm), dim3(BLOCK), 0, m, n, (const uint32_t *)ts_sorted.vals,
           (const uint32_t *)incl, rank, txn_of_rank);
    uint32_t *seen = ctx->get<uint32_t>("dup_seen", m);
    ACC_HIP(hipMemsetAsync(seen, 0, m * sizeof(uint32_t), st));
    launch(ctx, "dup_txn", k_dup_txn, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint32_t *)rank, seen, g);
    launch(ctx, "exec_ties", k_exec_ties, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint32_t *)rank, seen, g);
}

static TsPlan ts_plan(const uint64_t *hg)
{
    TsPlan plan;
    plan.r0 = make_runs(hg[0]); plan.r1 = make_runs(hg[1]); plan.r2 = make_runs(hg[2]);
    plan.b0 = plan.r0.bits; plan.b1 = plan.r1.bits; plan.b2 = plan.r2.bits;
    return plan;
}

// A batch whose sorted-batch dictionary met an executeAt tie (g[6], found after the caller's next sync when the check
// was deferred): the general dictionary instead, in place (same rank buffers). g[6] is then the exact-tie flag.
void redo_general_dictionary(acc_ctx *ctx, uint32_t n, const uint64_t *tm, const uint64_t *tl, const int32_t *tn,
                             const uint64_t *em, const uint64_t *el, const int32_t *en, uint64_t *g, Dictionary &d)
{
    ACC_HIP(hipMemsetAsync(g + 6, 0, sizeof(uint64_t), ctx->stream));
    general_ranks(ctx, n, tm, tl, tn, em, el, en, ts_plan(d.hg), g, d.rank, d.txn_of_rank);
    d.fast = false;
    d.ties_pending = false;
    ctx->stat("keydeps.fast_dictionary", 0);
}

// Validation (k_prep_txn: statuses, kinds, key order, TxnId order) and the order-rank dictionary of the 2N
// timestamps (rank[t] = TxnId of t, rank[n + t] = executeAt of t; equal <=> Timestamp.equals). Shared by the
// KeyDeps and RangeDeps paths. Throws the first validation error. defer_ties: the sorted-batch dictionary's tie check
// (g[6]) is left to the caller's next sync (out.ties_pending), which then calls redo_general_dictionary on a tie.
void prep_dictionary(acc_ctx *ctx, uint32_t n, size_t P, const uint64_t *tm, const uint64_t *tl, const int32_t *tn,
                     const uint64_t *em, const uint64_t *el, const int32_t *en, const uint8_t *status,
                     const uint32_t *key_off, const uint64_t *key_code, uint32_t *owner, uint64_t *g, Dictionary &out,
                     bool defer_ties)
{
    hipStream_t st = ctx->stream;
    // ---- 1. prep
    static_assert(8 * PREP_SLOTS <= acc_ctx::PINNED_WORDS - acc_ctx::PINNED_SLOTS, "slot rows fit the pinned area");
    static_assert(PREP_G_WORDS == 8 + 8 * PREP_SLOTS, "g and the prep slots share one buffer");
    uint64_t *gslots = g + 8;   // g has PREP_G_WORDS words
    ACC_HIP(hipMemsetAsync(g, 0, PREP_G_WORDS * sizeof(uint64_t), st));
    uint32_t *bflag = ctx->get<uint32_t>("bflag", n);
    launch(ctx, "prep_txn", k_prep_txn, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, P, tm, tl, tn, em, el, en, status,
           key_off, key_code, owner, bflag, gslots);
    // the last key_off entry must equal P
    uint64_t hg[8] = { 0, 0, 0, 0, 0, 0, 0, 0 };
    {
        // (key_off[n] == P is checked by the kernel: ERR_KEY_TOTAL)
        uint64_t *hs = ctx->pinned + acc_ctx::PINNED_SLOTS;
        ACC_HIP(hipMemcpyAsync(hs, gslots, 8 * PREP_SLOTS * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        ctx->sync();
        for (uint32_t r = 0; r < PREP_SLOTS; ++r) {
            for (int w = 0; w < 7; ++w) hg[w] |= hs[8 * r + w];
            hg[7] += hs[8 * r + 7];
        }
    }
    check_errors(hg[4]);
    const bool batch_sorted = hg[5] == 0;

    // ---- 2. dictionary: order ranks over 2N timestamps
    const TsPlan plan = ts_plan(hg);
    const size_t m = 2 * (size_t)n;
    uint32_t *rank = ctx->get<uint32_t>("rank", m);
    uint32_t *txn_of_rank = ctx->get<uint32_t>("txn_of_rank", m);
    const uint64_t nb = hg[7];
    bool fast_dict = batch_sorted && plan.b0 + plan.b1 + plan.b2 <= 64 && nb < n;
    out.ties_pending = false;
    if (fast_dict) {
        uint32_t *bidx = ctx->get<uint32_t>("bidx", (size_t)n + 1);
        scan<uint32_t, OpAdd<uint32_t>>(ctx, bflag, bidx, n, true, bidx + n);
        uint64_t *bkey = ctx->get<uint64_t>("bkey", nb);
        uint32_t *bsrc = ctx->get<uint32_t>("bsrc", nb);
        uint64_t *tkey = ctx->get<uint64_t>("tkey", n);
        launch(ctx, "b_compact", k_b_compact, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint32_t *)bflag,
               (const uint32_t *)bidx, em, el, en, tm, tl, tn, plan, bkey, bsrc, tkey);
        Sorted sb = radix_sort(ctx, "rs_b", bkey, nullptr, nb, plan.b0 + plan.b1 + plan.b2);
        launch(ctx, "rank_txn_sorted", k_rank_txn_sorted, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (uint32_t)nb,
               (const uint64_t *)tkey, (const uint64_t *)sb.keys, (const uint32_t *)bflag, rank, txn_of_rank, g);
        launch(ctx, "rank_b_sorted", k_rank_b_sorted, dim3(grid_for(nb, BLOCK)), dim3(BLOCK), 0, n, (uint32_t)nb,
               (const uint64_t *)tkey, (const uint64_t *)sb.keys, (const uint32_t *)sb.vals, (const uint32_t *)bsrc, rank, g);
        if (defer_ties) {
            out.ties_pending = true;
        } else {
            ACC_HIP(hipMemcpyAsync(ctx->pinned, g + 6, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
            ctx->sync();
            if (ctx->pinned[0]) {   // an executeAt equals another timestamp: dense ranks need the general dictionary
                ACC_HIP(hipMemsetAsync(g + 6, 0, sizeof(uint64_t), st));
                fast_dict = false;
            }
        }
    }
    if (!fast_dict) general_ranks(ctx, n, tm, tl, tn, em, el, en, plan, g, rank, txn_of_rank);
    ctx->stat("keydeps.fast_dictionary", fast_dict ? 1 : 0);
    out.rank = rank;
    out.txn_of_rank = txn_of_rank;
    out.rbits = bits_for(m - 1);
    out.batch_sorted = batch_sorted;
    out.fast = fast_dict;
    memcpy(out.hg, hg, sizeof hg);
}

static void keydeps_core(acc_ctx *ctx, const acc_batch_in *in, acc_keydeps_view *view, KdState *ks,
                         bool cfk_only = false)
{
    if (!in || !view) fail(ACC_E_ARG, "null argument");
    if (in->mem != ACC_MEM_HOST && in->mem != ACC_MEM_DEVICE) fail(ACC_E_ARG, "mem must be ACC_MEM_HOST or ACC_MEM_DEVICE");
    const uint32_t n = in->n_txn;
    const size_t P = (size_t)in->n_pairs;
    if (P >= 0xFFFFFFFFull) fail(ACC_E_ARG, "n_pairs must be < 2^32");
    hipStream_t st = ctx->stream;
    ctx->kd_valid = false;

    // ---- stage inputs
    const uint32_t *key_off = stage_in(ctx, "in_key_off", in->key_off, (size_t)n + 1, in->mem);
    if (n == 0 || P == 0) {
        // no pairs: every txn has KeyDeps.NONE
        uint64_t *arena_off = ctx->get<uint64_t>("arena_off", (size_t)n + 1);
        uint64_t *kd_off = ctx->get<uint64_t>("kd_off", (size_t)n + 1);
        uint64_t *u_off = ctx->get<uint64_t>("u_off", (size_t)n + 1);
        ACC_HIP(hipMemsetAsync(arena_off, 0, ((size_t)n + 1) * 8, st));
        ACC_HIP(hipMemsetAsync(kd_off, 0, ((size_t)n + 1) * 8, st));
        ACC_HIP(hipMemsetAsync(u_off, 0, ((size_t)n + 1) * 8, st));
        *view = acc_keydeps_view{ n, 0, 0, 0, 0, arena_off, ctx->get<int32_t>("arena", 1), kd_off,
                                  ctx->get<uint32_t>("key_idx", 1), u_off, ctx->get<uint32_t>("dep_txn", 1) };
        ctx->kd_view = *view;
        ctx->kd_valid = true;
        ctx->sync();
        return;
    }
    const uint64_t *tm = stage_in(ctx, "in_tm", in->txn_id.msb, n, in->mem);
    const uint64_t *tl = stage_in(ctx, "in_tl", in->txn_id.lsb, n, in->mem);
    const int32_t *tn = stage_in(ctx, "in_tn", in->txn_id.node, n, in->mem);
    const uint64_t *em = stage_in(ctx, "in_em", in->execute_at.msb, n, in->mem);
    const uint64_t *el = stage_in(ctx, "in_el", in->execute_at.lsb, n, in->mem);
    const int32_t *en = stage_in(ctx, "in_en", in->execute_at.node, n, in->mem);
    const uint8_t *status = stage_in(ctx, "in_status", in->status, n, in->mem);
    const uint64_t *key_code = stage_in(ctx, "in_key_code", in->key_code, P, in->mem);

    // ---- 1-2. prep + dictionary
    uint64_t *g = ctx->get<uint64_t>("g", PREP_G_WORDS);
    uint32_t *owner = ctx->get<uint32_t>("owner", P);
    Dictionary dict;
    // the sorted-batch dictionary's tie check is read at the CFK sync below (one host sync fewer)
    prep_dictionary(ctx, n, P, tm, tl, tn, em, el, en, status, key_off, key_code, owner, g, dict, true);
    uint64_t hg[8];
    memcpy(hg, dict.hg, sizeof hg);
    const bool batch_sorted = dict.batch_sorted;
    uint32_t *const rank = dict.rank, *const txn_of_rank = dict.txn_of_rank;
    const int rbits = dict.rbits;

    // ---- 3. CFK build: pairs sorted by (key, TxnId rank)
    uint4 *tinfo = ctx->get<uint4>("tinfo", n);
    uint32_t *bigflag = ctx->get<uint32_t>("v3_bigflag", n);
    bool tinfo_done = false;   // the txn records written by the pair-key launch
    PairPlan pp;
    pp.rk = make_runs(hg[3]);
    pp.rbits = rbits;
    uint64_t *pkey = ctx->get<uint64_t>("pair_key", P);
    const unsigned gP = grid_for(P, BLOCK);
    Sorted ps;
    int key_shift = 0;
    uint32_t *seg_flag = ctx->get<uint32_t>("seg_flag", P);
    bool flags_done = false;
    const uint64_t *sp_m4 = nullptr;   // mode 4: the sorted packed keys, unpacked by the CFK gather
    pp.sb = std::max(1, bits_for(hg[6]));   // bounds the key slot within a txn (hg[6] = OR of the key counts)
    if (batch_sorted && pp.rk.bits <= 32) {
        // pair index order is already TxnId order within every key: a stable keys-only sort of (key << 32 | pair index),
        // 8 B per element; the segment flags pass unpacks the permutation. Mode 4 packs (owner, slot) instead of the
        // pair index and the CFK gather unpacks it (one random read of the owner's record per pair, which carries
        // key_off[owner] for the pair index)
        const bool m4 = bits_for((uint64_t)n - 1) + pp.sb <= 32;
        pp.mode = m4 ? 4 : 3;
        TxnInfoArgs ti;   // the txn records (k_txn_info) by the same launch: the ranks are final unless ties turn up
        ti.n = n; ti.status = status; ti.tl = tl; ti.tinfo = tinfo; ti.bigflag = bigflag;
        launch(ctx, "pair_keys", k_pair_keys, dim3(grid_for(std::max<size_t>(P, n), BLOCK)), dim3(BLOCK), 0, P, key_code,
               (const uint32_t *)owner, key_off, (const uint32_t *)rank, (const uint32_t *)nullptr, pp, 0, pkey, ti);
        tinfo_done = true;
        const uint64_t *sp = radix_sort_keys(ctx, "rs_pair", pkey, P, 32, pp.rk.bits);
        uint32_t *perm = ctx->get<uint32_t>("pair_perm", P + V2_ITEMS);
        if (m4) sp_m4 = sp;
        else launch(ctx, "seg_flags", k_seg_flags_packed, dim3(gP), dim3(BLOCK), 0, P, sp, seg_flag, perm, -1, key_off,
                    (uint32_t *)nullptr);
        ps = { nullptr, perm };
        flags_done = true;
    } else if (batch_sorted) {
        pp.mode = 0;   // pair index order is already TxnId order within every key: stable sort by key
        launch(ctx, "pair_keys", k_pair_keys, dim3(gP), dim3(BLOCK), 0, P, key_code, (const uint32_t *)owner, key_off,
               (const uint32_t *)rank, (const uint32_t *)nullptr, pp, 0, pkey, TxnInfoArgs{});
        ps = radix_sort(ctx, "rs_pair", pkey, nullptr, P, pp.rk.bits);
    } else if (pp.rk.bits + rbits <= 64) {
        pp.mode = 1;
        launch(ctx, "pair_keys", k_pair_keys, dim3(gP), dim3(BLOCK), 0, P, key_code, (const uint32_t *)owner, key_off,
               (const uint32_t *)rank, (const uint32_t *)nullptr, pp, 0, pkey, TxnInfoArgs{});
        ps = radix_sort(ctx, "rs_pair", pkey, nullptr, P, pp.rk.bits + rbits);
        key_shift = rbits;
    } else {
        pp.mode = 2;
        launch(ctx, "pair_keys", k_pair_keys, dim3(gP), dim3(BLOCK), 0, P, key_code, (const uint32_t *)owner, key_off,
               (const uint32_t *)rank, (const uint32_t *)nullptr, pp, 1, pkey, TxnInfoArgs{});
        Sorted byrank = radix_sort(ctx, "rs_pair_r", pkey, nullptr, P, rbits);
        launch(ctx, "pair_keys", k_pair_keys, dim3(gP), dim3(BLOCK), 0, P, key_code, (const uint32_t *)owner, key_off,
               (const uint32_t *)rank, (const uint32_t *)byrank.vals, pp, 0, pkey, TxnInfoArgs{});
        ps = radix_sort(ctx, "rs_pair", pkey, byrank.vals, P, pp.rk.bits);
    }
    uint32_t *seg_incl = ctx->get<uint32_t>("seg_incl", P + V2_ITEMS);   // written by k_v2_apply (the multi-scan's column 8)
    if (!flags_done)
        launch(ctx, "seg_flags", k_seg_flags, dim3(gP), dim3(BLOCK), 0, P, (const uint64_t *)ps.keys, key_shift, seg_flag);

    uint32_t *seg_start = ctx->get<uint32_t>("seg_start", P + 1);
    uint64_t *seg_key_buf = ks ? ctx->get<uint64_t>("seg_key", P + 1) : nullptr;   // per segment its key code
    uint32_t *s_rank = ctx->get<uint32_t>("s_rank", P + V2_ITEMS);   // padded for the 16-B column loads
    uint32_t *s_exec = ctx->get<uint32_t>("s_exec", P + V2_ITEMS);
    uint8_t *s_info = ctx->get<uint8_t>("s_info", P + V2_ITEMS);
    uint32_t *pair_pos = ctx->get<uint32_t>("pair_pos", P);
    uint4 *ptinfo = sp_m4 ? nullptr : ctx->get<uint4>("pair_tinfo", P);
    bool have_pair_pos = ks != nullptr;
    uint64_t rk_mask = 0;   // the bits the key compaction keeps (k_v2_apply rebuilds segment key codes from them)
    for (int r = 0; r < pp.rk.n; ++r) rk_mask |= (pp.rk.len[r] >= 64 ? ~0ull : ((1ull << pp.rk.len[r]) - 1)) << pp.rk.lo[r];
    auto need_pair_pos = [&]() {
        if (have_pair_pos) return;
        launch(ctx, "pair_pos", k_pair_pos, dim3(gP), dim3(BLOCK), 0, P, (const uint32_t *)ps.vals, pair_pos);
        have_pair_pos = true;
    };
    const int segbits = bits_for(P);
    // ---- v2 structures (class lists, prefix counts, bumped committed list)
    const uint32_t nt = (uint32_t)((P + V2_TILE - 1) / V2_TILE);
    uint32_t *tile_sums = ctx->get<uint32_t>("v2_tile_sums", (size_t)NCNT * nt);
    uint32_t *tile_pref = ctx->get<uint32_t>("v2_tile_pref", (size_t)NCNT * nt);
    uint32_t *totals = ctx->get<uint32_t>("v2_totals", 16);
    uint32_t *bases = ctx->get<uint32_t>("v2_bases", 16);
    V2Cols cols;
    cols.rdir = ctx->get<uint4>("v2_rdir", 4 * (P / RD_W + 1));
    cols.list_rank = ctx->get<uint32_t>("v2_list_rank", P);
    cols.bc_rank = ctx->get<uint32_t>("v2_bc_rank", P);
    cols.bc_exec = ctx->get<uint32_t>("v2_bc_exec", P);
    cols.bc_kind = ctx->get<uint8_t>("v2_bc_kind", P);
    cols.bc_pm_in = ctx->get<uint64_t>("v2_bc_pm_in", P);
    cols.bc_key = ctx->get<uint64_t>("v2_bc_key", P);
    // the count / mark passes' accumulators, zeroed by the column kernels (txn records, k_v2_apply); bigflag above
    uint64_t *tot = ctx->get<uint64_t>("v3_tot", 4);   // E, big txns, a 9-16-key big txn, stream txns with a run record
    uint64_t *gstat = ctx->get<uint64_t>("v2_gstat", GSTAT_N + 6);   // + the batch totals and E / big counts (k_v3_ucompact)
    // the rank-dependent columns (run again when the deferred tie check finds the sorted-batch ranks invalid)
    auto build_columns = [&]() {
        if (!tinfo_done)
            launch(ctx, "txn_info", k_txn_info, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint32_t *)rank, status,
                   tl, key_off, tinfo, bigflag);
        tinfo_done = false;   // a second build (the ties re-rank) writes them again
        if (!sp_m4)
            launch(ctx, "pair_tinfo", k_pair_tinfo, dim3(gP), dim3(BLOCK), 0, P, (const uint32_t *)owner, (const uint4 *)tinfo, ptinfo);
        launch(ctx, "cfk_gather", k_cfk_gather4, dim3(nt), dim3(BLOCK), 0, P, ps.vals, (const uint4 *)ptinfo, sp_m4, pp.sb,
               (const uint4 *)tinfo, seg_flag, s_rank, s_exec, s_info, ks ? pair_pos : (uint32_t *)nullptr, tile_sums, nt);
        launch(ctx, "v2_tile_scans", k_v2_tile_scans, dim3(NCNT), dim3(BLOCK), 0, (const uint32_t *)tile_sums, tile_pref, nt, totals);
        launch(ctx, "v2_apply", k_v2_apply, dim3(nt), dim3(BLOCK), 0, P, (const uint32_t *)s_rank, (const uint32_t *)s_exec,
               (const uint8_t *)s_info, (const uint32_t *)seg_flag, (const uint32_t *)tile_pref, (const uint32_t *)totals, nt,
               rbits, cols, seg_incl, seg_start, (const uint32_t *)ps.vals, key_code, seg_key_buf, sp_m4, pp.rk, rk_mask,
               bases, tot, 4u, gstat, (uint32_t)GSTAT_N, (const uint64_t *)g, reinterpret_cast<uint64_t *>(totals) + 4);
    };
    build_columns();
    // totals, g[4..6] staged by k_v2_apply, the bumped-query count
    ACC_HIP(hipMemcpyAsync(ctx->pinned, totals, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    ctx->sync();
    if (dict.ties_pending && ctx->pinned[6]) {
        // an executeAt equals another timestamp: the sorted-batch ranks are not dense ranks; the general dictionary,
        // then the rank-dependent columns again (the pair order does not depend on ranks in a sorted batch)
        check_errors(ctx->pinned[4]);
        redo_general_dictionary(ctx, n, tm, tl, tn, em, el, en, g, dict);
        build_columns();
        ACC_HIP(hipMemcpyAsync(ctx->pinned, totals, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        ctx->sync();
    }
    dict.ties_pending = false;
    if (ks) { ks->have_dict = true; ks->dict = dict; ks->owner = owner; }
    uint32_t htot[16];
    memcpy(htot, ctx->pinned, sizeof htot);
    check_errors(ctx->pinned[4]);
    const bool ties = ctx->pinned[6] != 0;
    ctx->stat("keydeps.path_replay", ties || (ctx->flags & ACC_OPT_FORCE_REPLAY) ? 1 : 0);
    ctx->stat("keydeps.exec_ties", ties ? 1 : 0);
    ctx->stat("keydeps.batch_sorted", batch_sorted ? 1 : 0);
    if (ks) {
        ks->cfk = true; ks->n = n; ks->P = P; ks->rbits = rbits; ks->rank = rank; ks->txn_of_rank = txn_of_rank;
        ks->key_off = key_off; ks->owner = owner; ks->seg_incl = seg_incl; ks->seg_start = seg_start;
        ks->s_rank = s_rank; ks->s_exec = s_exec; ks->pair_pos = pair_pos; ks->perm = ps.vals; ks->s_info = s_info;
        ks->tl = tl; ks->key_code = key_code; ks->g = g; ks->seg_key = seg_key_buf;
        ks->tm = tm; ks->tn = tn; ks->em = em; ks->el = el; ks->en = en;
    }
    if (cfk_only) return;
    if (ties || (ctx->flags & ACC_OPT_FORCE_REPLAY)) {
        need_pair_pos();
        keydeps_v1_tail(ctx, view, n, P, rbits, tl, key_off, owner, rank, txn_of_rank, g, seg_incl, seg_start,
                        s_rank, s_exec, s_info, pair_pos, ks);
        return;
    }
    const uint32_t nbc = htot[6];
    if (segbits + rbits > 64) fail(ACC_E_ARG, "batch too large for the (segment, executeAt) composite key");
    Sorted bcs = radix_sort(ctx, "rs_bc", cols.bc_key, nullptr, nbc, segbits + rbits);
    uint32_t *bcs_exec = ctx->get<uint32_t>("v2_bcs_exec", nbc);
    uint64_t *bcs_lw_in = ctx->get<uint64_t>("v2_bcs_lw_in64", nbc), *bcs_lw64 = ctx->get<uint64_t>("v2_bcs_lastw64", nbc);
    launch(ctx, "v2_bcs_cols", k_v2_bcs_cols, dim3(grid_for(nbc, BLOCK)), dim3(BLOCK), 0, nbc, (const uint64_t *)bcs.keys,
           (const uint32_t *)bcs.vals, (const uint8_t *)cols.bc_kind, (uint64_t)((1ull << rbits) - 1), bcs_exec, bcs_lw_in);
    uint64_t *bc_pm64 = ctx->get<uint64_t>("v2_bc_pm64", nbc);
    {   // nearest-Write index and the segmented executeAt maximum: two prefix maxima in one launch (read as low words)
        const uint64_t *si[2] = { bcs_lw_in, cols.bc_pm_in };
        uint64_t *so[2] = { bcs_lw64, bc_pm64 };
        const size_t sn[2] = { nbc, nbc };
        scan_multi<uint64_t, OpMax<uint64_t>>(ctx, 2, si, so, sn, false, (uint64_t *const *)nullptr);
    }

    V2View vv{};
    vv.perm = ps.vals; vv.pair_pos = pair_pos; vv.seg_incl = seg_incl; vv.seg_start = seg_start;
    vv.s_rank = s_rank; vv.s_exec = s_exec; vv.s_info = s_info; vv.rdir = cols.rdir; vv.tinfo = tinfo;
    vv.list_rank = cols.list_rank; vv.bases = bases; vv.bc_rank = cols.bc_rank; vv.bc_exec = cols.bc_exec; vv.bc_pm = bc_pm64;
    vv.bc_kind = cols.bc_kind; vv.bcs_exec = bcs_exec; vv.bcs_lastw = bcs_lw64;
    // ---- count pass: per-pair records, big-txn flags, E
    if (P >= 0x80000000ull) fail(ACC_E_CAP, "n_pairs must be < 2^31 (count-pass record format)");
    RecOut ro;
    ro.rec = ctx->get<uint4>("v2_rec", 4 * P);
    ro.irec = ctx->get<uint4>("v2_irec", 2 * P);
    uint4 *rec = ro.rec;
    vv.irec32 = reinterpret_cast<const uint32_t *>(ro.irec);
    vv.rec = ro.rec;

    uint32_t *bpos = ctx->get<uint32_t>("v3_bpos", n);
    uint64_t *blk_e = ctx->get<uint64_t>("v3_blk_e", gP);
    uint32_t *psz = ctx->get<uint32_t>("v3_psz", P);   // the big txns' per-pair entry counts (mark pass -> bigfill)
#ifdef ACC_PHASE_PROF
    const size_t ct_rows = (size_t)gP * WAVES;
    unsigned long long *ct_buf = ctx->get<unsigned long long>("v2_ct_prof", 8 * ct_rows);
    ACC_HIP(hipMemsetAsync(ct_buf, 0, 8 * ct_rows * sizeof(unsigned long long), st));
    ACC_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_ct_prof), &ct_buf, sizeof ct_buf, 0, hipMemcpyHostToDevice, st));
#endif
    launch(ctx, "v2_count", k_v2_count, dim3(gP), dim3(BLOCK), 0, P, vv, (const uint32_t *)owner, ro, bigflag, blk_e);
#ifdef ACC_PHASE_PROF
    {
        std::vector<unsigned long long> h(8 * ct_rows);
        ACC_HIP(hipMemcpyAsync(h.data(), ct_buf, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
        ACC_HIP(hipStreamSynchronize(st));
        double sum[8] = {}, mx[3] = {};
        size_t w = 0;
        for (size_t r = 0; r < ct_rows; ++r) {
            if (!(h[8 * r + 7] >> 32)) continue;
            ++w;
            for (int i = 0; i < 7; ++i) sum[i] += (double)h[8 * r + i];
            sum[7] += (double)(h[8 * r + 7] & 0xFFFFFFFFu);
            for (int i = 0; i < 3; ++i) mx[i] = std::max(mx[i], (double)h[8 * r + i]);
        }
        const double d = w ? (double)w : 1.0;
        fprintf(stderr, "[ct_phase] waves=%zu avg cycles: query %.0f r3count %.0f inline+write %.0f | max %.0f %.0f %.0f | "
                "per pair: bumped %.4f seg-with-bc %.4f posM-search %.4f r3-candidates %.3f run-records %.4f\n",
                w, sum[0] / d, sum[1] / d, sum[2] / d, mx[0], mx[1], mx[2], sum[3] / P, sum[4] / P, sum[5] / P, sum[6] / P,
                sum[7] / P);
    }
#endif
    const uint32_t raw_cap = ST_RAW;
    uint64_t *kd_off = ctx->get<uint64_t>("kd_off", (size_t)n + 1);
    uint64_t *arena_off = ctx->get<uint64_t>("arena_off", (size_t)n + 1);
    uint64_t *szA = ctx->get<uint64_t>("v3_szA", n), *szK = ctx->get<uint64_t>("v3_szK", n);
    uint64_t *eb = ctx->get<uint64_t>("v3_eb", n), *dB = ctx->get<uint64_t>("v3_dB", (size_t)n + 1);
    uint32_t *runflag = ctx->get<uint32_t>("v3_runflag", n);
    launch(ctx, "v3_mark", k_v3_mark, dim3(grid_for((size_t)n * MK_G, BLOCK)), dim3(BLOCK), 0, n, key_off,
           (const uint32_t *)ro.irec, (const uint4 *)rec, psz, raw_cap, bigflag, szA, szK, tot + 2, eb, runflag);
    uint64_t *blk_pre = ctx->get<uint64_t>("v3_blk_pre", gP);
    {   // arena / key offsets, the count pass's per-block entry totals, the big txns' TxnId scratch bases: one launch
        const uint64_t *si[4] = { szA, szK, blk_e, eb };
        uint64_t *so[4] = { arena_off, kd_off, blk_pre, dB }, *stot[4] = { arena_off + n, kd_off + n, tot, dB + n };
        const size_t sn[4] = { n, n, gP, n };
        scan_multi<uint64_t, OpAdd<uint64_t>>(ctx, 4, si, so, sn, true, stot);
    }
    // the big-txn list in txn order (k_v3_bigfill's per-txn ranges abut: a big txn writes its end where the next
    // txn's first pair starts, equal values when the next txn is big too)
    scan<uint32_t, OpAdd<uint32_t>>(ctx, bigflag, bpos, n, true, reinterpret_cast<uint32_t *>(tot + 1));
    uint32_t *blist = ctx->get<uint32_t>("v3_blist", n);
    launch(ctx, "v3_compact", k_v3_compact, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint32_t *)bigflag,
           (const uint32_t *)bpos, blist);
    // the stream txns with a run record, for the RUNS stream pass
    uint32_t *rpos = ctx->get<uint32_t>("v3_rpos", n), *rlist = ctx->get<uint32_t>("v3_rlist", n);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, runflag, rpos, n, true, reinterpret_cast<uint32_t *>(tot + 3));
    launch(ctx, "v3_compact", k_v3_compact, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint32_t *)runflag,
           (const uint32_t *)rpos, rlist);
    // ---- E (dependency entries), the big-txn count and the 9-16-key flag reach the host here
    ACC_HIP(hipMemcpyAsync(ctx->pinned, tot, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t E = ctx->pinned[0];
    const uint32_t nbig = (uint32_t)ctx->pinned[1];
    const bool any16 = ctx->pinned[2] != 0;
    const uint32_t nrun = (uint32_t)ctx->pinned[3];
    if (E >= 0xFFFFFFFFull) fail(ACC_E_CAP, "more than 2^32-1 dependency entries in one batch");
    uint64_t *u_off = ctx->get<uint64_t>("u_off", (size_t)n + 1);
    uint64_t *u_cnt = ctx->get<uint64_t>("u_cnt", n);
    uint64_t *vdep_off = nullptr;
    uint32_t *dep_scr = nullptr;
    uint64_t nfb = 0, efb = 0, nmed = 0, nbig2 = 0;
    ctx->stat("keydeps.huge_txns", 0);
    V2Out wo{};
    bool win_ok = false;
    uint64_t *vcnt = nullptr;
    uint32_t *med_list = nullptr, *big_list = nullptr, *fb_list = nullptr;
    // the sorting tiers: medium (<= MED_CAP raw entries), block (<= BIG_E), huge (<= HUGE_E, fed by the block tier)
    auto sort_tiers = [&](bool with_med) {
        if (with_med)
            launch(ctx, "v2_write_med", k_v2_write_big<MED_CAP, BLOCK>, dim3(std::min<unsigned>(nbig, 2048)), dim3(BLOCK), 0,
                   (const uint32_t *)med_list, vv, (const uint64_t *)vcnt, wo);
        launch(ctx, "v2_write_big", k_v2_write_big<BIG_E, 512>, dim3(std::min<unsigned>(nbig, 1024)), dim3(512), 0,
               (const uint32_t *)big_list, vv, (const uint64_t *)vcnt, wo);
        launch(ctx, "v2_write_huge", k_v2_write_big<HUGE_E, 1024>, dim3(std::min<unsigned>(nbig, 64)), dim3(1024), 0,
               (const uint32_t *)wo.huge_list, vv, (const uint64_t *)vcnt, wo);
    };
    uint32_t *dep_st = ctx->get<uint32_t>("v3_dep_stream", (size_t)n * ST_SLOT);   // stream txns' TxnIds, slot t * ST_SLOT
    int32_t *const arena = ctx->get<int32_t>("arena", P + E);
    uint32_t *const key_idx = ctx->get<uint32_t>("key_idx", P);
    uint32_t *const dep_txn = ctx->get<uint32_t>("dep_txn", std::max<uint64_t>(E, 1));
    // ---- big txns' arena / keys into place, TxnId offsets and compaction. With global-path txns (known only after
    // the tiers ran) this is redone once they are written, so the common case pays one host sync here.
    auto finish = [&]() {
        scan<uint64_t, OpAdd<uint64_t>>(ctx, u_cnt, u_off, n, true, u_off + n);
        const uint32_t *tmap = nullptr, *ne_cnt = nullptr;
        const uint64_t *uo = u_off;
        if (ks && ks->sparse) {
            uint32_t *flag = ctx->get<uint32_t>("v3_ne_flag", n), *pos = ctx->get<uint32_t>("v3_ne_pos", n);
            uint32_t *cnt = ctx->get<uint32_t>("v3_ne_cnt", 1), *ne_t = ctx->get<uint32_t>("v3_ne_t", n);
            uint64_t *ne_uoff = ctx->get<uint64_t>("v3_ne_uoff", (size_t)n + 1);
            launch(ctx, "v3_neflag", k_v3_neflag, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint64_t *)u_cnt, flag);
            scan<uint32_t, OpAdd<uint32_t>>(ctx, flag, pos, n, true, cnt);
            launch(ctx, "v3_nelist", k_v3_nelist, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint32_t *)flag,
                   (const uint32_t *)pos, (const uint32_t *)cnt, (const uint64_t *)u_off, ne_t, ne_uoff);
            tmap = ne_t; ne_cnt = cnt; uo = ne_uoff;
        }
        launch(ctx, "v3_ucompact", k_v3_ucompact, dim3((unsigned)((E + UC_CHUNK - 1) / UC_CHUNK) + 1), dim3(BLOCK), 0, n,
               uo, (const uint64_t *)arena_off, (const uint64_t *)kd_off, (const uint32_t *)bigflag, key_off,
               (const uint64_t *)vdep_off, (const uint32_t *)dep_st, (const uint32_t *)dep_scr,
               tmap, ne_cnt, dep_txn, (const uint64_t *)u_off, gstat + GSTAT_N);
        ACC_HIP(hipMemcpyAsync(ctx->pinned, gstat, (GSTAT_N + 6) * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        ctx->sync();
    };
    // ---- big txns: v2 tiers, headers / key indices / entries into the final arrays, TxnIds into scratch
    if (nbig) {
        const unsigned gB = (nbig + WAVES - 1) / WAVES;
        vdep_off = ctx->get<uint64_t>("dep_off", P + 1);
        vcnt = ctx->get<uint64_t>("cnt", P);
        uint32_t *vcnz = ctx->get<uint32_t>("cnz", P + 1);
        dep_scr = ctx->get<uint32_t>("v2_dep_scratch", std::max<uint64_t>(E, 1));
        med_list = ctx->get<uint32_t>("v2_med_list", nbig);
        big_list = ctx->get<uint32_t>("v2_big_list", nbig);
        fb_list = ctx->get<uint32_t>("v2_fb_list", nbig);
        V3Big bg;
        bg.blist = blist; bg.key_off = key_off; bg.psz = psz; bg.dB = dB; bg.arena_off = arena_off; bg.kd_off = kd_off;
        bg.vdep_off = vdep_off; bg.vcnt = vcnt; bg.vcnz = vcnz; bg.u_cnt = u_cnt; bg.arena = arena; bg.key_idx = key_idx;
        const bool big_ok = rbits + 6 <= 31;
        win_ok = big_ok && !(ctx->flags & ACC_OPT_NO_WINDOW_TIER);   // (testing: the sorting tiers instead)
        launch(ctx, "v3_route", k_v3_route, dim3(grid_for(nbig, BLOCK)), dim3(BLOCK), 0, nbig, (const uint32_t *)blist,
               key_off, (const uint64_t *)eb, (int)big_ok, (int)win_ok, med_list, big_list, fb_list,
               ctx->get<uint32_t>("v2_w8_list", nbig), ctx->get<uint32_t>("v2_w16_list", nbig), gstat);
        launch(ctx, "v3_bigfill", k_v3_bigfill, dim3(gB), dim3(BLOCK), 0, nbig, bg);
        wo.key_off = key_off; wo.dep_off = vdep_off; wo.arena_off = arena_off; wo.cnz = vcnz; wo.txn_of_rank = txn_of_rank;
        wo.arena = arena; wo.dep_scratch = dep_scr; wo.u_cnt = u_cnt; wo.gstat = gstat;
        wo.rec = rec; wo.irec32 = vv.irec32; wo.med_list = med_list; wo.big_list = big_list; wo.fb_list = fb_list;
        wo.huge_list = ctx->get<uint32_t>("v2_huge_list", nbig);
        // persistent grids over device-side list counts (routing happened after the last host sync); the tiers run on a
        // side stream, concurrently with the stream pass (it needs only the big txns' sizes, set by bigfill)
        ctx->fork(nrun ? 2 : 1);
        ctx->launch_stream = ctx->aux[0];
        if (win_ok) {
#ifdef ACC_PHASE_PROF
            {
                unsigned long long *wpb = ctx->get<unsigned long long>("v2_win_prof", 10);
                ACC_HIP(hipMemsetAsync(wpb, 0, 80, ctx->aux[0]));
                ACC_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_win_prof), &wpb, sizeof wpb, 0, hipMemcpyHostToDevice, ctx->aux[0]));
            }
#endif
            // the window tier takes every big txn of <= 16 keys; the sorting tiers run after the next host sync, only
            // when it passed txns on or some txn has more keys (no launch without work)
            launch(ctx, "v2_write_win", k_v2_write_win<8>, dim3(std::min<unsigned>(nbig, 2048)), dim3(BLOCK), 0,
                   (const uint32_t *)ctx->get<uint32_t>("v2_w8_list", nbig), (const uint64_t *)(gstat + 7), vv,
                   (const uint64_t *)vcnt, wo);
            // (> 8 keys is rare: a small persistent grid, launched only when the mark pass saw a big txn of 9-16 keys)
            if (any16)
                launch(ctx, "v2_write_win16", k_v2_write_win<16>, dim3(std::min<unsigned>(nbig, 256)), dim3(BLOCK), 0,
                       (const uint32_t *)ctx->get<uint32_t>("v2_w16_list", nbig), (const uint64_t *)(gstat + 8), vv,
                       (const uint64_t *)vcnt, wo);
        } else if (big_ok) {
            sort_tiers(true);
        } else {
            // ranks beyond 25 bits: u64 records in the wave tier (k_v3_route sends everything else to the global path)
            launch(ctx, "v2_write_medium", k_v2_write_medium, dim3(std::min<unsigned>(gB, 2048)), dim3(BLOCK), 0,
                   (const uint64_t *)gstat, (const uint32_t *)med_list, vv, (const uint64_t *)vcnt, wo);
        }
        ctx->launch_stream = nullptr;
    }
    {
        // ---- stream pass: the stream txns' KeyDeps (a grid over every txn, 16 lanes per txn), TxnIds to scratch;
        // 256-thread workgroups co-schedule best with the 512-thread block tier
        constexpr int st_nt = 256;
        const uint32_t tt = (uint32_t)st_nt / ST_G;
        const uint32_t nblocks = (n + tt - 1) / tt;
        const uint32_t ntiles = nblocks * (uint32_t)(st_nt / 64);   // waves (phase-profile rows)
        V3Stream sp;
        sp.v = vv; sp.err = gstat + 5;
        sp.key_off = key_off; sp.bigflag = bigflag; sp.list = nullptr; sp.txn_of_rank = txn_of_rank;
        sp.rec = rec; sp.irec = ro.irec;
        sp.arena_off = arena_off; sp.kd_off = kd_off; sp.u_cnt_out = u_cnt; sp.arena = arena; sp.key_idx = key_idx;
        sp.dep_scr = dep_st; sp.n = n; sp.ntiles = ntiles;
#ifdef ACC_PHASE_PROF
        const size_t prof_rows = (size_t)ntiles;
        unsigned long long *prof_buf = ctx->get<unsigned long long>("v3_prof", 8 * prof_rows);
        ACC_HIP(hipMemsetAsync(prof_buf, 0, 8 * prof_rows * sizeof(unsigned long long), st));
        ACC_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_st_prof), &prof_buf, sizeof prof_buf, 0, hipMemcpyHostToDevice, st));
#endif
        if (nrun) {
            // the stream txns with a run record on side stream 1, concurrently with the lean pass below (their gathers
            // kept out of the lean pass: registers and a wave-uniform loop in every wave that holds one; config 2: 25%
            // of the txns)
            if (!nbig) ctx->fork(2);
            V3Stream sr = sp;
            sr.list = rlist; sr.n = nrun;
            const uint32_t rblocks = (nrun + tt - 1) / tt;
            ctx->launch_stream = ctx->aux[1];
            if (rbits <= 28) launch(ctx, "v3_stream_runs", k_v3_stream<uint32_t, st_nt, ST_G, ST_N2, true, true>, dim3(rblocks), dim3(st_nt), 0, sr);
            else launch(ctx, "v3_stream_runs", k_v3_stream<uint64_t, st_nt, ST_G, ST_N2, true, true>, dim3(rblocks), dim3(st_nt), 0, sr);
            ctx->launch_stream = nullptr;
        }
        if (rbits <= 28) launch(ctx, "v3_stream", k_v3_stream<uint32_t, st_nt, ST_G, ST_N2, false, false>, dim3(nblocks), dim3(st_nt), 0, sp);
        else launch(ctx, "v3_stream", k_v3_stream<uint64_t, st_nt, ST_G, ST_N2, false, false>, dim3(nblocks), dim3(st_nt), 0, sp);
#ifdef ACC_PHASE_PROF
        {
            std::vector<unsigned long long> h(8 * prof_rows);
            ACC_HIP(hipMemcpyAsync(h.data(), prof_buf, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
            ACC_HIP(hipStreamSynchronize(st));
            double sum[6] = {}, mx[6] = {};
            size_t w = 0;
            for (size_t r = 0; r < prof_rows; ++r) {
                if (!h[8 * r + 7]) continue;
                ++w;
                for (int i = 0; i < 6; ++i) { sum[i] += (double)h[8 * r + i]; mx[i] = std::max(mx[i], (double)h[8 * r + i]); }
            }
            const double d = w ? (double)w : 1.0;
            fprintf(stderr, "[st_phase] waves=%zu avg cycles: setup %.0f records %.0f gather %.0f sort %.0f emit-lds %.0f lookback+copy %.0f | max: %.0f %.0f %.0f %.0f %.0f %.0f\n",
                    w, sum[0] / d, sum[1] / d, sum[2] / d, sum[3] / d, sum[4] / d, sum[5] / d, mx[0], mx[1], mx[2], mx[3], mx[4], mx[5]);
        }
#endif
    }
    if (nbig || nrun) ctx->join(nrun ? 2 : 1);
#ifdef ACC_PHASE_PROF
    if (nbig && win_ok) {
        std::vector<unsigned long long> h(10);
        ACC_HIP(hipMemcpyAsync(h.data(), ctx->get<unsigned long long>("v2_win_prof", 10), 80, hipMemcpyDeviceToHost, st));
        ACC_HIP(hipStreamSynchronize(st));
        const double nt = h[6] ? (double)h[6] : 1.0;
        fprintf(stderr, "[win_phase] txns=%llu avg cycles per txn (thread 0 of each block): runs+lowend %.0f gather %.0f "
                "below-sort %.0f prefix %.0f span-writes %.0f rank-map %.0f list-wait %.0f | avg E %.1f span words %.1f below %.1f\n",
                h[6], h[0] / nt, h[1] / nt, h[2] / nt, h[3] / nt, h[4] / nt, h[5] / nt, h[9] / nt, h[7] / nt,
                (double)(h[8] >> 32) / nt, (double)(h[8] & 0xFFFFFFFFull) / nt);
    }
#endif
    finish();
    if (ctx->pinned[5]) fail(ACC_E_STATE, "internal: stream gather count differs from the count pass");
    if (ctx->pinned[2]) fail(ACC_E_STATE, "internal: v2 gather count differs from the count pass");
    if (nbig && win_ok && (ctx->pinned[0] || ctx->pinned[1])) {
        // txns the window tier could not take (> 16 keys, or too many entries below its span): the sorting tiers now,
        // on the context stream, then the copies / compaction again
        sort_tiers(ctx->pinned[0] != 0);
        finish();
        if (ctx->pinned[2]) fail(ACC_E_STATE, "internal: v2 gather count differs from the count pass");
    }
    if (nbig) {
        nmed = ctx->pinned[0]; nbig2 = ctx->pinned[1];
        nfb = ctx->pinned[3]; efb = ctx->pinned[4];
        ctx->stat("keydeps.huge_txns", ctx->pinned[6]);
        ctx->stat("keydeps.window_txns", ctx->pinned[7] + ctx->pinned[8]);
    }
    if (nfb) {
        need_pair_pos();
        uint64_t *vcnt = ctx->get<uint64_t>("cnt", P);
        uint32_t *vcnz = ctx->get<uint32_t>("cnz", P + 1);
        uint32_t *fb_list = ctx->get<uint32_t>("v2_fb_list", nbig);
        // txns beyond the block tiers (> 64 keys, > HUGE_E raw entries, or ranks beyond 25 bits): gather to global
        // memory, sort by (txn, value, key) for the TxnId array and by (txn, key, value) for the arena order
        uint64_t *fb_e = ctx->get<uint64_t>("v2_fb_e", nfb);
        uint64_t *fb_off = ctx->get<uint64_t>("v2_fb_off", nfb + 1);
        uint64_t *fb_maxk = ctx->get<uint64_t>("v2_fb_maxk", 1);
        ACC_HIP(hipMemsetAsync(fb_maxk, 0, sizeof(uint64_t), st));
        launch(ctx, "v2_fb_sizes", k_fb_sizes, dim3(grid_for(nfb, BLOCK)), dim3(BLOCK), 0, (uint32_t)nfb,
               (const uint32_t *)fb_list, key_off, (const uint64_t *)vdep_off, fb_e, fb_maxk);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, fb_e, fb_off, nfb, true, fb_off + nfb);
        ACC_HIP(hipMemcpyAsync(ctx->pinned, fb_maxk, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        ctx->sync();
        const int bbits = bits_for(nfb - 1);
        const int kbits = std::max(1, bits_for(ctx->pinned[0] - 1));   // key index within its txn
        if (bbits + rbits + kbits > 64) fail(ACC_E_CAP, "too many oversized txns for the global KeyDeps path");
        uint64_t *gkey = ctx->get<uint64_t>("v2_gkey", efb);
        launch(ctx, "v2_big_gather", k_v2_big_gather, dim3((unsigned)((nfb + WAVES - 1) / WAVES)), dim3(BLOCK), 0,
               (uint32_t)nfb, (const uint32_t *)fb_list, (const uint64_t *)fb_off, vv, (const uint64_t *)vcnt, key_off,
               rbits, kbits, gkey);
        Sorted s1 = radix_sort(ctx, "rs_big1", gkey, nullptr, efb, bbits + rbits + kbits);
        uint32_t *nflag = ctx->get<uint32_t>("v2_big_nflag", efb);
        uint32_t *nincl = ctx->get<uint32_t>("v2_big_nincl", efb);
        launch(ctx, "v2_big_newflag", k_v2_big_newflag, dim3(grid_for(efb, BLOCK)), dim3(BLOCK), 0, efb,
               (const uint64_t *)s1.keys, kbits, nflag);
        scan<uint32_t, OpAdd<uint32_t>>(ctx, nflag, nincl, efb, false);
        uint32_t *idx1 = ctx->get<uint32_t>("v2_big_idx1", efb);
        uint64_t *key2 = ctx->get<uint64_t>("v2_big_key2", efb);
        launch(ctx, "v2_big_rank", k_v2_big_rank, dim3(grid_for(efb, BLOCK)), dim3(BLOCK), 0, efb, (const uint64_t *)s1.keys,
               (const uint32_t *)nincl, (const uint32_t *)fb_list, (const uint64_t *)fb_off, rbits, kbits, key_off,
               (const uint64_t *)vdep_off, (const uint32_t *)txn_of_rank, dep_scr, u_cnt, idx1, key2);
        Sorted s2 = radix_sort(ctx, "rs_big2", key2, nullptr, efb, bbits + kbits + rbits);
        launch(ctx, "v2_big_arena", k_v2_big_arena, dim3(grid_for(efb, BLOCK)), dim3(BLOCK), 0, efb,
               (const uint32_t *)s2.vals, (const uint64_t *)s2.keys, (const uint32_t *)idx1, (const uint32_t *)fb_list,
               (const uint64_t *)fb_off, rbits, kbits, key_off, (const uint32_t *)vcnz, (const uint64_t *)arena_off, arena);
        finish();
    }
    ctx->stat("keydeps.stream_txns", n - nbig);
    ctx->stat("keydeps.stream_run_txns", nrun);
    ctx->stat("keydeps.big_path_txns", nbig);
    ctx->stat("keydeps.medium_txns", nmed);
    ctx->stat("keydeps.big_txns", nbig2);
    ctx->stat("keydeps.fallback_txns", nfb);
    ctx->stat("keydeps.fallback_entries", efb);
    ctx->stat("keydeps.bumped_committed", nbc);
    *view = acc_keydeps_view{ n, ctx->pinned[GSTAT_N], ctx->pinned[GSTAT_N + 1], ctx->pinned[GSTAT_N + 2], E, arena_off,
                              arena, kd_off, key_idx, u_off, dep_txn };
    ctx->kd_view = *view;
    ctx->kd_valid = true;
}


void keydeps_batch(acc_ctx *ctx, const acc_batch_in *in, acc_keydeps_view *view)
{
    keydeps_core(ctx, in, view, nullptr);
}

// ---------------------------------------------------------------- KeyDeps of a mixed key/range batch
//
// A range-domain txn T is no CommandsForKey member (SafeCommandStore.updateCommandsForKey registers key txns only,
// local/SafeCommandStore.java:217-240); as a query it visits every CFK whose key lies inside its store-sliced ranges
// (impl/InMemoryCommandStore.java:274-289: commandsForKey.subMap(start, startInclusive, end, endInclusive)) and runs
// the same mapReduceActive there. The key txns' results come from keydeps_core; each range txn's covered CFK keys
// become "virtual" queries (T, segment) answered by the exact-replay scan (make_query / run_query), then one sort of
// (txn, TxnId rank) gives every range txn's TxnId union and indices.

constexpr uint64_t MX_ERR_DOMAIN = 1, MX_ERR_EMPTY = 2, MX_ERR_UNSORTED = 4, MX_ERR_OFF = 8;
constexpr uint32_t MX_PIECE = 32;   // covered segments per work piece

// Bucket directory of the sorted CFK keys: bucket(x) = (x - seg_key[0]) >> shift over 2^tbits buckets, the shift
// making the key span fit; bstart[b] = first segment whose bucket is >= b (b in [0, 2^tbits]). A bound search then
// bisects one bucket (a few keys) instead of all segments: 2-3 dependent loads instead of ~25.
__device__ __forceinline__ uint32_t mx_shift(const uint64_t *seg_key, uint32_t nseg, uint32_t tbits)
{
    const uint64_t span = seg_key[nseg - 1] - seg_key[0];
    const uint32_t sb = span ? 64u - (uint32_t)__clzll((long long)span) : 0u;
    return sb > tbits ? sb - tbits : 0u;
}

// bend[b] = 1 + the last segment of bucket b (written by that segment; 0 for empty buckets, zeroed before): an
// exclusive max-scan of bend is bstart (keys are sorted, so the segments of buckets <= b are a prefix)
__global__ __launch_bounds__(BLOCK) void k_mx_buckets(uint32_t nseg, uint32_t tbits, const uint64_t *__restrict__ seg_key,
                                                      uint32_t *__restrict__ bend)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= nseg) return;
    const uint32_t sh = mx_shift(seg_key, nseg, tbits);
    const uint64_t k0 = seg_key[0], b = (seg_key[i] - k0) >> sh;
    if (i + 1 == nseg || ((seg_key[i + 1] - k0) >> sh) != b) bend[b] = i + 1;
}

// first segment m in [0, nseg) with seg_key[m] > x (upper) / >= x (!upper)
__device__ __forceinline__ uint32_t mx_bound(const uint64_t *seg_key, const uint32_t *bstart, uint32_t nseg, uint32_t sh,
                                             uint32_t tbits, uint64_t x, bool upper)
{
    const uint64_t k0 = seg_key[0];
    if (x < k0) return 0;
    uint64_t b = (x - k0) >> sh;
    if (b >= (1ull << tbits)) return nseg;
    uint32_t lo = bstart[b], hi = bstart[b + 1];
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (upper ? seg_key[m] <= x : seg_key[m] < x) lo = m + 1; else hi = m; }
    return lo;
}

// validation (TxnId.domain(), Range start < end, Ranges.ofSortedAndDeoverlapped) and, per range, its run of covered
// segments [ra, ra + rcnt) over the sorted CFK keys, its owner and its number of work pieces
__global__ __launch_bounds__(BLOCK) void k_mx_ranges(uint32_t n, const uint64_t *__restrict__ tl,
                                                     const uint32_t *__restrict__ key_off, const uint32_t *__restrict__ rng_off,
                                                     const uint64_t *__restrict__ rs, const uint64_t *__restrict__ re,
                                                     uint32_t end_inclusive, const uint64_t *__restrict__ seg_key, uint32_t nseg,
                                                     const uint32_t *__restrict__ bstart, uint32_t tbits,
                                                     uint32_t *__restrict__ ra, uint32_t *__restrict__ rowner,
                                                     uint64_t *__restrict__ rcnt, uint64_t *__restrict__ rpieces,
                                                     uint64_t *__restrict__ errs)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= n) return;
    const bool isr = (tl[t] & 1u) != 0;
    const uint32_t r0 = rng_off[t], r1 = rng_off[t + 1];
    uint64_t e = 0;
    if (r1 < r0) e |= MX_ERR_OFF;
    else {
        if (isr && key_off[t + 1] != key_off[t]) e |= MX_ERR_DOMAIN;
        if (!isr && r1 != r0) e |= MX_ERR_DOMAIN;
        for (uint32_t j = r0; j < r1; ++j) {
            const uint64_t s = rs[j], x = re[j];
            if (s >= x) e |= MX_ERR_EMPTY;
            if (j > r0 && re[j - 1] > s) e |= MX_ERR_UNSORTED;
            // EndInclusive (s, x]: keys > s .. <= x; StartInclusive [s, x): keys >= s .. < x
            uint32_t a = 0, b = 0;
            if (nseg) {
                const uint32_t sh = mx_shift(seg_key, nseg, tbits);
                a = mx_bound(seg_key, bstart, nseg, sh, tbits, s, end_inclusive != 0);
                b = mx_bound(seg_key, bstart, nseg, sh, tbits, x, end_inclusive != 0);
            }
            const uint32_t c = (e || b < a) ? 0u : b - a;
            ra[j] = a;
            rowner[j] = t;
            rcnt[j] = c;
            rpieces[j] = (c + MX_PIECE - 1) / MX_PIECE;
        }
    }
    if (e) atomicOr((unsigned long long *)errs, (unsigned long long)e);
}


// work pieces: piece p = (range, first covered segment), at most MX_PIECE segments each. Its record (one thread per
// range writes its pieces', so the count / emit passes read one record instead of a chain of dependent loads):
// prec[2p] = (owner txn, first segment, covered-key index of that segment within the txn's keys, queries),
// prec[2p + 1] = (T.executeAt rank S, T's TxnId rank, T.kind().witnesses() mask | p1 << 8, 0)
__global__ __launch_bounds__(BLOCK) void k_mx_pieces(uint32_t R, const uint64_t *__restrict__ poff, const uint32_t *__restrict__ ra,
                                                     const uint32_t *__restrict__ rowner, const uint64_t *__restrict__ rcnt,
                                                     const uint64_t *__restrict__ r_off, const uint32_t *__restrict__ rng_off,
                                                     const uint32_t *__restrict__ rank, uint32_t n, const uint64_t *__restrict__ tl,
                                                     uint4 *__restrict__ prec)
{
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= R) return;
    const uint64_t p0 = poff[j], p1 = poff[j + 1];
    if (p0 == p1) return;
    const uint32_t t = rowner[j], a = ra[j], c = (uint32_t)rcnt[j];
    const uint32_t kb = (uint32_t)(r_off[j] - r_off[rng_off[t]]);
    const uint32_t S = rank[n + t], tr = rank[t];
    const uint32_t wk = witnesses((uint32_t)(tl[t] >> 1) & 7u) | (S != tr ? 1u << 8 : 0u);
    for (uint64_t p = p0; p < p1; ++p) {
        const uint32_t k0 = (uint32_t)(p - p0) * MX_PIECE;
        prec[2 * p] = make_uint4(t, a + k0, kb + k0, min(c - k0, MX_PIECE));
        prec[2 * p + 1] = make_uint4(S, tr, wk, 0);
    }
}

// 32 lanes per piece, one covered segment (one query) per lane
__device__ __forceinline__ uint32_t mx_scan32(uint32_t x, uint32_t sub)   // inclusive, within the 32-lane half
{
#pragma unroll
    for (uint32_t d = 1; d < 32; d <<= 1) {
        const uint32_t u = __shfl_up(x, d, 64);
        if (sub >= d) x += u;
    }
    return x;
}

// count pass: entries and non-empty keys per piece. Each lane keeps its count in qc, or, for a single entry (nearly
// every non-empty (range txn, key) query: one conflicting key txn), the entry itself with MX_ONE set, so the emit pass
// replays the scan only for the rare lanes with two or more entries
constexpr uint32_t MX_ONE = 0x80000000u;
__device__ __forceinline__ uint32_t mx_qcount(uint32_t q) { return (q & MX_ONE) ? 1u : q; }

// A segment holding one CFK entry (nearly every covered key of a sparse key space) is answered in place: with
// s1 = s0 + 1, make_query_ts / run_query reduce to one test of that entry. Its committed[] is itself or empty, so any
// maxCommittedBefore M is its own executeAt, which the prefix-max prune (executeAt < M) never removes; nothing of the
// segment lies below scanStart = s0; the scan [s0, insertPos) is the entry exactly when its TxnId is below T.executeAt.
// Queries over longer segments go to deferred lists that k_mx_pdefer answers densely, adding into the piece totals:
// MX_DSLOTS lists (block b appends to list b % MX_DSLOTS with wave-aggregated atomics on that list's counter, so the
// appends spread over many addresses), list s holding at most dcap entries (its blocks' lanes); dlist null: every
// query in place.
constexpr uint32_t MX_DSLOTS = 1024;
__global__ __launch_bounds__(BLOCK) void k_mx_pcount(uint64_t NP, const uint4 *__restrict__ prec, CfkView v,
                                                     uint64_t *__restrict__ pe_cnt, uint32_t *__restrict__ pk_cnt,
                                                     uint32_t *__restrict__ qc, uint32_t pack, uint32_t *__restrict__ dlist,
                                                     uint32_t *__restrict__ dcnt, uint32_t dcap)
{
    const uint64_t p = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) >> 5;
    const uint32_t sub = threadIdx.x & 31u, g0 = lane_id() & 32u;
    uint32_t c = 0;
    bool dfr = false;
    if (p < NP) {
        const uint4 pr = prec[2 * p], pq = prec[2 * p + 1];
        uint32_t f = 0;
        if (sub < pr.w) {
            const uint32_t seg = pr.y + sub;
            const uint32_t s0 = v.seg_start[seg], s1 = v.seg_start[seg + 1];
            if (dlist && s1 - s0 == 1) {
                const uint32_t S = pq.x, trank = pq.y, wk = pq.z & 0xFFu;
                const uint32_t r = v.s_rank[s0], info = v.s_info[s0], st = info & 7u;
                c = (r < S && ((wk >> (info >> 3)) & 1u) && st != 0 && st != 7 && !((pq.z >> 8) && r == trank)) ? 1u : 0u;
                f = r;
            } else if (dlist) dfr = true;
            else c = run_query<false, true>(v, make_query_ts(v, pr.x, seg), &f);
        }
        qc[p * 32 + sub] = (pack && c == 1) ? (MX_ONE | f) : c;
    }
    const uint64_t db = __ballot(dfr);
    if (db) {
        const uint32_t slot = blockIdx.x % MX_DSLOTS;
        uint32_t base = 0;
        const uint32_t lead = (uint32_t)__ffsll((unsigned long long)db) - 1;
        if (lane_id() == lead) base = atomicAdd(&dcnt[slot], (uint32_t)__popcll(db));
        base = __shfl(base, (int)lead, 64);
        if (dfr) dlist[(size_t)slot * dcap + base + (uint32_t)__popcll(db & ((1ull << lane_id()) - 1))] = (uint32_t)(p * 32 + sub);
    }
    const uint32_t ce = mx_scan32(c, sub), ck = mx_scan32(c != 0 ? 1u : 0u, sub);
    const uint32_t te = __shfl(ce, (int)(g0 + 31), 64), tk = __shfl(ck, (int)(g0 + 31), 64);
    if (p < NP && sub == 0) { pe_cnt[p] = te; pk_cnt[p] = tk; }
}

// the deferred queries (segments of two or more entries): the exact-replay scan, one lane each; blockIdx.y = list,
// a grid-stride loop over its device-side count
__global__ __launch_bounds__(BLOCK) void k_mx_pdefer(const uint4 *__restrict__ prec, CfkView v, const uint32_t *__restrict__ dlist,
                                                     const uint32_t *__restrict__ dcnt, uint32_t dcap, uint64_t *__restrict__ pe_cnt,
                                                     uint32_t *__restrict__ pk_cnt, uint32_t *__restrict__ qc, uint32_t pack)
{
    const uint32_t nd = dcnt[blockIdx.y];
    const uint32_t *lst = dlist + (size_t)blockIdx.y * dcap;
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < nd; i += gridDim.x * BLOCK) {
        const uint32_t q = lst[i], p = q >> 5, sub = q & 31u;
        const uint4 pr = prec[2 * (uint64_t)p];
        uint32_t f = 0;
        const uint32_t c = run_query<false, true>(v, make_query_ts(v, pr.x, pr.y + sub), &f);
        qc[q] = (pack && c == 1) ? (MX_ONE | f) : c;
        if (c) {
            atomicAdd((unsigned long long *)&pe_cnt[p], (unsigned long long)c);
            atomicAdd(&pk_cnt[p], 1u);
        }
    }
}

struct MxE {   // emitted entries and key records of the range txns
    uint32_t *deps, *owner;          // [Ex]: TxnId rank, owning txn
    uint32_t *kx_idx, *kx_end;       // [Kx]: covered-key index, end of its entries (absolute entry index)
    uint64_t *kx_code;               // [Kx]: key code
};

__global__ __launch_bounds__(BLOCK) void k_mx_pemit(uint64_t NP, const uint4 *__restrict__ prec, const uint64_t *__restrict__ seg_key,
                                                    CfkView v, const uint64_t *__restrict__ pe_off,
                                                    const uint32_t *__restrict__ pk_off, MxE x, const uint32_t *__restrict__ qc)
{
    const uint64_t p = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) >> 5;
    const uint32_t sub = threadIdx.x & 31u;
    uint32_t c = 0, q = 0;
    uint4 pr = make_uint4(0, 0, 0, 0);
    bool act = false;
    if (p < NP) {
        pr = prec[2 * p];
        q = qc[p * 32 + sub];
        act = sub < pr.w;
        c = act ? mx_qcount(q) : 0u;
    }
    const uint32_t ce = mx_scan32(c, sub), ck = mx_scan32(c != 0 ? 1u : 0u, sub);
    if (!act || c == 0) return;
    const uint64_t e = pe_off[p] + (ce - c);
    const uint32_t seg = pr.y + sub;
    if (q & MX_ONE) x.deps[e] = q & ~MX_ONE;
    else run_query<true>(v, make_query_ts(v, pr.x, seg), x.deps + e);
    const uint32_t kr = pk_off[p] + ck - 1;
    x.kx_idx[kr] = pr.z + sub;
    x.kx_code[kr] = seg_key[seg];
    x.kx_end[kr] = (uint32_t)(e + c);
}

__global__ __launch_bounds__(BLOCK) void k_mx_toff(uint32_t n, const uint32_t *__restrict__ rng_off, const uint64_t *__restrict__ poff,
                                                   const uint64_t *__restrict__ pe_off, const uint32_t *__restrict__ pk_off,
                                                   uint64_t *__restrict__ etoff, uint32_t *__restrict__ ktoff)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t > n) return;
    const uint64_t p = poff[rng_off[t]];
    etoff[t] = pe_off[p];
    ktoff[t] = pk_off[p];
}

// the owning txn of every emitted entry (fallback union only)
__global__ __launch_bounds__(BLOCK) void k_mx_owner(uint32_t n, const uint64_t *__restrict__ etoff, uint32_t *__restrict__ owner)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= n) return;
    for (uint64_t e = etoff[t]; e < etoff[t + 1]; ++e) owner[e] = t;
}

// sort keys (txn, TxnId rank) of the emitted entries (fallback union)
__global__ __launch_bounds__(BLOCK) void k_mx_sortkeys(uint64_t E, const uint32_t *__restrict__ deps, const uint32_t *__restrict__ owner,
                                                       int rbits, uint64_t *__restrict__ key)
{
    const uint64_t e = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e < E) key[e] = ((uint64_t)owner[e] << rbits) | deps[e];
}

__global__ __launch_bounds__(BLOCK) void k_mx_uflag(uint64_t E, const uint64_t *__restrict__ sk, uint32_t *__restrict__ f)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < E) f[i] = i == 0 || sk[i] != sk[i - 1];
}

struct MxKv {   // the key-txn KeyDeps (keydeps_core's view)
    const uint64_t *arena_off, *kd_off, *u_off;
    const int32_t *arena;
    const uint32_t *key_idx, *dep_txn;
};
struct MxOut {
    uint64_t *arena_off, *kd_off, *u_off;
    int32_t *arena;
    uint32_t *key_idx, *dep_txn;
    uint64_t *kd_key;
};
// per-txn TxnId union of the emitted entries: idx_of_e[e] = index of entry e's TxnId in its txn's union,
// dep_scr[e0 + i] = batch index of the i-th union TxnId, ucnt[t] = union size
struct MxU {
    const uint32_t *deps;
    const uint64_t *etoff;
    const uint32_t *txn_of_rank;
    uint32_t *idx_of_e, *dep_scr, *ucnt;
};

// per txn: entry count routing into tier lists (txns without entries: none): E <= 16, <= 32, <= 64 (lane groups),
// <= MX_MID_E (wave, LDS), <= MX_BLK_E (block); beyond: the sorted fallback (flag gst[1]).
// gst: [0] block count, [1] fallback flag, [2] mid count, [3..5] 16 / 32 / 64-lane counts
constexpr uint32_t MX_MID_E = 512, MX_BLK_E = 4096;
struct MxLists {
    uint32_t *l[5];   // 16, 32, 64, mid, block
};
// MX_RT chunks of BLOCK txns per workgroup: one list-counter add per list and workgroup (the five counters share one
// line: per-256-txn adds serialised there); list order is free (each txn writes its own outputs)
constexpr int MX_RT = 16;
__global__ __launch_bounds__(BLOCK) void k_mx_route(uint32_t n, const uint64_t *__restrict__ etoff, MxLists L,
                                                    uint64_t *__restrict__ gst)
{
    __shared__ uint32_t wcnt[5][MX_RT * WAVES], base[5];
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    int cs[MX_RT];
    bool ovf = false;
#pragma unroll
    for (int r = 0; r < MX_RT; ++r) {
        const uint32_t t = (blockIdx.x * MX_RT + (uint32_t)r) * BLOCK + threadIdx.x;
        int c = -1;
        if (t < n) {
            const uint64_t E = etoff[t + 1] - etoff[t];
            if (E == 0) c = -1;
            else if (E <= 16) c = 0;
            else if (E <= 32) c = 1;
            else if (E <= 64) c = 2;
            else if (E <= MX_MID_E) c = 3;
            else if (E <= MX_BLK_E) c = 4;
            else ovf = true;
        }
        cs[r] = c;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint32_t cnt = (uint32_t)__popcll(__ballot(c == k));
            if (lane == 0) wcnt[k][r * WAVES + w] = cnt;
        }
    }
    if (ovf) atomicOr((unsigned long long *)&gst[1], 1ull);
    __syncthreads();
    if (threadIdx.x < 5) {
        uint32_t tot = 0;
        for (int q = 0; q < MX_RT * WAVES; ++q) { const uint32_t x = wcnt[threadIdx.x][q]; wcnt[threadIdx.x][q] = tot; tot += x; }
        const int slot = threadIdx.x == 4 ? 0 : threadIdx.x == 3 ? 2 : 3 + (int)threadIdx.x;
        base[threadIdx.x] = tot ? (uint32_t)atomicAdd((unsigned long long *)&gst[slot], (unsigned long long)tot) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MX_RT; ++r) {
        const int c = cs[r];
        const uint32_t t = (blockIdx.x * MX_RT + (uint32_t)r) * BLOCK + threadIdx.x;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint64_t bal = __ballot(c == k);
            if (c == k) L.l[k][base[k] + wcnt[k][r * WAVES + w] + (uint32_t)__popcll(bal & lt)] = t;
        }
    }
}

// groups of S lanes (S = 16, 32, 64), one listed txn each (E <= S): register bitonic of (rank << 32 | local entry)
template <int S>
__global__ __launch_bounds__(BLOCK) void k_mx_union_seg(const uint32_t *__restrict__ list, const uint64_t *__restrict__ cnt, MxU u)
{
    constexpr uint32_t G = 64 / S;
    const uint32_t lane = lane_id(), grp = lane / S, sub = lane & (S - 1);
    const uint32_t li = (blockIdx.x * WAVES + (threadIdx.x >> 6)) * G + grp;
    const bool live = li < (uint32_t)*cnt;
    const uint32_t t = live ? list[li] : 0;
    const uint64_t e0 = live ? u.etoff[t] : 0;
    const uint32_t E = live ? (uint32_t)(u.etoff[t + 1] - e0) : 0;
    const bool in = sub < E;
    uint64_t x = in ? (((uint64_t)u.deps[e0 + sub] << 32) | sub) : ~0ull;
#pragma unroll
    for (uint32_t k = 2; k <= (uint32_t)S; k <<= 1) {
#pragma unroll
        for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
            const uint64_t y = xor_lanes(x, (int)jj);
            const bool up = k == (uint32_t)S || (lane & k) == 0, lower = (lane & jj) == 0;   // ascending per group
            const uint64_t mn = x < y ? x : y, mx = x < y ? y : x;
            x = (lower == up) ? mn : mx;
        }
    }
    const uint64_t prev = shfl_up(x, 1);
    const bool nw = in && (sub == 0 || (prev >> 32) != (x >> 32));
    const uint64_t gmask = S == 64 ? ~0ull : (((1ull << S) - 1) << (grp * S));
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const uint64_t bal = __ballot(nw) & gmask;
    const uint32_t idx = (uint32_t)__popcll(bal & lt) + (nw ? 1u : 0u) - 1u;
    if (in) {
        u.idx_of_e[e0 + (uint32_t)x] = idx;
        if (nw) u.dep_scr[e0 + idx] = u.txn_of_rank[(uint32_t)(x >> 32)];
    }
    if (live && sub == 0) u.ucnt[t] = (uint32_t)__popcll(bal);
}

// R values per lane sorted across the wave (element r * 64 + lane), ascending: partners 64 or more apart are registers
// of the same lane, the others lanes (shuffles)
template <int R>
__device__ __forceinline__ void wave_reg_sort(uint64_t (&v)[R])
{
    const uint32_t lane = lane_id();
#pragma unroll
    for (uint32_t k = 2; k <= 64u * R; k <<= 1) {
#pragma unroll
        for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
            if (jj >= 64) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int r2 = r ^ (int)(jj >> 6);
                    if (r2 > r) {
                        const bool up = ((((uint32_t)r << 6) | lane) & k) == 0;
                        const uint64_t a = v[r], b = v[r2];
                        if ((a > b) == up) { v[r] = b; v[r2] = a; }
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint64_t y = xor_lanes(v[r], (int)jj);
                    const bool up = ((((uint32_t)r << 6) | lane) & k) == 0, lower = (lane & jj) == 0;
                    const uint64_t mn = v[r] < y ? v[r] : y, mx = v[r] < y ? y : v[r];
                    v[r] = (lower == up) ? mn : mx;
                }
            }
        }
    }
}

// a txn's union over E <= 64 R entries in registers: sort (rank << 32 | entry), distinct ranks -> indices
template <int R>
__device__ __forceinline__ void mx_union_regs(const MxU &u, uint32_t t, uint64_t e0, uint32_t E)
{
    const uint32_t lane = lane_id();
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    uint64_t v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i = ((uint32_t)r << 6) | lane;
        v[r] = i < E ? (((uint64_t)u.deps[e0 + i] << 32) | i) : ~0ull;
    }
    wave_reg_sort<R>(v);
    uint32_t base = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint64_t x = v[r];
        uint64_t prev = shfl_up(x, 1);
        if (r > 0) {
            const uint64_t pl = shfl_idx(v[r - 1], 63);
            if (lane == 0) prev = pl;
        }
        const uint32_t i = ((uint32_t)r << 6) | lane;
        const bool in = i < E;
        const bool nw = in && (i == 0 || (prev >> 32) != (x >> 32));
        const uint64_t bal = __ballot(nw);
        const uint32_t idx = base + (uint32_t)__popcll(bal & lt) + (nw ? 1u : 0u) - 1u;
        if (in) {
            u.idx_of_e[e0 + (uint32_t)x] = idx;
            if (nw) u.dep_scr[e0 + idx] = u.txn_of_rank[(uint32_t)(x >> 32)];
        }
        base += (uint32_t)__popcll(bal);
    }
    if (lane == 0) u.ucnt[t] = base;
}

// wave per listed txn, 64 < E <= MX_MID_E: registers up to 256 entries, one wave's LDS bitonic beyond
__global__ __launch_bounds__(BLOCK) void k_mx_union_mid(const uint32_t *__restrict__ list, const uint64_t *__restrict__ gst, MxU u)
{
    __shared__ uint64_t sbuf[WAVES][MX_MID_E];
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6, i = blockIdx.x * WAVES + w;
    if (i >= (uint32_t)gst[2]) return;
    const uint32_t t = list[i];
    uint64_t *buf = sbuf[w];
    const uint64_t e0 = u.etoff[t];
    const uint32_t E = (uint32_t)(u.etoff[t + 1] - e0);
    if (E <= 128) { mx_union_regs<2>(u, t, e0, E); return; }   // wave-uniform
    if (E <= 256) { mx_union_regs<4>(u, t, e0, E); return; }
    uint32_t n2 = 128;
    while (n2 < E) n2 <<= 1;
    for (uint32_t q = lane; q < n2; q += 64) buf[q] = q < E ? (((uint64_t)u.deps[e0 + q] << 32) | q) : ~0ull;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    wave_bitonic_lds(buf, n2);
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    uint32_t distinct = 0;
    for (uint32_t q0 = 0; q0 < E; q0 += 64) {
        const uint32_t q = q0 + lane;
        const bool in = q < E;
        const uint64_t x = in ? buf[q] : 0;
        const bool nw = in && (q == 0 || (buf[q - 1] >> 32) != (x >> 32));
        const uint64_t bal = __ballot(nw);
        const uint32_t idx = distinct + (uint32_t)__popcll(bal & lt) + (nw ? 1u : 0u) - 1u;
        if (in) {
            u.idx_of_e[e0 + (uint32_t)x] = idx;
            if (nw) u.dep_scr[e0 + idx] = u.txn_of_rank[(uint32_t)(x >> 32)];
        }
        distinct += (uint32_t)__popcll(bal);
    }
    if (lane == 0) u.ucnt[t] = distinct;
}

// block per listed txn, 64 < E <= MX_BLK_E: LDS bitonic
__global__ __launch_bounds__(BLOCK) void k_mx_union_block(const uint32_t *__restrict__ list, const uint64_t *__restrict__ gst, MxU u)
{
    __shared__ uint64_t buf[MX_BLK_E];
    __shared__ uint32_t lds[WAVES];
    const uint32_t b = blockIdx.x;
    if (b >= (uint32_t)gst[0]) return;
    const uint32_t t = list[b], tid = threadIdx.x;
    const uint64_t e0 = u.etoff[t];
    const uint32_t E = (uint32_t)(u.etoff[t + 1] - e0);
    uint32_t n2 = 128;
    while (n2 < E) n2 <<= 1;
    for (uint32_t i = tid; i < n2; i += BLOCK) buf[i] = i < E ? (((uint64_t)u.deps[e0 + i] << 32) | i) : ~0ull;
    __syncthreads();
    for (uint32_t k = 2; k <= n2; k <<= 1)
        for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
            for (uint32_t pi = tid; pi < (n2 >> 1); pi += BLOCK) {
                const uint32_t i = ((pi & ~(jj - 1)) << 1) | (pi & (jj - 1)), l = i | jj;
                const uint64_t xa = buf[i], ya = buf[l];
                if ((xa > ya) == ((i & k) == 0)) { buf[i] = ya; buf[l] = xa; }
            }
            __syncthreads();
        }
    // distinct index: chunked scan of the "new value" flags (contiguous chunks per thread)
    const uint32_t per = (E + BLOCK - 1) / BLOCK, lo = min(E, tid * per), hi = min(E, lo + per);
    uint32_t c = 0;
    for (uint32_t i = lo; i < hi; ++i) c += i == 0 || (buf[i] >> 32) != (buf[i - 1] >> 32);
    uint32_t total;
    uint32_t run = block_exclusive(c, OpAdd<uint32_t>(), lds, total);
    for (uint32_t i = lo; i < hi; ++i) {
        const uint64_t x = buf[i];
        const bool nw = i == 0 || (x >> 32) != (buf[i - 1] >> 32);
        run += nw;
        u.idx_of_e[e0 + (uint32_t)x] = run - 1;
        if (nw) u.dep_scr[e0 + run - 1] = u.txn_of_rank[(uint32_t)(x >> 32)];
    }
    if (tid == 0) u.ucnt[t] = total;
}

// global fallback (some txn beyond MX_BLK_E): from the (txn, rank) sort
__global__ __launch_bounds__(BLOCK) void k_mx_union_sorted(uint64_t E, const uint64_t *__restrict__ sk, const uint32_t *__restrict__ sperm,
                                                           const uint32_t *__restrict__ uflag, const uint32_t *__restrict__ ucum,
                                                           const uint32_t *__restrict__ owner, int rbits, MxU u)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= E) return;
    const uint32_t e = sperm[i];
    const uint64_t e0 = u.etoff[owner[e]];
    const uint32_t idx = ucum[i] + uflag[i] - 1 - ucum[e0];
    u.idx_of_e[e] = idx;
    if (uflag[i]) u.dep_scr[e0 + idx] = u.txn_of_rank[(uint32_t)(sk[i] & ((1ull << rbits) - 1))];
}
__global__ __launch_bounds__(BLOCK) void k_mx_ucnt_sorted(uint32_t n, const uint64_t *__restrict__ etoff, const uint32_t *__restrict__ ucum,
                                                          uint32_t *__restrict__ ucnt)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t < n) ucnt[t] = ucum[etoff[t + 1]] - ucum[etoff[t]];
}

__global__ __launch_bounds__(BLOCK) void k_mx_sizes(uint32_t n, MxKv kv, const uint64_t *__restrict__ etoff,
                                                    const uint32_t *__restrict__ ktoff, const uint32_t *__restrict__ ucnt,
                                                    uint64_t *__restrict__ a_cnt, uint64_t *__restrict__ kd_cnt,
                                                    uint64_t *__restrict__ u_cnt)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t == n) { a_cnt[n] = 0; kd_cnt[n] = 0; u_cnt[n] = 0; }   // the exclusive scans over n + 1 end in the totals
    if (t >= n) return;
    const uint64_t ex = etoff[t + 1] - etoff[t];
    const uint64_t kd = ktoff[t + 1] - ktoff[t];
    a_cnt[t] = (kv.arena_off[t + 1] - kv.arena_off[t]) + kd + ex;
    kd_cnt[t] = (kv.kd_off[t + 1] - kv.kd_off[t]) + kd;
    u_cnt[t] = (kv.u_off[t + 1] - kv.u_off[t]) + (ex ? ucnt[t] : 0u);
}

// the combined layout. A workgroup owns BLOCK consecutive txns, whose output runs are one contiguous range of each
// output array: each output element takes its txn from a chunk owner map (chunk_owners) and reads from that txn's
// source (key txns: keydeps_core's result, with key codes; range txns: their key records, per-entry union indices and
// union TxnIds), so every write is a whole-line access.
__global__ __launch_bounds__(BLOCK) void k_mx_write(uint32_t n, MxKv kv, const uint64_t *__restrict__ etoff,
                                                    const uint32_t *__restrict__ ktoff, MxE x,
                                                    const uint32_t *__restrict__ idx_of_e, const uint32_t *__restrict__ dep_scr,
                                                    const uint32_t *__restrict__ key_off, const uint64_t *__restrict__ key_code,
                                                    MxOut o)
{
    __shared__ uint64_t ao[BLOCK + 1], ko[BLOCK + 1], uo[BLOCK + 1];   // output offsets
    __shared__ uint64_t sa[BLOCK], sk[BLOCK], su[BLOCK];                // source bases: arena / keys / TxnIds
    __shared__ uint32_t kdn[BLOCK], kofs[BLOCK];                        // range txn: key records; key txn: key_off
    __shared__ uint32_t own[8 * BLOCK], red[WAVES];                     // chunk owner map (chunk_owners)
    const uint32_t t0 = blockIdx.x * BLOCK, nt = min((uint32_t)BLOCK, n - t0), tid = threadIdx.x;
    if (tid < nt) {
        const uint32_t t = t0 + tid;
        ao[tid] = o.arena_off[t]; ko[tid] = o.kd_off[t]; uo[tid] = o.u_off[t];
        const uint64_t e0 = etoff[t], ex = etoff[t + 1] - e0;
        if (ex) {
            const uint32_t k0 = ktoff[t];
            kdn[tid] = ktoff[t + 1] - k0;
            sa[tid] = e0; sk[tid] = k0; su[tid] = e0;
        } else {
            kdn[tid] = 0xFFFFFFFFu;   // a key txn
            sa[tid] = kv.arena_off[t]; sk[tid] = kv.kd_off[t]; su[tid] = kv.u_off[t];
            kofs[tid] = key_off[t];
        }
    }
    if (tid == 0) { ao[nt] = o.arena_off[t0 + nt]; ko[nt] = o.kd_off[t0 + nt]; uo[nt] = o.u_off[t0 + nt]; }
    __syncthreads();
    // per array, chunks of U * BLOCK outputs: the owner map of the chunk (chunk_owners), then U outputs per thread,
    // interleaved across the block (whole-line stores), each reading its txn from the map
    constexpr int U = 8;
    uint32_t carry = 0;
    for (uint64_t c0 = ao[0]; c0 < ao[nt]; c0 += (uint64_t)U * BLOCK) {
        chunk_owners<U>(nt, ao, c0, own, red, carry);
        int32_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t p = (uint32_t)u * BLOCK + tid;
            const uint64_t j = c0 + p;
            v[u] = 0;
            if (j < ao[nt]) {
                const uint32_t a = own[p];
                const uint64_t i = j - ao[a];
                const uint32_t kd = kdn[a];
                if (kd == 0xFFFFFFFFu) v[u] = kv.arena[sa[a] + i];
                else if (i < kd) v[u] = (int32_t)(kd + (x.kx_end[sk[a] + i] - (uint32_t)sa[a]));
                else v[u] = (int32_t)idx_of_e[sa[a] + i - kd];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = c0 + (uint64_t)u * BLOCK + tid;
            if (j < ao[nt]) o.arena[j] = v[u];
        }
    }
    carry = 0;
    for (uint64_t c0 = ko[0]; c0 < ko[nt]; c0 += (uint64_t)U * BLOCK) {
        chunk_owners<U>(nt, ko, c0, own, red, carry);
        uint32_t ki[U];
        uint64_t kc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t p = (uint32_t)u * BLOCK + tid;
            const uint64_t j = c0 + p;
            ki[u] = 0; kc[u] = 0;
            if (j < ko[nt]) {
                const uint32_t a = own[p];
                const uint64_t i = j - ko[a];
                if (kdn[a] == 0xFFFFFFFFu) {
                    ki[u] = kv.key_idx[sk[a] + i];
                    kc[u] = key_code[kofs[a] + ki[u]];
                } else {
                    ki[u] = x.kx_idx[sk[a] + i];
                    kc[u] = x.kx_code[sk[a] + i];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = c0 + (uint64_t)u * BLOCK + tid;
            if (j < ko[nt]) { o.key_idx[j] = ki[u]; o.kd_key[j] = kc[u]; }
        }
    }
    carry = 0;
    for (uint64_t c0 = uo[0]; c0 < uo[nt]; c0 += (uint64_t)U * BLOCK) {
        chunk_owners<U>(nt, uo, c0, own, red, carry);
        uint32_t d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t p = (uint32_t)u * BLOCK + tid;
            const uint64_t j = c0 + p;
            d[u] = 0;
            if (j < uo[nt]) {
                const uint32_t a = own[p];
                const uint64_t i = j - uo[a];
                d[u] = kdn[a] == 0xFFFFFFFFu ? kv.dep_txn[su[a] + i] : dep_scr[su[a] + i];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = c0 + (uint64_t)u * BLOCK + tid;
            if (j < uo[nt]) o.dep_txn[j] = d[u];
        }
    }
}

void keydeps_mixed(acc_ctx *ctx, const acc_range_batch_in *in, acc_keydeps_view *view, SharedDict *shared)
{
    if (!in || !view) fail(ACC_E_ARG, "null argument");
    if (in->mem != ACC_MEM_HOST && in->mem != ACC_MEM_DEVICE) fail(ACC_E_ARG, "mem must be ACC_MEM_HOST or ACC_MEM_DEVICE");
    if (in->end_inclusive > 1) fail(ACC_E_ARG, "end_inclusive must be 0 (StartInclusive) or 1 (EndInclusive)");
    const uint32_t n = in->n_txn;
    const size_t R = (size_t)in->n_ranges;
    if (R >= 0xFFFFFFFFull) fail(ACC_E_ARG, "n_ranges must be < 2^32");
    hipStream_t st = ctx->stream;
    ctx->kd_valid = false;

    // ---- key txns (and the CFK snapshot): keydeps_core over the key part of the batch
    acc_batch_in kin{ n, in->mem, in->n_pairs, in->txn_id, in->execute_at, in->status, in->key_off, in->key_code };
    acc_keydeps_view kv{};
    KdState ks;
    ks.sparse = R > 0;
    keydeps_core(ctx, &kin, &kv, &ks);
    ctx->kd_valid = false;
    if (shared) {
        shared->valid = ks.have_dict; shared->dict = ks.dict; shared->owner = ks.owner;
        if (shared->ready && shared->valid) shared->ready(*shared);
    }
    if (n == 0) {
        kv.kd_key = ctx->get<uint64_t>("mx_kd_key", 1);
        *view = kv;
        ctx->kd_view = kv;
        ctx->kd_valid = true;
        return;
    }
    const uint32_t *key_off = stage_in(ctx, "in_key_off", in->key_off, (size_t)n + 1, in->mem);
    const uint64_t *key_code = stage_in(ctx, "in_key_code", in->key_code, (size_t)in->n_pairs, in->mem);
    const uint64_t *tl = stage_in(ctx, "in_tl", in->txn_id.lsb, n, in->mem);
    const uint32_t *rng_off = stage_in(ctx, "in_rng_off", in->rng_off, (size_t)n + 1, in->mem);
    const uint64_t *rs = stage_in(ctx, "in_rng_start", in->rng_start, R, in->mem);
    const uint64_t *re = stage_in(ctx, "in_rng_end", in->rng_end, R, in->mem);

    // ---- covered segments per range, work pieces
    uint32_t nseg = 0;
    if (ks.cfk) {
        ACC_HIP(hipMemcpyAsync(ctx->pinned, ks.seg_incl + ks.P - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        ctx->sync();
        nseg = (uint32_t)(ctx->pinned[0] & 0xFFFFFFFFu);
    }
    const uint64_t *seg_key = ks.cfk ? ks.seg_key : ctx->get<uint64_t>("mx_seg_key", 1);   // written by k_v2_apply
    // bucket directory: about one key per bucket
    const uint32_t tbits = nseg ? (uint32_t)std::min(26, std::max(0, bits_for(nseg) - 1)) : 0u;
    const size_t nbk = (size_t)1 << tbits;
    uint32_t *bstart = ctx->get<uint32_t>("mx_bstart", nbk + 1);
    if (nseg) {
        uint32_t *bend = ctx->get<uint32_t>("mx_bend", nbk);
        ACC_HIP(hipMemsetAsync(bend, 0, nbk * sizeof(uint32_t), st));
        launch(ctx, "mx_buckets", k_mx_buckets, dim3(grid_for(nseg, BLOCK)), dim3(BLOCK), 0, nseg, tbits,
               (const uint64_t *)seg_key, bend);
        scan<uint32_t, OpMax<uint32_t>>(ctx, bend, bstart, nbk, true, bstart + nbk);
    }
    uint32_t *ra = ctx->get<uint32_t>("mx_ra", R + 1);
    uint32_t *rowner = ctx->get<uint32_t>("mx_rowner", R + 1);
    uint64_t *rcnt = ctx->get<uint64_t>("mx_rcnt", R + 1);
    uint64_t *rpieces = ctx->get<uint64_t>("mx_rpieces", R + 1);
    uint64_t *r_off = ctx->get<uint64_t>("mx_r_off", R + 2);
    uint64_t *poff = ctx->get<uint64_t>("mx_poff", R + 2);
    uint64_t *errs = ctx->get<uint64_t>("mx_errs", 1);
    ACC_HIP(hipMemsetAsync(errs, 0, 8, st));
    launch(ctx, "mx_ranges", k_mx_ranges, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, tl, key_off, rng_off, rs, re,
           in->end_inclusive, (const uint64_t *)seg_key, nseg, (const uint32_t *)bstart, tbits, ra, rowner, rcnt, rpieces, errs);
    if (R) {
        const uint64_t *si[2] = { rcnt, rpieces };
        uint64_t *so[2] = { r_off, poff }, *stot[2] = { r_off + R, poff + R };
        const size_t sn[2] = { R, R };
        scan_multi<uint64_t, OpAdd<uint64_t>>(ctx, 2, si, so, sn, true, stot);
    } else {
        ACC_HIP(hipMemsetAsync(r_off, 0, 8, st));
        ACC_HIP(hipMemsetAsync(poff, 0, 8, st));
    }
    ACC_HIP(hipMemcpyAsync(ctx->pinned, errs, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, r_off + R, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 2, poff + R, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t merr = ctx->pinned[0];
    if (merr & MX_ERR_DOMAIN) fail(ACC_E_ARG, "a range-domain txn lists keys or a key-domain txn lists ranges (TxnId.domain())");
    if (merr & MX_ERR_EMPTY) fail(ACC_E_ARG, "range start must be below its end (Range: start >= end)");
    if (merr & MX_ERR_UNSORTED) fail(ACC_E_ARG, "ranges of a txn must be sorted and deoverlapped (Ranges.ofSortedAndDeoverlapped)");
    if (merr & MX_ERR_OFF) fail(ACC_E_ARG, "rng_off must be non-decreasing");
    const uint64_t V = ctx->pinned[1], NP = ctx->pinned[2];
    if (V >= 0xFFFFFFFFull) fail(ACC_E_CAP, "more than 2^32-1 (range txn, covered key) queries in one batch");
    ctx->stat("keydeps.range_key_queries", V);

    // ---- count and emit per piece with the exact-replay scan
    uint64_t *pe_cnt = ctx->get<uint64_t>("mx_pe_cnt", NP + 1);
    uint64_t *pe_off = ctx->get<uint64_t>("mx_pe_off", NP + 2);
    uint32_t *pk_cnt = ctx->get<uint32_t>("mx_pk_cnt", NP + 1);
    uint32_t *pk_off = ctx->get<uint32_t>("mx_pk_off", NP + 2);
    uint64_t *etoff = ctx->get<uint64_t>("mx_etoff", (size_t)n + 1);
    uint32_t *ktoff = ctx->get<uint32_t>("mx_ktoff", (size_t)n + 1);
    uint64_t Ex = 0, Kx = 0;
    CfkView v{};
    uint32_t *qc = ctx->get<uint32_t>("mx_qc", NP * 32);
    uint4 *prec = ctx->get<uint4>("mx_prec", 2 * NP + 2);
    if (NP) {
        const uint32_t pack = ks.rbits <= 31;
        const bool defer = NP * 32 < 0xFFFFFFFFull;
        if (!ks.v1) {
            // with deferral and packed single results the exact-replay scan only ever runs on segments of two or more
            // entries (pcount / pdefer; pemit replays only lanes of two or more entries)
            ks.v1view = build_v1_cfk(ctx, n, ks.P, ks.rbits, ks.tl, ks.owner, ks.rank, ks.seg_incl, ks.seg_start, ks.s_rank,
                                     ks.s_exec, ks.s_info, ks.pair_pos, defer && pack);
            ks.v1 = true;
        }
        v = ks.v1view;
        launch(ctx, "mx_pieces", k_mx_pieces, dim3(grid_for(R, BLOCK)), dim3(BLOCK), 0, (uint32_t)R, (const uint64_t *)poff,
               (const uint32_t *)ra, (const uint32_t *)rowner, (const uint64_t *)rcnt, (const uint64_t *)r_off, rng_off, ks.rank,
               n, ks.tl, prec);
        const unsigned gcount = grid_for(NP * 32, BLOCK);
        const uint32_t dcap = ((gcount + MX_DSLOTS - 1) / MX_DSLOTS) * BLOCK;   // lanes of the blocks of one list
        uint32_t *dlist = defer ? ctx->get<uint32_t>("mx_dlist", (size_t)MX_DSLOTS * dcap) : nullptr;
        uint32_t *dcnt = ctx->get<uint32_t>("mx_dcnt", MX_DSLOTS);
        if (defer) ACC_HIP(hipMemsetAsync(dcnt, 0, MX_DSLOTS * sizeof(uint32_t), st));
        launch(ctx, "mx_pcount", k_mx_pcount, dim3(gcount), dim3(BLOCK), 0, NP, (const uint4 *)prec, v, pe_cnt, pk_cnt, qc, pack,
               dlist, dcnt, dcap);
        if (defer)
            launch(ctx, "mx_pdefer", k_mx_pdefer, dim3(8, MX_DSLOTS), dim3(BLOCK), 0, (const uint4 *)prec, v, (const uint32_t *)dlist,
                   (const uint32_t *)dcnt, dcap, pe_cnt, pk_cnt, qc, pack);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, pe_cnt, pe_off, NP, true, pe_off + NP);
        scan<uint32_t, OpAdd<uint32_t>>(ctx, pk_cnt, pk_off, NP, true, pk_off + NP);
        ACC_HIP(hipMemcpyAsync(ctx->pinned, pe_off + NP, 8, hipMemcpyDeviceToHost, st));
        ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, pk_off + NP, 4, hipMemcpyDeviceToHost, st));
        ctx->sync();
        Ex = ctx->pinned[0];
        Kx = ctx->pinned[1] & 0xFFFFFFFFull;
        if (Ex >= 0xFFFFFFFFull) fail(ACC_E_CAP, "more than 2^32-1 range-txn KeyDeps entries in one batch");
    } else {
        ACC_HIP(hipMemsetAsync(pe_off, 0, 8, st));
        ACC_HIP(hipMemsetAsync(pk_off, 0, 4, st));
    }
    launch(ctx, "mx_toff", k_mx_toff, dim3(grid_for((size_t)n + 1, BLOCK)), dim3(BLOCK), 0, n, rng_off, (const uint64_t *)poff,
           (const uint64_t *)pe_off, (const uint32_t *)pk_off, etoff, ktoff);
    MxE mx;
    mx.deps = ctx->get<uint32_t>("mx_deps", Ex + 1);
    mx.owner = ctx->get<uint32_t>("mx_owner", Ex + 1);
    mx.kx_idx = ctx->get<uint32_t>("mx_kx_idx", Kx + 1);
    mx.kx_end = ctx->get<uint32_t>("mx_kx_end", Kx + 1);
    mx.kx_code = ctx->get<uint64_t>("mx_kx_code", Kx + 1);
    uint32_t *ucnt = ctx->get<uint32_t>("mx_ucnt", (size_t)n + 1);
    uint32_t *idx_of_e = ctx->get<uint32_t>("mx_idx_of_e", Ex + 1);
    uint32_t *dep_scr = ctx->get<uint32_t>("mx_dep_scr", Ex + 1);
    MxU mu{ mx.deps, etoff, ks.txn_of_rank, idx_of_e, dep_scr, ucnt };
    if (Ex) {
        launch(ctx, "mx_pemit", k_mx_pemit, dim3(grid_for(NP * 32, BLOCK)), dim3(BLOCK), 0, NP, (const uint4 *)prec,
               (const uint64_t *)seg_key, v, (const uint64_t *)pe_off, (const uint32_t *)pk_off, mx, (const uint32_t *)qc);
        // per-txn TxnId unions: wave / block tiers, or one (txn, rank) sort when some txn is beyond the block tier
        MxLists L;
        static const char *lnames[5] = { "mx_l16", "mx_l32", "mx_l64", "mx_mid_list", "mx_blk_list" };
        for (int k = 0; k < 5; ++k) L.l[k] = ctx->get<uint32_t>(lnames[k], n);
        uint32_t *const mid_list = L.l[3], *const blk_list = L.l[4];
        uint64_t *gst = ctx->get<uint64_t>("mx_gst", 6);
        ACC_HIP(hipMemsetAsync(gst, 0, 48, st));
        launch(ctx, "mx_route", k_mx_route, dim3(grid_for(n, (size_t)BLOCK * MX_RT)), dim3(BLOCK), 0, n, (const uint64_t *)etoff, L,
               gst);
        ACC_HIP(hipMemcpyAsync(ctx->pinned, gst, 48, hipMemcpyDeviceToHost, st));
        ctx->sync();
        const uint64_t nblk = ctx->pinned[0], nmid = ctx->pinned[2];
        const uint64_t nsmall[3] = { ctx->pinned[3], ctx->pinned[4], ctx->pinned[5] };
        ctx->stat("keydeps.range_block_txns", nblk);
        ctx->stat("keydeps.range_mid_txns", nmid);
        if (!ctx->pinned[1]) {
            if (nsmall[0])
                launch(ctx, "mx_union_s16", k_mx_union_seg<16>, dim3((unsigned)((nsmall[0] + 4 * WAVES - 1) / (4 * WAVES))),
                       dim3(BLOCK), 0, (const uint32_t *)L.l[0], (const uint64_t *)(gst + 3), mu);
            if (nsmall[1])
                launch(ctx, "mx_union_s32", k_mx_union_seg<32>, dim3((unsigned)((nsmall[1] + 2 * WAVES - 1) / (2 * WAVES))),
                       dim3(BLOCK), 0, (const uint32_t *)L.l[1], (const uint64_t *)(gst + 4), mu);
            if (nsmall[2])
                launch(ctx, "mx_union_s64", k_mx_union_seg<64>, dim3((unsigned)((nsmall[2] + WAVES - 1) / WAVES)),
                       dim3(BLOCK), 0, (const uint32_t *)L.l[2], (const uint64_t *)(gst + 5), mu);
            if (nmid)
                launch(ctx, "mx_union_mid", k_mx_union_mid, dim3((unsigned)((nmid + WAVES - 1) / WAVES)), dim3(BLOCK), 0,
                       (const uint32_t *)mid_list, (const uint64_t *)gst, mu);
            if (nblk)
                launch(ctx, "mx_union_block", k_mx_union_block, dim3((unsigned)nblk), dim3(BLOCK), 0,
                       (const uint32_t *)blk_list, (const uint64_t *)gst, mu);
        } else {
            const int tbits = bits_for(n);
            if (tbits + ks.rbits > 64) fail(ACC_E_CAP, "batch too large for the (txn, TxnId rank) composite key");
            uint64_t *skey = ctx->get<uint64_t>("mx_skey", Ex);
            uint32_t *uflag = ctx->get<uint32_t>("mx_uflag", Ex + 1);
            uint32_t *ucum = ctx->get<uint32_t>("mx_ucum", Ex + 1);
            launch(ctx, "mx_owner", k_mx_owner, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint64_t *)etoff, mx.owner);
            launch(ctx, "mx_sortkeys", k_mx_sortkeys, dim3(grid_for(Ex, BLOCK)), dim3(BLOCK), 0, Ex, (const uint32_t *)mx.deps,
                   (const uint32_t *)mx.owner, ks.rbits, skey);
            Sorted so = radix_sort(ctx, "mx_rs", skey, nullptr, Ex, tbits + ks.rbits);
            launch(ctx, "mx_uflag", k_mx_uflag, dim3(grid_for(Ex, BLOCK)), dim3(BLOCK), 0, Ex, (const uint64_t *)so.keys, uflag);
            scan<uint32_t, OpAdd<uint32_t>>(ctx, uflag, ucum, Ex, true, ucum + Ex);
            launch(ctx, "mx_union_sorted", k_mx_union_sorted, dim3(grid_for(Ex, BLOCK)), dim3(BLOCK), 0, Ex,
                   (const uint64_t *)so.keys, (const uint32_t *)so.vals, (const uint32_t *)uflag, (const uint32_t *)ucum,
                   (const uint32_t *)mx.owner, ks.rbits, mu);
            launch(ctx, "mx_ucnt_sorted", k_mx_ucnt_sorted, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint64_t *)etoff,
                   (const uint32_t *)ucum, ucnt);
        }
    }

    // ---- combined offsets and the combined layout
    MxKv mkv{ kv.arena_off, kv.kd_off, kv.u_off, kv.arena, kv.key_idx, kv.dep_txn };
    uint64_t *a_cnt = ctx->get<uint64_t>("mx_a_cnt", (size_t)n + 1);
    uint64_t *kd_cnt = ctx->get<uint64_t>("mx_kd_cnt", (size_t)n + 1);
    uint64_t *u_cnt = ctx->get<uint64_t>("mx_u_cnt", (size_t)n + 1);
    launch(ctx, "mx_sizes", k_mx_sizes, dim3(grid_for((size_t)n + 1, BLOCK)), dim3(BLOCK), 0, n, mkv, (const uint64_t *)etoff,
           (const uint32_t *)ktoff, (const uint32_t *)ucnt, a_cnt, kd_cnt, u_cnt);
    MxOut o;
    o.arena_off = ctx->get<uint64_t>("mx_arena_off", (size_t)n + 1);
    o.kd_off = ctx->get<uint64_t>("mx_kd_off", (size_t)n + 1);
    o.u_off = ctx->get<uint64_t>("mx_u_off", (size_t)n + 1);
    uint64_t *mtot = ctx->get<uint64_t>("mx_totals", 3);
    {   // the three combined offset arrays in one launch (over n + 1: the last element is each total), totals staged
        const uint64_t *si[3] = { a_cnt, kd_cnt, u_cnt };
        uint64_t *so[3] = { o.arena_off, o.kd_off, o.u_off }, *stot[3] = { mtot, mtot + 1, mtot + 2 };
        const size_t sn[3] = { (size_t)n + 1, (size_t)n + 1, (size_t)n + 1 };
        scan_multi<uint64_t, OpAdd<uint64_t>>(ctx, 3, si, so, sn, true, stot);
    }
    ACC_HIP(hipMemcpyAsync(ctx->pinned, mtot, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t TA = ctx->pinned[0], TK = ctx->pinned[1], TU = ctx->pinned[2];
    o.arena = ctx->get<int32_t>("mx_arena", TA + 1);
    o.key_idx = ctx->get<uint32_t>("mx_key_idx", TK + 1);
    o.kd_key = ctx->get<uint64_t>("mx_kd_key", TK + 1);
    o.dep_txn = ctx->get<uint32_t>("mx_dep_txn", TU + 1);
    launch(ctx, "mx_write", k_mx_write, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, mkv, (const uint64_t *)etoff,
           (const uint32_t *)ktoff, mx, (const uint32_t *)idx_of_e, (const uint32_t *)dep_scr, key_off, key_code, o);
    ctx->sync();
    *view = acc_keydeps_view{ n, TA, TK, TU, kv.total_edges + Ex, o.arena_off, o.arena, o.kd_off, o.key_idx, o.u_off,
                              o.dep_txn, o.kd_key };
    ctx->kd_view = *view;
    ctx->kd_valid = true;
}

// ---------------------------------------------------------------- CFK snapshot for the other scans (recovery.hip)

void cfk_snapshot(acc_ctx *ctx, const acc_batch_in *in, CfkSnapshot &out)
{
    acc_keydeps_view kv{};
    KdState ks;
    keydeps_core(ctx, in, &kv, &ks, true);
    ctx->kd_valid = false;
    out = CfkSnapshot{};
    out.n = in->n_txn;
    out.P = (size_t)in->n_pairs;
    if (!ks.cfk) return;
    ACC_HIP(hipMemcpyAsync(ctx->pinned, ks.seg_incl + ks.P - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
    const uint32_t nseg = (uint32_t)(ctx->pinned[0] & 0xFFFFFFFFu);   // seg_incl = inclusive count of segment starts
    const uint64_t *seg_key = ks.seg_key;   // written by k_v2_apply
    out.cfk = true; out.nseg = nseg; out.rbits = ks.rbits; out.rank = ks.rank; out.txn_of_rank = ks.txn_of_rank;
    out.seg_start = ks.seg_start; out.seg_key = seg_key; out.s_rank = ks.s_rank; out.s_exec = ks.s_exec;
    out.s_info = ks.s_info; out.perm = ks.perm; out.tm = ks.tm; out.tl = ks.tl; out.tn = ks.tn; out.em = ks.em;
    out.el = ks.el; out.en = ks.en; out.key_off = ks.key_off;
}

}  // namespace acc
