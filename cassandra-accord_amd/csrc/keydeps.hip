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
#include "prims.hpp"

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

enum : uint32_t {
    ERR_BAD_STATUS = 1u << 0,
    ERR_BAD_KIND = 1u << 1,
    ERR_LOCAL_ONLY = 1u << 2,
    ERR_KEYS_UNSORTED = 1u << 3,
    ERR_DUP_TXNID = 1u << 4,
    ERR_KEY_OFF = 1u << 5,
};

// g[0..2] ts word masks, g[3] key mask, g[4] error bits, g[5] batch-not-in-TxnId-order flag
__device__ __forceinline__ void block_or(uint64_t v, uint64_t *dst)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v |= shfl_idx(v, (int)(lane_id() ^ d));
    if (lane_id() == 0 && v) atomicOr((unsigned long long *)dst, (unsigned long long)v);
}

__global__ __launch_bounds__(BLOCK) void k_prep_txn(uint32_t n, const uint64_t *__restrict__ tm, const uint64_t *__restrict__ tl,
                                                    const int32_t *__restrict__ tn, const uint64_t *__restrict__ em,
                                                    const uint64_t *__restrict__ el, const int32_t *__restrict__ en,
                                                    const uint8_t *__restrict__ status, const uint32_t *__restrict__ key_off,
                                                    const uint64_t *__restrict__ key_code, uint32_t *__restrict__ owner,
                                                    uint64_t *__restrict__ g)
{
    uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    uint64_t m0 = 0, m1 = 0, m2 = 0, errs = 0, unsorted = 0;
    if (t < n) {
        const uint64_t r0 = tm[0], r1 = ts_w1(tl[0]), r2 = ts_w2(tn[0]);
        m0 = (tm[t] ^ r0) | (em[t] ^ r0);
        m1 = (ts_w1(tl[t]) ^ r1) | (ts_w1(el[t]) ^ r1);
        m2 = (ts_w2(tn[t]) ^ r2) | (ts_w2(en[t]) ^ r2);
        if (status[t] > 7) errs |= ERR_BAD_STATUS;
        uint32_t kind = (uint32_t)(tl[t] >> 1) & 7u;
        if (kind >= 6) errs |= ERR_BAD_KIND;
        else if (kind == 5) errs |= ERR_LOCAL_ONLY;
        if (t + 1 < n && ts_cmp(tm[t], tl[t], tn[t], tm[t + 1], tl[t + 1], tn[t + 1]) >= 0) unsorted = 1;
        uint32_t a = key_off[t], b = key_off[t + 1];
        if (b < a) errs |= ERR_KEY_OFF;
        else {
            for (uint32_t j = a; j < b; ++j) {
                owner[j] = t;
                if (j > a && key_code[j - 1] >= key_code[j]) errs |= ERR_KEYS_UNSORTED;
            }
        }
    }
    block_or(m0, &g[0]);
    block_or(m1, &g[1]);
    block_or(m2, &g[2]);
    block_or(errs, &g[4]);
    block_or(unsorted, &g[5]);
}

__global__ __launch_bounds__(BLOCK) void k_prep_keys(size_t P, const uint64_t *__restrict__ key_code, uint64_t *__restrict__ g)
{
    size_t j = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    uint64_t m = 0;
    if (j < P) m = key_code[j] ^ key_code[0];
    block_or(m, &g[3]);
}

// ---------------------------------------------------------------- dictionary (order ranks)

struct TsPlan {
    Runs r0, r1, r2;
    int b0, b1, b2;
};

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
    block_or(err, &g[4]);
}

// ---------------------------------------------------------------- CFK build

struct PairPlan {
    Runs rk;       // key code compaction
    int rbits;     // txn-rank bits in the composite (0 when the batch is already in TxnId order)
    int mode;      // 0: key only (sorted batch), 1: (key << rbits) | rank, 2: key only after a rank pre-sort
};

__global__ __launch_bounds__(BLOCK) void k_pair_keys(size_t P, const uint64_t *__restrict__ key_code,
                                                     const uint32_t *__restrict__ owner, const uint32_t *__restrict__ rank,
                                                     const uint32_t *__restrict__ perm, PairPlan plan,
                                                     int rank_only, uint64_t *__restrict__ out)
{
    size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= P) return;
    size_t j = perm ? perm[i] : i;
    if (rank_only) { out[i] = rank[owner[j]]; return; }
    uint64_t kc = pext_runs(key_code[j], plan.rk);
    out[i] = plan.mode == 1 ? ((kc << plan.rbits) | rank[owner[j]]) : kc;
}

__global__ __launch_bounds__(BLOCK) void k_seg_flags(size_t P, const uint64_t *__restrict__ skeys, int key_shift,
                                                     uint32_t *__restrict__ flag)
{
    size_t p = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p >= P) return;
    flag[p] = p == 0 || (skeys[p] >> key_shift) != (skeys[p - 1] >> key_shift);
}

// Gather per-position CFK columns; fill seg_start; classify committed (C) / uncommitted (U).
__global__ __launch_bounds__(BLOCK) void k_cfk_gather(size_t P, uint32_t n, const uint32_t *__restrict__ perm,
                                                      const uint32_t *__restrict__ owner, const uint32_t *__restrict__ rank,
                                                      const uint8_t *__restrict__ status, const uint64_t *__restrict__ tl,
                                                      const uint32_t *__restrict__ seg_incl, const uint32_t *__restrict__ seg_flag,
                                                      uint32_t *__restrict__ seg_start, uint32_t *__restrict__ s_rank,
                                                      uint32_t *__restrict__ s_exec, uint8_t *__restrict__ s_info,
                                                      uint32_t *__restrict__ pair_pos, uint32_t *__restrict__ cflag,
                                                      uint32_t *__restrict__ uflag, uint64_t *__restrict__ pmax_in)
{
    size_t p = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p >= P) return;
    uint32_t j = perm[p];
    uint32_t t = owner[j];
    uint32_t seg = seg_incl[p] - 1;
    if (seg_flag[p]) seg_start[seg] = (uint32_t)p;
    if (p == P - 1) seg_start[seg + 1] = (uint32_t)P;
    uint32_t st = status[t];
    uint32_t kind = (uint32_t)(tl[t] >> 1) & 7u;
    uint32_t er = rank[n + t];
    s_rank[p] = rank[t];
    s_exec[p] = er;
    s_info[p] = (uint8_t)(st | (kind << 3));
    pair_pos[j] = (uint32_t)p;
    bool c = st >= 4 && st <= 6;
    cflag[p] = c;
    uflag[p] = st >= 1 && st <= 3;
    // segmented prefix-max via a segment-id prefix: max over (seg << 32 | exec+1) never crosses segments
    pmax_in[p] = ((uint64_t)seg << 32) | (c ? (uint64_t)er + 1 : 0);
}

__global__ __launch_bounds__(BLOCK) void k_low32(size_t P, const uint64_t *__restrict__ in, uint32_t *__restrict__ out)
{
    size_t p = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p < P) out[p] = (uint32_t)in[p];
}

// Committed entries -> (seg << ebits | execRank) composite for the stable (seg, executeAt) sort; pads
// (all ones in `bits`) fill [NC, P) so the sort runs on the host-known size P.
__global__ __launch_bounds__(BLOCK) void k_committed_keys(size_t P, const uint32_t *__restrict__ cflag, const uint32_t *__restrict__ cum_c,
                                                          const uint32_t *__restrict__ seg_incl, const uint32_t *__restrict__ s_exec,
                                                          const uint32_t *__restrict__ uflag, const uint32_t *__restrict__ cum_u,
                                                          int ebits, int bits, uint64_t *__restrict__ ckey,
                                                          uint32_t *__restrict__ cpos, uint32_t *__restrict__ u_pos)
{
    size_t p = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p >= P) return;
    uint32_t nc = cum_c[P];
    if (cflag[p]) {
        uint32_t c = cum_c[p];
        ckey[c] = ((uint64_t)(seg_incl[p] - 1) << ebits) | s_exec[p];
        cpos[c] = (uint32_t)p;
    }
    if (p >= nc) {
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

__device__ __forceinline__ Query make_query(const CfkView &v, uint32_t j)
{
    Query q;
    uint32_t t = v.owner[j];
    uint32_t p = v.pair_pos[j];
    uint32_t seg = v.seg_incl[p] - 1;
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

template <bool EMIT>
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

// ---------------------------------------------------------------- host orchestration

static void check_errors(uint64_t errs)
{
    if (errs & ERR_BAD_STATUS) fail(ACC_E_ARG, "invalid InternalStatus ordinal (> INVALID_OR_TRUNCATED)");
    if (errs & ERR_BAD_KIND) fail(ACC_E_ARG, "Kind.ofOrdinal: invalid kind ordinal in TxnId flags");
    if (errs & ERR_KEY_OFF) fail(ACC_E_ARG, "key_off must be non-decreasing");
    if (errs & ERR_KEYS_UNSORTED) fail(ACC_E_ARG, "keys of a txn must be sorted and unique (Keys.ofSortedUnique)");
    if (errs & ERR_DUP_TXNID) fail(ACC_E_ARG, "TxnIds of a batch must be distinct (CommandsForKey txns are sorted unique)");
    if (errs & ERR_LOCAL_ONLY) fail(ACC_E_STATE, "Kind.witnesses(): unhandled kind LocalOnly (AssertionError)");
}

void keydeps_batch(acc_ctx *ctx, const acc_batch_in *in, acc_keydeps_view *view)
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

    // ---- 1. prep
    uint64_t *g = ctx->get<uint64_t>("g", 8);
    uint32_t *owner = ctx->get<uint32_t>("owner", P);
    ACC_HIP(hipMemsetAsync(g, 0, 8 * sizeof(uint64_t), st));
    launch(ctx, "prep_txn", k_prep_txn, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, tm, tl, tn, em, el, en, status,
           key_off, key_code, owner, g);
    launch(ctx, "prep_keys", k_prep_keys, dim3(grid_for(P, BLOCK)), dim3(BLOCK), 0, P, key_code, g);
    // the last key_off entry must equal P
    {
        uint32_t last = 0;
        ACC_HIP(hipMemcpyAsync(ctx->pinned, g, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        ACC_HIP(hipMemcpyAsync(ctx->pinned + 8, key_off + n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        ctx->sync();
        memcpy(&last, ctx->pinned + 8, sizeof(uint32_t));
        if (last != P) fail(ACC_E_ARG, "key_off[n_txn] must equal n_pairs");
    }
    uint64_t hg[8];
    memcpy(hg, ctx->pinned, sizeof hg);
    check_errors(hg[4]);
    const bool batch_sorted = hg[5] == 0;

    // ---- 2. dictionary: order ranks over 2N timestamps
    TsPlan plan;
    plan.r0 = make_runs(hg[0]); plan.r1 = make_runs(hg[1]); plan.r2 = make_runs(hg[2]);
    plan.b0 = plan.r0.bits; plan.b1 = plan.r1.bits; plan.b2 = plan.r2.bits;
    const size_t m = 2 * (size_t)n;
    uint32_t *rank = ctx->get<uint32_t>("rank", m);
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
    uint32_t *txn_of_rank = ctx->get<uint32_t>("txn_of_rank", m);
    launch(ctx, "rank_scatter", k_rank_scatter, dim3(gm), dim3(BLOCK), 0, m, n, (const uint32_t *)ts_sorted.vals,
           (const uint32_t *)incl, rank, txn_of_rank);
    {
        uint32_t *seen = ctx->get<uint32_t>("dup_seen", m);
        ACC_HIP(hipMemsetAsync(seen, 0, m * sizeof(uint32_t), st));
        launch(ctx, "dup_txn", k_dup_txn, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint32_t *)rank, seen, g);
    }
    const int rbits = bits_for(m - 1);

    // ---- 3. CFK build: pairs sorted by (key, TxnId rank)
    PairPlan pp;
    pp.rk = make_runs(hg[3]);
    pp.rbits = rbits;
    uint64_t *pkey = ctx->get<uint64_t>("pair_key", P);
    const unsigned gP = grid_for(P, BLOCK);
    Sorted ps;
    int key_shift = 0;
    if (batch_sorted) {
        pp.mode = 0;   // pair index order is already TxnId order within every key: stable sort by key
        launch(ctx, "pair_keys", k_pair_keys, dim3(gP), dim3(BLOCK), 0, P, key_code, (const uint32_t *)owner,
               (const uint32_t *)rank, (const uint32_t *)nullptr, pp, 0, pkey);
        ps = radix_sort(ctx, "rs_pair", pkey, nullptr, P, pp.rk.bits);
    } else if (pp.rk.bits + rbits <= 64) {
        pp.mode = 1;
        launch(ctx, "pair_keys", k_pair_keys, dim3(gP), dim3(BLOCK), 0, P, key_code, (const uint32_t *)owner,
               (const uint32_t *)rank, (const uint32_t *)nullptr, pp, 0, pkey);
        ps = radix_sort(ctx, "rs_pair", pkey, nullptr, P, pp.rk.bits + rbits);
        key_shift = rbits;
    } else {
        pp.mode = 2;
        launch(ctx, "pair_keys", k_pair_keys, dim3(gP), dim3(BLOCK), 0, P, key_code, (const uint32_t *)owner,
               (const uint32_t *)rank, (const uint32_t *)nullptr, pp, 1, pkey);
        Sorted byrank = radix_sort(ctx, "rs_pair_r", pkey, nullptr, P, rbits);
        launch(ctx, "pair_keys", k_pair_keys, dim3(gP), dim3(BLOCK), 0, P, key_code, (const uint32_t *)owner,
               (const uint32_t *)rank, (const uint32_t *)byrank.vals, pp, 0, pkey);
        ps = radix_sort(ctx, "rs_pair", pkey, byrank.vals, P, pp.rk.bits);
    }
    uint32_t *seg_flag = ctx->get<uint32_t>("seg_flag", P);
    uint32_t *seg_incl = ctx->get<uint32_t>("seg_incl", P);
    launch(ctx, "seg_flags", k_seg_flags, dim3(gP), dim3(BLOCK), 0, P, (const uint64_t *)ps.keys, key_shift, seg_flag);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, seg_flag, seg_incl, P, false);

    uint32_t *seg_start = ctx->get<uint32_t>("seg_start", P + 1);
    uint32_t *s_rank = ctx->get<uint32_t>("s_rank", P);
    uint32_t *s_exec = ctx->get<uint32_t>("s_exec", P);
    uint8_t *s_info = ctx->get<uint8_t>("s_info", P);
    uint32_t *pair_pos = ctx->get<uint32_t>("pair_pos", P);
    uint32_t *cflag = ctx->get<uint32_t>("cflag", P);
    uint32_t *uflag = ctx->get<uint32_t>("uflag", P);
    uint64_t *pmax_in = ctx->get<uint64_t>("pmax_in", P);
    launch(ctx, "cfk_gather", k_cfk_gather, dim3(gP), dim3(BLOCK), 0, P, n, (const uint32_t *)ps.vals,
           (const uint32_t *)owner, (const uint32_t *)rank, status, tl, (const uint32_t *)seg_incl,
           (const uint32_t *)seg_flag, seg_start, s_rank, s_exec, s_info, pair_pos, cflag, uflag, pmax_in);
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
           (const uint32_t *)cum_u, rbits, cbits, ckey, cpos, u_pos);
    Sorted cs = radix_sort(ctx, "rs_cl", ckey, cpos, P, cbits);
    uint32_t *cl_exec = ctx->get<uint32_t>("cl_exec", P);
    uint32_t *lastw_in = ctx->get<uint32_t>("lastw_in", P);
    uint32_t *lastw = ctx->get<uint32_t>("lastw", P);
    launch(ctx, "committed_cols", k_committed_cols, dim3(gP), dim3(BLOCK), 0, P, (const uint32_t *)cs.vals,
           (const uint32_t *)s_exec, (const uint8_t *)s_info, (const uint32_t *)cum_c, cl_exec, lastw_in);
    scan<uint32_t, OpMax<uint32_t>>(ctx, lastw_in, lastw, P, false);
    uint32_t *cl_start = ctx->get<uint32_t>("cl_start", P + 1);
    launch(ctx, "seg_committed_start", k_seg_committed_start, dim3(grid_for(P + 1, BLOCK)), dim3(BLOCK), 0, P,
           (const uint32_t *)seg_incl, (const uint32_t *)seg_start, (const uint32_t *)cum_c, cl_start);

    // ---- 4. conflict scan: count, scan, emit
    CfkView v;
    v.seg_start = seg_start; v.s_rank = s_rank; v.s_exec = s_exec; v.seg_incl = seg_incl; v.pair_pos = pair_pos;
    v.owner = owner; v.rank = rank; v.s_info = s_info; v.cl_start = cl_start; v.cl_exec = cl_exec; v.lastw = lastw;
    v.pmax = pmax; v.cum_u = cum_u; v.u_pos = u_pos; v.tl = tl; v.n = n;
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

}  // namespace acc
