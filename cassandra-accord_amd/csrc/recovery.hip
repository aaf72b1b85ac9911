// recovery.hip — batched CommandsForKey.mapReduceFull (SURVEY.md §8(f) N3 = §8(a) A7).
//
// BeginRecovery asks every replica four questions about the txn X being recovered
// (messages/BeginRecovery.java:334-378), each a SafeCommandStore.mapReduceFull over X's keys
// (impl/InMemoryCommandStore.java:874-881) = per key CommandsForKey.mapReduceFull (local/CommandsForKey.java:553-612):
// a window of the key's txns (before / from / all around X's insert position), a kind test
// (X.kind().witnessedBy()), a status test and, for WITH / WITHOUT, whether X is in the entry's missing[].
//
// Device plan (the CFK snapshot of keydeps.hip, stages 1-3, is shared):
//   1. query ranks    X need not be a batch member: binary search of X over the dictionary's distinct timestamps
//                     gives lo = #timestamps < X and eq = (one equals X), so "TxnId < X" is rank < lo and
//                     "executeAt <= X" is exec rank < lo + eq.
//   2. items          per (query, key): its segment (binary search of the sorted segment keys), the binarySearch
//                     insert position of X among the segment's TxnId ranks, the window, its 256-entry chunks.
//   3. count / emit   one wave per chunk evaluates the entry predicate (kind, status, hasInfo, executeAt, missing[]
//                     membership by binary search over TxnId ranks) and compacts matches in position order, so each
//                     query's entries come out key by key in TxnId order (the map visiting order).
//   4. build          Deps.Builder: keys with >= 1 entry, one (query, TxnId rank) radix sort for the sorted unique
//                     TxnIds and each entry's index, the Java keysToTxnIds layout.
#include "dict.hpp"

namespace acc {

constexpr uint32_t RC_CH = 256;   // CFK entries per work chunk: one wave, four per lane

enum : uint64_t {
    RC_ERR_KIND_STATE = 1, RC_ERR_KIND_ARG = 2, RC_ERR_KEYS = 4, RC_ERR_QOFF = 8,
    RC_ERR_MISS_IDX = 16, RC_ERR_MISS_SORT = 32, RC_ERR_MISS_OFF = 64,
};

struct RcParams {
    uint32_t started_at, test_dep, test_status, exec_after;
};

// Timestamp.compareTo (primitives/Timestamp.java:208-217): msb, then lsb >>> 16 and lsb & 0x1E (both inside
// lsb & IDENTITY_LSB, unsigned), then signed node
__device__ __forceinline__ int rc_ts_cmp(uint64_t am, uint64_t al, int32_t an, uint64_t bm, uint64_t bl, int32_t bn)
{
    constexpr uint64_t ID = 0xFFFFFFFFFFFF001EULL;
    if (am != bm) return am < bm ? -1 : 1;
    const uint64_t a1 = al & ID, b1 = bl & ID;
    if (a1 != b1) return a1 < b1 ? -1 : 1;
    if (an != bn) return an < bn ? -1 : 1;
    return 0;
}

// Kind.witnessedBy() (primitives/Txn.java:247-262) as a mask over Kind ordinals: EphemeralRead -> Nothing,
// Read -> WsOrSyncPoints, Write -> AnyGloballyVisible, SyncPoint / ExclusiveSyncPoint -> ExclusiveSyncPoints
__device__ __forceinline__ int witnessed_by(uint32_t kind)
{
    switch (kind) {
    case 2:         return 0;
    case 0:         return (1 << 1) | (1 << 3) | (1 << 4);
    case 1:         return (1 << 0) | (1 << 1) | (1 << 3) | (1 << 4);
    case 3: case 4: return 1 << 4;
    default:        return -1;
    }
}

template <class T>
__device__ __forceinline__ uint32_t rc_lower(const T *a, uint32_t lo, uint32_t hi, T v)
{
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (a[m] < v) lo = m + 1; else hi = m; }
    return lo;
}

// first index in [0, n) with a[idx] > v
__device__ __forceinline__ uint32_t rc_upper64(const uint64_t *a, uint32_t n, uint64_t v)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (a[m] <= v) lo = m + 1; else hi = m; }
    return lo;
}

__global__ __launch_bounds__(BLOCK) void k_rc_src_of_rank(size_t m, const uint32_t *__restrict__ rank,
                                                          uint32_t *__restrict__ src_of_rank, uint32_t *__restrict__ nranks)
{
    const size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    uint32_t r = 0;
    if (i < m) {
        r = rank[i] + 1;
        src_of_rank[r - 1] = (uint32_t)i;   // equal timestamps share a rank: any of them represents it
    }
    r = wave_inclusive(r, OpMax<uint32_t>());
    if (lane_id() == 63 && r) atomicMax(nranks, r);
}

// missing[] of every input pair: batch indices, strictly ascending by TxnId (Arrays.binarySearch needs sorted input)
__global__ __launch_bounds__(BLOCK) void k_rc_missing(size_t P, uint32_t n, uint64_t n_missing, const uint32_t *__restrict__ off,
                                                      const uint32_t *__restrict__ txn, const uint32_t *__restrict__ rank,
                                                      uint64_t *__restrict__ errs)
{
    const size_t j = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    uint64_t e = 0;
    if (j < P) {
        const uint32_t m0 = off[j], m1 = off[j + 1];
        if (m1 < m0 || m1 > n_missing || (j == P - 1 && m1 != n_missing) || (j == 0 && m0 != 0)) e |= RC_ERR_MISS_OFF;
        else
            for (uint32_t x = m0; x < m1; ++x) {
                if (txn[x] >= n) { e |= RC_ERR_MISS_IDX; break; }
                if (x > m0 && rank[txn[x - 1]] >= rank[txn[x]]) { e |= RC_ERR_MISS_SORT; break; }
            }
    }
    if (__ballot(e != 0) && e) atomicOr((unsigned long long *)errs, (unsigned long long)e);
}

struct RcSnap {
    const uint64_t *tm, *tl, *em, *el;
    const int32_t *tn, *en;
    const uint32_t *src_of_rank, *nranks;
    uint32_t n;
};

// per query: lo = #dictionary timestamps below testTxnId, eq = testTxnId is one of them, the Kinds mask
__global__ __launch_bounds__(BLOCK) void k_rc_query(uint32_t nq, const uint64_t *__restrict__ qm, const uint64_t *__restrict__ ql,
                                                    const int32_t *__restrict__ qn, const uint32_t *__restrict__ qoff,
                                                    const uint64_t *__restrict__ qkey, RcSnap s, int test_kinds,
                                                    uint32_t *__restrict__ qlo, uint8_t *__restrict__ qeq,
                                                    uint8_t *__restrict__ qmask, uint64_t *__restrict__ errs)
{
    const uint32_t q = blockIdx.x * BLOCK + threadIdx.x;
    if (q >= nq) return;
    uint64_t e = 0;
    const uint64_t xm = qm[q], xl = ql[q];
    const int32_t xn = qn[q];
    const uint32_t nr = s.nranks ? *s.nranks : 0u;
    uint32_t lo = 0, hi = nr;
    auto cmp_rank = [&](uint32_t r) {
        const uint32_t src = s.src_of_rank[r];
        return src < s.n ? rc_ts_cmp(s.tm[src], s.tl[src], s.tn[src], xm, xl, xn)
                         : rc_ts_cmp(s.em[src - s.n], s.el[src - s.n], s.en[src - s.n], xm, xl, xn);
    };
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (cmp_rank(m) < 0) lo = m + 1; else hi = m; }
    qlo[q] = lo;
    qeq[q] = lo < nr && cmp_rank(lo) == 0;
    const uint32_t kind = (uint32_t)(xl >> 1) & 7u;
    int mask = test_kinds;
    if (mask < 0) {
        mask = witnessed_by(kind);
        if (mask < 0) e |= kind == 5 ? RC_ERR_KIND_STATE : RC_ERR_KIND_ARG;   // LocalOnly: AssertionError; > 5: ofOrdinal
    }
    qmask[q] = (uint8_t)(mask < 0 ? 0 : mask);
    const uint32_t k0 = qoff[q], k1 = qoff[q + 1];
    if (k1 < k0) e |= RC_ERR_QOFF;
    else
        for (uint32_t j = k0 + 1; j < k1; ++j)
            if (qkey[j - 1] >= qkey[j]) { e |= RC_ERR_KEYS; break; }
    if (e) atomicOr((unsigned long long *)errs, (unsigned long long)e);
}

struct RcCfk {
    const uint64_t *seg_key;
    const uint32_t *seg_start, *s_rank, *s_exec, *perm, *rank, *miss_off, *miss_txn;
    const uint8_t *s_info;
    uint32_t nseg;
    uint32_t P;
};

// per (query, key): the CommandsForKey.mapReduceFull window [start, end) of the key's segment
__global__ __launch_bounds__(BLOCK) void k_rc_items(uint32_t Qp, uint32_t nq, const uint32_t *__restrict__ qoff,
                                                    const uint64_t *__restrict__ qkey, RcCfk c, RcParams p,
                                                    const uint32_t *__restrict__ qlo, const uint8_t *__restrict__ qeq,
                                                    uint32_t *__restrict__ item_q, uint32_t *__restrict__ item_a,
                                                    uint32_t *__restrict__ item_w, uint64_t *__restrict__ item_chunks)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= Qp) return;
    uint32_t lo = 0, hi = nq + 1;   // q = (first index with qoff > i) - 1
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (qoff[m] <= i) lo = m + 1; else hi = m; }
    const uint32_t q = lo - 1;
    item_q[i] = q;
    uint32_t a = 0, w = 0;
    const uint64_t k = qkey[i];
    const uint32_t s = c.nseg ? rc_lower<uint64_t>(c.seg_key, 0, c.nseg, k) : 0;
    if (s < c.nseg && c.seg_key[s] == k) {
        const uint32_t sb = c.seg_start[s], se = s + 1 < c.nseg ? c.seg_start[s + 1] : c.P;
        const uint32_t x = qlo[q];
        // Arrays.binarySearch(txns, testTxnId): found <=> X is a member; insertPos = its index or the insert point
        const uint32_t pos = rc_lower<uint32_t>(c.s_rank, sb, se, x);
        const bool known = qeq[q] && pos < se && c.s_rank[pos] == x;
        if (known || p.test_dep != 0) {
            const uint32_t start = p.started_at == 1 ? pos : sb;
            const uint32_t end = p.started_at == 0 ? pos : se;
            a = start;
            w = end - start;
        }
    }
    item_a[i] = a;
    item_w[i] = w;
    item_chunks[i] = (w + RC_CH - 1) / RC_CH;
}

// the per-entry tests of CommandsForKey.mapReduceFull (:577-607) plus the optional executeAt > testTxnId map filter
__device__ __forceinline__ bool rc_match(const RcCfk &c, const RcParams &p, uint32_t e, uint32_t mask, uint32_t x, bool eq)
{
    const uint32_t info = c.s_info[e];
    const uint32_t status = info & 7u, kind = info >> 3;
    if (!((mask >> kind) & 1u)) return false;
    switch (p.test_status) {
    case 1: if (status != 3 && status != 4) return false; break;   // IS_PROPOSED: ACCEPTED, COMMITTED
    case 2: if (status < 5 || status >= 7) return false; break;    // IS_STABLE: STABLE <= s < INVALID_OR_TRUNCATED
    default: if (status == 0) return false; break;                 // ANY_STATUS: not TRANSITIVELY_KNOWN
    }
    const uint32_t ex = c.s_exec[e];
    const bool exec_after = ex >= x + (eq ? 1u : 0u);             // executeAt > testTxnId
    if (p.test_dep != 2) {
        if (status < 3 || status > 6) return false;               // !InternalStatus.hasInfo
        if (!exec_after) return false;
        bool in_missing = false;
        if (eq) {                                                 // only a batch member can be in missing[]
            const uint32_t j = c.perm[e];
            uint32_t lo = c.miss_off[j], hi = c.miss_off[j + 1];
            while (lo < hi) {
                const uint32_t m = (lo + hi) >> 1;
                const uint32_t r = c.rank[c.miss_txn[m]];
                if (r < x) lo = m + 1; else if (r > x) hi = m; else { in_missing = true; break; }
            }
        }
        if (in_missing == (p.test_dep == 0)) return false;        // hasAsDep != (testDep == WITH)
    }
    if (p.exec_after && !exec_after) return false;
    return true;
}

struct RcChunks {
    const uint64_t *chunk_off;   // [Qp+1] exclusive scan of item_chunks
    const uint32_t *item_q, *item_a, *item_w, *qlo;
    const uint8_t *qeq, *qmask;
    uint32_t Qp;
};

// one wave per chunk: match count (and its item's running total)
__global__ __launch_bounds__(BLOCK) void k_rc_count(uint64_t nchunks, RcCfk c, RcParams p, RcChunks ch,
                                                    uint32_t *__restrict__ chunk_cnt, unsigned long long *__restrict__ item_cnt)
{
    const uint64_t cw = (uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    if (cw >= nchunks) return;
    const uint32_t item = rc_upper64(ch.chunk_off, ch.Qp + 1, cw) - 1;
    const uint32_t q = ch.item_q[item];
    const uint32_t base = ch.item_a[item] + (uint32_t)(cw - ch.chunk_off[item]) * RC_CH;
    const uint32_t end = ch.item_a[item] + ch.item_w[item];
    const uint32_t x = ch.qlo[q], mask = ch.qmask[q];
    const bool eq = ch.qeq[q] != 0;
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t u = 0; u < RC_CH / 64; ++u) {
        const uint32_t e = base + u * 64 + lane_id();
        cnt += (uint32_t)__popcll(__ballot(e < end && rc_match(c, p, e, mask, x, eq)));
    }
    if (lane_id() == 0) {
        chunk_cnt[cw] = cnt;
        if (cnt) atomicAdd(&item_cnt[item], (unsigned long long)cnt);
    }
}

// the same walk, compacting matches in position order: (query << rbits | TxnId rank) per emitted entry
__global__ __launch_bounds__(BLOCK) void k_rc_emit(uint64_t nchunks, RcCfk c, RcParams p, RcChunks ch,
                                                   const uint64_t *__restrict__ chunk_eoff, int rbits, uint64_t *__restrict__ ent)
{
    const uint64_t cw = (uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    if (cw >= nchunks) return;
    const uint32_t item = rc_upper64(ch.chunk_off, ch.Qp + 1, cw) - 1;
    const uint32_t q = ch.item_q[item];
    const uint32_t base = ch.item_a[item] + (uint32_t)(cw - ch.chunk_off[item]) * RC_CH;
    const uint32_t end = ch.item_a[item] + ch.item_w[item];
    const uint32_t x = ch.qlo[q], mask = ch.qmask[q];
    const bool eq = ch.qeq[q] != 0;
    const uint64_t lt = (1ull << lane_id()) - 1;
    uint64_t out = chunk_eoff[cw];
#pragma unroll
    for (uint32_t u = 0; u < RC_CH / 64; ++u) {
        const uint32_t e = base + u * 64 + lane_id();
        const bool m = e < end && rc_match(c, p, e, mask, x, eq);
        const uint64_t bal = __ballot(m);
        if (m) ent[out + (uint64_t)__popcll(bal & lt)] = ((uint64_t)q << rbits) | c.s_rank[e];
        out += (uint64_t)__popcll(bal);
    }
}

__global__ __launch_bounds__(BLOCK) void k_rc_widen(uint64_t n, const uint32_t *__restrict__ in, uint64_t *__restrict__ out)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) out[i] = in[i];
}

__global__ __launch_bounds__(BLOCK) void k_rc_kept(uint32_t Qp, const unsigned long long *__restrict__ item_cnt,
                                                   uint64_t *__restrict__ kept)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < Qp) kept[i] = item_cnt[i] ? 1u : 0u;
}

// per query (and the end sentinel): arena and key offsets from the item scans
__global__ __launch_bounds__(BLOCK) void k_rc_qoff(uint32_t nq, const uint32_t *__restrict__ qoff, const uint64_t *__restrict__ kpos,
                                                   const uint64_t *__restrict__ epos, uint64_t *__restrict__ arena_off,
                                                   uint64_t *__restrict__ kd_off)
{
    const uint32_t q = blockIdx.x * BLOCK + threadIdx.x;
    if (q > nq) return;
    const uint32_t b = qoff[q];
    arena_off[q] = kpos[b] + epos[b];
    kd_off[q] = kpos[b];
}

// AbstractBuilder: a key with entries gets its end offset (keys.length + entries through it) and its key index
__global__ __launch_bounds__(BLOCK) void k_rc_header(uint32_t Qp, const uint32_t *__restrict__ item_q,
                                                     const unsigned long long *__restrict__ item_cnt, const uint32_t *__restrict__ qoff,
                                                     const uint64_t *__restrict__ kpos, const uint64_t *__restrict__ epos,
                                                     const uint64_t *__restrict__ arena_off, int32_t *__restrict__ arena,
                                                     uint32_t *__restrict__ key_idx)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= Qp) return;
    const uint64_t cnt = item_cnt[i];
    if (!cnt) return;
    const uint32_t q = item_q[i], b = qoff[q], e = qoff[q + 1];
    const uint64_t kd = kpos[e] - kpos[b];
    arena[arena_off[q] + (kpos[i] - kpos[b])] = (int32_t)(kd + (epos[i] + cnt - epos[b]));
    key_idx[kpos[i]] = i - b;
}

__global__ __launch_bounds__(BLOCK) void k_rc_uflag(uint64_t E, const uint64_t *__restrict__ keys, int rbits,
                                                    uint32_t *__restrict__ uflag, unsigned long long *__restrict__ u_cnt)
{
    const uint64_t p = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p >= E) return;
    const bool f = p == 0 || keys[p] != keys[p - 1];
    uflag[p] = f ? 1u : 0u;
    if (f) atomicAdd(&u_cnt[keys[p] >> rbits], 1ull);
}

// every entry's index into its query's sorted unique TxnIds; the TxnIds themselves as batch indices
__global__ __launch_bounds__(BLOCK) void k_rc_body(uint64_t E, const uint64_t *__restrict__ keys, const uint32_t *__restrict__ src,
                                                   const uint32_t *__restrict__ uflag, const uint32_t *__restrict__ uincl, int rbits,
                                                   const uint32_t *__restrict__ qoff, const uint64_t *__restrict__ kpos,
                                                   const uint64_t *__restrict__ epos, const uint64_t *__restrict__ arena_off,
                                                   const uint64_t *__restrict__ u_off, const uint32_t *__restrict__ txn_of_rank,
                                                   int32_t *__restrict__ arena, uint32_t *__restrict__ dep_txn)
{
    const uint64_t p = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p >= E) return;
    const uint64_t key = keys[p];
    const uint32_t q = (uint32_t)(key >> rbits), r = (uint32_t)(key & ((1ull << rbits) - 1));
    const uint64_t uid = (uint64_t)uincl[p] - 1;
    const uint32_t b = qoff[q], e = qoff[q + 1];
    const uint64_t kd = kpos[e] - kpos[b];
    arena[arena_off[q] + kd + ((uint64_t)src[p] - epos[b])] = (int32_t)(uid - u_off[q]);
    if (uflag[p]) dep_txn[uid] = txn_of_rank[r];
}

static void check_rc_errors(uint64_t e)
{
    if (e & RC_ERR_KIND_STATE) fail(ACC_E_STATE, "Kind.witnessedBy(): unhandled kind LocalOnly (AssertionError)");
    if (e & RC_ERR_KIND_ARG) fail(ACC_E_ARG, "Kind.ofOrdinal: invalid kind ordinal in a testTxnId");
    if (e & RC_ERR_QOFF) fail(ACC_E_ARG, "query key_off must be non-decreasing");
    if (e & RC_ERR_KEYS) fail(ACC_E_ARG, "keys of a query must be sorted and unique (Keys.ofSortedUnique)");
    if (e & RC_ERR_MISS_OFF) fail(ACC_E_ARG, "missing_off must be non-decreasing from 0 to n_missing");
    if (e & RC_ERR_MISS_IDX) fail(ACC_E_ARG, "missing[] entry is not a batch txn");
    if (e & RC_ERR_MISS_SORT) fail(ACC_E_ARG, "missing[] must be sorted unique by TxnId (Arrays.binarySearch)");
}

void map_reduce_full(acc_ctx *ctx, const acc_batch_in *in, const acc_recovery_in *rq, acc_keydeps_view *view)
{
    if (!in || !rq || !view) fail(ACC_E_ARG, "null argument");
    if (rq->mem != ACC_MEM_HOST && rq->mem != ACC_MEM_DEVICE) fail(ACC_E_ARG, "mem must be ACC_MEM_HOST or ACC_MEM_DEVICE");
    if (rq->started_at > 2 || rq->test_dep > 2 || rq->test_status > 2)
        fail(ACC_E_ARG, "started_at / test_dep / test_status must be TestStartedAt / TestDep / TestStatus ordinals");
    if (rq->flags & ~ACC_FULL_EXECUTES_AFTER) fail(ACC_E_ARG, "unknown flags");
    if (rq->test_kinds > 0x3F) fail(ACC_E_ARG, "test_kinds must be a mask over the six Kind ordinals, or -1");
    hipStream_t st = ctx->stream;
    ctx->kd_valid = false;
    CfkSnapshot s;
    cfk_snapshot(ctx, in, s);
    const uint32_t nq = rq->n_query, n = s.n;
    const size_t P = s.P;
    const uint32_t mem = rq->mem;

    const uint32_t *qoff = stage_in(ctx, "rc_qoff", rq->key_off, (size_t)nq + 1, mem);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, qoff + nq, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint32_t Qp = (uint32_t)(ctx->pinned[0] & 0xFFFFFFFFu);
    const uint64_t *qm = stage_in(ctx, "rc_qm", rq->test_txn.msb, nq, mem);
    const uint64_t *ql = stage_in(ctx, "rc_ql", rq->test_txn.lsb, nq, mem);
    const int32_t *qn = stage_in(ctx, "rc_qn", rq->test_txn.node, nq, mem);
    const uint64_t *qkey = stage_in(ctx, "rc_qkey", rq->key_code, Qp, mem);
    const uint32_t *moff = stage_in(ctx, "rc_moff", rq->missing_off, P + 1, mem);
    const uint32_t *mtxn = stage_in(ctx, "rc_mtxn", rq->missing_txn, (size_t)rq->n_missing, mem);

    uint64_t *errs = ctx->get<uint64_t>("rc_errs", 1);
    uint32_t *nranks = ctx->get<uint32_t>("rc_nranks", 1);
    ACC_HIP(hipMemsetAsync(errs, 0, 8, st));
    ACC_HIP(hipMemsetAsync(nranks, 0, 4, st));
    RcSnap rs{ s.tm, s.tl, s.em, s.el, s.tn, s.en, nullptr, nranks, n };
    if (s.cfk) {
        const size_t m = 2 * (size_t)n;
        uint32_t *sor = ctx->get<uint32_t>("rc_src_of_rank", m);
        launch(ctx, "rc_src_of_rank", k_rc_src_of_rank, dim3(grid_for(m, BLOCK)), dim3(BLOCK), 0, m, s.rank, sor, nranks);
        rs.src_of_rank = sor;
        launch(ctx, "rc_missing", k_rc_missing, dim3(grid_for(P, BLOCK)), dim3(BLOCK), 0, P, n, rq->n_missing, moff, mtxn,
               s.rank, errs);
    }
    uint32_t *qlo = ctx->get<uint32_t>("rc_qlo", nq);
    uint8_t *qeq = ctx->get<uint8_t>("rc_qeq", nq);
    uint8_t *qmask = ctx->get<uint8_t>("rc_qmask", nq);
    launch(ctx, "rc_query", k_rc_query, dim3(grid_for(nq, BLOCK)), dim3(BLOCK), 0, nq, qm, ql, qn, qoff, qkey, rs,
           (int)rq->test_kinds, qlo, qeq, qmask, errs);

    const RcParams prm{ rq->started_at, rq->test_dep, rq->test_status, (uint32_t)(rq->flags & ACC_FULL_EXECUTES_AFTER) };
    RcCfk c{ s.seg_key, s.seg_start, s.s_rank, s.s_exec, s.perm, s.rank, moff, mtxn, s.s_info, s.cfk ? s.nseg : 0u,
             (uint32_t)P };
    uint32_t *item_q = ctx->get<uint32_t>("rc_item_q", Qp);
    uint32_t *item_a = ctx->get<uint32_t>("rc_item_a", Qp);
    uint32_t *item_w = ctx->get<uint32_t>("rc_item_w", Qp);
    uint64_t *item_chunks = ctx->get<uint64_t>("rc_item_chunks", Qp);
    uint64_t *chunk_off = ctx->get<uint64_t>("rc_chunk_off", (size_t)Qp + 1);
    if (Qp) {
        launch(ctx, "rc_items", k_rc_items, dim3(grid_for(Qp, BLOCK)), dim3(BLOCK), 0, Qp, nq, qoff, qkey, c, prm,
               (const uint32_t *)qlo, (const uint8_t *)qeq, item_q, item_a, item_w, item_chunks);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, item_chunks, chunk_off, Qp, true, chunk_off + Qp);
    } else {
        ACC_HIP(hipMemsetAsync(chunk_off, 0, 8, st));
    }
    ACC_HIP(hipMemcpyAsync(ctx->pinned, errs, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, chunk_off + Qp, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    check_rc_errors(ctx->pinned[0]);
    const uint64_t NC = ctx->pinned[1];

    // ---- count, scan, emit
    unsigned long long *item_cnt = ctx->get<unsigned long long>("rc_item_cnt", Qp);
    uint32_t *chunk_cnt = ctx->get<uint32_t>("rc_chunk_cnt", NC);
    uint64_t *chunk_cnt64 = ctx->get<uint64_t>("rc_chunk_cnt64", NC);
    uint64_t *chunk_eoff = ctx->get<uint64_t>("rc_chunk_eoff", NC + 1);
    ACC_HIP(hipMemsetAsync(item_cnt, 0, (size_t)Qp * 8, st));
    RcChunks chs{ chunk_off, item_q, item_a, item_w, qlo, qeq, qmask, Qp };
    const unsigned gW = (unsigned)((NC + WAVES - 1) / WAVES);
    if (NC) {
        launch(ctx, "rc_count", k_rc_count, dim3(gW), dim3(BLOCK), 0, NC, c, prm, chs, chunk_cnt, item_cnt);
        launch(ctx, "rc_widen", k_rc_widen, dim3(grid_for(NC, BLOCK)), dim3(BLOCK), 0, NC, (const uint32_t *)chunk_cnt, chunk_cnt64);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, chunk_cnt64, chunk_eoff, NC, true, chunk_eoff + NC);
    } else {
        ACC_HIP(hipMemsetAsync(chunk_eoff, 0, 8, st));
    }
    uint64_t *kept = ctx->get<uint64_t>("rc_kept", Qp);
    uint64_t *kpos = ctx->get<uint64_t>("rc_kpos", (size_t)Qp + 1);
    uint64_t *epos = ctx->get<uint64_t>("rc_epos", (size_t)Qp + 1);
    if (Qp) {
        launch(ctx, "rc_kept", k_rc_kept, dim3(grid_for(Qp, BLOCK)), dim3(BLOCK), 0, Qp, (const unsigned long long *)item_cnt, kept);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, kept, kpos, Qp, true, kpos + Qp);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, reinterpret_cast<const uint64_t *>(item_cnt), epos, Qp, true, epos + Qp);
    } else {
        ACC_HIP(hipMemsetAsync(kpos, 0, 8, st));
        ACC_HIP(hipMemsetAsync(epos, 0, 8, st));
    }
    ACC_HIP(hipMemcpyAsync(ctx->pinned, chunk_eoff + NC, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, kpos + Qp, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t E = ctx->pinned[0], TK = ctx->pinned[1];
    if (E >= 0xFFFFFFFFull) fail(ACC_E_CAP, "more than 2^32-1 recovery-scan entries in one call");
    const int rbits = s.rbits;
    const int qbits = bits_for(nq ? nq - 1 : 0);
    if (E && qbits + rbits > 64) fail(ACC_E_CAP, "too many queries for the (query, TxnId rank) composite key");
    uint64_t *ent = ctx->get<uint64_t>("rc_ent", E);
    if (E) launch(ctx, "rc_emit", k_rc_emit, dim3(gW), dim3(BLOCK), 0, NC, c, prm, chs, (const uint64_t *)chunk_eoff, rbits, ent);

    // ---- Deps.Builder layout
    uint64_t *arena_off = ctx->get<uint64_t>("rc_arena_off", (size_t)nq + 1);
    uint64_t *kd_off = ctx->get<uint64_t>("rc_kd_off", (size_t)nq + 1);
    uint64_t *u_off = ctx->get<uint64_t>("rc_u_off", (size_t)nq + 1);
    int32_t *arena = ctx->get<int32_t>("rc_arena", TK + E);
    uint32_t *key_idx = ctx->get<uint32_t>("rc_key_idx", TK);
    uint32_t *dep_txn = ctx->get<uint32_t>("rc_dep_txn", E);
    unsigned long long *u_cnt = ctx->get<unsigned long long>("rc_u_cnt", nq);
    ACC_HIP(hipMemsetAsync(u_cnt, 0, (size_t)nq * 8, st));
    launch(ctx, "rc_qoff", k_rc_qoff, dim3(grid_for((size_t)nq + 1, BLOCK)), dim3(BLOCK), 0, nq, qoff, (const uint64_t *)kpos,
           (const uint64_t *)epos, arena_off, kd_off);
    if (Qp)
        launch(ctx, "rc_header", k_rc_header, dim3(grid_for(Qp, BLOCK)), dim3(BLOCK), 0, Qp, (const uint32_t *)item_q,
               (const unsigned long long *)item_cnt, qoff, (const uint64_t *)kpos, (const uint64_t *)epos,
               (const uint64_t *)arena_off, arena, key_idx);
    if (E) {
        Sorted so = radix_sort(ctx, "rc_rs", ent, nullptr, E, qbits + rbits);
        uint32_t *uflag = ctx->get<uint32_t>("rc_uflag", E);
        uint32_t *uincl = ctx->get<uint32_t>("rc_uincl", E);
        launch(ctx, "rc_uflag", k_rc_uflag, dim3(grid_for(E, BLOCK)), dim3(BLOCK), 0, E, (const uint64_t *)so.keys, rbits, uflag, u_cnt);
        scan<uint32_t, OpAdd<uint32_t>>(ctx, uflag, uincl, E, false);
        if (nq) scan<uint64_t, OpAdd<uint64_t>>(ctx, reinterpret_cast<const uint64_t *>(u_cnt), u_off, nq, true, u_off + nq);
        launch(ctx, "rc_body", k_rc_body, dim3(grid_for(E, BLOCK)), dim3(BLOCK), 0, E, (const uint64_t *)so.keys,
               (const uint32_t *)so.vals, (const uint32_t *)uflag, (const uint32_t *)uincl, rbits, qoff, (const uint64_t *)kpos,
               (const uint64_t *)epos, (const uint64_t *)arena_off, (const uint64_t *)u_off, s.txn_of_rank, arena, dep_txn);
    } else {
        ACC_HIP(hipMemsetAsync(u_off, 0, ((size_t)nq + 1) * 8, st));
    }
    ACC_HIP(hipMemcpyAsync(ctx->pinned, u_off + nq, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t TU = ctx->pinned[0];
    ctx->stat("recovery.items", Qp);
    ctx->stat("recovery.chunks", NC);
    ctx->stat("recovery.entries", E);
    *view = acc_keydeps_view{ nq, TK + E, TK, TU, E, arena_off, arena, kd_off, key_idx, u_off, dep_txn, nullptr };
    ctx->kd_view = *view;
    ctx->kd_valid = true;
}

}  // namespace acc
