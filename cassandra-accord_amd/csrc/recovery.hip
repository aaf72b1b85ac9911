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

// ================================================================ range-command half
// InMemorySafeStore.mapReduceRangesInternal (impl/InMemoryCommandStore.java:883-1016) for a batch of recovery queries:
//   1. table        validation, TxnId ranks of the (TxnId-sorted) command table, the distinct-range dictionary
//                   (two stable radix sorts: by end, then by start = Range::compare order)
//   2. windows      per query the table window its TestStartedAt admits (binary searches of testTxnId), 64-entry chunks
//   3. count / emit one wave per chunk, one lane per command: the status / kind / executeAt / Deps.intersects tests, then
//                   every range of the command that intersects the query's participants (Routables.foldl) gives an
//                   entry (query, range id, TxnId rank)
//   4. build        the TreeMap<Range, List> + Deps.Builder result = sorted unique entries; RangeDeps layout per query
//                   (a second (query, TxnId rank) sort gives the sorted unique TxnIds and each entry's index)

enum : uint64_t {
    RR_ERR_ORDER = 1, RR_ERR_STATUS = 2, RR_ERR_RANGES = 4, RR_ERR_DEPS = 8, RR_ERR_PARTS = 16,
    RR_ERR_KIND_STATE = 32, RR_ERR_KIND_ARG = 64, RR_ERR_OFF = 128,
};

struct RrCmds {
    const uint64_t *tm, *tl, *em, *el;
    const int32_t *tn, *en;
    const uint8_t *status, *flags;
    const uint32_t *roff;
    const uint64_t *rs, *re;
    const uint32_t *doff;
    const uint64_t *dm, *dl;
    const int32_t *dn;
    const uint64_t *ds, *de;
    const uint8_t *dk;
    const uint32_t *trank, *rid;
    uint32_t n, end_incl;
    uint64_t R, D;
};

struct RrQueries {
    const uint64_t *qm, *ql;
    const int32_t *qn;
    const uint8_t *isr;
    const uint32_t *poff;
    const uint64_t *ps, *pe;
    uint32_t nq;
};

__device__ __forceinline__ bool rr_contains(uint64_t s, uint64_t e, uint64_t k, bool ei)
{
    return ei ? (s < k && k <= e) : (s <= k && k < e);   // Range.contains (Range.java:40-138)
}

__global__ __launch_bounds__(BLOCK) void k_rr_check(RrCmds c, uint32_t *__restrict__ tflag, uint64_t *__restrict__ errs)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= c.n) return;
    uint64_t e = 0;
    int prev = 1;
    if (i > 0) {
        prev = rc_ts_cmp(c.tm[i - 1], c.tl[i - 1], c.tn[i - 1], c.tm[i], c.tl[i], c.tn[i]);
        if (prev > 0) e |= RR_ERR_ORDER;
    }
    tflag[i] = prev != 0 ? 1u : 0u;
    if (c.status[i] > 10 || (c.flags[i] & ~7u)) e |= RR_ERR_STATUS;
    const uint32_t r0 = c.roff[i], r1 = c.roff[i + 1];
    if (r1 < r0 || r1 > c.R || (i == 0 && r0 != 0) || (i == c.n - 1 && r1 != c.R)) e |= RR_ERR_OFF;
    else
        for (uint32_t j = r0; j < r1; ++j)
            if (c.rs[j] >= c.re[j] || (j > r0 && c.re[j - 1] > c.rs[j])) { e |= RR_ERR_RANGES; break; }
    const uint32_t d0 = c.doff[i], d1 = c.doff[i + 1];
    if (d1 < d0 || d1 > c.D || (i == 0 && d0 != 0) || (i == c.n - 1 && d1 != c.D)) e |= RR_ERR_OFF;
    else
        for (uint32_t j = d0; j < d1; ++j) {
            if (!c.dk[j] && c.ds[j] >= c.de[j]) { e |= RR_ERR_DEPS; break; }
            if (j > d0 && rc_ts_cmp(c.dm[j - 1], c.dl[j - 1], c.dn[j - 1], c.dm[j], c.dl[j], c.dn[j]) > 0) { e |= RR_ERR_DEPS; break; }
        }
    if (e) atomicOr((unsigned long long *)errs, (unsigned long long)e);
}

__global__ __launch_bounds__(BLOCK) void k_rr_first(uint32_t n, const uint32_t *__restrict__ tflag, const uint32_t *__restrict__ tincl,
                                                    uint32_t *__restrict__ trank, uint32_t *__restrict__ first_of)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = tincl[i] - 1;
    trank[i] = r;
    if (tflag[i]) first_of[r] = i;
}

__global__ __launch_bounds__(BLOCK) void k_rr_gather64(uint64_t n, const uint32_t *__restrict__ perm, const uint64_t *__restrict__ in,
                                                       uint64_t *__restrict__ out)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) out[i] = in[perm[i]];
}

// sorted (start, end) -> dictionary flags (a new distinct range)
__global__ __launch_bounds__(BLOCK) void k_rr_dflag(uint64_t R, const uint64_t *__restrict__ ss, const uint32_t *__restrict__ perm,
                                                    const uint64_t *__restrict__ re, uint32_t *__restrict__ dflag)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= R) return;
    dflag[i] = (i == 0 || ss[i] != ss[i - 1] || re[perm[i]] != re[perm[i - 1]]) ? 1u : 0u;
}

__global__ __launch_bounds__(BLOCK) void k_rr_dict(uint64_t R, const uint64_t *__restrict__ ss, const uint32_t *__restrict__ perm,
                                                   const uint64_t *__restrict__ re, const uint32_t *__restrict__ dflag,
                                                   const uint32_t *__restrict__ dincl, uint32_t *__restrict__ rid,
                                                   uint64_t *__restrict__ dict_s, uint64_t *__restrict__ dict_e)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= R) return;
    const uint32_t d = dincl[i] - 1, j = perm[i];
    rid[j] = d;
    if (dflag[i]) { dict_s[d] = ss[i]; dict_e[d] = re[j]; }
}

// per query: Kinds mask, participant validation, the table window TestStartedAt admits, its 64-entry chunks
__global__ __launch_bounds__(BLOCK) void k_rr_query(RrQueries Q, RrCmds c, int test_kinds, uint32_t started_at,
                                                    uint8_t *__restrict__ qmask, uint32_t *__restrict__ qa, uint32_t *__restrict__ qw,
                                                    uint64_t *__restrict__ qchunks, uint64_t *__restrict__ errs)
{
    const uint32_t q = blockIdx.x * BLOCK + threadIdx.x;
    if (q >= Q.nq) return;
    uint64_t e = 0;
    const uint64_t xm = Q.qm[q], xl = Q.ql[q];
    const int32_t xn = Q.qn[q];
    int mask = test_kinds;
    if (mask < 0) {
        mask = witnessed_by((uint32_t)(xl >> 1) & 7u);
        if (mask < 0) e |= ((xl >> 1) & 7u) == 5 ? RR_ERR_KIND_STATE : RR_ERR_KIND_ARG;
    }
    qmask[q] = (uint8_t)(mask < 0 ? 0 : mask);
    const uint32_t p0 = Q.poff[q], p1 = Q.poff[q + 1];
    if (p1 < p0 || Q.isr[q] > 1) e |= RR_ERR_PARTS;
    else if (Q.isr[q]) {
        for (uint32_t j = p0; j < p1; ++j)
            if (Q.ps[j] >= Q.pe[j] || (j > p0 && Q.pe[j - 1] > Q.ps[j])) { e |= RR_ERR_PARTS; break; }
    } else {
        for (uint32_t j = p0 + 1; j < p1; ++j)
            if (Q.ps[j - 1] >= Q.ps[j]) { e |= RR_ERR_PARTS; break; }
    }
    // lower = #entries with TxnId < X, upper = #entries with TxnId <= X
    uint32_t lo = 0, hi = c.n;
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (rc_ts_cmp(c.tm[m], c.tl[m], c.tn[m], xm, xl, xn) < 0) lo = m + 1; else hi = m; }
    const uint32_t lower = lo;
    hi = c.n;
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (rc_ts_cmp(c.tm[m], c.tl[m], c.tn[m], xm, xl, xn) <= 0) lo = m + 1; else hi = m; }
    const uint32_t upper = lo;
    uint32_t a = 0, w = c.n;
    if (started_at == 0) w = lower;                     // STARTED_BEFORE: txnId < X (:897-898)
    else if (started_at == 1) { a = upper; w = c.n - upper; }   // STARTED_AFTER: txnId > X (:894-896)
    qa[q] = a;
    qw[q] = w;
    qchunks[q] = (w + 63) / 64;
    if (e) atomicOr((unsigned long long *)errs, (unsigned long long)e);
}

// Deps.intersects(X, ranges of entry i): a KeyDeps entry of X whose key one of the ranges contains, or a RangeDeps entry
// of X whose range intersects one of them
__device__ bool rr_deps_intersect(const RrCmds &c, uint32_t i, uint64_t xm, uint64_t xl, int32_t xn)
{
    uint32_t lo = c.doff[i], hi = c.doff[i + 1];
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (rc_ts_cmp(c.dm[m], c.dl[m], c.dn[m], xm, xl, xn) < 0) lo = m + 1; else hi = m; }
    const uint32_t r0 = c.roff[i], r1 = c.roff[i + 1];
    const bool ei = c.end_incl != 0;
    for (uint32_t j = lo; j < c.doff[i + 1] && rc_ts_cmp(c.dm[j], c.dl[j], c.dn[j], xm, xl, xn) == 0; ++j) {
        const uint64_t s = c.ds[j];
        if (c.dk[j]) {
            uint32_t a = r0, b = r1;   // first range whose end reaches the key
            while (a < b) { const uint32_t m = (a + b) >> 1; if (ei ? c.re[m] < s : c.re[m] <= s) a = m + 1; else b = m; }
            if (a < r1 && rr_contains(c.rs[a], c.re[a], s, ei)) return true;
        } else {
            const uint64_t t = c.de[j];
            uint32_t a = r0, b = r1;   // first range ending after s
            while (a < b) { const uint32_t m = (a + b) >> 1; if (c.re[m] <= s) a = m + 1; else b = m; }
            if (a < r1 && c.rs[a] < t) return true;
        }
    }
    return false;
}

// does range (s, e) of a command intersect the query's participants (Routables.foldl over rangeCommand.ranges, sliced)
__device__ __forceinline__ bool rr_hits_query(const RrQueries &Q, uint32_t q, uint64_t s, uint64_t e, bool ei)
{
    uint32_t a = Q.poff[q], b = Q.poff[q + 1];
    const uint32_t end = b;
    if (Q.isr[q]) {
        while (a < b) { const uint32_t m = (a + b) >> 1; if (Q.pe[m] <= s) a = m + 1; else b = m; }
        return a < end && Q.ps[a] < e;   // Range.compareIntersecting == 0
    }
    while (a < b) { const uint32_t m = (a + b) >> 1; if (ei ? Q.ps[m] <= s : Q.ps[m] < s) a = m + 1; else b = m; }
    return a < end && rr_contains(s, e, Q.ps[a], ei);
}

// the per-command tests of mapReduceRangesInternal (:889-933) plus the optional executeAt > testTxnId map filter
__device__ bool rr_command_passes(const RrCmds &c, const RcParams &p, uint32_t i, uint32_t mask, uint64_t xm, uint64_t xl, int32_t xn)
{
    const uint32_t f = c.flags[i];
    const bool hist = (f & ACC_RCMD_HISTORICAL) != 0;
    if (!(((mask >> ((c.tl[i] >> 1) & 7u)) & 1u))) return false;   // testKind.test(txnId.kind())
    if (hist) {
        if (p.test_status != 0 || p.test_dep != 2) return false;      // historical: ANY_STATUS + ANY_DEPS only
        if (p.exec_after && rc_ts_cmp(c.tm[i], c.tl[i], c.tn[i], xm, xl, xn) <= 0) return false;   // executeAt = txnId
        return true;
    }
    if (f & ACC_RCMD_ERASED) return false;
    const int ex_cmp = rc_ts_cmp(c.em[i], c.el[i], c.en[i], xm, xl, xn);
    // STARTED_BEFORE falls through into ANY's test (:897-901)
    if (p.started_at != 1 && p.test_dep != 2 && ex_cmp < 0) return false;
    const uint32_t st = c.status[i];
    if (p.test_status == 1 && !(st == 3 || st == 4 || st == 5)) return false;   // IS_PROPOSED: Accepted, PreCommitted, Committed
    if (p.test_status == 2 && !(st >= 6 && st < 9)) return false;               // IS_STABLE: Stable <= s < Truncated
    if (p.test_dep != 2) {
        if (!(f & ACC_RCMD_HAS_DEPS)) return false;
        const bool has = rr_deps_intersect(c, i, xm, xl, xn);
        if ((p.test_dep == 0) == !has) return false;
    }
    if (p.exec_after && ex_cmp <= 0) return false;
    return true;
}

struct RrChunks {
    const uint64_t *chunk_off;   // [nq+1]
    const uint32_t *qa, *qw;
    const uint8_t *qmask;
    uint32_t nq;
    int rb, tb;                  // entry key = (q << (rb + tb)) | (range id << tb) | TxnId rank
};

template <bool EMIT>
__global__ __launch_bounds__(BLOCK) void k_rr_scan(uint64_t nchunks, RrCmds c, RrQueries Q, RcParams p, RrChunks ch,
                                                   uint32_t *__restrict__ chunk_cnt, const uint64_t *__restrict__ chunk_eoff,
                                                   uint64_t *__restrict__ ent)
{
    const uint64_t cw = (uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    if (cw >= nchunks) return;
    const uint32_t q = rc_upper64(ch.chunk_off, ch.nq + 1, cw) - 1;
    const uint32_t i = ch.qa[q] + (uint32_t)(cw - ch.chunk_off[q]) * 64u + lane_id();
    const uint64_t xm = Q.qm[q], xl = Q.ql[q];
    const int32_t xn = Q.qn[q];
    const bool ei = c.end_incl != 0;
    uint32_t cnt = 0;
    const bool live = i < ch.qa[q] + ch.qw[q] && rr_command_passes(c, p, i, ch.qmask[q], xm, xl, xn);
    if (live)
        for (uint32_t j = c.roff[i]; j < c.roff[i + 1]; ++j) cnt += rr_hits_query(Q, q, c.rs[j], c.re[j], ei) ? 1u : 0u;
    const uint32_t incl = wave_inclusive(cnt, OpAdd<uint32_t>());
    if constexpr (!EMIT) {
        if (lane_id() == 63) chunk_cnt[cw] = incl;
    } else {
        if (cnt) {
            uint64_t o = chunk_eoff[cw] + incl - cnt;
            const uint64_t qk = (uint64_t)q << (ch.rb + ch.tb), tr = c.trank[i];
            for (uint32_t j = c.roff[i]; j < c.roff[i + 1]; ++j)
                if (rr_hits_query(Q, q, c.rs[j], c.re[j], ei)) ent[o++] = qk | ((uint64_t)c.rid[j] << ch.tb) | tr;
        }
    }
}

__global__ __launch_bounds__(BLOCK) void k_rr_uniq(uint64_t E, const uint64_t *__restrict__ k, uint32_t *__restrict__ f)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < E) f[i] = (i == 0 || k[i] != k[i - 1]) ? 1u : 0u;
}

__global__ __launch_bounds__(BLOCK) void k_rr_compact(uint64_t E, const uint64_t *__restrict__ k, const uint32_t *__restrict__ f,
                                                      const uint32_t *__restrict__ incl, uint64_t *__restrict__ uk)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < E && f[i]) uk[incl[i] - 1] = k[i];
}

// per unique entry: a new (query, range) group?
__global__ __launch_bounds__(BLOCK) void k_rr_gflag(uint64_t U, const uint64_t *__restrict__ uk, int tb, uint32_t *__restrict__ g)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < U) g[i] = (i == 0 || (uk[i] >> tb) != (uk[i - 1] >> tb)) ? 1u : 0u;
}

// per query (and the end sentinel): first entry (lower bound of q in the sorted keys) and first group
__global__ __launch_bounds__(BLOCK) void k_rr_qoff(uint32_t nq, uint64_t U, const uint64_t *__restrict__ uk, int qshift,
                                                   const uint32_t *__restrict__ gexcl, uint64_t *__restrict__ eoff,
                                                   uint64_t *__restrict__ rd_off, uint64_t *__restrict__ arena_off)
{
    const uint32_t q = blockIdx.x * BLOCK + threadIdx.x;
    if (q > nq) return;
    uint64_t lo = 0, hi = U;
    while (lo < hi) { const uint64_t m = (lo + hi) >> 1; if ((uk[m] >> qshift) < q) lo = m + 1; else hi = m; }
    eoff[q] = lo;
    rd_off[q] = gexcl[lo];
    arena_off[q] = gexcl[lo] + lo;
}

// RangeDeps.Builder header: each (query, range) group's end offset; its range id
__global__ __launch_bounds__(BLOCK) void k_rr_header(uint64_t U, const uint64_t *__restrict__ uk, int rb, int tb,
                                                     const uint32_t *__restrict__ gflag, const uint32_t *__restrict__ gexcl,
                                                     const uint64_t *__restrict__ eoff, const uint64_t *__restrict__ rd_off,
                                                     const uint64_t *__restrict__ arena_off, int32_t *__restrict__ arena,
                                                     uint32_t *__restrict__ range_id)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= U) return;
    const uint64_t k = uk[i];
    const uint32_t q = (uint32_t)(k >> (rb + tb));
    const uint32_t g = gexcl[i] + gflag[i] - 1;
    if (gflag[i]) range_id[g] = (uint32_t)((k >> tb) & ((1ull << rb) - 1));
    if (i + 1 == U || gflag[i + 1]) {
        const uint64_t nr = rd_off[q + 1] - rd_off[q];
        arena[arena_off[q] + (g - rd_off[q])] = (int32_t)(nr + (i + 1 - eoff[q]));
    }
}

__global__ __launch_bounds__(BLOCK) void k_rr_tkey(uint64_t U, const uint64_t *__restrict__ uk, int rb, int tb, uint64_t *__restrict__ tk)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < U) tk[i] = ((uk[i] >> (rb + tb)) << tb) | (uk[i] & ((1ull << tb) - 1));
}

__global__ __launch_bounds__(BLOCK) void k_rr_uoff(uint32_t nq, uint64_t U, const uint64_t *__restrict__ tk, int tb,
                                                   const uint32_t *__restrict__ uexcl, uint64_t *__restrict__ u_off)
{
    const uint32_t q = blockIdx.x * BLOCK + threadIdx.x;
    if (q > nq) return;
    uint64_t lo = 0, hi = U;
    while (lo < hi) { const uint64_t m = (lo + hi) >> 1; if ((tk[m] >> tb) < q) lo = m + 1; else hi = m; }
    u_off[q] = uexcl[lo];
}

// every entry's index into its query's sorted unique TxnIds; the TxnIds as the first table index holding them
__global__ __launch_bounds__(BLOCK) void k_rr_body(uint64_t U, const uint64_t *__restrict__ tk, const uint32_t *__restrict__ src, int tb,
                                                   const uint32_t *__restrict__ uflag, const uint32_t *__restrict__ uexcl,
                                                   const uint64_t *__restrict__ eoff, const uint64_t *__restrict__ rd_off,
                                                   const uint64_t *__restrict__ arena_off, const uint64_t *__restrict__ u_off,
                                                   const uint32_t *__restrict__ first_of, int32_t *__restrict__ arena,
                                                   uint32_t *__restrict__ dep_txn)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= U) return;
    const uint64_t k = tk[i];
    const uint32_t q = (uint32_t)(k >> tb), tr = (uint32_t)(k & ((1ull << tb) - 1));
    const uint64_t uid = (uint64_t)uexcl[i] + uflag[i] - 1;
    const uint64_t nr = rd_off[q + 1] - rd_off[q];
    arena[arena_off[q] + nr + ((uint64_t)src[i] - eoff[q])] = (int32_t)(uid - u_off[q]);
    if (uflag[i]) dep_txn[uid] = first_of[tr];
}

static void check_rr_errors(uint64_t e)
{
    if (e & RR_ERR_KIND_STATE) fail(ACC_E_STATE, "Kind.witnessedBy(): unhandled kind LocalOnly (AssertionError)");
    if (e & RR_ERR_KIND_ARG) fail(ACC_E_ARG, "Kind.ofOrdinal: invalid kind ordinal in a testTxnId");
    if (e & RR_ERR_ORDER) fail(ACC_E_ARG, "the range-command table must be sorted by TxnId");
    if (e & RR_ERR_STATUS) fail(ACC_E_ARG, "invalid Status ordinal or ACC_RCMD_* flags");
    if (e & RR_ERR_OFF) fail(ACC_E_ARG, "rng_off / dep_off must be non-decreasing from 0 to their totals");
    if (e & RR_ERR_RANGES) fail(ACC_E_ARG, "a command's ranges must be sorted, non-overlapping, start < end");
    if (e & RR_ERR_DEPS) fail(ACC_E_ARG, "a command's deps must be sorted by TxnId, ranges with start < end");
    if (e & RR_ERR_PARTS) fail(ACC_E_ARG, "query participants: keys sorted unique, ranges sorted non-overlapping start < end");
}

void map_reduce_full_ranges(acc_ctx *ctx, const acc_range_cmds_in *ci, const acc_recovery_ranges_in *ri, acc_rangedeps_view *view)
{
    if (!ci || !ri || !view) fail(ACC_E_ARG, "null argument");
    for (uint32_t m : { ci->mem, ri->mem })
        if (m != ACC_MEM_HOST && m != ACC_MEM_DEVICE) fail(ACC_E_ARG, "mem must be ACC_MEM_HOST or ACC_MEM_DEVICE");
    if (ri->started_at > 2 || ri->test_dep > 2 || ri->test_status > 2)
        fail(ACC_E_ARG, "started_at / test_dep / test_status must be TestStartedAt / TestDep / TestStatus ordinals");
    if (ri->flags & ~ACC_FULL_EXECUTES_AFTER) fail(ACC_E_ARG, "unknown flags");
    if (ri->test_kinds > 0x3F) fail(ACC_E_ARG, "test_kinds must be a mask over the six Kind ordinals, or -1");
    if (ci->end_inclusive > 1) fail(ACC_E_ARG, "end_inclusive must be 0 or 1");
    hipStream_t st = ctx->stream;
    ctx->rd_valid = false;
    const uint32_t n = ci->n_cmd, nq = ri->n_query;
    const uint32_t cm = ci->mem, qmem = ri->mem;

    // ---- sizes: the offset totals
    const uint32_t *roff = stage_in(ctx, "rr_roff", ci->rng_off, (size_t)n + 1, cm);
    const uint32_t *doff = stage_in(ctx, "rr_doff", ci->dep_off, (size_t)n + 1, cm);
    const uint32_t *poff = stage_in(ctx, "rr_poff", ri->part_off, (size_t)nq + 1, qmem);
    uint32_t *tot = reinterpret_cast<uint32_t *>(ctx->pinned);
    ACC_HIP(hipMemcpyAsync(tot + 0, roff + n, 4, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(tot + 1, doff + n, 4, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(tot + 2, poff + nq, 4, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t R = tot[0], D = tot[1], NP = tot[2];

    RrCmds c{};
    c.tm = stage_in(ctx, "rr_tm", ci->txn_id.msb, n, cm);
    c.tl = stage_in(ctx, "rr_tl", ci->txn_id.lsb, n, cm);
    c.tn = stage_in(ctx, "rr_tn", ci->txn_id.node, n, cm);
    c.em = stage_in(ctx, "rr_em", ci->execute_at.msb, n, cm);
    c.el = stage_in(ctx, "rr_el", ci->execute_at.lsb, n, cm);
    c.en = stage_in(ctx, "rr_en", ci->execute_at.node, n, cm);
    c.status = stage_in(ctx, "rr_status", ci->status, n, cm);
    c.flags = stage_in(ctx, "rr_flags", ci->flags, n, cm);
    c.roff = roff;
    c.rs = stage_in(ctx, "rr_rs", ci->rng_start, R, cm);
    c.re = stage_in(ctx, "rr_re", ci->rng_end, R, cm);
    c.doff = doff;
    c.dm = stage_in(ctx, "rr_dm", ci->dep_txn.msb, D, cm);
    c.dl = stage_in(ctx, "rr_dl", ci->dep_txn.lsb, D, cm);
    c.dn = stage_in(ctx, "rr_dn", ci->dep_txn.node, D, cm);
    c.ds = stage_in(ctx, "rr_ds", ci->dep_start, D, cm);
    c.de = stage_in(ctx, "rr_de", ci->dep_end, D, cm);
    c.dk = stage_in(ctx, "rr_dk", ci->dep_is_key, D, cm);
    c.n = n;
    c.end_incl = ci->end_inclusive;
    c.R = R;
    c.D = D;
    RrQueries Q{};
    Q.qm = stage_in(ctx, "rr_qm", ri->test_txn.msb, nq, qmem);
    Q.ql = stage_in(ctx, "rr_ql", ri->test_txn.lsb, nq, qmem);
    Q.qn = stage_in(ctx, "rr_qn", ri->test_txn.node, nq, qmem);
    Q.isr = stage_in(ctx, "rr_isr", ri->part_is_range, nq, qmem);
    Q.poff = poff;
    Q.ps = stage_in(ctx, "rr_ps", ri->part_start, NP, qmem);
    Q.pe = stage_in(ctx, "rr_pe", ri->part_end, NP, qmem);
    Q.nq = nq;

    // ---- 1. table: validation, TxnId ranks, range dictionary
    uint64_t *errs = ctx->get<uint64_t>("rr_errs", 1);
    ACC_HIP(hipMemsetAsync(errs, 0, 8, st));
    uint32_t *tflag = ctx->get<uint32_t>("rr_tflag", n);
    uint32_t *tincl = ctx->get<uint32_t>("rr_tincl", n);
    uint32_t *trank = ctx->get<uint32_t>("rr_trank", n);
    uint32_t *first_of = ctx->get<uint32_t>("rr_first_of", n);
    if (n) {
        launch(ctx, "rr_check", k_rr_check, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, c, tflag, errs);
        scan<uint32_t, OpAdd<uint32_t>>(ctx, tflag, tincl, n, false);
        launch(ctx, "rr_first", k_rr_first, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint32_t *)tflag,
               (const uint32_t *)tincl, trank, first_of);
    }
    uint32_t *rid = ctx->get<uint32_t>("rr_rid", R);
    uint64_t *dict_s = ctx->get<uint64_t>("rr_dict_s", R);
    uint64_t *dict_e = ctx->get<uint64_t>("rr_dict_e", R);
    uint32_t *dincl = ctx->get<uint32_t>("rr_dincl", R);
    if (R) {
        Sorted by_end = radix_sort(ctx, "rr_rs1", c.re, nullptr, R, 64);
        uint64_t *sg = ctx->get<uint64_t>("rr_sg", R);
        launch(ctx, "rr_gather", k_rr_gather64, dim3(grid_for(R, BLOCK)), dim3(BLOCK), 0, R, (const uint32_t *)by_end.vals, c.rs, sg);
        Sorted by_start = radix_sort(ctx, "rr_rs2", sg, by_end.vals, R, 64);
        uint32_t *dflag = ctx->get<uint32_t>("rr_dflag", R);
        launch(ctx, "rr_dflag", k_rr_dflag, dim3(grid_for(R, BLOCK)), dim3(BLOCK), 0, R, (const uint64_t *)by_start.keys,
               (const uint32_t *)by_start.vals, c.re, dflag);
        scan<uint32_t, OpAdd<uint32_t>>(ctx, dflag, dincl, R, false);
        launch(ctx, "rr_dict", k_rr_dict, dim3(grid_for(R, BLOCK)), dim3(BLOCK), 0, R, (const uint64_t *)by_start.keys,
               (const uint32_t *)by_start.vals, c.re, (const uint32_t *)dflag, (const uint32_t *)dincl, rid, dict_s, dict_e);
    }
    c.trank = trank;
    c.rid = rid;

    // ---- 2. windows
    uint8_t *qmask = ctx->get<uint8_t>("rr_qmask", nq);
    uint32_t *qa = ctx->get<uint32_t>("rr_qa", nq);
    uint32_t *qw = ctx->get<uint32_t>("rr_qw", nq);
    uint64_t *qchunks = ctx->get<uint64_t>("rr_qchunks", nq);
    uint64_t *chunk_off = ctx->get<uint64_t>("rr_chunk_off", (size_t)nq + 1);
    if (nq) {
        launch(ctx, "rr_query", k_rr_query, dim3(grid_for(nq, BLOCK)), dim3(BLOCK), 0, Q, c, (int)ri->test_kinds,
               (uint32_t)ri->started_at, qmask, qa, qw, qchunks, errs);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, qchunks, chunk_off, nq, true, chunk_off + nq);
    } else {
        ACC_HIP(hipMemsetAsync(chunk_off, 0, 8, st));
    }
    ACC_HIP(hipMemcpyAsync(ctx->pinned, errs, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, chunk_off + nq, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 2, n ? (const void *)(tincl + n - 1) : (const void *)errs, 4, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(reinterpret_cast<uint32_t *>(ctx->pinned + 2) + 1, R ? (const void *)(dincl + R - 1) : (const void *)errs,
                           4, hipMemcpyDeviceToHost, st));
    ctx->sync();
    check_rr_errors(ctx->pinned[0]);
    const uint64_t NC = ctx->pinned[1];
    const uint32_t NT = n ? reinterpret_cast<uint32_t *>(ctx->pinned + 2)[0] : 0u;
    const uint32_t ND = R ? reinterpret_cast<uint32_t *>(ctx->pinned + 2)[1] : 0u;
    const int qb = bits_for(nq ? nq - 1 : 0), rb = std::max(1, bits_for(ND ? ND - 1 : 0)), tb = std::max(1, bits_for(NT ? NT - 1 : 0));
    const RcParams prm{ ri->started_at, ri->test_dep, ri->test_status, (uint32_t)(ri->flags & ACC_FULL_EXECUTES_AFTER) };
    if (NC && qb + rb + tb > 64) fail(ACC_E_CAP, "too many queries / ranges / TxnIds for the (query, range, TxnId) key");

    // ---- 3. count / emit
    RrChunks ch{ chunk_off, qa, qw, qmask, nq, rb, tb };
    uint32_t *chunk_cnt = ctx->get<uint32_t>("rr_chunk_cnt", NC);
    uint64_t *chunk_cnt64 = ctx->get<uint64_t>("rr_chunk_cnt64", NC);
    uint64_t *chunk_eoff = ctx->get<uint64_t>("rr_chunk_eoff", NC + 1);
    const unsigned gW = (unsigned)((NC + WAVES - 1) / WAVES);
    if (NC) {
        launch(ctx, "rr_count", k_rr_scan<false>, dim3(gW), dim3(BLOCK), 0, NC, c, Q, prm, ch, chunk_cnt,
               (const uint64_t *)nullptr, (uint64_t *)nullptr);
        launch(ctx, "rr_widen", k_rc_widen, dim3(grid_for(NC, BLOCK)), dim3(BLOCK), 0, NC, (const uint32_t *)chunk_cnt, chunk_cnt64);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, chunk_cnt64, chunk_eoff, NC, true, chunk_eoff + NC);
    } else {
        ACC_HIP(hipMemsetAsync(chunk_eoff, 0, 8, st));
    }
    ACC_HIP(hipMemcpyAsync(ctx->pinned, chunk_eoff + NC, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t E = ctx->pinned[0];
    if (E >= 0xFFFFFFFFull) fail(ACC_E_CAP, "more than 2^32-1 range recovery-scan entries in one call");
    uint64_t *ent = ctx->get<uint64_t>("rr_ent", E);
    if (E) launch(ctx, "rr_emit", k_rr_scan<true>, dim3(gW), dim3(BLOCK), 0, NC, c, Q, prm, ch, (uint32_t *)nullptr,
                  (const uint64_t *)chunk_eoff, ent);

    // ---- 4. TreeMap<Range, List> + Deps.Builder: sorted unique (query, range, TxnId)
    uint64_t U = 0;
    const uint64_t *uk = nullptr;
    if (E) {
        Sorted so = radix_sort(ctx, "rr_rs3", ent, nullptr, E, qb + rb + tb);
        uint32_t *f = ctx->get<uint32_t>("rr_ef", E);
        uint32_t *fi = ctx->get<uint32_t>("rr_efi", E);
        launch(ctx, "rr_uniq", k_rr_uniq, dim3(grid_for(E, BLOCK)), dim3(BLOCK), 0, E, (const uint64_t *)so.keys, f);
        scan<uint32_t, OpAdd<uint32_t>>(ctx, f, fi, E, false);
        ACC_HIP(hipMemcpyAsync(ctx->pinned, fi + E - 1, 4, hipMemcpyDeviceToHost, st));
        ctx->sync();
        U = reinterpret_cast<uint32_t *>(ctx->pinned)[0];
        uint64_t *ukw = ctx->get<uint64_t>("rr_uk", U);
        launch(ctx, "rr_compact", k_rr_compact, dim3(grid_for(E, BLOCK)), dim3(BLOCK), 0, E, (const uint64_t *)so.keys,
               (const uint32_t *)f, (const uint32_t *)fi, ukw);
        uk = ukw;
    }
    uint32_t *gflag = ctx->get<uint32_t>("rr_gflag", U);
    uint32_t *gexcl = ctx->get<uint32_t>("rr_gexcl", U + 1);
    uint64_t *eoff = ctx->get<uint64_t>("rr_eoff", (size_t)nq + 1);
    uint64_t *rd_off = ctx->get<uint64_t>("rr_rd_off", (size_t)nq + 1);
    uint64_t *arena_off = ctx->get<uint64_t>("rr_arena_off", (size_t)nq + 1);
    uint64_t *u_off = ctx->get<uint64_t>("rr_u_off", (size_t)nq + 1);
    if (U) {
        launch(ctx, "rr_gflag", k_rr_gflag, dim3(grid_for(U, BLOCK)), dim3(BLOCK), 0, U, uk, tb, gflag);
        scan<uint32_t, OpAdd<uint32_t>>(ctx, gflag, gexcl, U, true, gexcl + U);
    } else {
        ACC_HIP(hipMemsetAsync(gexcl, 0, 4, st));
    }
    launch(ctx, "rr_qoff", k_rr_qoff, dim3(grid_for((size_t)nq + 1, BLOCK)), dim3(BLOCK), 0, nq, U, uk, rb + tb,
           (const uint32_t *)gexcl, eoff, rd_off, arena_off);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, gexcl + U, 4, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t G = reinterpret_cast<uint32_t *>(ctx->pinned)[0];
    int32_t *arena = ctx->get<int32_t>("rr_arena", G + U);
    uint32_t *range_id = ctx->get<uint32_t>("rr_range_id", G);
    uint32_t *dep_txn = ctx->get<uint32_t>("rr_dep_txn", U);
    uint64_t TU = 0;
    if (U) {
        launch(ctx, "rr_header", k_rr_header, dim3(grid_for(U, BLOCK)), dim3(BLOCK), 0, U, uk, rb, tb, (const uint32_t *)gflag,
               (const uint32_t *)gexcl, (const uint64_t *)eoff, (const uint64_t *)rd_off, (const uint64_t *)arena_off, arena, range_id);
        uint64_t *tk = ctx->get<uint64_t>("rr_tk", U);
        launch(ctx, "rr_tkey", k_rr_tkey, dim3(grid_for(U, BLOCK)), dim3(BLOCK), 0, U, uk, rb, tb, tk);
        Sorted s2 = radix_sort(ctx, "rr_rs4", tk, nullptr, U, qb + tb);
        uint32_t *uf = ctx->get<uint32_t>("rr_uf", U);
        uint32_t *ux = ctx->get<uint32_t>("rr_ux", U + 1);
        launch(ctx, "rr_uniq", k_rr_uniq, dim3(grid_for(U, BLOCK)), dim3(BLOCK), 0, U, (const uint64_t *)s2.keys, uf);
        scan<uint32_t, OpAdd<uint32_t>>(ctx, uf, ux, U, true, ux + U);
        launch(ctx, "rr_uoff", k_rr_uoff, dim3(grid_for((size_t)nq + 1, BLOCK)), dim3(BLOCK), 0, nq, U, (const uint64_t *)s2.keys, tb,
               (const uint32_t *)ux, u_off);
        launch(ctx, "rr_body", k_rr_body, dim3(grid_for(U, BLOCK)), dim3(BLOCK), 0, U, (const uint64_t *)s2.keys,
               (const uint32_t *)s2.vals, tb, (const uint32_t *)uf, (const uint32_t *)ux, (const uint64_t *)eoff,
               (const uint64_t *)rd_off, (const uint64_t *)arena_off, (const uint64_t *)u_off, (const uint32_t *)first_of, arena,
               dep_txn);
        ACC_HIP(hipMemcpyAsync(ctx->pinned, ux + U, 4, hipMemcpyDeviceToHost, st));
        ctx->sync();
        TU = reinterpret_cast<uint32_t *>(ctx->pinned)[0];
    } else {
        ACC_HIP(hipMemsetAsync(u_off, 0, ((size_t)nq + 1) * 8, st));
    }
    ctx->stat("recovery.range_chunks", NC);
    ctx->stat("recovery.range_entries", U);
    *view = acc_rangedeps_view{ nq, ND, G + U, G, TU, U, dict_s, dict_e, arena_off, arena, rd_off, range_id, u_off, dep_txn };
    ctx->rd_view = *view;
    ctx->rd_valid = true;
}

}  // namespace acc
