// conflicts.hip — MaxConflicts and the PreAccept executeAt proposal (local/MaxConflicts.java:31-96,
// local/CommandStore.java:280-290, 320-345).
//
// A CommandStore's MaxConflicts is a ReducingRangeMap<Timestamp>: sorted boundaries with one value per interval,
// updated by MaxConflicts.merge(map, create(keysOrRanges, executeAt)) (ReducingIntervalMap.merge with Timestamp::max)
// and read by MaxConflicts.get(keys) = foldl(keys, Timestamp::max, NONE) over the intervals the query touches. A key k
// enters as k.asRange() (ReducingRangeMap.create(Keys), utils/ReducingRangeMap.java:379-406), which holds exactly k.
//
// Device form (acc_maxconflicts, persistent across calls): disjoint closed intervals [st_i, en_i] over the u64 key
// codes, ascending, each with its Timestamp (intervals without a value are not stored, adjacent equal values are
// coalesced as the builder does); a range (s, e] (EndInclusive) is [s + 1, e], [s, e) (StartInclusive) is [s, e - 1],
// a key k is [k, k]. Per 256 intervals one block maximum for long range queries.
//   update (a batch of commands; Timestamp::max is associative and commutative, so the batch merges at once):
//     1. every update part and every stored interval as a closed interval with a value;
//     2. their cut points (a, b + 1) sorted unique = elementary slots; the values ranked (Timestamp.compareTo);
//     3. range chmax of the value ranks over the slots through a segment tree (atomicMax on the O(log) canonical nodes
//        of each interval), each slot's value = the max on its root path;
//     4. runs of equal non-empty slots compacted into the new interval list, block maxima rebuilt.
//   get (a batch of PreAccept queries): a wave per query, a lane per part: two binary searches give the intervals the
//     part intersects, their max through the block maxima; the wave folds the lanes' maxima under Timestamp.compareTo
//     and sets the fast-path bit txnId.compareTo(minNonConflicting) >= 0 (CommandStore.preaccept :320-345).
// acc_max_conflicts (every update and every query of a store in one call) is create + update + get.
#include "dict.hpp"

#include <algorithm>

struct acc_maxconflicts {
    int device = 0;
    uint32_t end_inclusive = 1;
    uint64_t nv = 0, cap = 0;                         // intervals, allocated capacity
    uint64_t *st = nullptr, *en = nullptr;            // [cap] closed interval bounds
    uint64_t *vm = nullptr, *vl = nullptr;            // [cap] values (msb, lsb)
    int32_t *vn = nullptr;                            // [cap] values (node)
    uint64_t *bm = nullptr, *bl = nullptr;            // [cap / MC_BLK + 1] block maxima
    int32_t *bn = nullptr;
};

namespace acc {
namespace mc {

constexpr uint64_t IDENTITY_LSB = 0xFFFFFFFFFFFF001EULL;
constexpr uint32_t MC_BLK = 256;
constexpr uint64_t MAXC = ~0ull;
enum : uint64_t { E_OFF = 1, E_SORT = 2, E_RANGE = 4 };

struct Ts {
    uint64_t m, l;
    int32_t n;
};
__device__ __forceinline__ int cmp(const Ts &a, const Ts &b)
{
    if (a.m != b.m) return a.m < b.m ? -1 : 1;
    const uint64_t a1 = a.l & IDENTITY_LSB, b1 = b.l & IDENTITY_LSB;
    if (a1 != b1) return a1 < b1 ? -1 : 1;
    if (a.n != b.n) return a.n < b.n ? -1 : 1;
    return 0;
}
__device__ __forceinline__ Ts tmax(const Ts &a, const Ts &b) { return cmp(a, b) >= 0 ? a : b; }   // Timestamp.max

struct Upd {
    const uint64_t *xm, *xl;
    const int32_t *xn;
    const uint32_t *key_off, *rng_off;
    const uint64_t *key, *rs, *re;
    uint32_t n;
    uint64_t K, R;
    int ei;
};

// validation (offsets from 0 to the totals, keys sorted unique, ranges sorted non-overlapping with start < end); the
// host reads the flags before any kernel indexes through the offsets
__global__ __launch_bounds__(BLOCK) void k_mc_check(Upd u, uint64_t *__restrict__ err)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= u.n) return;
    uint64_t e = 0;
    const uint32_t a = u.key_off[i], b = u.key_off[i + 1], c = u.rng_off[i], d = u.rng_off[i + 1];
    if (b < a || b > u.K || (i == 0 && a != 0) || (i + 1 == u.n && b != u.K)) e |= E_OFF;
    else
        for (uint32_t j = a + 1; j < b; ++j)
            if (u.key[j - 1] >= u.key[j]) e |= E_SORT;
    if (d < c || d > u.R || (i == 0 && c != 0) || (i + 1 == u.n && d != u.R)) e |= E_OFF;
    else
        for (uint32_t j = c; j < d; ++j)
            if (u.rs[j] >= u.re[j] || (j > c && u.re[j - 1] > u.rs[j])) e |= E_RANGE;
    if (e) atomicOr((unsigned long long *)err, (unsigned long long)e);
}

// closed interval of a range of the store's bound type
__device__ __forceinline__ void range_closed(uint64_t s, uint64_t e, int ei, uint64_t &a, uint64_t &b)
{
    if (ei) { a = s + 1; b = e; } else { a = s; b = e - 1; }
}

// the values to rank: the updates' executeAts, then the stored intervals' values (3 words: msb, lsb, node as an
// order-preserving u64)
__global__ __launch_bounds__(BLOCK) void k_mc_values(Upd u, uint64_t nv, const uint64_t *__restrict__ vm,
                                                     const uint64_t *__restrict__ vl, const int32_t *__restrict__ vn,
                                                     uint64_t *__restrict__ w0, uint64_t *__restrict__ w1, uint64_t *__restrict__ w2)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= u.n + nv) return;
    uint64_t m, l;
    int32_t nd;
    // the stored values first, then the updates in batch order: the lowest index of a rank is the instance the
    // reference's sequential merge keeps (Timestamp.max returns its first argument on compareTo == 0, and
    // MaxConflicts.merge(existing, update) passes the existing value first; MaxConflicts.java:77-79)
    if (i < nv) { m = vm[i]; l = vl[i]; nd = vn[i]; }
    else { m = u.xm[i - nv]; l = u.xl[i - nv]; nd = u.xn[i - nv]; }
    w0[i] = m; w1[i] = l; w2[i] = (uint64_t)((uint32_t)nd ^ 0x80000000u);
}

// per part (update keys, update ranges, stored intervals): its closed interval and value index, and both cut points
struct Parts {
    uint64_t *a, *b, *cut;   // [Q], [Q], [2Q] (MAXC + 1 cuts become MAXC: the end of the code space)
    uint32_t *val;           // [Q] value index into the ranked values
};
__global__ __launch_bounds__(BLOCK) void k_mc_parts(Upd u, const uint32_t *__restrict__ kown, const uint32_t *__restrict__ rown,
                                                    uint64_t nv, const uint64_t *__restrict__ st, const uint64_t *__restrict__ en,
                                                    Parts p)
{
    const uint64_t q = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    const uint64_t Q = u.K + u.R + nv;
    if (q >= Q) return;
    uint64_t a, b;
    uint32_t v;
    if (q < u.K) { a = b = u.key[q]; v = (uint32_t)nv + kown[q]; }
    else if (q < u.K + u.R) { range_closed(u.rs[q - u.K], u.re[q - u.K], u.ei, a, b); v = (uint32_t)nv + rown[q - u.K]; }
    else { a = st[q - u.K - u.R]; b = en[q - u.K - u.R]; v = (uint32_t)(q - u.K - u.R); }
    p.a[q] = a; p.b[q] = b; p.val[q] = v;
    p.cut[2 * q] = a;
    p.cut[2 * q + 1] = b == MAXC ? MAXC : b + 1;
}

// owner update of every key / range (from the validated offsets)
__global__ __launch_bounds__(BLOCK) void k_mc_owners(Upd u, uint32_t *__restrict__ kown, uint32_t *__restrict__ rown)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= u.n) return;
    for (uint32_t j = u.key_off[i]; j < u.key_off[i + 1]; ++j) kown[j] = i;
    for (uint32_t j = u.rng_off[i]; j < u.rng_off[i + 1]; ++j) rown[j] = i;
}

__device__ __forceinline__ uint32_t lower_u64(const uint64_t *a, uint32_t n, uint64_t v)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (a[m] < v) lo = m + 1; else hi = m; }
    return lo;
}

// distinct cut points (dense ranks of the sorted cuts) -> slot starts
__global__ __launch_bounds__(BLOCK) void k_mc_slots(uint64_t nc, const uint64_t *__restrict__ cut, const uint32_t *__restrict__ crank,
                                                    uint64_t *__restrict__ slot)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < nc) slot[crank[i]] = cut[i];
}

// range chmax over the part's slots [i0, i1]: atomicMax on the canonical segment-tree nodes of
// (value rank + 1) << 32 | ~value index -- the largest value, and among values equal under compareTo the lowest index:
// the stored instance, then the earliest update of the batch, which is the instance the reference's sequential
// MaxConflicts.merge(existing, update) keeps (Timestamp.max returns its first argument on a tie, Timestamp.java:265-268)
__global__ __launch_bounds__(BLOCK) void k_mc_chmax(uint64_t Q, Parts p, const uint32_t *__restrict__ vrank,
                                                    const uint64_t *__restrict__ slot, uint32_t m, uint32_t M,
                                                    unsigned long long *__restrict__ tree)
{
    const uint64_t q = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (q >= Q) return;
    const uint64_t a = p.a[q], b = p.b[q];
    const uint32_t i0 = lower_u64(slot, m, a);
    const uint32_t i1 = b == MAXC ? m - 1 : lower_u64(slot, m, b + 1) - 1;
    const unsigned long long v = ((unsigned long long)(vrank[p.val[q]] + 1) << 32) | (0xFFFFFFFFu - p.val[q]);
    uint32_t l = i0 + M, r = i1 + M + 1;   // half-open [l, r) over the leaves
    while (l < r) {
        if (l & 1) atomicMax(&tree[l++], v);
        if (r & 1) atomicMax(&tree[--r], v);
        l >>= 1; r >>= 1;
    }
}

// each slot's value (max on its root path) and the run boundaries of equal non-empty values
__global__ __launch_bounds__(BLOCK) void k_mc_leaves(uint32_t m, uint32_t M, const unsigned long long *__restrict__ tree,
                                                     uint64_t *__restrict__ sval)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= m) return;
    unsigned long long v = 0;
    for (uint32_t nd = i + M; nd >= 1; nd >>= 1) v = max(v, tree[nd]);
    sval[i] = v;
}
// runs of slots whose values are equal (Timestamp.equals: the same rank) coalesce into one interval holding the run's
// first instance, as the builder skips an appended value equal to the last one
__global__ __launch_bounds__(BLOCK) void k_mc_runflag(uint32_t m, const uint64_t *__restrict__ sval, uint32_t *__restrict__ f)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < m) f[i] = sval[i] != 0 && (i == 0 || (sval[i - 1] >> 32) != (sval[i] >> 32));
}

// the new interval list: a run's first slot writes its start and value, its last slot its end
__global__ __launch_bounds__(BLOCK) void k_mc_emit(uint32_t m, const uint64_t *__restrict__ slot, const uint64_t *__restrict__ sval,
                                                   const uint32_t *__restrict__ f, const uint32_t *__restrict__ fincl,
                                                   const uint64_t *__restrict__ w0,
                                                   const uint64_t *__restrict__ w1, const uint64_t *__restrict__ w2,
                                                   uint64_t *__restrict__ st, uint64_t *__restrict__ en, uint64_t *__restrict__ vm,
                                                   uint64_t *__restrict__ vl, int32_t *__restrict__ vn)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= m || sval[i] == 0) return;
    const uint32_t k = fincl[i] - 1;
    if (f[i]) {
        const uint32_t src = 0xFFFFFFFFu - (uint32_t)sval[i];   // the slot's instance
        st[k] = slot[i];
        vm[k] = w0[src]; vl[k] = w1[src]; vn[k] = (int32_t)((uint32_t)w2[src] ^ 0x80000000u);
    }
    if (i + 1 == m || (sval[i + 1] >> 32) != (sval[i] >> 32)) en[k] = i + 1 == m ? MAXC : slot[i + 1] - 1;
}

__global__ __launch_bounds__(BLOCK) void k_mc_blockmax(uint64_t nv, const uint64_t *__restrict__ vm, const uint64_t *__restrict__ vl,
                                                       const int32_t *__restrict__ vn, uint64_t *__restrict__ bm,
                                                       uint64_t *__restrict__ bl, int32_t *__restrict__ bn)
{
    const uint64_t b = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    const uint64_t a0 = b * MC_BLK;
    if (a0 >= nv) return;
    Ts best{ vm[a0], vl[a0], vn[a0] };
    for (uint64_t i = a0 + 1; i < min(nv, a0 + MC_BLK); ++i) best = tmax(best, Ts{ vm[i], vl[i], vn[i] });
    bm[b] = best.m; bl[b] = best.l; bn[b] = best.n;
}

struct Map {
    const uint64_t *st, *en, *vm, *vl, *bm, *bl;
    const int32_t *vn, *bn;
    uint64_t nv;
    int ei;
};
struct Qs {
    const uint64_t *qm, *ql, *ps, *pe;
    const int32_t *qn;
    const uint8_t *isr;
    const uint32_t *poff;
    uint32_t nq;
    uint64_t np;
    uint64_t *om, *ol;
    int32_t *on;
    uint8_t *fast;
};

__device__ __forceinline__ uint64_t lower64(const uint64_t *a, uint64_t n, uint64_t v)   // first index with a[i] >= v
{
    uint64_t lo = 0, hi = n;
    while (lo < hi) { const uint64_t m = (lo + hi) >> 1; if (a[m] < v) lo = m + 1; else hi = m; }
    return lo;
}

// one wave per query, a lane per part: the intervals [i0, i1] the part's closed interval [a, b] intersects (first with
// en >= a, last with st <= b), their max through the block maxima
__global__ __launch_bounds__(BLOCK) void k_mc_query(Qs q, Map mp, uint64_t *__restrict__ err)
{
    const uint32_t qi = blockIdx.x * WAVES + (threadIdx.x >> 6), lane = lane_id();
    if (qi >= q.nq) return;
    bool have = false;
    Ts best{ 0, 0, 0 };
    auto take = [&](const Ts &t) { best = have ? tmax(best, t) : t; have = true; };
    uint32_t p0 = q.poff[qi], p1 = q.poff[qi + 1];
    const bool isr = q.isr[qi] != 0;
    uint64_t e = 0;
    if (p1 < p0 || p1 > q.np || (qi == 0 && p0 != 0) || (qi + 1 == q.nq && p1 != q.np) || q.isr[qi] > 1) {
        e |= E_OFF;
        p1 = p0;   // never index through bad offsets
    }
    // each lane takes a contiguous chunk of the parts, so folding the lanes in order visits the intervals in key order
    // and a tie keeps the first maximum visited, as foldl with Timestamp::max does (MaxConflicts.get)
    const uint32_t per = (p1 - p0 + 63) / 64, pa = min(p1, p0 + lane * per), pb = min(p1, pa + per);
    for (uint32_t p = pa; p < pb; ++p) {
        const uint64_t s = q.ps[p], t = isr ? q.pe[p] : s;
        if (isr && s >= t) { e |= E_RANGE; continue; }
        if (p > p0 && (isr ? q.pe[p - 1] > s : q.ps[p - 1] >= s)) e |= E_SORT;
        uint64_t a, b;
        if (isr) range_closed(s, t, mp.ei, a, b);
        else a = b = s;
        const uint64_t i0 = lower64(mp.en, mp.nv, a);
        const uint64_t i1e = b == MAXC ? mp.nv : lower64(mp.st, mp.nv, b + 1);   // intervals with st <= b: [0, i1e)
        if (i0 >= i1e) continue;
        const uint64_t bl0 = (i0 + MC_BLK - 1) / MC_BLK, bl1 = i1e / MC_BLK;
        if (bl0 < bl1) {
            for (uint64_t i = i0; i < bl0 * MC_BLK; ++i) take(Ts{ mp.vm[i], mp.vl[i], mp.vn[i] });
            for (uint64_t bb = bl0; bb < bl1; ++bb) take(Ts{ mp.bm[bb], mp.bl[bb], mp.bn[bb] });
            for (uint64_t i = bl1 * MC_BLK; i < i1e; ++i) take(Ts{ mp.vm[i], mp.vl[i], mp.vn[i] });
        } else {
            for (uint64_t i = i0; i < i1e; ++i) take(Ts{ mp.vm[i], mp.vl[i], mp.vn[i] });
        }
    }
    // wave max under Timestamp.compareTo: lanes park their maxima in LDS, lane 0 folds them in lane order
    __shared__ Ts red[WAVES][64];
    __shared__ uint32_t red_have[WAVES][64];
    const uint32_t w = threadIdx.x >> 6;
    red[w][lane] = best;
    red_have[w][lane] = have ? 1u : 0u;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (lane == 0) {
        for (uint32_t l = 1; l < 64; ++l) {
            if (!red_have[w][l]) continue;
            const Ts o = red[w][l];
            best = have ? tmax(best, o) : o;
            have = true;
        }
        if (!have) best = Ts{ 0, 0, 0 };   // Timestamp.NONE
        q.om[qi] = best.m; q.ol[qi] = best.l; q.on[qi] = best.n;
        q.fast[qi] = cmp(Ts{ q.qm[qi], q.ql[qi], q.qn[qi] }, best) >= 0 ? 1 : 0;   // txnId.compareTo(minNonConflicting) >= 0
    }
    if (e) atomicOr((unsigned long long *)err, (unsigned long long)e);
}

template <class T>
static void grow(T *&p, uint64_t count)
{
    if (p) ACC_HIP(hipFree(p));
    p = nullptr;
    ACC_HIP(hipMalloc(&p, std::max<uint64_t>(count, 1) * sizeof(T)));
}

}  // namespace mc

acc_maxconflicts *mc_new(int device, uint32_t end_inclusive)
{
    if (end_inclusive > 1) fail(ACC_E_ARG, "end_inclusive must be 0 or 1");
    auto *m = new acc_maxconflicts();
    m->device = device;
    m->end_inclusive = end_inclusive;
    return m;
}

void mc_free(acc_maxconflicts *m)
{
    if (!m) return;
    for (void *p : { (void *)m->st, (void *)m->en, (void *)m->vm, (void *)m->vl, (void *)m->vn, (void *)m->bm, (void *)m->bl,
                     (void *)m->bn })
        if (p) (void)hipFree(p);
    delete m;
}

uint64_t mc_size(const acc_maxconflicts *m) { return m ? m->nv : 0; }

// MaxConflicts.update of every command of the batch (CommandStore.updateMaxConflicts, local/CommandStore.java:280-290)
void mc_update(acc_ctx *ctx, acc_maxconflicts *M, const acc_conflicts_in *ui)
{
    using namespace mc;
    if (!ui || !M) fail(ACC_E_ARG, "null argument");
    if (ui->mem != ACC_MEM_HOST && ui->mem != ACC_MEM_DEVICE) fail(ACC_E_ARG, "mem must be ACC_MEM_HOST or ACC_MEM_DEVICE");
    if (ui->end_inclusive != M->end_inclusive) fail(ACC_E_ARG, "updates' Range bound type differs from the map's");
    if (ui->n_keys >= 0xFFFFFFFFull || ui->n_ranges >= 0xFFFFFFFFull) fail(ACC_E_CAP, "more than 2^32-1 keys / ranges");
    hipStream_t st = ctx->stream;
    const uint32_t n = ui->n_upd;
    const uint64_t K = ui->n_keys, R = ui->n_ranges;
    if (n == 0) {
        if (K || R) fail(ACC_E_ARG, "keys / ranges without updates");
        return;
    }
    Upd u{};
    u.xm = stage_in(ctx, "mc_xm", ui->execute_at.msb, n, ui->mem);
    u.xl = stage_in(ctx, "mc_xl", ui->execute_at.lsb, n, ui->mem);
    u.xn = stage_in(ctx, "mc_xn", ui->execute_at.node, n, ui->mem);
    u.key_off = stage_in(ctx, "mc_koff", ui->key_off, (size_t)n + 1, ui->mem);
    u.rng_off = stage_in(ctx, "mc_roff", ui->rng_off, (size_t)n + 1, ui->mem);
    u.key = stage_in(ctx, "mc_key", ui->key, K, ui->mem);
    u.rs = stage_in(ctx, "mc_rs", ui->rng_start, R, ui->mem);
    u.re = stage_in(ctx, "mc_re", ui->rng_end, R, ui->mem);
    u.n = n; u.K = K; u.R = R; u.ei = (int)ui->end_inclusive;
    uint64_t *errs = ctx->get<uint64_t>("mc_errs", 1);
    ACC_HIP(hipMemsetAsync(errs, 0, 8, st));
    launch(ctx, "mc_check", k_mc_check, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, u, errs);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, errs, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();   // nothing below indexes through unvalidated offsets
    const uint64_t e0 = ctx->pinned[0];
    if (e0 & E_OFF) fail(ACC_E_ARG, "key_off / rng_off must be non-decreasing from 0 to their totals");
    if (e0 & E_SORT) fail(ACC_E_ARG, "keys of an update must be sorted unique");
    if (e0 & E_RANGE) fail(ACC_E_ARG, "ranges of an update must be sorted, non-overlapping, start < end");
    if (K + R == 0) return;
    // 1. values (updates' executeAts, stored values) ranked under Timestamp.compareTo
    const uint64_t nv = M->nv, V = n + nv;
    uint64_t *w0 = ctx->get<uint64_t>("mc_w0", V), *w1 = ctx->get<uint64_t>("mc_w1", V), *w2 = ctx->get<uint64_t>("mc_w2", V);
    launch(ctx, "mc_values", k_mc_values, dim3(grid_for(V, BLOCK)), dim3(BLOCK), 0, u, nv, (const uint64_t *)M->vm,
           (const uint64_t *)M->vl, (const int32_t *)M->vn, w0, w1, w2);
    const uint64_t *vw[3] = { w0, w1, w2 };
    const uint64_t vand[3] = { ~0ull, IDENTITY_LSB, ~0ull };
    DenseRank vr = dense_rank(ctx, "mc_vdict", V, 3, vw, vand, nullptr, true);
    // 2. parts and cut points
    uint32_t *kown = ctx->get<uint32_t>("mc_kown", K), *rown = ctx->get<uint32_t>("mc_rown", R);
    launch(ctx, "mc_owners", k_mc_owners, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, u, kown, rown);
    const uint64_t Q = K + R + nv;
    Parts pt;
    pt.a = ctx->get<uint64_t>("mc_pa", Q); pt.b = ctx->get<uint64_t>("mc_pb", Q);
    pt.cut = ctx->get<uint64_t>("mc_cut", 2 * Q); pt.val = ctx->get<uint32_t>("mc_pv", Q);
    launch(ctx, "mc_parts", k_mc_parts, dim3(grid_for(Q, BLOCK)), dim3(BLOCK), 0, u, (const uint32_t *)kown,
           (const uint32_t *)rown, nv, (const uint64_t *)M->st, (const uint64_t *)M->en, pt);
    const uint64_t *cw[1] = { pt.cut };
    DenseRank cr = dense_rank(ctx, "mc_cdict", 2 * Q, 1, cw, nullptr, nullptr, false);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, cr.count_dev, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t m64 = ctx->pinned[0];
    if (m64 >= 0x7FFFFFFFull) fail(ACC_E_CAP, "MaxConflicts too large (>= 2^31 boundaries)");
    const uint32_t m = (uint32_t)m64;
    uint64_t *slot = ctx->get<uint64_t>("mc_slot", m);
    launch(ctx, "mc_slots", k_mc_slots, dim3(grid_for(2 * Q, BLOCK)), dim3(BLOCK), 0, 2 * Q, (const uint64_t *)pt.cut,
           (const uint32_t *)cr.rank, slot);
    // 3. range chmax through a segment tree over the slots
    uint32_t Mp = 1;
    while (Mp < m) Mp <<= 1;
    unsigned long long *tree = ctx->get<unsigned long long>("mc_tree64", 2 * (size_t)Mp);
    ACC_HIP(hipMemsetAsync(tree, 0, 2 * (size_t)Mp * 8, st));
    launch(ctx, "mc_chmax", k_mc_chmax, dim3(grid_for(Q, BLOCK)), dim3(BLOCK), 0, Q, pt, (const uint32_t *)vr.rank,
           (const uint64_t *)slot, m, Mp, tree);
    uint64_t *sval = ctx->get<uint64_t>("mc_sval64", m);
    uint32_t *f = ctx->get<uint32_t>("mc_f", m), *fi = ctx->get<uint32_t>("mc_fi", m);
    launch(ctx, "mc_leaves", k_mc_leaves, dim3(grid_for(m, BLOCK)), dim3(BLOCK), 0, m, Mp, (const unsigned long long *)tree, sval);
    launch(ctx, "mc_runflag", k_mc_runflag, dim3(grid_for(m, BLOCK)), dim3(BLOCK), 0, m, (const uint64_t *)sval, f);
    uint32_t *nnew = ctx->get<uint32_t>("mc_nnew", 1);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, f, fi, m, false, nnew);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, nnew, 4, hipMemcpyDeviceToHost, st));
    ctx->sync();
    uint32_t nn;
    memcpy(&nn, ctx->pinned, 4);
    // 4. the new interval list (fresh buffers: the old ones are read by this batch's kernels)
    acc_maxconflicts nm = *M;
    nm.st = nm.en = nm.vm = nm.vl = nm.bm = nm.bl = nullptr;
    nm.vn = nm.bn = nullptr;
    const uint64_t cap = std::max<uint64_t>(nn, 1);
    auto free_new = [&]() {
        for (void *p : { (void *)nm.st, (void *)nm.en, (void *)nm.vm, (void *)nm.vl, (void *)nm.vn, (void *)nm.bm, (void *)nm.bl,
                         (void *)nm.bn })
            if (p) (void)hipFree(p);
    };
    try {
        grow(nm.st, cap); grow(nm.en, cap); grow(nm.vm, cap); grow(nm.vl, cap); grow(nm.vn, cap);
        const uint64_t nb = (cap + MC_BLK - 1) / MC_BLK;
        grow(nm.bm, nb); grow(nm.bl, nb); grow(nm.bn, nb);
    } catch (...) {
        free_new();
        throw;
    }
    launch(ctx, "mc_emit", k_mc_emit, dim3(grid_for(m, BLOCK)), dim3(BLOCK), 0, m, (const uint64_t *)slot, (const uint64_t *)sval,
           (const uint32_t *)f, (const uint32_t *)fi, (const uint64_t *)w0, (const uint64_t *)w1,
           (const uint64_t *)w2, nm.st, nm.en, nm.vm, nm.vl, nm.vn);
    nm.nv = nn;
    nm.cap = cap;
    if (nn) launch(ctx, "mc_blockmax", k_mc_blockmax, dim3(grid_for((nn + MC_BLK - 1) / MC_BLK, BLOCK)), dim3(BLOCK), 0, (uint64_t)nn,
                   (const uint64_t *)nm.vm, (const uint64_t *)nm.vl, (const int32_t *)nm.vn, nm.bm, nm.bl, nm.bn);
    ctx->sync();
    for (void *p : { (void *)M->st, (void *)M->en, (void *)M->vm, (void *)M->vl, (void *)M->vn, (void *)M->bm, (void *)M->bl,
                     (void *)M->bn })
        if (p) ACC_HIP(hipFree(p));
    *M = nm;
    ctx->stat("conflicts.intervals", nn);
    ctx->stat("conflicts.slots", m);
}

// MaxConflicts.get per PreAccept query and the fast-path test (CommandStore.preaccept, local/CommandStore.java:320-345)
void mc_get(acc_ctx *ctx, const acc_maxconflicts *M, const acc_preaccept_in *qi, acc_preaccept_out *out)
{
    using namespace mc;
    if (!qi || !out || !M) fail(ACC_E_ARG, "null argument");
    for (uint32_t mm : { qi->mem, out->mem })
        if (mm != ACC_MEM_HOST && mm != ACC_MEM_DEVICE) fail(ACC_E_ARG, "mem must be ACC_MEM_HOST or ACC_MEM_DEVICE");
    hipStream_t st = ctx->stream;
    const uint32_t nq = qi->n_query;
    const uint64_t NP = qi->n_parts;
    if (nq == 0) return;
    Qs q{};
    q.qm = stage_in(ctx, "mc_qm", qi->txn_id.msb, nq, qi->mem);
    q.ql = stage_in(ctx, "mc_ql", qi->txn_id.lsb, nq, qi->mem);
    q.qn = stage_in(ctx, "mc_qn", qi->txn_id.node, nq, qi->mem);
    q.isr = stage_in(ctx, "mc_qisr", qi->is_range, nq, qi->mem);
    q.poff = stage_in(ctx, "mc_qoff", qi->part_off, (size_t)nq + 1, qi->mem);
    q.ps = stage_in(ctx, "mc_qps", qi->part_start, NP, qi->mem);
    q.pe = stage_in(ctx, "mc_qpe", qi->part_end, NP, qi->mem);
    q.nq = nq;
    q.np = NP;
    const bool host_out = out->mem == ACC_MEM_HOST;
    q.om = host_out ? ctx->get<uint64_t>("mc_om", nq) : out->max_msb;
    q.ol = host_out ? ctx->get<uint64_t>("mc_ol", nq) : out->max_lsb;
    q.on = host_out ? ctx->get<int32_t>("mc_on", nq) : out->max_node;
    q.fast = host_out ? ctx->get<uint8_t>("mc_fast", nq) : out->fast_path;
    Map mp{ M->st, M->en, M->vm, M->vl, M->bm, M->bl, M->vn, M->bn, M->nv, (int)M->end_inclusive };
    uint64_t *errs = ctx->get<uint64_t>("mc_errs", 1);
    ACC_HIP(hipMemsetAsync(errs, 0, 8, st));
    launch(ctx, "mc_query", k_mc_query, dim3((nq + WAVES - 1) / WAVES), dim3(BLOCK), 0, q, mp, errs);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, errs, 8, hipMemcpyDeviceToHost, st));
    if (host_out) {
        ACC_HIP(hipMemcpyAsync(out->max_msb, q.om, (size_t)nq * 8, hipMemcpyDeviceToHost, st));
        ACC_HIP(hipMemcpyAsync(out->max_lsb, q.ol, (size_t)nq * 8, hipMemcpyDeviceToHost, st));
        ACC_HIP(hipMemcpyAsync(out->max_node, q.on, (size_t)nq * 4, hipMemcpyDeviceToHost, st));
        ACC_HIP(hipMemcpyAsync(out->fast_path, q.fast, nq, hipMemcpyDeviceToHost, st));
    }
    ctx->sync();
    const uint64_t e1 = ctx->pinned[0];
    if (e1 & E_OFF) fail(ACC_E_ARG, "query part_off must be non-decreasing from 0 to n_parts; is_range 0 or 1");
    if (e1 & E_SORT) fail(ACC_E_ARG, "query keys / ranges must be sorted (unique / non-overlapping)");
    if (e1 & E_RANGE) fail(ACC_E_ARG, "query ranges must have start < end");
}

// every update and every query of a store in one call: a transient map
void max_conflicts(acc_ctx *ctx, const acc_conflicts_in *ui, const acc_preaccept_in *qi, acc_preaccept_out *out)
{
    if (!ui || !qi || !out) fail(ACC_E_ARG, "null argument");
    if (ui->end_inclusive > 1) fail(ACC_E_ARG, "end_inclusive must be 0 or 1");
    acc_maxconflicts *m = mc_new(ctx->device, ui->end_inclusive);
    try {
        mc_update(ctx, m, ui);
        mc_get(ctx, m, qi, out);
    } catch (...) {
        mc_free(m);
        throw;
    }
    ctx->stat("conflicts.distinct_keys", m->nv);
    mc_free(m);
}

}  // namespace acc
