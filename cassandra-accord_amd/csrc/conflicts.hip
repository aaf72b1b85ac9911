// conflicts.hip — MaxConflicts and the PreAccept executeAt proposal (local/MaxConflicts.java:31-96,
// local/CommandStore.java:280-290, 320-345).
//
// A CommandStore's MaxConflicts is the pointwise max of every (keysOrRanges, executeAt) it was updated with
// (updateMaxConflicts: MaxConflicts.merge(map, create(keysOrRanges, executeAt)), a ReducingRangeMap folded with
// Timestamp::max), so MaxConflicts.get(keys) is the max executeAt of the updates whose keys / ranges intersect the
// query's. Batched on device:
//   1. the updates' keys radix sorted (values = update index), one max per distinct key (a lane per key run), and one
//      max per 256 distinct keys for range queries;
//   2. one wave per query: a key part takes its key's max (binary search); a range part the maxima of the distinct
//      keys it holds (block maxima for whole blocks); every part is tested against the updates' ranges (lanes stride
//      over them); a wave max reduction under Timestamp.compareTo; then the fast-path test txnId >= the max.
#include "dict.hpp"

namespace acc {
namespace mc {

constexpr uint64_t IDENTITY_LSB = 0xFFFFFFFFFFFF001EULL;
constexpr uint32_t MC_BLK = 256;
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

__global__ __launch_bounds__(BLOCK) void k_mc_check(Upd u, uint32_t *__restrict__ kown, uint64_t *__restrict__ err)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= u.n) return;
    uint64_t e = 0;
    const uint32_t a = u.key_off[i], b = u.key_off[i + 1], c = u.rng_off[i], d = u.rng_off[i + 1];
    if (b < a || b > u.K || (i == 0 && a != 0) || (i + 1 == u.n && b != u.K)) e |= E_OFF;
    else
        for (uint32_t j = a; j < b; ++j) {
            kown[j] = i;
            if (j > a && u.key[j - 1] >= u.key[j]) e |= E_SORT;
        }
    if (d < c || d > u.R || (i == 0 && c != 0) || (i + 1 == u.n && d != u.R)) e |= E_OFF;
    else
        for (uint32_t j = c; j < d; ++j)
            if (u.rs[j] >= u.re[j] || (j > c && u.re[j - 1] > u.rs[j])) e |= E_RANGE;
    if (e) atomicOr((unsigned long long *)err, (unsigned long long)e);
}

__global__ __launch_bounds__(BLOCK) void k_mc_flag(uint64_t K, const uint64_t *__restrict__ sk, uint32_t *__restrict__ f)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < K) f[i] = (i == 0 || sk[i] != sk[i - 1]) ? 1u : 0u;
}

// one lane per distinct key: the max executeAt over its run of sorted pairs
__global__ __launch_bounds__(BLOCK) void k_mc_keymax(uint64_t K, const uint64_t *__restrict__ sk, const uint32_t *__restrict__ sv,
                                                     const uint32_t *__restrict__ f, const uint32_t *__restrict__ fi,
                                                     const uint32_t *__restrict__ kown, Upd u, uint64_t *__restrict__ dk,
                                                     uint64_t *__restrict__ dm, uint64_t *__restrict__ dl, int32_t *__restrict__ dn)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= K || !f[i]) return;
    const uint32_t d = fi[i] - 1;
    uint32_t o = kown[sv[i]];
    Ts best{ u.xm[o], u.xl[o], u.xn[o] };
    for (uint64_t q = i + 1; q < K && !f[q]; ++q) {
        o = kown[sv[q]];
        best = tmax(best, Ts{ u.xm[o], u.xl[o], u.xn[o] });
    }
    dk[d] = sk[i];
    dm[d] = best.m; dl[d] = best.l; dn[d] = best.n;
}

__global__ __launch_bounds__(BLOCK) void k_mc_blockmax(uint32_t nd, const uint64_t *__restrict__ dm, const uint64_t *__restrict__ dl,
                                                       const int32_t *__restrict__ dn, uint64_t *__restrict__ bm,
                                                       uint64_t *__restrict__ bl, int32_t *__restrict__ bn)
{
    const uint32_t b = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t a0 = b * MC_BLK;
    if (a0 >= nd) return;
    Ts best{ dm[a0], dl[a0], dn[a0] };
    for (uint32_t i = a0 + 1; i < min(nd, a0 + MC_BLK); ++i) best = tmax(best, Ts{ dm[i], dl[i], dn[i] });
    bm[b] = best.m; bl[b] = best.l; bn[b] = best.n;
}

struct Keys {
    const uint64_t *dk, *dm, *dl, *bm, *bl;
    const int32_t *dn, *bn;
    uint32_t nd;
};
struct Qs {
    const uint64_t *qm, *ql, *ps, *pe;
    const int32_t *qn;
    const uint8_t *isr;
    const uint32_t *poff;
    uint32_t nq;
    uint64_t *om, *ol;
    int32_t *on;
    uint8_t *fast;
};

__device__ __forceinline__ uint32_t lower_u64(const uint64_t *a, uint32_t n, uint64_t v)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (a[m] < v) lo = m + 1; else hi = m; }
    return lo;
}

// one wave per query
__global__ __launch_bounds__(BLOCK) void k_mc_query(Qs q, Keys k, Upd u, uint64_t *__restrict__ err)
{
    const uint32_t qi = blockIdx.x * WAVES + (threadIdx.x >> 6), lane = lane_id();
    if (qi >= q.nq) return;
    bool have = false;
    Ts best{ 0, 0, 0 };
    auto take = [&](const Ts &t) { best = have ? tmax(best, t) : t; have = true; };
    const uint32_t p0 = q.poff[qi], p1 = q.poff[qi + 1];
    const bool isr = q.isr[qi] != 0;
    const bool ei = u.ei != 0;
    uint64_t e = 0;
    if (p1 < p0 || q.isr[qi] > 1) e |= E_OFF;
    for (uint32_t p = p0; p < p1 && !e; ++p) {
        const uint64_t a = q.ps[p], b = isr ? q.pe[p] : q.ps[p];
        if (isr && a >= b) { e |= E_RANGE; break; }
        if (p > p0 && (isr ? q.pe[p - 1] > a : q.ps[p - 1] >= a)) { e |= E_SORT; break; }
        // distinct update keys this part holds: a key part the one equal key; a range part the keys it contains
        uint32_t lo, hi;
        if (!isr) {
            lo = lower_u64(k.dk, k.nd, a);
            hi = (lo < k.nd && k.dk[lo] == a) ? lo + 1 : lo;
        } else if (ei) {   // (a, b]
            lo = lower_u64(k.dk, k.nd, a + 1);
            hi = lower_u64(k.dk, k.nd, b + 1 > b ? b + 1 : b);
            if (b == ~0ull) hi = k.nd;
        } else {           // [a, b)
            lo = lower_u64(k.dk, k.nd, a);
            hi = lower_u64(k.dk, k.nd, b);
        }
        // partial blocks element-wise, whole blocks through their maxima
        const uint32_t bl0 = (lo + MC_BLK - 1) / MC_BLK, bl1 = hi / MC_BLK;
        if (bl0 < bl1) {
            for (uint32_t i = lo + lane; i < bl0 * MC_BLK; i += 64) take(Ts{ k.dm[i], k.dl[i], k.dn[i] });
            for (uint32_t bb = bl0 + lane; bb < bl1; bb += 64) take(Ts{ k.bm[bb], k.bl[bb], k.bn[bb] });
            for (uint32_t i = bl1 * MC_BLK + lane; i < hi; i += 64) take(Ts{ k.dm[i], k.dl[i], k.dn[i] });
        } else {
            for (uint32_t i = lo + lane; i < hi; i += 64) take(Ts{ k.dm[i], k.dl[i], k.dn[i] });
        }
        // the updates' ranges: a key part contained (Range.contains), a range part intersecting
        for (uint32_t r = lane; r < (uint32_t)u.R; r += 64) {
            const uint64_t s = u.rs[r], t = u.re[r];
            bool hit;
            if (isr) hit = s < b && t > a;
            else hit = ei ? (s < a && a <= t) : (s <= a && a < t);
            if (hit) {
                // the update owning range r: its executeAt
                uint32_t lo2 = 0, hi2 = u.n;   // last update with rng_off <= r
                while (hi2 - lo2 > 1) { const uint32_t m = (lo2 + hi2) >> 1; if (u.rng_off[m] <= r) lo2 = m; else hi2 = m; }
                take(Ts{ u.xm[lo2], u.xl[lo2], u.xn[lo2] });
            }
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
    }
    if (lane == 0) {
        if (!have) best = Ts{ 0, 0, 0 };   // Timestamp.NONE
        q.om[qi] = best.m; q.ol[qi] = best.l; q.on[qi] = best.n;
        q.fast[qi] = cmp(Ts{ q.qm[qi], q.ql[qi], q.qn[qi] }, best) >= 0 ? 1 : 0;   // txnId.compareTo(minNonConflicting) >= 0
    }
    if (e && lane == 0) atomicOr((unsigned long long *)err, (unsigned long long)e);
}

}  // namespace mc

void max_conflicts(acc_ctx *ctx, const acc_conflicts_in *ui, const acc_preaccept_in *qi, acc_preaccept_out *out)
{
    using namespace mc;
    if (!ui || !qi || !out) fail(ACC_E_ARG, "null argument");
    for (uint32_t m : { ui->mem, qi->mem, out->mem })
        if (m != ACC_MEM_HOST && m != ACC_MEM_DEVICE) fail(ACC_E_ARG, "mem must be ACC_MEM_HOST or ACC_MEM_DEVICE");
    if (ui->end_inclusive > 1) fail(ACC_E_ARG, "end_inclusive must be 0 or 1");
    if (ui->n_keys >= 0xFFFFFFFFull || ui->n_ranges >= 0xFFFFFFFFull) fail(ACC_E_CAP, "more than 2^32-1 keys / ranges");
    hipStream_t st = ctx->stream;
    const uint32_t n = ui->n_upd, nq = qi->n_query;
    const uint64_t K = ui->n_keys, R = ui->n_ranges, NP = qi->n_parts;
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
    if (n == 0 && (K || R)) fail(ACC_E_ARG, "keys / ranges without updates");
    uint64_t *errs = ctx->get<uint64_t>("mc_errs", 1);
    ACC_HIP(hipMemsetAsync(errs, 0, 8, st));
    uint32_t *kown = ctx->get<uint32_t>("mc_kown", K);
    if (n) launch(ctx, "mc_check", k_mc_check, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, u, kown, errs);
    // distinct keys and their maxima
    uint32_t nd = 0;
    uint64_t *dk = ctx->get<uint64_t>("mc_dk", K), *dm = ctx->get<uint64_t>("mc_dm", K), *dl = ctx->get<uint64_t>("mc_dl", K);
    int32_t *dn = ctx->get<int32_t>("mc_dn", K);
    if (K) {
        Sorted so = radix_sort(ctx, "mc_rs", u.key, nullptr, K, 64);
        uint32_t *f = ctx->get<uint32_t>("mc_f", K), *fi = ctx->get<uint32_t>("mc_fi", K);
        launch(ctx, "mc_flag", k_mc_flag, dim3(grid_for(K, BLOCK)), dim3(BLOCK), 0, K, (const uint64_t *)so.keys, f);
        scan<uint32_t, OpAdd<uint32_t>>(ctx, f, fi, K, false);
        launch(ctx, "mc_keymax", k_mc_keymax, dim3(grid_for(K, BLOCK)), dim3(BLOCK), 0, K, (const uint64_t *)so.keys,
               (const uint32_t *)so.vals, (const uint32_t *)f, (const uint32_t *)fi, (const uint32_t *)kown, u, dk, dm, dl, dn);
        ACC_HIP(hipMemcpyAsync(ctx->pinned, fi + K - 1, 4, hipMemcpyDeviceToHost, st));
    }
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, errs, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    if (K) nd = reinterpret_cast<uint32_t *>(ctx->pinned)[0];
    const uint64_t e0 = ctx->pinned[1];
    if (e0 & E_OFF) fail(ACC_E_ARG, "key_off / rng_off must be non-decreasing from 0 to their totals");
    if (e0 & E_SORT) fail(ACC_E_ARG, "keys of an update must be sorted unique");
    if (e0 & E_RANGE) fail(ACC_E_ARG, "ranges of an update must be sorted, non-overlapping, start < end");
    const uint32_t nb = (nd + MC_BLK - 1) / MC_BLK;
    uint64_t *bm = ctx->get<uint64_t>("mc_bm", nb), *bl = ctx->get<uint64_t>("mc_bl", nb);
    int32_t *bn = ctx->get<int32_t>("mc_bn", nb);
    if (nb) launch(ctx, "mc_blockmax", k_mc_blockmax, dim3(grid_for(nb, BLOCK)), dim3(BLOCK), 0, nd, (const uint64_t *)dm,
                   (const uint64_t *)dl, (const int32_t *)dn, bm, bl, bn);
    Keys kk{ dk, dm, dl, bm, bl, dn, bn, nd };
    Qs q{};
    q.qm = stage_in(ctx, "mc_qm", qi->txn_id.msb, nq, qi->mem);
    q.ql = stage_in(ctx, "mc_ql", qi->txn_id.lsb, nq, qi->mem);
    q.qn = stage_in(ctx, "mc_qn", qi->txn_id.node, nq, qi->mem);
    q.isr = stage_in(ctx, "mc_qisr", qi->is_range, nq, qi->mem);
    q.poff = stage_in(ctx, "mc_qoff", qi->part_off, (size_t)nq + 1, qi->mem);
    q.ps = stage_in(ctx, "mc_qps", qi->part_start, NP, qi->mem);
    q.pe = stage_in(ctx, "mc_qpe", qi->part_end, NP, qi->mem);
    q.nq = nq;
    const bool host_out = out->mem == ACC_MEM_HOST;
    q.om = host_out ? ctx->get<uint64_t>("mc_om", nq) : out->max_msb;
    q.ol = host_out ? ctx->get<uint64_t>("mc_ol", nq) : out->max_lsb;
    q.on = host_out ? ctx->get<int32_t>("mc_on", nq) : out->max_node;
    q.fast = host_out ? ctx->get<uint8_t>("mc_fast", nq) : out->fast_path;
    ACC_HIP(hipMemsetAsync(errs, 0, 8, st));
    if (nq) launch(ctx, "mc_query", k_mc_query, dim3((nq + WAVES - 1) / WAVES), dim3(BLOCK), 0, q, kk, u, errs);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, errs, 8, hipMemcpyDeviceToHost, st));
    if (host_out && nq) {
        ACC_HIP(hipMemcpyAsync(out->max_msb, q.om, (size_t)nq * 8, hipMemcpyDeviceToHost, st));
        ACC_HIP(hipMemcpyAsync(out->max_lsb, q.ol, (size_t)nq * 8, hipMemcpyDeviceToHost, st));
        ACC_HIP(hipMemcpyAsync(out->max_node, q.on, (size_t)nq * 4, hipMemcpyDeviceToHost, st));
        ACC_HIP(hipMemcpyAsync(out->fast_path, q.fast, nq, hipMemcpyDeviceToHost, st));
    }
    ctx->sync();
    const uint64_t e1 = ctx->pinned[0];
    if (e1 & E_OFF) fail(ACC_E_ARG, "query part_off must be non-decreasing; is_range 0 or 1");
    if (e1 & E_SORT) fail(ACC_E_ARG, "query keys / ranges must be sorted (unique / non-overlapping)");
    if (e1 & E_RANGE) fail(ACC_E_ARG, "query ranges must have start < end");
    ctx->stat("conflicts.distinct_keys", nd);
}

}  // namespace acc
