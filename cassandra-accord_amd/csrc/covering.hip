// covering.hip — PartialDeps.covering (primitives/PartialDeps.java:31-58, 80-86).
//
// A store computes every txn's PartialDeps with covering = the store's Ranges (PreAccept.calculatePartialDeps: new
// PartialDeps.Builder(ranges), messages/PreAccept.java:245-265), and the constructor asserts
// covering.containsAll(keyDeps.keys) and rangeDeps.isCoveredBy(covering) (PartialDeps.java:52-58,
// IllegalStateException). PreAccept.reduce folds the replies of the stores a txn touches with PartialDeps.with, whose
// covering is that.covering.with(this.covering) (PartialDeps.java:80-86).
//
// On the device: a workgroup lane per txn (group) checks its keys / ranges against its covering (a few ranges: the
// binary searches stay in cache). The covering of a reduced txn is the fold over the stores that replied for it; a
// node has few stores, so the distinct store sets are few: their coverings are folded on the host with the restated
// Ranges.with (ranges.hpp) and each txn carries the index of its set's covering.
#include "prims.hpp"
#include "ranges.hpp"

#include <map>
#include <vector>

namespace acc {

namespace cov {

// AbstractRanges.indexOf(key) >= 0 over [lo, hi) of the covering (Range.compareTo(key), Range.java:48-55 / 98-105)
__device__ __forceinline__ bool contains_key(const uint64_t *cs, const uint64_t *ce, uint64_t lo, uint64_t hi, uint64_t k, int ei)
{
    while (lo < hi) {
        const uint64_t m = (lo + hi) >> 1;
        const int c = ei ? (k <= cs[m] ? 1 : k > ce[m] ? -1 : 0) : (k < cs[m] ? 1 : k >= ce[m] ? -1 : 0);   // -r.compareTo(k)
        if (c == 0) return true;
        if (c > 0) hi = m; else lo = m + 1;   // key before the range: search left
    }
    return false;
}

// RangeDeps.isCoveredBy's test for one entry range [s, e) of the covering [lo, hi) (RangeDeps.java:595-613): the loop
// accepts an entry whose start lies inside some covering range; an entry starting in the gap before covering range j
// (after range j - 1) must intersect range j; an entry starting after the last range fails
__device__ __forceinline__ bool covered(const uint64_t *cs, const uint64_t *ce, uint64_t lo, uint64_t hi, uint64_t s, uint64_t e)
{
    uint64_t a = lo, b = hi;   // j = first covering range with start > s
    while (a < b) { const uint64_t m = (a + b) >> 1; if (cs[m] <= s) a = m + 1; else b = m; }
    const uint64_t j = a;
    if (j > lo && s < ce[j - 1]) return true;
    if (j == hi) return false;
    return !(cs[j] >= e || ce[j] <= s);   // Range.compareIntersecting == 0
}

// keys: group g's keys key_code[key_off[g] .. key_off[g+1]); ranges: group g's ranges [rng_off[g], rng_off[g+1]) as
// (rs, re) or, with rid, dictionary ids into (rs, re). cov_id (null: covering 0) selects the group's covering.
struct Groups {
    uint32_t n;
    const uint64_t *key_off, *key_code;
    const uint64_t *rng_off, *rs, *re;
    const uint32_t *rid;
    const uint32_t *cov_id;
};
struct Table {
    const uint64_t *off, *cs, *ce;
    int ei;
};

__global__ __launch_bounds__(BLOCK) void k_cov_check(Groups g, Table t, uint64_t *__restrict__ err)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= g.n) return;
    const uint32_t c = g.cov_id ? g.cov_id[i] : 0u;
    const uint64_t lo = t.off[c], hi = t.off[c + 1];
    uint64_t e = 0;
    if (g.key_off)
        for (uint64_t k = g.key_off[i]; k < g.key_off[i + 1]; ++k)
            if (!contains_key(t.cs, t.ce, lo, hi, g.key_code[k], t.ei)) { e |= 1; break; }
    if (g.rng_off)
        for (uint64_t r = g.rng_off[i]; r < g.rng_off[i + 1]; ++r) {
            const uint64_t x = g.rid ? g.rid[r] : r;
            if (!covered(t.cs, t.ce, lo, hi, g.rs[x], g.re[x])) { e |= 2; break; }
        }
    if (e) atomicOr((unsigned long long *)err, (unsigned long long)e);
}

// participation: every received (global txn index) from source s sets bit s of its home group's store mask
__global__ __launch_bounds__(BLOCK) void k_cov_mask(uint64_t n, const uint32_t *__restrict__ gidx, const uint64_t *__restrict__ src_off,
                                                    uint32_t world, uint32_t nsrc, unsigned long long *__restrict__ mask)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    uint32_t s = 0;
    while (s + 1 < nsrc && src_off[s + 1] <= i) ++s;
    atomicOr(&mask[gidx[i] / world], 1ull << s);
}

// the store's txns by home rank (global index mod world): counts, then a scatter with a cursor per destination
__global__ __launch_bounds__(BLOCK) void k_cov_dest_count(uint32_t n, const uint32_t *__restrict__ gidx, uint32_t world,
                                                          uint32_t *__restrict__ cnt)
{
    __shared__ uint32_t h[64];
    if (threadIdx.x < 64) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) atomicAdd(&h[gidx[i] % world], 1u);
    __syncthreads();
    if (threadIdx.x < world && h[threadIdx.x]) atomicAdd(&cnt[threadIdx.x], h[threadIdx.x]);
}
__global__ __launch_bounds__(BLOCK) void k_cov_dest_scatter(uint32_t n, const uint32_t *__restrict__ gidx, uint32_t world,
                                                            uint32_t *__restrict__ cursor, uint32_t *__restrict__ out)
{
    __shared__ uint32_t h[64], base[64];
    if (threadIdx.x < 64) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    uint32_t d = 0, r = 0;
    if (i < n) { d = gidx[i] % world; r = atomicAdd(&h[d], 1u); }
    __syncthreads();
    if (threadIdx.x < world && h[threadIdx.x]) base[threadIdx.x] = atomicAdd(&cursor[threadIdx.x], h[threadIdx.x]);
    __syncthreads();
    if (i < n) out[base[d] + r] = gidx[i];
}

}  // namespace cov

// The store covering of the last acc_partial_deps_batch on ctx: every txn's KeyDeps keys and RangeDeps ranges
// against it (ACC_E_STATE on a violation, as the PartialDeps constructor throws).
void partial_deps_covering(acc_ctx *ctx, const acc_rlist *covering, uint32_t end_inclusive)
{
    using namespace cov;
    if (!covering) fail(ACC_E_ARG, "null covering");
    if (!ctx->kd_valid || !ctx->rd_valid) fail(ACC_E_STATE, "no acc_partial_deps_batch result on this context");
    const rg::V c = rg::check_sorted_deoverlapped(rg::load(covering));
    hipStream_t st = ctx->stream;
    const acc_keydeps_view &kv = ctx->kd_view;
    const acc_rangedeps_view &rv = ctx->rd_view;
    if (kv.n_txn != rv.n_txn) fail(ACC_E_STATE, "internal: PartialDeps halves of different batches");
    const size_t nc = c.size();
    std::vector<uint64_t> h(2 + 2 * nc);
    h[0] = 0; h[1] = nc;
    for (size_t i = 0; i < nc; ++i) { h[2 + i] = c[i].s; h[2 + nc + i] = c[i].e; }
    uint64_t *d = ctx->get<uint64_t>("cov_table1", h.size());
    ACC_HIP(hipMemcpyAsync(d, h.data(), h.size() * 8, hipMemcpyHostToDevice, st));
    uint64_t *err = ctx->get<uint64_t>("cov_err", 1);
    ACC_HIP(hipMemsetAsync(err, 0, 8, st));
    Groups g{ kv.n_txn, kv.kd_key ? kv.kd_off : nullptr, kv.kd_key, rv.rd_off, rv.rng_start, rv.rng_end, rv.range_id, nullptr };
    const Table t{ d, d + 2, d + 2 + nc, (int)end_inclusive };
    if (g.n) launch(ctx, "cov_check", k_cov_check, dim3(grid_for(g.n, BLOCK)), dim3(BLOCK), 0, g, t, err);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, err, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    if (ctx->pinned[0] & 1) fail(ACC_E_STATE, "PartialDeps: covering does not contain every KeyDeps key (PartialDeps.java:56)");
    if (ctx->pinned[0] & 2) fail(ACC_E_STATE, "PartialDeps: RangeDeps not covered by covering (PartialDeps.java:57)");
}

// Reduce side. send: the store's txns by home rank (u32 global indices) and the store covering (one copy per
// destination), as exchange streams qp (participation) and qc (covering ranges as (start, end) u64 pairs).
void covering_pack(acc_ctx *ctx, const acc_rlist *covering, const uint32_t *txn_global_dev, uint32_t n_store, uint32_t world,
                   void *send[2], std::vector<uint64_t> off[2])
{
    using namespace cov;
    if (world > 64) fail(ACC_E_CAP, "PartialDeps.covering over more than 64 stores");
    const rg::V c = rg::check_sorted_deoverlapped(rg::load(covering));
    hipStream_t st = ctx->stream;
    uint32_t *cnt = ctx->get<uint32_t>("cov_cnt", 2 * 64);
    ACC_HIP(hipMemsetAsync(cnt, 0, 2 * 64 * 4, st));
    uint32_t *part = ctx->get<uint32_t>("cov_part", std::max<uint32_t>(n_store, 1));
    if (n_store) launch(ctx, "cov_dest_count", k_cov_dest_count, dim3(grid_for(n_store, BLOCK)), dim3(BLOCK), 0, n_store,
                        txn_global_dev, world, cnt);
    std::vector<uint32_t> hc(64);
    ACC_HIP(hipMemcpyAsync(hc.data(), cnt, 64 * 4, hipMemcpyDeviceToHost, st));
    ctx->sync();
    off[0].assign(world + 1, 0);
    for (uint32_t d = 0; d < world; ++d) off[0][d + 1] = off[0][d] + hc[d];
    std::vector<uint32_t> cur(64, 0);
    for (uint32_t d = 0; d < world; ++d) cur[d] = (uint32_t)off[0][d];
    ACC_HIP(hipMemcpyAsync(cnt + 64, cur.data(), 64 * 4, hipMemcpyHostToDevice, st));
    if (n_store) launch(ctx, "cov_dest_scatter", k_cov_dest_scatter, dim3(grid_for(n_store, BLOCK)), dim3(BLOCK), 0, n_store,
                        txn_global_dev, world, cnt + 64, part);
    send[0] = part;
    // the covering, one copy per destination: (start, end) pairs
    const size_t nc = c.size();
    std::vector<uint64_t> hs(2 * nc * world);
    for (uint32_t d = 0; d < world; ++d)
        for (size_t i = 0; i < nc; ++i) { hs[2 * (nc * d + i)] = c[i].s; hs[2 * (nc * d + i) + 1] = c[i].e; }
    uint64_t *cs = ctx->get<uint64_t>("cov_send", std::max<size_t>(hs.size(), 1));
    if (!hs.empty()) ACC_HIP(hipMemcpyAsync(cs, hs.data(), hs.size() * 8, hipMemcpyHostToDevice, st));
    send[1] = cs;
    off[1].assign(world + 1, 0);
    for (uint32_t d = 0; d < world; ++d) off[1][d + 1] = off[1][d] + nc;
    ctx->sync();   // cur and hs are pageable host vectors: their copies complete before they go out of scope
}

// Home side: the store mask of every home txn, the distinct masks' coverings folded on the host in store order
// (acc = next.with(acc): PreAccept.reduce's ok1.deps.with(ok2.deps) gives that.covering.with(this.covering)), the
// table and each txn's covering index on the device; then the invariants of the reduced PartialDeps.
void covering_merge(acc_ctx *ctx, uint32_t world, uint32_t rank, uint32_t n_global, uint32_t end_inclusive,
                    const std::vector<uint64_t> &n_part, const void *recv_part, const std::vector<uint64_t> &n_cov,
                    const void *recv_cov, const acc_merge_view *kv, const acc_deps_merge_view *rv, acc_covering_view *out)
{
    using namespace cov;
    hipStream_t st = ctx->stream;
    const uint32_t ng = n_global > rank ? (n_global - rank + world - 1) / world : 0;
    // checked before any copy from a host vector is queued (a throw would free them under a pending copy)
    if (kv->n_groups != ng || rv->n_groups != ng) fail(ACC_E_STATE, "internal: reduced halves of different home sets");
    // the stores' coverings (a few ranges each)
    uint64_t ncov_all = 0;
    for (uint32_t s = 0; s < world; ++s) ncov_all += n_cov[s];
    std::vector<uint64_t> hcv(2 * ncov_all);
    if (ncov_all) ACC_HIP(hipMemcpyAsync(hcv.data(), recv_cov, hcv.size() * 8, hipMemcpyDeviceToHost, st));
    // store masks
    uint64_t npart = 0;
    std::vector<uint64_t> poff(world + 1, 0);
    for (uint32_t s = 0; s < world; ++s) { poff[s + 1] = poff[s] + n_part[s]; }
    npart = poff[world];
    unsigned long long *mask = ctx->get<unsigned long long>("cov_mask", std::max<uint32_t>(ng, 1));
    ACC_HIP(hipMemsetAsync(mask, 0, (size_t)std::max<uint32_t>(ng, 1) * 8, st));
    uint64_t *dpoff = ctx->get<uint64_t>("cov_poff", world + 1);
    ACC_HIP(hipMemcpyAsync(dpoff, poff.data(), (world + 1) * 8, hipMemcpyHostToDevice, st));
    if (npart) launch(ctx, "cov_mask", k_cov_mask, dim3((unsigned)((npart + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, npart,
                      static_cast<const uint32_t *>(recv_part), (const uint64_t *)dpoff, world, world, mask);
    std::vector<uint64_t> hm(ng);
    if (ng) ACC_HIP(hipMemcpyAsync(hm.data(), mask, (size_t)ng * 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    std::vector<rg::V> sc(world);
    {
        uint64_t x = 0;
        for (uint32_t s = 0; s < world; ++s)
            for (uint64_t i = 0; i < n_cov[s]; ++i, ++x) sc[s].push_back({ hcv[2 * x], hcv[2 * x + 1] });
    }
    std::map<uint64_t, uint32_t> ids;
    for (uint32_t i = 0; i < ng; ++i) ids.emplace(hm[i], 0u);
    std::vector<uint64_t> toff(1, 0), ts, te;
    uint32_t k = 0;
    for (auto &kvp : ids) {
        kvp.second = k++;
        rg::V acc;
        bool first = true;
        for (uint32_t s = 0; s < world; ++s) {
            if (!((kvp.first >> s) & 1ull)) continue;
            acc = first ? sc[s] : rg::with(sc[s], acc);
            first = false;
        }
        for (const auto &r : acc) { ts.push_back(r.s); te.push_back(r.e); }
        toff.push_back(ts.size());
    }
    std::vector<uint32_t> cid(ng);
    for (uint32_t i = 0; i < ng; ++i) cid[i] = ids[hm[i]];
    const uint32_t nd = (uint32_t)ids.size();
    uint64_t *doff = ctx->get<uint64_t>("cov_off", (size_t)nd + 1);
    uint64_t *dts = ctx->get<uint64_t>("cov_start", std::max<size_t>(ts.size(), 1));
    uint64_t *dte = ctx->get<uint64_t>("cov_end", std::max<size_t>(te.size(), 1));
    uint32_t *dcid = ctx->get<uint32_t>("cov_id", std::max<uint32_t>(ng, 1));
    ACC_HIP(hipMemcpyAsync(doff, toff.data(), toff.size() * 8, hipMemcpyHostToDevice, st));
    if (!ts.empty()) {
        ACC_HIP(hipMemcpyAsync(dts, ts.data(), ts.size() * 8, hipMemcpyHostToDevice, st));
        ACC_HIP(hipMemcpyAsync(dte, te.data(), te.size() * 8, hipMemcpyHostToDevice, st));
    }
    if (ng) ACC_HIP(hipMemcpyAsync(dcid, cid.data(), (size_t)ng * 4, hipMemcpyHostToDevice, st));
    // invariants of the reduced PartialDeps (the constructor's checks on the final fold)
    uint64_t *err = ctx->get<uint64_t>("cov_err", 1);
    ACC_HIP(hipMemsetAsync(err, 0, 8, st));
    Groups g{ ng, kv->key_off, kv->key_code, rv->range_deps.key_off, rv->range_deps.key_a, rv->range_deps.key_b, nullptr, dcid };
    const Table t{ doff, dts, dte, (int)end_inclusive };
    if (ng) launch(ctx, "cov_check", k_cov_check, dim3(grid_for(ng, BLOCK)), dim3(BLOCK), 0, g, t, err);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, err, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    if (ctx->pinned[0] & 1) fail(ACC_E_STATE, "PartialDeps: covering does not contain every KeyDeps key (PartialDeps.java:56)");
    if (ctx->pinned[0] & 2) fail(ACC_E_STATE, "PartialDeps: RangeDeps not covered by covering (PartialDeps.java:57)");
    *out = acc_covering_view{ ng, nd, dcid, doff, dts, dte, (const uint64_t *)mask, (uint64_t)ts.size() };
}

}  // namespace acc
