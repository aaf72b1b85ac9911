// latest.hip — recovery merge of LatestDeps replies: LatestDeps.mergeProposal / mergeCommit
// (primitives/LatestDeps.java:306-326) as Recover calls them for a batch of recovering txns (coordinate/Recover.java:295-355).
//
// A LatestDeps is a ReducingRangeMap (utils/ReducingIntervalMap.java) over RoutingKey intervals whose entries carry a
// KnownDeps phase, a Ballot, the coordinated Deps and the replica's local Deps. Recover folds the replies into one map
// (Merge.merge = mergeIntervals with MergeEntry.reduce, LatestDeps.java:228-241, 338-345; AbstractEntry.reduce :77-95),
// then per interval picks deps objects by phase (forProposal :371-382 / forCommit :384-413), slices each to its
// interval (KeyDeps.slice / RangeDeps.slice) and merges the slices (KeyDeps.merge / RangeDeps.merge).
//
// Split: the interval fold is a handful of entries per reply: host C++ below, restated step for step (builder
// coalescing of equal neighbours included, since it decides which phase later reductions see). The data-parallel part
// — gathering every selected (deps object, interval) item, KeyDeps/RangeDeps.slice + trimUnusedValues, and the batched
// Deps.merge of all items of all groups — runs on device (rmm.hip slice, depsmerge.hip merge).
#include "prims.hpp"

#include <vector>

namespace acc {

void rmm_slice(acc_ctx *ctx, const acc_rmm_batch *in, const acc_ranges_in *select, acc_slice_view *out);
void deps_merge(acc_ctx *ctx, const acc_deps_merge_in *in, acc_deps_merge_view *view);

namespace ld {

// KnownDeps ordinals (local/Status.java:539-578) and whether their Phase tie-breaks with the ballot (:99-115)
enum : uint8_t { DEPS_UNKNOWN = 0, DEPS_PROPOSED = 1, DEPS_COMMITTED = 2, DEPS_ERASED = 3, DEPS_KNOWN = 4, NO_DEPS = 5 };
inline bool tie_break_with_ballot(uint8_t known) { return known == DEPS_PROPOSED || known == DEPS_COMMITTED; }

struct Ballot { uint64_t msb, lsb; int32_t node; };

// Timestamp.compareTo (primitives/Timestamp.java:208-217)
inline int ts_cmp(const Ballot &a, const Ballot &b)
{
    constexpr uint64_t ID = 0xFFFFFFFFFFFF001EULL;
    if (a.msb != b.msb) return a.msb < b.msb ? -1 : 1;
    const uint64_t a1 = a.lsb & ID, b1 = b.lsb & ID;
    if (a1 != b1) return a1 < b1 ? -1 : 1;
    if (a.node != b.node) return a.node < b.node ? -1 : 1;
    return 0;
}

// MergeEntry (LatestDeps.java:249-275): deps objects are caller ids (the identity the Java compares with ==), -1 = null
struct Entry {
    uint8_t known;
    Ballot ballot;
    int32_t coord;
    std::vector<int32_t> merge;
};

struct Map {   // ReducingRangeMap: starts.size() == values.size() + 1 (or both empty); value -1 = null
    std::vector<uint64_t> starts;
    std::vector<int> values;
};

struct Pool {
    std::vector<Entry> e;
    int add(Entry x) { e.push_back(std::move(x)); return (int)e.size() - 1; }
};

// AbstractEntry.reduce (:77-95) with MergeEntry.reduce's merge function (:266-270), which builds the merged entry from
// the ARGUMENTS a and b as passed (not from the higher-phase one), whenever the higher-phase entry is <= DepsProposed
inline int reduce(Pool &p, int a, int b)
{
    const Entry &A = p.e[a], &B = p.e[b];
    int c = (A.known > B.known) - (A.known < B.known);
    if (c == 0 && tie_break_with_ballot(A.known)) c = ts_cmp(A.ballot, B.ballot);
    const int hi = c < 0 ? b : a;
    if (p.e[hi].known <= DEPS_PROPOSED) {
        Entry m{ A.known, A.ballot, A.coord, A.merge };
        m.merge.insert(m.merge.end(), B.merge.begin(), B.merge.end());
        return p.add(std::move(m));
    }
    return hi;
}

// MergeBuilder.tryMergeEqual (:420-435): same coordinatedDeps and merge lists element for element (by identity)
inline bool merge_equal(const Pool &p, int a, int b)
{
    const Entry &A = p.e[a], &B = p.e[b];
    if (A.coord != B.coord || A.merge.size() != B.merge.size()) return false;
    for (size_t i = 0; i < A.merge.size(); ++i)
        if (A.merge[i] != B.merge[i]) return false;
    return true;
}

// AbstractIntervalBuilder (utils/ReducingIntervalMap.java:522-575)
struct Builder {
    const Pool &p;
    Map m;
    bool has_prev = false;
    uint64_t prev_end = 0;
    explicit Builder(const Pool &pool) : p(pool) {}
    void append(uint64_t start, uint64_t end, int v)
    {
        if (has_prev) {
            if (prev_end > start) fail(ACC_E_STATE, "LatestDeps intervals out of order (AbstractIntervalBuilder.append)");
            if (prev_end < start) { m.starts.push_back(prev_end); m.values.push_back(-1); }
        }
        const size_t n = m.starts.size();
        if (n && m.values[n - 1] >= 0 && merge_equal(p, m.values[n - 1], v)) {
            // the tail entry stays (tryMergeEqual returns it)
        } else {
            m.starts.push_back(start);
            m.values.push_back(v);
        }
        prev_end = end;
        has_prev = true;
    }
    Map build()
    {
        if (has_prev) { m.starts.push_back(prev_end); has_prev = false; }
        return std::move(m);
    }
};

struct Iter {
    const Map &m;
    size_t i = 0;
    bool has() const { return i < m.values.size(); }
    uint64_t start() const { return m.starts[i]; }
    uint64_t end() const { return m.starts[i + 1]; }
    int value() const { return m.values[i]; }
};

// ReducingIntervalMap.mergeIntervals (:202-273) with MergeBuilder (slice = identity)
Map merge_intervals(Pool &p, const Map &L, const Map &R)
{
    if (L.values.empty()) return R;
    if (R.values.empty()) return L;
    Builder b(p);
    Iter left{ L }, right{ R };
    uint64_t start;
    {
        Iter &first = left.start() <= right.start() ? left : right;
        Iter &second = &first == &left ? right : left;
        while (first.has() && first.end() <= second.start()) {
            if (first.value() >= 0) b.append(first.start(), first.end(), first.value());
            ++first.i;
        }
        start = second.start();
        if (first.has() && first.start() < start && first.value() >= 0) b.append(first.start(), start, first.value());
    }
    while (left.has() && right.has()) {
        const uint64_t le = left.end(), re = right.end();
        const uint64_t end = le <= re ? le : re;
        const int lv = left.value(), rv = right.value();
        const int v = lv < 0 ? rv : rv < 0 ? lv : reduce(p, lv, rv);
        if (le <= re) ++left.i;
        if (le >= re) ++right.i;
        if (v >= 0) b.append(start, end, v);
        start = end;
    }
    Iter &rem = left.has() ? left : right;
    while (rem.has()) {
        const uint64_t end = rem.end();
        if (rem.value() >= 0) b.append(start, end, rem.value());
        start = end;
        ++rem.i;
    }
    return b.build();
}

struct Item {
    int32_t obj;
    uint64_t s, e;
};

}  // namespace ld

// ---------------------------------------------------------------- device part

struct LdObjs {   // the deps objects of one half (staged)
    const uint64_t *key_off, *val_off, *k2v_off, *key_a, *key_b, *msb, *lsb;
    const int32_t *node, *k2v;
};

__global__ __launch_bounds__(BLOCK) void k_ld_sizes(uint32_t n, const int32_t *__restrict__ obj, LdObjs o, uint64_t *__restrict__ nk,
                                                    uint64_t *__restrict__ nv, uint64_t *__restrict__ no)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const int32_t d = obj[i];
    nk[i] = o.key_off[d + 1] - o.key_off[d];
    nv[i] = o.val_off[d + 1] - o.val_off[d];
    no[i] = o.k2v_off[d + 1] - o.k2v_off[d];
}

// one wave per item: the object's keys (ranges) and int[] copied into the item batch the slice runs over
__global__ __launch_bounds__(BLOCK) void k_ld_gather(uint32_t n, const int32_t *__restrict__ obj, LdObjs o,
                                                     const uint64_t *__restrict__ ik, const uint64_t *__restrict__ io,
                                                     uint64_t *__restrict__ ka, uint64_t *__restrict__ kb, int32_t *__restrict__ k2v)
{
    const uint32_t i = blockIdx.x * WAVES + (threadIdx.x >> 6);
    if (i >= n) return;
    const int32_t d = obj[i];
    const uint64_t k0 = o.key_off[d], nk = ik[i + 1] - ik[i];
    for (uint64_t x = lane_id(); x < nk; x += 64) {
        ka[ik[i] + x] = o.key_a[k0 + x];
        if (kb) kb[ik[i] + x] = o.key_b[k0 + x];
    }
    const uint64_t o0 = o.k2v_off[d], no = io[i + 1] - io[i];
    for (uint64_t x = lane_id(); x < no; x += 64) k2v[io[i] + x] = o.k2v[o0 + x];
}

// one wave per item: the sliced keys and the kept TxnIds as values (the slice's int[] is used as it is)
__global__ __launch_bounds__(BLOCK) void k_ld_half(uint32_t n, const int32_t *__restrict__ obj, LdObjs o, acc_slice_view sv,
                                                   uint64_t *__restrict__ ka, uint64_t *__restrict__ kb, uint64_t *__restrict__ msb,
                                                   uint64_t *__restrict__ lsb, int32_t *__restrict__ node)
{
    const uint32_t i = blockIdx.x * WAVES + (threadIdx.x >> 6);
    if (i >= n) return;
    const int32_t d = obj[i];
    const uint64_t k0 = o.key_off[d], v0 = o.val_off[d];
    for (uint64_t x = sv.key_off[i] + lane_id(); x < sv.key_off[i + 1]; x += 64) {
        const uint64_t src = k0 + sv.key_idx[x];
        ka[x] = o.key_a[src];
        if (kb) kb[x] = o.key_b[src];
    }
    for (uint64_t y = sv.val_off[i] + lane_id(); y < sv.val_off[i + 1]; y += 64) {
        const uint64_t src = v0 + sv.val_idx[y];
        msb[y] = o.msb[src];
        lsb[y] = o.lsb[src];
        node[y] = o.node[src];
    }
}

namespace {

LdObjs stage_objs(acc_ctx *ctx, const acc_rmm_in &in, uint32_t nd, uint32_t mem, bool is_range)
{
    LdObjs o{};
    o.key_off = stage_in(ctx, "ld_key_off", in.key_off, (size_t)nd + 1, mem);
    o.val_off = stage_in(ctx, "ld_val_off", in.val_off, (size_t)nd + 1, mem);
    o.k2v_off = stage_in(ctx, "ld_k2v_off", in.k2v_off, (size_t)nd + 1, mem);
    hipStream_t st = ctx->stream;
    ACC_HIP(hipMemcpyAsync(ctx->pinned, o.key_off + nd, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, o.val_off + nd, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 2, o.k2v_off + nd, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t NK = ctx->pinned[0], NV = ctx->pinned[1], NO = ctx->pinned[2];
    o.key_a = stage_in(ctx, "ld_key_a", in.key_a, NK, mem);
    o.key_b = is_range ? stage_in(ctx, "ld_key_b", in.key_b, NK, mem) : nullptr;
    o.msb = stage_in(ctx, "ld_msb", in.txn.msb, NV, mem);
    o.lsb = stage_in(ctx, "ld_lsb", in.txn.lsb, NV, mem);
    o.node = stage_in(ctx, "ld_node", in.txn.node, NV, mem);
    o.k2v = stage_in(ctx, "ld_k2v", in.k2v, NO, mem);
    return o;
}

// the items of one half: gather, slice to their intervals, gather the slices into an acc_rmm_in (device pointers)
acc_rmm_in slice_items(acc_ctx *ctx, const char *ns, const acc_rmm_in &in, uint32_t nd, uint32_t mem, bool is_range,
                       uint32_t ni, const int32_t *d_obj, const uint64_t *d_sel_off, const uint64_t *d_sel_s,
                       const uint64_t *d_sel_e, uint32_t end_inclusive)
{
    NsScope scope(ctx, ns);
    if (!in.key_off) return acc_rmm_in{};
    if (!in.val_off || !in.k2v_off || (is_range && !in.key_b)) fail(ACC_E_ARG, "incomplete deps half (null offsets or range ends)");
    const LdObjs o = stage_objs(ctx, in, nd, mem, is_range);
    uint64_t *nk = ctx->get<uint64_t>("ld_nk", ni), *nv = ctx->get<uint64_t>("ld_nv", ni), *no = ctx->get<uint64_t>("ld_no", ni);
    uint64_t *ik = ctx->get<uint64_t>("ld_ik", (size_t)ni + 1), *iv = ctx->get<uint64_t>("ld_iv", (size_t)ni + 1);
    uint64_t *io = ctx->get<uint64_t>("ld_io", (size_t)ni + 1);
    if (ni) launch(ctx, "ld_sizes", k_ld_sizes, dim3(grid_for(ni, BLOCK)), dim3(BLOCK), 0, ni, d_obj, o, nk, nv, no);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, nk, ik, ni, true, ik + ni);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, nv, iv, ni, true, iv + ni);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, no, io, ni, true, io + ni);
    hipStream_t st = ctx->stream;
    ACC_HIP(hipMemcpyAsync(ctx->pinned, ik + ni, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, io + ni, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t TK = ctx->pinned[0], TO = ctx->pinned[1];
    uint64_t *ka = ctx->get<uint64_t>("ld_item_ka", TK + 1);
    uint64_t *kb = is_range ? ctx->get<uint64_t>("ld_item_kb", TK + 1) : nullptr;
    int32_t *k2v = ctx->get<int32_t>("ld_item_k2v", TO + 1);
    if (ni) launch(ctx, "ld_gather", k_ld_gather, dim3((ni + WAVES - 1) / WAVES), dim3(BLOCK), 0, ni, d_obj, o,
                   (const uint64_t *)ik, (const uint64_t *)io, ka, kb, k2v);
    acc_rmm_batch ib{ ACC_MEM_DEVICE, ni, ik, ka, kb, iv, io, k2v };
    acc_ranges_in sel{ d_sel_off, d_sel_s, d_sel_e, end_inclusive, 0 };
    acc_slice_view sv{};
    rmm_slice(ctx, &ib, &sel, &sv);
    uint64_t *hka = ctx->get<uint64_t>("ld_h_ka", sv.total_keys + 1);
    uint64_t *hkb = is_range ? ctx->get<uint64_t>("ld_h_kb", sv.total_keys + 1) : nullptr;
    uint64_t *hm = ctx->get<uint64_t>("ld_h_msb", sv.total_vals + 1), *hl = ctx->get<uint64_t>("ld_h_lsb", sv.total_vals + 1);
    int32_t *hn = ctx->get<int32_t>("ld_h_node", sv.total_vals + 1);
    if (ni) launch(ctx, "ld_half", k_ld_half, dim3((ni + WAVES - 1) / WAVES), dim3(BLOCK), 0, ni, d_obj, o, sv, hka, hkb, hm, hl, hn);
    acc_rmm_in h{};
    h.key_off = sv.key_off; h.key_a = hka; h.key_b = hkb; h.val_off = sv.val_off;
    h.txn = acc_ts_cols{ hm, hl, hn };
    h.k2v_off = sv.k2v_off; h.k2v = sv.k2v;
    return h;
}

}  // namespace

void latest_deps_merge(acc_ctx *ctx, const acc_latest_in *in, acc_latest_view *view)
{
    using namespace ld;
    if (!in || !view) fail(ACC_E_ARG, "null argument");
    if (in->mode > ACC_LATEST_COMMIT) fail(ACC_E_ARG, "mode must be ACC_LATEST_PROPOSAL or ACC_LATEST_COMMIT");
    if (in->deps_mem != ACC_MEM_HOST && in->deps_mem != ACC_MEM_DEVICE) fail(ACC_E_ARG, "deps_mem must be ACC_MEM_HOST or ACC_MEM_DEVICE");
    if (in->end_inclusive > 1) fail(ACC_E_ARG, "end_inclusive must be 0 or 1");
    ctx->dm_valid = false;
    const uint32_t ng = in->n_groups, nd = in->n_deps;
    if (ng && (!in->grp_off || !in->iv_off)) fail(ACC_E_ARG, "null grp_off / iv_off");
    const bool commit = in->mode == ACC_LATEST_COMMIT;

    // ---- host: fold every group's replies (LatestDeps.merge(list, getter) :228-241), then pick the items
    std::vector<Item> items;
    std::vector<uint64_t> item_grp(1, 0);
    ctx->latest_suff_off.assign(1, 0);
    ctx->latest_suff_s.clear();
    ctx->latest_suff_e.clear();
    for (uint32_t g = 0; g < ng; ++g) {
        Pool pool;
        Map acc;
        for (uint32_t r = in->grp_off[g]; r < in->grp_off[g + 1]; ++r) {
            Map cur;   // new Merge(LatestDeps): entries converted one for one, nulls where the map has gaps
            for (uint32_t i = in->iv_off[r]; i < in->iv_off[r + 1]; ++i) {
                const uint64_t s = in->iv_start[i], e = in->iv_end[i];
                if (s >= e) fail(ACC_E_ARG, "LatestDeps interval start must be below its end");
                if (in->known[i] > NO_DEPS) fail(ACC_E_ARG, "invalid KnownDeps ordinal");
                const int32_t cd = in->coord_deps ? in->coord_deps[i] : -1, lc = in->local_deps ? in->local_deps[i] : -1;
                if (cd >= (int32_t)nd || lc >= (int32_t)nd || cd < -1 || lc < -1) fail(ACC_E_ARG, "deps object id out of range");
                if (!cur.starts.empty()) {
                    if (cur.starts.back() > s) fail(ACC_E_ARG, "LatestDeps intervals must be sorted and non-overlapping");
                    if (cur.starts.back() < s) { cur.values.push_back(-1); cur.starts.push_back(s); }
                } else {
                    cur.starts.push_back(s);
                }
                Entry en{ in->known[i], Ballot{ in->ballot.msb[i], in->ballot.lsb[i], in->ballot.node[i] }, cd, {} };
                if (lc >= 0) en.merge.push_back(lc);
                cur.values.push_back(pool.add(std::move(en)));
                cur.starts.push_back(e);   // the next interval starts here, or after a null gap
            }
            acc = merge_intervals(pool, acc, cur);
        }
        // Merge.mergeProposal (:350-358) / mergeCommit (:360-369): items in stream order (intervals ascending)
        bool use_local = false;
        if (commit) {
            const Ballot t{ in->txn_id.msb[g], in->txn_id.lsb[g], in->txn_id.node[g] };
            const Ballot x{ in->execute_at.msb[g], in->execute_at.lsb[g], in->execute_at.node[g] };
            use_local = ts_cmp(t, x) == 0;   // txnId.equals(executeAt)
        }
        std::vector<std::pair<uint64_t, uint64_t>> suff;
        for (size_t i = 0; i < acc.values.size(); ++i) {
            if (acc.values[i] < 0) continue;
            const Entry &en = pool.e[acc.values[i]];
            const uint64_t s = acc.starts[i], e = acc.starts[i + 1];
            auto add = [&](int32_t d) {
                if (d < 0) fail(ACC_E_STATE, "null coordinatedDeps in a LatestDeps entry that needs it (NullPointerException)");
                items.push_back(Item{ d, s, e });
            };
            if (!commit) {   // forProposal (:371-382)
                if (en.known == DEPS_PROPOSED) add(en.coord);
                else if (en.known == DEPS_UNKNOWN) for (int32_t d : en.merge) add(d);
                else fail(ACC_E_STATE, "Invalid KnownDeps for proposal (AssertionError)");
            } else {         // forCommit (:384-413)
                switch (en.known) {
                case DEPS_UNKNOWN:
                    if (!use_local) break;
                    suff.emplace_back(s, e);
                    for (int32_t d : en.merge) add(d);
                    break;
                case DEPS_PROPOSED:
                    if (!use_local) break;
                    suff.emplace_back(s, e);
                    add(en.coord);
                    for (int32_t d : en.merge) add(d);
                    break;
                case DEPS_KNOWN: case DEPS_COMMITTED:
                    suff.emplace_back(s, e);
                    add(en.coord);
                    break;
                default:
                    fail(ACC_E_STATE, "Invalid KnownDeps for commit (AssertionError)");
                }
            }
        }
        // sufficientFor = Ranges.of(list): sorted, overlapping ranges merged, adjacent ones kept (AbstractRanges.java:688-784);
        // the map's intervals are ascending and disjoint, so the list (added once per half) reduces to them
        for (auto &r : suff) { ctx->latest_suff_s.push_back(r.first); ctx->latest_suff_e.push_back(r.second); }
        ctx->latest_suff_off.push_back(ctx->latest_suff_s.size());
        item_grp.push_back(items.size());
    }

    // ---- device: slice every item to its interval, then one batched Deps.merge per group
    const uint32_t ni = (uint32_t)items.size();
    std::vector<int32_t> h_obj(ni);
    std::vector<uint64_t> h_off(ni + 1), h_s(ni), h_e(ni);
    for (uint32_t i = 0; i < ni; ++i) { h_obj[i] = items[i].obj; h_off[i] = i; h_s[i] = items[i].s; h_e[i] = items[i].e; }
    h_off[ni] = ni;
    const int32_t *d_obj = stage_in(ctx, "ld_obj", h_obj.data(), ni, ACC_MEM_HOST);
    const uint64_t *d_off = stage_in(ctx, "ld_sel_off", h_off.data(), (size_t)ni + 1, ACC_MEM_HOST);
    const uint64_t *d_s = stage_in(ctx, "ld_sel_s", h_s.data(), ni, ACC_MEM_HOST);
    const uint64_t *d_e = stage_in(ctx, "ld_sel_e", h_e.data(), ni, ACC_MEM_HOST);
    const uint64_t *d_grp = stage_in(ctx, "ld_grp", item_grp.data(), (size_t)ng + 1, ACC_MEM_HOST);
    const acc_rmm_in kh = slice_items(ctx, "ldk.", in->key_deps, nd, in->deps_mem, false, ni, d_obj, d_off, d_s, d_e, in->end_inclusive);
    const acc_rmm_in rh = slice_items(ctx, "ldr.", in->range_deps, nd, in->deps_mem, true, ni, d_obj, d_off, d_s, d_e, in->end_inclusive);
    acc_deps_merge_in dmi{ ACC_MEM_DEVICE, ng, ni, d_grp, kh, rh };
    acc_deps_merge_view dv{};
    deps_merge(ctx, &dmi, &dv);
    ctx->stat("latest.items", ni);
    *view = acc_latest_view{ dv, (uint64_t)ctx->latest_suff_s.size(), ctx->latest_suff_off.data(), ctx->latest_suff_s.data(),
                             ctx->latest_suff_e.data() };
}

}  // namespace acc
