// depsmerge.hip — Deps.merge over raw deps objects (primitives/Deps.java:256-260): KeyDeps.merge
// (primitives/KeyDeps.java:115-135) and RangeDeps.merge (primitives/RangeDeps.java:101-134) of many replies per
// coordinated txn, on the arrays KeyDeps/RangeDeps.SerializerSupport expose (primitives/KeyDeps.java:55-73,
// primitives/RangeDeps.java:55-73): keys (u64 codes) or ranges ((start, end) codes), raw TxnId columns, and the Java
// keysToTxnIds / rangesToTxnIds int[].
//
// Each half:
//   1. dictionaries: dense order ranks of the keys (u64, or (start, end) under Range::compare) and of the TxnIds
//      (Timestamp.compareTo over the identity bits; equal rank <=> Timestamp.equals) of every reply;
//   2. the batched rank-space union (merge.hip: LDS tier / global radix path) = the LinearMerger fold's result, which
//      is the canonical union (KeyDepsTest.testMergedProperty, KeyDepsTest.java:275-283);
//   3. TxnId instances: Timestamp.equals ignores the flag bits outside IDENTITY_LSB (domain, REJECTED, ...), so equal
//      TxnIds may differ in raw bits. The Java keeps the instance SortedArrays.linearUnion picks
//      (utils/SortedArrays.java:152-281: ties keep LEFT, except inside the superset candidate's matched prefix when
//      the right side is longer) and RelationMultiMap.linearUnion's pass-through returns (utils/RelationMultiMap.java:
//      583-711). Every output TxnId first takes its first occurrence in fold order; groups where some tie differs in
//      raw bits then replay the fold exactly (one lane per such group, k_rep_exact) to pick the same instance;
//   4. output: codes / ranges / raw TxnIds mapped back from the dictionaries.
#include "dict.hpp"

namespace acc {

void keydeps_merge(acc_ctx *ctx, const acc_merge_in *in, acc_merge_view *view);

namespace {


__global__ __launch_bounds__(BLOCK) void k_dm_node_word(size_t n, const int32_t *__restrict__ node, uint64_t *__restrict__ out)
{
    const size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) out[i] = (uint64_t)((uint32_t)node[i] ^ 0x80000000u);   // Node.Id signed order as unsigned
}

__global__ __launch_bounds__(BLOCK) void k_dm_widen(size_t n, const uint32_t *__restrict__ in, uint64_t *__restrict__ out)
{
    const size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) out[i] = in[i];
}

// Range start < end (Range ctor); err |= 1
__global__ __launch_bounds__(BLOCK) void k_dm_range_check(size_t n, const uint64_t *__restrict__ s, const uint64_t *__restrict__ e,
                                                          uint64_t *__restrict__ err)
{
    const size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    bool bad = i < n && s[i] >= e[i];
    if (__ballot(bad) && lane_id() == 0) atomicOr((unsigned long long *)err, 1ull);
}

__device__ __forceinline__ uint64_t ub_u64(const uint64_t *a, uint64_t lo, uint64_t hi, uint64_t v)   // first a[i] > v
{
    while (lo < hi) { const uint64_t m = (lo + hi) >> 1; if (a[m] <= v) lo = m + 1; else hi = m; }
    return lo;
}
__device__ __forceinline__ uint64_t lb_u32(const uint32_t *a, uint64_t lo, uint64_t hi, uint32_t v)
{
    while (lo < hi) { const uint64_t m = (lo + hi) >> 1; if (a[m] < v) lo = m + 1; else hi = m; }
    return lo;
}

struct Rep {
    const uint64_t *grp_off, *key_off, *val_off, *k2v_off;   // inputs (device)
    uint64_t R, NV;
    uint32_t ng;
    const uint32_t *vrank, *krank;
    const int32_t *k2v;
    const uint64_t *msb, *lsb;
    const int32_t *node;
    const uint64_t *out_val_off;   // merged view
    const uint32_t *out_rank;
    uint32_t *rep;                 // [TV] kept instance (input slot) of each merged TxnId
    uint32_t *flag;                // [ng] some equals-tie of the group differs in raw bits
    uint64_t *nflag;
};

// reply of value slot i (replies own contiguous slot ranges), group of reply r
__device__ __forceinline__ uint64_t reply_of(const Rep &p, uint64_t i) { return ub_u64(p.val_off, 0, p.R + 1, i) - 1; }
__device__ __forceinline__ uint32_t group_of(const Rep &p, uint64_t r) { return (uint32_t)(ub_u64(p.grp_off, 0, (uint64_t)p.ng + 1, r) - 1); }
__device__ __forceinline__ bool reply_empty(const Rep &p, uint64_t r)   // RelationMultiMap.isEmpty (:1012-1015)
{
    return p.k2v_off[r + 1] - p.k2v_off[r] == p.key_off[r + 1] - p.key_off[r];
}

// first occurrence in fold order (reply order, empty replies skipped: KeyDeps.merge / RangeDeps.merge skip them)
__global__ __launch_bounds__(BLOCK) void k_rep_first(Rep p)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= p.NV) return;
    const uint64_t r = reply_of(p, i);
    if (reply_empty(p, r)) return;
    const uint32_t g = group_of(p, r);
    const uint64_t pos = lb_u32(p.out_rank, p.out_val_off[g], p.out_val_off[g + 1], p.vrank[i]);
    atomicMin(&p.rep[pos], (uint32_t)i);
}

__global__ __launch_bounds__(BLOCK) void k_rep_check(Rep p)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= p.NV) return;
    const uint64_t r = reply_of(p, i);
    if (reply_empty(p, r)) return;
    const uint32_t g = group_of(p, r);
    const uint64_t pos = lb_u32(p.out_rank, p.out_val_off[g], p.out_val_off[g + 1], p.vrank[i]);
    const uint32_t s = p.rep[pos];
    if (s == (uint32_t)i) return;
    if (p.msb[s] != p.msb[i] || p.lsb[s] != p.lsb[i] || p.node[s] != p.node[i]) {
        if (atomicExch(&p.flag[g], 1u) == 0u) atomicAdd((unsigned long long *)p.nflag, 1ull);
    }
}

// ---- exact instance replay (rare: only groups with raw-bit-differing ties). One lane per flagged group runs the
// LinearMerger fold in rank space with value INSTANCES (input slots), following SortedArrays.linearUnion and
// RelationMultiMap.linearUnion (same structure as oracle/accord_oracle_rmm.c's restatement). Scratch: two
// accumulators (keys, slots, ints) at the group's input offsets, plus two remap arrays.

struct Acc {
    uint32_t *k; uint32_t *v; int32_t *o;
    uint64_t nk, nv, no;
};

struct Exact {
    Rep p;
    uint32_t *k[2], *v[2];
    int32_t *o[2];
    int32_t *rmL, *rmR;
    uint32_t *keybuf;   // union keys of the current step
    uint32_t *valbuf;   // union values (slots) of the current step
};

__device__ __forceinline__ int cmpu(uint32_t a, uint32_t b) { return a < b ? -1 : a > b ? 1 : 0; }

// SortedArrays.linearUnion over u32 items with a ranking function; returns 1 (left), 2 (right) or 0 (new: out).
template <class Rank>
__device__ int sa_union(const uint32_t *L, uint64_t nl, const uint32_t *R, uint64_t nr, uint32_t *out, uint64_t &no, Rank rk)
{
    uint64_t li = 0, ri = 0, rs = 0;
    bool built = false;
    if (nl >= nr) {
        while (li < nl && ri < nr) {
            const int c = L[li] == R[ri] ? 0 : cmpu(rk(L[li]), rk(R[ri]));
            if (c <= 0) { li += 1; ri += c == 0 ? 1 : 0; }
            else { for (uint64_t q = 0; q < li; ++q) out[q] = L[q]; rs = li; out[rs++] = R[ri++]; built = true; break; }
        }
        if (!built) {
            if (ri == nr) { no = nl; return 1; }
            for (uint64_t q = 0; q < li; ++q) out[q] = L[q];
            rs = li;
        }
    } else {
        while (li < nl && ri < nr) {
            const int c = L[li] == R[ri] ? 0 : cmpu(rk(L[li]), rk(R[ri]));
            if (c >= 0) { ri += 1; li += c == 0 ? 1 : 0; }
            else { for (uint64_t q = 0; q < ri; ++q) out[q] = R[q]; rs = ri; out[rs++] = L[li++]; built = true; break; }
        }
        if (!built) {
            if (li == nl) { no = nr; return 2; }
            for (uint64_t q = 0; q < ri; ++q) out[q] = R[q];
            rs = ri;
        }
    }
    while (li < nl && ri < nr) {
        const int c = L[li] == R[ri] ? 0 : cmpu(rk(L[li]), rk(R[ri]));
        if (c == 0) { out[rs++] = L[li]; li++; ri++; }
        else if (c < 0) out[rs++] = L[li++];
        else out[rs++] = R[ri++];
    }
    while (li < nl) out[rs++] = L[li++];
    while (ri < nr) out[rs++] = R[ri++];
    no = rs;
    return 0;
}

__global__ __launch_bounds__(64) void k_rep_exact(Exact x)
{
    const uint32_t g = blockIdx.x * 64 + threadIdx.x;
    const Rep &p = x.p;
    if (g >= p.ng || !p.flag[g]) return;
    const uint64_t r0 = p.grp_off[g], r1 = p.grp_off[g + 1];
    const uint64_t KA = p.key_off[r0], VA = p.val_off[r0], OA = p.k2v_off[r0];
    auto vr = [&](uint32_t slot) { return p.vrank[slot]; };
    auto kr = [&](uint32_t key) { return key; };   // keys are stored as ranks already
    int cur = -1;
    Acc A{};
    for (uint64_t r = r0; r < r1; ++r) {
        if (reply_empty(p, r)) continue;
        // the reply as an Acc view: keys (ranks), values (slots), ints
        const uint64_t ka = p.key_off[r], va = p.val_off[r], oa = p.k2v_off[r];
        Acc B{};
        B.nk = p.key_off[r + 1] - ka; B.nv = p.val_off[r + 1] - va; B.no = p.k2v_off[r + 1] - oa;
        if (cur < 0) {   // LinearMerger.update, first input: the accumulator is the reply itself
            cur = 0;
            A.k = x.k[0] + KA; A.v = x.v[0] + VA; A.o = x.o[0] + OA;
            for (uint64_t q = 0; q < B.nk; ++q) A.k[q] = p.krank[ka + q];
            for (uint64_t q = 0; q < B.nv; ++q) A.v[q] = (uint32_t)(va + q);
            for (uint64_t q = 0; q < B.no; ++q) A.o[q] = p.k2v[oa + q];
            A.nk = B.nk; A.nv = B.nv; A.no = B.no;
            continue;
        }
        // B's arrays: keys and slots materialised in the key/val buffers of the other accumulator's tail region is not
        // possible (it is the output); read them through index arithmetic instead
        const int nxt = cur ^ 1;
        uint32_t *Bk = x.keybuf + KA;   // reply keys (ranks) copied once per step
        uint32_t *Bv = x.valbuf + VA;   // reply slots
        for (uint64_t q = 0; q < B.nk; ++q) Bk[q] = p.krank[ka + q];
        for (uint64_t q = 0; q < B.nv; ++q) Bv[q] = (uint32_t)(va + q);
        const int32_t *Bo = p.k2v + oa;
        uint32_t *ok_ = x.k[nxt] + KA;
        uint32_t *ov_ = x.v[nxt] + VA;
        int32_t *oo_ = x.o[nxt] + OA;
        uint64_t nko = 0, nvo = 0;
        const int kw = sa_union(A.k, A.nk, Bk, B.nk, ok_, nko, kr);
        const int vw = sa_union(A.v, A.nv, Bv, B.nv, ov_, nvo, vr);
        const uint32_t *outK = kw == 1 ? A.k : kw == 2 ? Bk : ok_;
        const uint32_t *outV = vw == 1 ? A.v : vw == 2 ? Bv : ov_;
        // remapToSuperset (:1196-1223): null when the lengths are equal
        const bool rlN = nvo == A.nv, rrN = nvo == B.nv;
        int32_t *rmL = x.rmL + VA, *rmR = x.rmR + VA;
        if (!rlN) { uint64_t j = 0; for (uint64_t i = 0; i < A.nv; ++i) { while (vr(outV[j]) < vr(A.v[i])) ++j; rmL[i] = (int32_t)j++; } }
        if (!rrN) { uint64_t j = 0; for (uint64_t i = 0; i < B.nv; ++i) { while (vr(outV[j]) < vr(Bv[i])) ++j; rmR[i] = (int32_t)j++; } }
        auto mapL = [&](int32_t i) { return rlN ? i : rmL[i]; };
        auto mapR = [&](int32_t i) { return rrN ? i : rmR[i]; };
        int kind = 0;   // 1: result = A as is, 2: result = B as is, 0: built
        if (rlN && rrN && A.no == B.no && A.nk == B.nk) {
            bool eq = true;
            for (uint64_t q = 0; q < B.no && eq; ++q) eq = A.o[q] == Bo[q];
            for (uint64_t q = 0; q < B.nk && eq; ++q) eq = A.k[q] == Bk[q];
            if (eq) kind = 1;
        }
        if (kind == 0 && rlN && kw == 1) {
            // left knows every TxnId and key: pass-through unless right holds an entry left lacks (:592-651)
            uint64_t lk = 0, rk = 0, l = A.nk, rr = B.nk;
            bool conflict = false;
            while (lk < A.nk && rk < B.nk && !conflict) {
                const int ck = cmpu(A.k[lk], Bk[rk]);
                if (ck < 0) { l = (uint64_t)A.o[lk]; lk++; }
                else if (ck > 0) { conflict = true; }
                else {
                    while (l < (uint64_t)A.o[lk] && rr < (uint64_t)Bo[rk]) {
                        const int32_t nl = A.o[l], nr = mapR(Bo[rr]);
                        if (nl < nr) l++;
                        else if (nr < nl) { conflict = true; break; }
                        else { l++; rr++; }
                    }
                    if (conflict) break;
                    if (l < (uint64_t)A.o[lk]) l = (uint64_t)A.o[lk];
                    else if (rr < (uint64_t)Bo[rk]) { conflict = true; break; }
                    rk++; lk++;
                }
            }
            if (!conflict) kind = 1;
        } else if (kind == 0 && rrN && kw == 2) {
            uint64_t lk = 0, rk = 0, l = A.nk, rr = B.nk;
            bool conflict = false;
            while (lk < A.nk && rk < B.nk && !conflict) {
                const int ck = cmpu(A.k[lk], Bk[rk]);
                if (ck < 0) { conflict = true; }
                else if (ck > 0) { rr = (uint64_t)Bo[rk]; rk++; }
                else {
                    while (l < (uint64_t)A.o[lk] && rr < (uint64_t)Bo[rk]) {
                        const int32_t nl = mapL(A.o[l]), nr = Bo[rr];
                        if (nl < nr) { conflict = true; break; }
                        else if (nr < nl) rr++;
                        else { l++; rr++; }
                    }
                    if (conflict) break;
                    if (l < (uint64_t)A.o[lk]) { conflict = true; break; }
                    else if (rr < (uint64_t)Bo[rk]) rr = (uint64_t)Bo[rk];
                    rk++; lk++;
                }
            }
            if (!conflict) kind = 2;
        }
        if (kind == 1) continue;   // the accumulator stays as is
        Acc N{};
        N.k = ok_; N.v = ov_; N.o = oo_;
        if (kind == 2) {
            for (uint64_t q = 0; q < B.nk; ++q) N.k[q] = Bk[q];
            for (uint64_t q = 0; q < B.nv; ++q) N.v[q] = Bv[q];
            for (uint64_t q = 0; q < B.no; ++q) N.o[q] = Bo[q];
            N.nk = B.nk; N.nv = B.nv; N.no = B.no;
        } else {
            // the general union (:713-795); only its value instances matter to the caller, but the structure is
            // rebuilt so the next step sees the same accumulator the Java holds
            if (kw != 0) for (uint64_t q = 0; q < nko; ++q) N.k[q] = outK[q];
            if (vw != 0) for (uint64_t q = 0; q < nvo; ++q) N.v[q] = outV[q];
            uint64_t lk = 0, rk = 0, ok = 0, l = A.nk, rr = B.nk, olen = nko;
            while (lk < A.nk && rk < B.nk) {
                const int ck = cmpu(A.k[lk], Bk[rk]);
                if (ck < 0) { while (l < (uint64_t)A.o[lk]) N.o[olen++] = mapL(A.o[l++]); N.o[ok++] = (int32_t)olen; lk++; }
                else if (ck > 0) { while (rr < (uint64_t)Bo[rk]) N.o[olen++] = mapR(Bo[rr++]); N.o[ok++] = (int32_t)olen; rk++; }
                else {
                    while (l < (uint64_t)A.o[lk] && rr < (uint64_t)Bo[rk]) {
                        const int32_t nl = mapL(A.o[l]), nr = mapR(Bo[rr]);
                        if (nl <= nr) { N.o[olen++] = nl; l += 1; rr += nl == nr ? 1 : 0; }
                        else { N.o[olen++] = nr; ++rr; }
                    }
                    while (l < (uint64_t)A.o[lk]) N.o[olen++] = mapL(A.o[l++]);
                    while (rr < (uint64_t)Bo[rk]) N.o[olen++] = mapR(Bo[rr++]);
                    N.o[ok++] = (int32_t)olen; rk++; lk++;
                }
            }
            while (lk < A.nk) { while (l < (uint64_t)A.o[lk]) N.o[olen++] = mapL(A.o[l++]); N.o[ok++] = (int32_t)olen; lk++; }
            while (rk < B.nk) { while (rr < (uint64_t)Bo[rk]) N.o[olen++] = mapR(Bo[rr++]); N.o[ok++] = (int32_t)olen; rk++; }
            N.nk = nko; N.nv = nvo; N.no = olen;
        }
        A = N;
        cur = nxt;
    }
    // the accumulator's value instances, in TxnId order = the merged view's order
    const uint64_t o0 = p.out_val_off[g];
    for (uint64_t q = 0; q < A.nv; ++q) p.rep[o0 + q] = A.v[q];
}

struct Gather {
    const uint32_t *rep, *kfirst, *out_krank;
    const uint64_t *msb, *lsb, *key_a, *key_b;
    const int32_t *node;
    uint64_t *o_msb, *o_lsb, *o_key_a, *o_key_b;
    int32_t *o_node;
    uint64_t TV, TK;
};

__global__ __launch_bounds__(BLOCK) void k_dm_gather(Gather x)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < x.TV) {
        const uint32_t s = x.rep[i];
        x.o_msb[i] = x.msb[s]; x.o_lsb[i] = x.lsb[s]; x.o_node[i] = x.node[s];
    }
    if (i < x.TK) {
        const uint32_t src = x.kfirst[x.out_krank[i]];
        x.o_key_a[i] = x.key_a[src];
        if (x.key_b) x.o_key_b[i] = x.key_b[src];
    }
}

__global__ __launch_bounds__(BLOCK) void k_dm_u32_of_u64(size_t n, const uint64_t *__restrict__ in, uint32_t *__restrict__ out)
{
    const size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) out[i] = (uint32_t)in[i];
}

// one half (KeyDeps or RangeDeps) of Deps.merge
void merge_half(acc_ctx *ctx, const char *ns, uint32_t mem, uint32_t ng, uint64_t R, const uint64_t *grp_off, const acc_rmm_in &in,
                bool is_range, acc_rmm_view &out, uint64_t &in_entries)
{
    NsScope scope(ctx, ns);
    hipStream_t st = ctx->stream;
    out = acc_rmm_view{};
    if (!in.key_off) {   // no such half: every group merges to NONE
        uint64_t *z = ctx->get<uint64_t>("dm_zero_off", (size_t)ng + 1);
        ACC_HIP(hipMemsetAsync(z, 0, ((size_t)ng + 1) * 8, st));
        out.key_off = out.val_off = out.k2v_off = z;
        return;
    }
    if (!in.val_off || !in.k2v_off || (is_range && !in.key_b)) fail(ACC_E_ARG, "incomplete deps half (null offsets or range ends)");
    const uint64_t *key_off = stage_in(ctx, "dm_key_off", in.key_off, R + 1, mem);
    const uint64_t *val_off = stage_in(ctx, "dm_val_off", in.val_off, R + 1, mem);
    const uint64_t *k2v_off = stage_in(ctx, "dm_k2v_off", in.k2v_off, R + 1, mem);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, key_off + R, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, val_off + R, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 2, k2v_off + R, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t NK = ctx->pinned[0], NV = ctx->pinned[1], NO = ctx->pinned[2];
    if (NK >= 0xFFFFFFFFull || NV >= 0xFFFFFFFFull || NO >= 0xFFFFFFFFull) fail(ACC_E_CAP, "deps merge input too large");
    in_entries += NO - NK;
    const uint64_t *key_a = stage_in(ctx, "dm_key_a", in.key_a, NK, mem);
    const uint64_t *key_b = is_range ? stage_in(ctx, "dm_key_b", in.key_b, NK, mem) : nullptr;
    const uint64_t *msb = stage_in(ctx, "dm_msb", in.txn.msb, NV, mem);
    const uint64_t *lsb = stage_in(ctx, "dm_lsb", in.txn.lsb, NV, mem);
    const int32_t *node = stage_in(ctx, "dm_node", in.txn.node, NV, mem);
    const int32_t *k2v = stage_in(ctx, "dm_k2v", in.k2v, NO, mem);
    if (is_range && NK) {
        uint64_t *err = ctx->get<uint64_t>("dm_err", 1);
        ACC_HIP(hipMemsetAsync(err, 0, 8, st));
        launch(ctx, "dm_range_check", k_dm_range_check, dim3(grid_for(NK, BLOCK)), dim3(BLOCK), 0, (size_t)NK, key_a, key_b, err);
        ACC_HIP(hipMemcpyAsync(ctx->pinned + 3, err, 8, hipMemcpyDeviceToHost, st));
    }
    // ---- dictionaries
    const uint64_t *kw[2] = { key_a, key_b };
    DenseRank kd = dense_rank(ctx, "dm_kdict", NK, is_range ? 2 : 1, kw, nullptr, nullptr, true);
    if (is_range && NK && ctx->pinned[3]) fail(ACC_E_ARG, "Range start must be below its end");
    uint64_t *nodew = ctx->get<uint64_t>("dm_nodew", NV);
    launch(ctx, "dm_node_word", k_dm_node_word, dim3(grid_for(NV, BLOCK)), dim3(BLOCK), 0, (size_t)NV, node, nodew);
    const uint64_t *vw[3] = { msb, lsb, nodew };
    const uint64_t vand[3] = { ~0ull, 0xFFFFFFFFFFFF001EULL, ~0ull };   // Timestamp.IDENTITY_LSB (Timestamp.java:41)
    DenseRank vd = dense_rank(ctx, "dm_vdict", NV, 3, vw, vand, nullptr, false);
    uint64_t *krank64 = ctx->get<uint64_t>("dm_krank64", NK);
    launch(ctx, "dm_widen", k_dm_widen, dim3(grid_for(NK, BLOCK)), dim3(BLOCK), 0, (size_t)NK, (const uint32_t *)kd.rank, krank64);
    // ---- the rank-space union (validation included: sorted unique keys / TxnIds, headers, entry ranges)
    acc_merge_in mi{ ACC_MEM_DEVICE, ng, R, grp_off, key_off, krank64, val_off, vd.rank, k2v_off, k2v };
    acc_merge_view mv{};
    keydeps_merge(ctx, &mi, &mv);
    const uint64_t TK = mv.total_keys, TV = mv.total_vals, TO = mv.total_k2v;
    // ---- TxnId instances
    Rep p{};
    p.grp_off = grp_off; p.key_off = key_off; p.val_off = val_off; p.k2v_off = k2v_off;
    p.R = R; p.NV = NV; p.ng = ng; p.vrank = vd.rank; p.krank = kd.rank; p.k2v = k2v;
    p.msb = msb; p.lsb = lsb; p.node = node;
    p.out_val_off = mv.val_off; p.out_rank = mv.txn_rank;
    p.rep = ctx->get<uint32_t>("dm_rep", TV + 1);
    p.flag = ctx->get<uint32_t>("dm_flag", (size_t)ng + 1);
    p.nflag = ctx->get<uint64_t>("dm_nflag", 1);
    ACC_HIP(hipMemsetAsync(p.rep, 0xFF, (TV + 1) * 4, st));
    ACC_HIP(hipMemsetAsync(p.flag, 0, ((size_t)ng + 1) * 4, st));
    ACC_HIP(hipMemsetAsync(p.nflag, 0, 8, st));
    const unsigned gv = grid_for(NV, BLOCK);
    if (NV) {
        launch(ctx, "dm_rep_first", k_rep_first, dim3(gv), dim3(BLOCK), 0, p);
        launch(ctx, "dm_rep_check", k_rep_check, dim3(gv), dim3(BLOCK), 0, p);
    }
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 4, p.nflag, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t nflag = ctx->pinned[4];
    ctx->stat(is_range ? "deps_merge.range_exact_groups" : "deps_merge.key_exact_groups", nflag);
    if (nflag) {
        Exact x{};
        x.p = p;
        for (int b = 0; b < 2; ++b) {
            x.k[b] = ctx->get<uint32_t>(b ? "dm_x_k1" : "dm_x_k0", NK + 1);
            x.v[b] = ctx->get<uint32_t>(b ? "dm_x_v1" : "dm_x_v0", NV + 1);
            x.o[b] = ctx->get<int32_t>(b ? "dm_x_o1" : "dm_x_o0", NO + 1);
        }
        x.rmL = ctx->get<int32_t>("dm_x_rml", NV + 1);
        x.rmR = ctx->get<int32_t>("dm_x_rmr", NV + 1);
        x.keybuf = ctx->get<uint32_t>("dm_x_kb", NK + 1);
        x.valbuf = ctx->get<uint32_t>("dm_x_vb", NV + 1);
        launch(ctx, "dm_rep_exact", k_rep_exact, dim3((ng + 63) / 64), dim3(64), 0, x);
    }
    // ---- outputs
    Gather gx{};
    gx.rep = p.rep; gx.kfirst = kd.first; gx.msb = msb; gx.lsb = lsb; gx.node = node; gx.key_a = key_a; gx.key_b = key_b;
    uint32_t *out_krank = ctx->get<uint32_t>("dm_out_krank", TK + 1);
    launch(ctx, "dm_u32", k_dm_u32_of_u64, dim3(grid_for(TK, BLOCK)), dim3(BLOCK), 0, (size_t)TK, mv.key_code, out_krank);
    gx.out_krank = out_krank;
    gx.o_msb = ctx->get<uint64_t>("dm_o_msb", TV + 1);
    gx.o_lsb = ctx->get<uint64_t>("dm_o_lsb", TV + 1);
    gx.o_node = ctx->get<int32_t>("dm_o_node", TV + 1);
    gx.o_key_a = ctx->get<uint64_t>("dm_o_key_a", TK + 1);
    gx.o_key_b = is_range ? ctx->get<uint64_t>("dm_o_key_b", TK + 1) : nullptr;
    gx.TV = TV; gx.TK = TK;
    launch(ctx, "dm_gather", k_dm_gather, dim3(grid_for(std::max(TV, TK), BLOCK)), dim3(BLOCK), 0, gx);
    out.total_keys = TK; out.total_vals = TV; out.total_k2v = TO;
    out.key_off = mv.key_off; out.key_a = gx.o_key_a; out.key_b = gx.o_key_b;
    out.val_off = mv.val_off; out.txn_msb = gx.o_msb; out.txn_lsb = gx.o_lsb; out.txn_node = gx.o_node; out.txn_src = p.rep;
    out.k2v_off = mv.k2v_off; out.k2v = mv.k2v;
}

}  // namespace

void deps_merge(acc_ctx *ctx, const acc_deps_merge_in *in, acc_deps_merge_view *view)
{
    if (!in || !view) fail(ACC_E_ARG, "null argument");
    if (in->mem != ACC_MEM_HOST && in->mem != ACC_MEM_DEVICE) fail(ACC_E_ARG, "mem must be ACC_MEM_HOST or ACC_MEM_DEVICE");
    ctx->dm_valid = false;
    ctx->merge_valid = false;
    const uint32_t ng = in->n_groups;
    const uint64_t R = in->n_replies;
    const uint64_t *grp_off = stage_in(ctx, "dm_grp_off", in->grp_off, (size_t)ng + 1, in->mem);
    acc_deps_merge_view v{};
    v.n_groups = ng;
    merge_half(ctx, "dmk.", in->mem, ng, R, grp_off, in->key_deps, false, v.key_deps, v.total_in_entries);
    merge_half(ctx, "dmr.", in->mem, ng, R, grp_off, in->range_deps, true, v.range_deps, v.total_in_entries);
    ctx->sync();
    ctx->merge_valid = false;   // the rank-space views of the halves are internal
    *view = v;
    ctx->dm_view = v;
    ctx->dm_valid = true;
}

void rmm_without_dev(acc_ctx *ctx, uint32_t ng, const acc_rmm_in &h, uint64_t NK, uint64_t NV, uint64_t NO,
                     const acc_txn_sets *sa, const acc_txn_sets *sb, acc_without_view *out);   // rmm.hip

// The recovery coordinator's fold of the replies' recovery deps (coordinate/Recover.java:320-322; pairwise,
// BeginRecovery.RecoverOk.reduce, messages/BeginRecovery.java:180-183): earlierCommittedWitness = Deps.merge of the
// replies'; earlierAcceptedNoWitness = Deps.merge of the replies', then .without(earlierCommittedWitness::contains) on
// both halves (Deps.without, primitives/Deps.java:122-124) with the merged committed key and range TxnIds as the sets
// (Deps.contains = KeyDeps.contains || RangeDeps.contains). Everything stays on the device between the steps.
void recovery_deps_reduce(acc_ctx *ctx, const acc_deps_merge_in *cw, const acc_deps_merge_in *anw, acc_recovery_deps_view *view)
{
    if (!cw || !anw || !view) fail(ACC_E_ARG, "null argument");
    if (cw->n_groups != anw->n_groups) fail(ACC_E_ARG, "committed and accepted deps must cover the same recovered txns");
    acc_recovery_deps_view v{};
    {
        NsScope s(ctx, "rcw.");
        deps_merge(ctx, cw, &v.committed);
    }
    {
        NsScope s(ctx, "ran.");
        deps_merge(ctx, anw, &v.accepted_merged);
    }
    const uint32_t ng = anw->n_groups;
    const acc_rmm_view &ck = v.committed.key_deps, &cr = v.committed.range_deps;
    const acc_txn_sets sa{ ck.val_off, acc_ts_cols{ ck.txn_msb, ck.txn_lsb, ck.txn_node } };
    const acc_txn_sets sb{ cr.val_off, acc_ts_cols{ cr.txn_msb, cr.txn_lsb, cr.txn_node } };
    for (int half = 0; half < 2; ++half) {
        const acc_rmm_view &m = half ? v.accepted_merged.range_deps : v.accepted_merged.key_deps;
        acc_rmm_in h{};
        h.key_off = m.key_off; h.key_a = m.key_a; h.key_b = m.key_b; h.val_off = m.val_off;
        h.txn = acc_ts_cols{ m.txn_msb, m.txn_lsb, m.txn_node };
        h.k2v_off = m.k2v_off; h.k2v = m.k2v;
        NsScope s(ctx, half ? "rwr." : "rwk.");
        rmm_without_dev(ctx, ng, h, m.total_keys, m.total_vals, m.total_k2v, &sa, &sb,
                        half ? &v.accepted_range : &v.accepted_key);
    }
    *view = v;
}

}  // namespace acc
