// dictionary.hip — dense order ranks of composite keys (up to three u64 words compared unsigned, most significant
// first). Used wherever the reference compares objects the device cannot hold as one machine word:
//   * TxnId / Timestamp (Timestamp.compareTo, primitives/Timestamp.java:208-217) as (msb, lsb & IDENTITY_LSB,
//     node ^ 2^31), so equal rank <=> Timestamp.equals (:244-249);
//   * Range keys of RangeDeps (Range::compare, primitives/Range.java:310-317) as (start, end);
//   * u64 key codes whose varying bits leave no room for a group field in a composite sort key.
// Each word is bit-compacted to its varying bits (order preserving); the words are sorted by one LSD radix sort over
// the concatenation when it fits 64 bits, else word by word (least significant first, stable), then runs of equal
// keys get one rank. first[r] = the smallest input index of rank r (stable sort: the first occurrence).
#include "dict.hpp"

namespace acc {

namespace {

constexpr int DMAXW = 3;

struct DWords {
    const uint64_t *w[DMAXW];
    uint64_t xor_mask[DMAXW];   // applied before compaction (sign flips of signed words), 0 = none
    uint64_t and_mask[DMAXW];   // identity masks (IDENTITY_LSB), ~0 = none
};

__device__ __forceinline__ uint64_t dword(const DWords &d, int k, size_t i)
{
    return (d.w[k][i] & d.and_mask[k]) ^ d.xor_mask[k];
}

// g[k] |= word_k(i) ^ word_k(0) over every i: the varying bits of each word
__global__ __launch_bounds__(BLOCK) void k_dict_masks(size_t n, DWords d, int nw, uint64_t *__restrict__ g)
{
    uint64_t m[DMAXW] = { 0, 0, 0 };
    uint64_t ref[DMAXW];
    for (int k = 0; k < nw; ++k) ref[k] = dword(d, k, 0);
    for (size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (size_t)gridDim.x * BLOCK)
        for (int k = 0; k < nw; ++k) m[k] |= dword(d, k, i) ^ ref[k];
    __shared__ uint64_t part[WAVES][DMAXW];
    for (int k = 0; k < DMAXW; ++k) {
        uint64_t x = m[k];
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) x |= shfl_xor(x, s);
        if (lane_id() == 0) part[threadIdx.x >> 6][k] = x;
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)nw) {
        uint64_t x = 0;
        for (int q = 0; q < WAVES; ++q) x |= part[q][threadIdx.x];
        if (x) atomicOr((unsigned long long *)&g[threadIdx.x], (unsigned long long)x);
    }
}

struct DPlan {
    Runs r[DMAXW];
    int shift[DMAXW];   // position of word k in the single composite (when it fits 64 bits)
};

// composite of every compacted word (sel < 0), or word `sel` alone, optionally gathered through perm
__global__ __launch_bounds__(BLOCK) void k_dict_compact(size_t n, DWords d, int nw, DPlan p, int sel, const uint32_t *__restrict__ perm,
                                                        uint64_t *__restrict__ out)
{
    const size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const size_t src = perm ? perm[i] : i;
    if (sel >= 0) { out[i] = pext_runs(dword(d, sel, src), p.r[sel]); return; }
    uint64_t c = 0;
    for (int k = 0; k < nw; ++k)
        if (p.r[k].bits) c |= pext_runs(dword(d, k, src), p.r[k]) << p.shift[k];
    out[i] = c;
}

// flag[i] = sorted key i differs from sorted key i-1
__global__ __launch_bounds__(BLOCK) void k_dict_flags(size_t n, const uint64_t *__restrict__ sorted_single, const uint32_t *__restrict__ perm,
                                                      DWords d, int nw, uint32_t *__restrict__ flag)
{
    const size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    uint32_t f = 1;
    if (i > 0) {
        if (sorted_single) f = sorted_single[i] != sorted_single[i - 1];
        else {
            const uint32_t a = perm[i], b = perm[i - 1];
            f = 0;
            for (int k = 0; k < nw; ++k) f |= dword(d, k, a) != dword(d, k, b);
        }
    }
    flag[i] = f;
}

__global__ __launch_bounds__(BLOCK) void k_dict_scatter(size_t n, const uint32_t *__restrict__ perm, const uint32_t *__restrict__ flag,
                                                        const uint32_t *__restrict__ incl, uint32_t *__restrict__ rank,
                                                        uint32_t *__restrict__ first, uint64_t *__restrict__ count)
{
    const size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t src = perm[i], r = incl[i] - 1;
    rank[src] = r;
    if (first && flag[i]) first[r] = src;
    if (i == n - 1) *count = incl[i];
}

}  // namespace

DenseRank dense_rank(acc_ctx *ctx, const char *tag, size_t n, int nw, const uint64_t *const *words, const uint64_t *and_mask,
                     const uint64_t *xor_mask, bool want_first)
{
    if (nw < 1 || nw > DMAXW) fail(ACC_E_STATE, "internal: dense_rank supports 1..3 words");
    if (n >= 0xFFFFFFFFull) fail(ACC_E_CAP, "dictionary too large (>= 2^32 keys)");
    hipStream_t st = ctx->stream;
    char nm[64];
    auto name = [&](const char *s) { snprintf(nm, sizeof nm, "%s.%s", tag, s); return nm; };
    DenseRank out;
    out.rank = ctx->get<uint32_t>(name("rank"), n);
    out.first = want_first ? ctx->get<uint32_t>(name("first"), n) : nullptr;
    out.count_dev = ctx->get<uint64_t>(name("count"), 1);
    if (n == 0) {
        ACC_HIP(hipMemsetAsync(out.count_dev, 0, 8, st));
        out.count = 0;
        return out;
    }
    DWords d{};
    for (int k = 0; k < DMAXW; ++k) {
        d.w[k] = k < nw ? words[k] : nullptr;
        d.and_mask[k] = (k < nw && and_mask) ? and_mask[k] : ~0ull;
        d.xor_mask[k] = (k < nw && xor_mask) ? xor_mask[k] : 0ull;
    }
    uint64_t *g = ctx->get<uint64_t>(name("masks"), DMAXW);
    ACC_HIP(hipMemsetAsync(g, 0, DMAXW * 8, st));
    launch(ctx, "dict_masks", k_dict_masks, dim3(std::min<unsigned>(grid_for(n, BLOCK), 1024u)), dim3(BLOCK), 0, n, d, nw, g);
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 32, g, DMAXW * 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    DPlan p{};
    int total = 0;
    for (int k = nw - 1; k >= 0; --k) {
        p.r[k] = make_runs(ctx->pinned[32 + k]);
        p.shift[k] = total;
        total += p.r[k].bits;
    }
    const unsigned gn = grid_for(n, BLOCK);
    uint32_t *flag = ctx->get<uint32_t>(name("flag"), n);
    uint32_t *incl = ctx->get<uint32_t>(name("incl"), n);
    const uint32_t *perm;
    if (total <= 64) {
        uint64_t *ck = ctx->get<uint64_t>(name("ckey"), n);
        launch(ctx, "dict_compact", k_dict_compact, dim3(gn), dim3(BLOCK), 0, n, d, nw, p, -1, (const uint32_t *)nullptr, ck);
        Sorted s = radix_sort(ctx, name("rs"), ck, nullptr, n, total);
        perm = s.vals;
        launch(ctx, "dict_flags", k_dict_flags, dim3(gn), dim3(BLOCK), 0, n, (const uint64_t *)s.keys, (const uint32_t *)nullptr,
               d, nw, flag);
    } else {
        // stable LSD over the words, least significant first; each pass gathers its word through the running order
        uint64_t *wk = ctx->get<uint64_t>(name("wkey"), n);
        uint32_t *pb = ctx->get<uint32_t>(name("perm"), n);
        const uint32_t *cur = nullptr;
        for (int k = nw - 1; k >= 0; --k) {
            if (!p.r[k].bits) continue;
            launch(ctx, "dict_compact", k_dict_compact, dim3(gn), dim3(BLOCK), 0, n, d, nw, p, k, cur, wk);
            Sorted s = radix_sort(ctx, name("rs"), wk, cur, n, p.r[k].bits);
            ACC_HIP(hipMemcpyAsync(pb, s.vals, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
            cur = pb;
        }
        perm = cur;
        launch(ctx, "dict_flags", k_dict_flags, dim3(gn), dim3(BLOCK), 0, n, (const uint64_t *)nullptr, perm, d, nw, flag);
    }
    scan<uint32_t, OpAdd<uint32_t>>(ctx, flag, incl, n, false);
    launch(ctx, "dict_scatter", k_dict_scatter, dim3(gn), dim3(BLOCK), 0, n, perm, (const uint32_t *)flag, (const uint32_t *)incl,
           out.rank, out.first, out.count_dev);
    out.count = ~0ull;   // on device until the caller's next sync (count_dev)
    out.perm = perm;
    return out;
}

}  // namespace acc
