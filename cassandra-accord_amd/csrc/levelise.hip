// levelise.hip — execution-order levelisation of a dependency graph.
//
// A txn waits on each dependency whose executeAt is earlier than its own (Commands.updateWaitingOn drops
// the others, local/Commands.java:804-810). Deterministic restatement: level(t) = 0 without such deps,
// else 1 + max level(dep); order = txns sorted by (level, executeAt rank, index).
//
// Every counted edge goes from a lower to a higher executeAt rank, so levels are final in executeAt order.
// One workgroup walks the txns in executeAt order (k_lv_walk); a dep's level is awaited by polling its
// published value, so the walk's length is the graph's dependency-chain depth at LDS latency.
#include "prims.hpp"

namespace acc {

__global__ __launch_bounds__(BLOCK) void k_lv_keys(uint32_t n, const uint32_t *__restrict__ exec_rank, uint64_t *__restrict__ key)
{
    uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t < n) key[t] = exec_rank[t];
}

__global__ __launch_bounds__(BLOCK) void k_lv_check(uint32_t n, const uint64_t *__restrict__ off, const uint32_t *__restrict__ dep,
                                                    uint32_t *__restrict__ err)
{
    uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= n) return;
    uint64_t a = off[t], b = off[t + 1];
    if (b < a) { atomicOr(err, 1u); return; }
    for (uint64_t e = a; e < b; ++e)
        if (dep[e] >= n) { atomicOr(err, 2u); return; }
}

// One workgroup of LV_THREADS lanes; lane j owns the txns at exec-order positions j, j + LV_THREADS, ... and
// walks them in that order. Per txn it advances a cursor over the txn's deps: deps with exec rank >= its own
// are skipped; a counted dep whose level is still unpublished (0) stops the cursor and the lane polls it again
// on its next iteration (no barrier: lanes and waves progress independently). The txn at the earliest
// pending position only depends on published txns, so the walk always advances and every lane's loop ends.
// Published value = level + 1, indexed by txn. kLds: the level and exec-rank columns (8 B per txn) live in
// LDS (n <= LV_LDS_MAX); otherwise levels are global (agent-scope atomics bypass the non-coherent L1) and
// exec ranks are read from global.
constexpr int LV_THREADS = 1024;
constexpr int LV_UNROLL = 4;
constexpr uint32_t LV_LDS_MAX = 20000;   // 8 B/txn of the 160 KiB LDS

template <bool kLds>
__global__ __launch_bounds__(LV_THREADS) void k_lv_walk(uint32_t n, const uint32_t *__restrict__ order_exec,
                                                        const uint64_t *__restrict__ off, const uint32_t *__restrict__ dep,
                                                        const uint32_t *__restrict__ exec_rank, uint32_t *__restrict__ level_g,
                                                        uint32_t *__restrict__ max_level)
{
    extern __shared__ uint32_t lds[];
    uint32_t *lv = kLds ? lds : level_g;             // level + 1 per txn, 0 = pending
    const uint32_t *er_col = kLds ? lds + n : exec_rank;
    if (kLds) {
        for (uint32_t t = threadIdx.x; t < n; t += LV_THREADS) { lds[t] = 0; lds[n + t] = exec_rank[t]; }
        __syncthreads();
    }
    auto ld = [&](uint32_t d) -> uint32_t {
        if (kLds) return __hip_atomic_load(&lv[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return __hip_atomic_load(&lv[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    uint32_t my_max = 0;
    uint32_t i = threadIdx.x;
    uint32_t t = 0, er = 0, l = 0;
    uint64_t cur = 0, b = 0;
    if (i < n) { t = order_exec[i]; er = er_col[t]; cur = off[t]; b = off[t + 1]; }
    while (__any(i < n)) {
        if (i < n) {
            bool pending = false;
            // LV_UNROLL deps per round: independent global loads in flight together
            while (cur < b && !pending) {
                uint32_t dd[LV_UNROLL];
#pragma unroll
                for (int q = 0; q < LV_UNROLL; ++q) dd[q] = cur + q < b ? dep[cur + q] : 0xFFFFFFFFu;
#pragma unroll
                for (int q = 0; q < LV_UNROLL; ++q) {
                    if (pending || dd[q] == 0xFFFFFFFFu) continue;
                    if (er_col[dd[q]] >= er) { ++cur; continue; }
                    uint32_t v = ld(dd[q]);
                    if (v == 0) { pending = true; continue; }
                    l = max(l, v);           // v = level(dep) + 1
                    ++cur;
                }
            }
            if (!pending) {
                if (kLds) __hip_atomic_store(&lv[t], l + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                else __hip_atomic_store(&lv[t], l + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                my_max = max(my_max, l);
                i += LV_THREADS;
                l = 0;
                if (i < n) { t = order_exec[i]; er = er_col[t]; cur = off[t]; b = off[t + 1]; }
            }
        }
    }
    __syncthreads();
    if (kLds)
        for (uint32_t u = threadIdx.x; u < n; u += LV_THREADS) level_g[u] = lds[u];
    // block max of levels -> n_levels - 1
    __shared__ uint32_t red[LV_THREADS / 64];
    uint32_t v = my_max;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t m = 0;
        for (int q = 0; q < LV_THREADS / 64; ++q) m = max(m, red[q]);
        *max_level = m;
    }
}

// published level + 1 -> level
__global__ __launch_bounds__(BLOCK) void k_lv_unbias(uint32_t n, uint32_t *__restrict__ level)
{
    uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t < n) level[t] -= 1;
}

__global__ __launch_bounds__(BLOCK) void k_lv_pos(uint32_t n, const uint32_t *__restrict__ order_exec, uint32_t *__restrict__ pos)
{
    uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) pos[order_exec[i]] = i;
}

// order key: (level, executeAt position) -- the exec-order position is already (exec rank, index) stable
__global__ __launch_bounds__(BLOCK) void k_lv_order_keys(uint32_t n, const uint32_t *__restrict__ level, const uint32_t *__restrict__ pos,
                                                         int pbits, uint64_t *__restrict__ key)
{
    uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t < n) key[t] = ((uint64_t)level[t] << pbits) | pos[t];
}

void levelise(acc_ctx *ctx, const acc_graph_in *in, uint32_t *level_out, uint32_t *order_out, uint32_t *n_levels)
{
    if (!in || !level_out || !order_out) fail(ACC_E_ARG, "null argument");
    if (in->mem != ACC_MEM_HOST && in->mem != ACC_MEM_DEVICE) fail(ACC_E_ARG, "mem must be ACC_MEM_HOST or ACC_MEM_DEVICE");
    const uint32_t n = in->n;
    hipStream_t st = ctx->stream;
    if (n == 0) { if (n_levels) *n_levels = 0; return; }
    const uint64_t *off = stage_in(ctx, "lv_off", in->off, (size_t)n + 1, in->mem);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, off + n, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t E = ctx->pinned[0];
    const uint32_t *dep = stage_in(ctx, "lv_dep", in->dep, E, in->mem);
    const uint32_t *exec_rank = stage_in(ctx, "lv_exec", in->exec_rank, n, in->mem);
    uint32_t *err = ctx->get<uint32_t>("lv_err", 4);
    ACC_HIP(hipMemsetAsync(err, 0, 16, st));
    launch(ctx, "lv_check", k_lv_check, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, off, dep, err);
    uint64_t *key = ctx->get<uint64_t>("lv_key", n);
    launch(ctx, "lv_keys", k_lv_keys, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, exec_rank, key);
    Sorted se = radix_sort(ctx, "lv_rs_exec", key, nullptr, n, 32);
    uint32_t *order_exec = ctx->get<uint32_t>("lv_order_exec", n);
    ACC_HIP(hipMemcpyAsync(order_exec, se.vals, (size_t)n * 4, hipMemcpyDeviceToDevice, st));
    uint32_t *pos = ctx->get<uint32_t>("lv_pos", n);
    launch(ctx, "lv_pos", k_lv_pos, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint32_t *)order_exec, pos);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, err, 4, hipMemcpyDeviceToHost, st));
    ctx->sync();
    uint32_t e0;
    memcpy(&e0, ctx->pinned, 4);
    if (e0 & 1) fail(ACC_E_ARG, "graph offsets must be non-decreasing");
    if (e0 & 2) fail(ACC_E_ARG, "dependency index out of range");
    uint32_t *level = ctx->get<uint32_t>("lv_level", n);
    uint32_t *maxl = ctx->get<uint32_t>("lv_max", 4);
    if (n <= LV_LDS_MAX) {
        const size_t lds = (size_t)n * 8;
        if (lds > 64 * 1024)
            ACC_HIP(hipFuncSetAttribute((const void *)k_lv_walk<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        launch(ctx, "lv_walk", k_lv_walk<true>, dim3(1), dim3(LV_THREADS), lds, n, (const uint32_t *)order_exec, off, dep,
               exec_rank, level, maxl);
    } else {
        ACC_HIP(hipMemsetAsync(level, 0, (size_t)n * 4, st));
        launch(ctx, "lv_walk", k_lv_walk<false>, dim3(1), dim3(LV_THREADS), 0, n, (const uint32_t *)order_exec, off, dep,
               exec_rank, level, maxl);
    }
    launch(ctx, "lv_unbias", k_lv_unbias, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, level);
    const int pbits = bits_for(n - 1);
    launch(ctx, "lv_order_keys", k_lv_order_keys, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint32_t *)level,
           (const uint32_t *)pos, pbits, key);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, maxl, 4, hipMemcpyDeviceToHost, st));
    ctx->sync();
    uint32_t ml;
    memcpy(&ml, ctx->pinned, 4);
    Sorted so = radix_sort(ctx, "lv_rs_order", key, nullptr, n, pbits + bits_for(ml));
    hipMemcpyKind kind = in->mem == ACC_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    ACC_HIP(hipMemcpyAsync(level_out, level, (size_t)n * 4, kind, st));
    ACC_HIP(hipMemcpyAsync(order_out, so.vals, (size_t)n * 4, kind, st));
    ctx->sync();
    if (n_levels) *n_levels = ml + 1;
}

}  // namespace acc
