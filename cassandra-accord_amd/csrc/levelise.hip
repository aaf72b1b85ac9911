// levelise.hip — execution-order levelisation of a dependency graph.
//
// A txn waits on each dependency whose executeAt is earlier than its own (Commands.updateWaitingOn drops
// the others, local/Commands.java:804-810). Deterministic restatement: level(t) = 0 without such deps,
// else 1 + max level(dep); order = txns sorted by (level, executeAt rank, index).
//
// Every counted edge goes from a lower to a higher executeAt rank, so levels are final in executeAt order.
// One workgroup walks the txns in executeAt order in windows of LV_WIN: each thread owns one txn; deps in
// earlier windows are final in global memory; deps inside the window are waited for through LDS (level+1,
// 0 = pending). The earliest pending txn of a window only depends on finished txns, so every spin round
// retires at least one txn: the wait is bounded by the window's dependency-chain depth, at LDS latency.
#include "prims.hpp"

namespace acc {

constexpr int LV_WIN = 1024;

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

__global__ __launch_bounds__(1024) void k_lv_walk(uint32_t n, const uint32_t *__restrict__ order_exec, const uint32_t *__restrict__ pos,
                                                  const uint64_t *__restrict__ off, const uint32_t *__restrict__ dep,
                                                  const uint32_t *__restrict__ exec_rank, uint32_t *__restrict__ level,
                                                  uint32_t *__restrict__ max_level)
{
    __shared__ uint32_t win[LV_WIN];
    uint32_t my_max = 0;
    for (uint32_t w0 = 0; w0 < n; w0 += LV_WIN) {
        const uint32_t slot = threadIdx.x;
        const uint32_t i = w0 + slot;
        win[slot] = 0;
        __syncthreads();
        bool active = i < n;
        uint32_t t = 0, er = 0, base = 0;   // base: 1 + max level of deps in earlier windows (0 = none)
        uint64_t a = 0, b = 0;
        if (active) {
            t = order_exec[i];
            er = exec_rank[t];
            a = off[t]; b = off[t + 1];
            for (uint64_t e = a; e < b; ++e) {
                uint32_t d = dep[e];
                if (exec_rank[d] >= er) continue;
                uint32_t pd = pos[d];
                if (pd < w0) base = max(base, level[d] + 1);
            }
        }
        bool done = !active;
        // spin until every in-window dep has published its level
        while (__syncthreads_or(!done)) {
            if (!done) {
                uint32_t l = base;
                bool ready = true;
                for (uint64_t e = a; e < b && ready; ++e) {
                    uint32_t d = dep[e];
                    if (exec_rank[d] >= er) continue;
                    uint32_t pd = pos[d];
                    if (pd < w0) continue;
                    uint32_t v = __hip_atomic_load(&win[pd - w0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (v == 0) ready = false;
                    else l = max(l, v);           // v = level(d) + 1
                }
                if (ready) {
                    level[t] = l;                  // level = 1 + max dep level (0 without deps)
                    __hip_atomic_store(&win[slot], l + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    my_max = max(my_max, l);
                    done = true;
                }
            }
        }
        __syncthreads();
    }
    // block max of levels -> n_levels - 1
    __shared__ uint32_t red[16];
    uint32_t v = my_max;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t m = 0;
        for (int q = 0; q < 16; ++q) m = max(m, red[q]);
        *max_level = m;
    }
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
    launch(ctx, "lv_walk", k_lv_walk, dim3(1), dim3(1024), 0, n, (const uint32_t *)order_exec, (const uint32_t *)pos, off, dep,
           exec_rank, level, maxl);
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
