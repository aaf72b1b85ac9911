// levelise.hip — execution-order levelisation of a dependency graph.
//
// A txn waits on each dependency whose executeAt is earlier than its own (Commands.updateWaitingOn drops
// the others, local/Commands.java:804-810). Deterministic restatement: level(t) = 0 without such deps,
// else 1 + max level(dep); order = txns sorted by (level, executeAt rank, index).
//
// Every counted edge goes from a lower to a higher executeAt rank, so levels are final in executeAt order.
// A persistent grid of waves walks the txns in executeAt order, one txn per wave (k_lv_waves); a dep's level is
// awaited by polling its published value.
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

// Wave-per-txn walk: every wave of a persistent grid takes tickets (positions in executeAt order) from one counter;
// for its txn, the 64 lanes read the dep list 64 at a time, keep the deps with an earlier executeAt (Commands.
// updateWaitingOn drops the others, local/Commands.java:804-810), read their published levels (level + 1, agent scope:
// the XCDs' L2s are not coherent) and re-poll the ones still unpublished, then the wave publishes 1 + max. A dep always
// has an earlier ticket, held by a running wave, so the earliest pending txn only waits on published ones and every
// wave's loop ends. The critical path is the graph's dependency depth at one memory round trip per level (~2 us:
// config 5's 709 levels in 1.5 ms); the deps of a txn are read in parallel. (A tiled variant resolving intra-tile hops
// in LDS measured 7x slower: each wave then walks its share of the tile serially at global-load latency.)
constexpr int LV_PEND = 4;   // unpublished deps a lane tracks in registers before it waits in place

__device__ __forceinline__ uint32_t lv_load(const uint32_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

__global__ __launch_bounds__(BLOCK) void k_lv_waves(uint32_t n, const uint32_t *__restrict__ order_exec, const uint64_t *__restrict__ off,
                                                    const uint32_t *__restrict__ dep, const uint32_t *__restrict__ exec_rank,
                                                    uint32_t *__restrict__ lv, uint32_t *__restrict__ ticket,
                                                    uint32_t *__restrict__ max_level)
{
    const uint32_t lane = lane_id();
    uint32_t my_max = 0;
    while (true) {
        uint32_t i = 0;
        if (lane == 0) i = atomicAdd(ticket, 1u);
        i = __shfl(i, 0, 64);
        if (i >= n) break;
        const uint32_t t = order_exec[i];
        const uint32_t er = exec_rank[t];
        const uint64_t a = off[t], b = off[t + 1];
        uint32_t l = 0;
        uint32_t pend[LV_PEND];
        uint32_t np = 0;
        for (uint64_t c = a; c < b; c += 64) {
            const uint64_t e = c + lane;
            if (e < b) {
                const uint32_t d = dep[e];
                if (exec_rank[d] < er) {
                    uint32_t v = lv_load(&lv[d]);
                    if (v) l = max(l, v);
                    else if (np < LV_PEND) {
#pragma unroll
                        for (int q = 0; q < LV_PEND; ++q) if ((uint32_t)q == np) pend[q] = d;
                        ++np;
                    } else {
                        while ((v = lv_load(&lv[d])) == 0) __builtin_amdgcn_s_sleep(1);
                        l = max(l, v);
                    }
                }
            }
        }
#pragma unroll
        for (int q = 0; q < LV_PEND; ++q) {
            if ((uint32_t)q < np) {
                uint32_t v;
                while ((v = lv_load(&lv[pend[q]])) == 0) __builtin_amdgcn_s_sleep(1);
                l = max(l, v);
            }
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) l = max(l, (uint32_t)__shfl_xor(l, d, 64));
        if (lane == 0) __hip_atomic_store(&lv[t], l + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        my_max = max(my_max, l);
    }
    if (lane == 0 && my_max) atomicMax(max_level, my_max);
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
    uint32_t *maxl = ctx->get<uint32_t>("lv_max", 4);   // [0] max level, [1] ticket counter
    ACC_HIP(hipMemsetAsync(level, 0, (size_t)n * 4, st));
    ACC_HIP(hipMemsetAsync(maxl, 0, 16, st));
    // a persistent grid of up to 4096 waves (16 per CU): enough txns in flight to cover the memory round trips
    const uint32_t waves = std::min<uint32_t>(n, 4096u);
    launch(ctx, "lv_walk", k_lv_waves, dim3((waves + WAVES - 1) / WAVES), dim3(BLOCK), 0, n, (const uint32_t *)order_exec, off, dep,
           exec_rank, level, maxl + 1, maxl);
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
