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

#include <cstdio>
#include <vector>

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
#ifndef ACC_LV_PEND
#define ACC_LV_PEND 4
#endif
constexpr int LV_PEND = ACC_LV_PEND;   // unpublished deps a lane tracks in registers

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

// ---- LDS tier (n <= LV_LDS_MAX_N): one 1024-thread workgroup walks the whole graph with every level in LDS, so a
// dependency hop costs an LDS round trip instead of a cross-XCD memory round trip (~2 us per level above).
//
// 1. k_lv_fcount / k_lv_fwrite (whole GPU, wave per exec-order position i): the waiting deps of txn order_exec[i]
//    (exec rank below its own, Commands.java:804-810) as their exec-order positions, u16, in exec order: a CSR
//    (foff, fdep) the walker streams front to back.
// 2. k_lv_lds: fdep is consumed in chunks of CH entries; round c walks the positions whose lists end in chunk c
//    (rstart[c] .. rstart[c+1]) while chunk c+1 is in flight into registers, then stored to LDS (three chunk slots:
//    a list of <= CH entries spans chunks c-1 and c; longer lists are read from HBM). Group g (16 lanes) of the
//    workgroup takes positions rstart[c] + g + 64 j; a wave's four groups advance together and re-read their deps'
//    levels until every one is published, which always terminates: the smallest unfinished position has all of its
//    deps finished and its wave is on it.
constexpr int LV_LDS = 69632;          // u16 slots of LDS: levels (level + 1, 0 = unpublished) + three chunk slots
constexpr int LV_FB = 2048;            // foff entries of a round staged in LDS (x2 buffers); beyond: read from HBM
constexpr uint32_t LV_LDS_MAX_N = 65535;
constexpr int LV_NT = 1024;
#ifndef ACC_LV_G
#define ACC_LV_G 16
#endif
constexpr int LV_G = ACC_LV_G;         // lanes per position (16: one DPP row)
constexpr uint32_t LV_CH_MAX = 16384;  // entries per chunk
constexpr int LV_PF = LV_CH_MAX / 8 / LV_NT;   // uint4 of a chunk per thread

// also the graph validation of k_lv_check (the LDS tier skips that pass): err |= 1 decreasing offsets, 2 a dep >= n
__global__ __launch_bounds__(BLOCK) void k_lv_fcount(uint32_t n, const uint32_t *__restrict__ order_exec,
                                                     const uint64_t *__restrict__ off, const uint32_t *__restrict__ dep,
                                                     const uint32_t *__restrict__ exec_rank, uint32_t *__restrict__ cnt,
                                                     uint32_t *__restrict__ err)
{
    const uint32_t i = blockIdx.x * WAVES + (threadIdx.x >> 6), lane = lane_id();
    if (i >= n) return;
    const uint32_t t = order_exec[i], er = exec_rank[t];
    const uint64_t a = off[t], b = off[t + 1];
    if (b < a && lane == 0) atomicOr(err, 1u);
    uint32_t c = 0;
    for (uint64_t e = a + lane; e < b; e += 64) {
        const uint32_t d = dep[e];
        if (d >= n) { atomicOr(err, 2u); continue; }
        c += exec_rank[d] < er;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
    if (lane == 0) cnt[i] = c;
}

__global__ __launch_bounds__(BLOCK) void k_lv_fwrite(uint32_t n, const uint32_t *__restrict__ order_exec,
                                                     const uint64_t *__restrict__ off, const uint32_t *__restrict__ dep,
                                                     const uint32_t *__restrict__ exec_rank, const uint32_t *__restrict__ pos,
                                                     const uint32_t *__restrict__ foff, uint16_t *__restrict__ fdep,
                                                     const uint32_t *__restrict__ err)
{
    const uint32_t i = blockIdx.x * WAVES + (threadIdx.x >> 6), lane = lane_id();
    if (i >= n || *err) return;   // an invalid graph (k_lv_fcount): its counts may exceed fdep, write nothing
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const uint32_t t = order_exec[i], er = exec_rank[t];
    const uint64_t a = off[t], b = off[t + 1];
    uint32_t w = foff[i];
    for (uint64_t c0 = a; c0 < b; c0 += 64) {
        const uint64_t e = c0 + lane;
        uint32_t d = 0;
        bool keep = false;
        if (e < b) { d = dep[e]; keep = d < n && exec_rank[d] < er; }
        const uint64_t bal = __ballot(keep);
        if (keep) fdep[w + (uint32_t)__popcll(bal & lt)] = (uint16_t)pos[d];
        w += (uint32_t)__popcll(bal);
    }
}

// rstart[c] = first position whose list ends in chunk >= c (lists ending at entry 0 count as chunk 0); rstart[R] = n
__device__ __forceinline__ uint32_t lv_rounds_of(uint32_t Ef, int ch_shift)
{
    return max(1u, (uint32_t)(((uint64_t)Ef + (1u << ch_shift) - 1) >> ch_shift));
}

__global__ __launch_bounds__(BLOCK) void k_lv_rounds(uint32_t n, int ch_shift, const uint32_t *__restrict__ foff,
                                                     uint32_t *__restrict__ rstart, const uint32_t *__restrict__ err)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n || *err) return;
    const uint32_t R = lv_rounds_of(foff[n], ch_shift);
    auto round_of = [&](uint32_t j) { const uint32_t e = foff[j + 1]; return e == 0 ? 0u : (e - 1) >> ch_shift; };
    const uint32_t r = round_of(i);
    const uint32_t rp = i == 0 ? 0u : round_of(i - 1) + 1;
    for (uint32_t c = i == 0 ? 0u : rp; c <= r; ++c) rstart[c] = i;
    if (i == n - 1)
        for (uint32_t c = r + 1; c <= R; ++c) rstart[c] = n;
}

// max over the 16 lanes of a DPP row (row_ror 1, 2, 4, 8): every lane of the row gets it, no LDS round trips
__device__ __forceinline__ uint32_t row_max16(uint32_t x)
{
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x121, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x122, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x124, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x128, 0xF, 0xF, false));
    return x;
}

#ifdef ACC_LV_PROF
// tuning build only: per wave, cycles in the walk loops, waiting at the round barriers, and first-scan passes
__device__ unsigned long long *g_lv_prof;
#endif

__device__ __forceinline__ uint32_t lv_lds_ld(const uint16_t *p) { return *(const volatile uint16_t *)p; }

__global__ __launch_bounds__(LV_NT) void k_lv_lds(uint32_t n, uint32_t npad, int ch_shift,
                                                  const uint32_t *__restrict__ foff, const uint16_t *__restrict__ fdep,
                                                  const uint32_t *__restrict__ rstart, const uint32_t *__restrict__ order_exec,
                                                  uint32_t *__restrict__ level, uint32_t *__restrict__ max_level,
                                                  const uint32_t *__restrict__ err)
{
    if (*err) return;   // invalid graph: the lists were not written (the host fails after the walk)
    const uint32_t Ef = foff[n], R = lv_rounds_of(Ef, ch_shift);   // sizes stay on the device (no host round trip)
    __shared__ __attribute__((aligned(16))) uint16_t L[LV_LDS];
    __shared__ uint32_t fb[2][LV_FB];   // foff of the round's positions (double-buffered)
    const uint32_t CH = 1u << ch_shift;
    uint16_t *lvl = L, *slots = L + npad;
    const uint32_t tid = threadIdx.x, lane = lane_id(), sub = lane & (LV_G - 1), gi = lane / LV_G;
    for (uint32_t i = tid; i < n; i += LV_NT) lvl[i] = 0;
    // chunk c -> slot c % 3: CH / 8 uint4 of fdep (reads may run past Ef into the buffer's padding)
    const uint32_t nv = CH / 8;
    const uint4 *src4 = reinterpret_cast<const uint4 *>(fdep);
    uint4 *dst4 = reinterpret_cast<uint4 *>(slots);
    if (Ef) for (uint32_t v = tid; v < nv; v += LV_NT) dst4[v] = src4[v];
    uint32_t r0 = rstart[0], r1 = R >= 1 ? rstart[1] : n, r2 = R >= 2 ? rstart[2] : n;
    for (uint32_t v = tid; v < LV_FB && r0 + v <= r1; v += LV_NT) fb[0][v] = foff[r0 + v];
    __syncthreads();
    uint32_t my_max = 0;
#ifdef ACC_LV_PROF
    unsigned long long prof_walk = 0, prof_wait = 0, prof_pass = 0;
#endif
    for (uint32_t c = 0; c < R; ++c) {
        // in flight during the walk: chunk c + 1 of fdep, foff of round c + 1, rstart[c + 3]
        static_assert(LV_PF == 2 && LV_FB == 2 * LV_NT, "two prefetch slots per thread");
        uint4 pf0 = {}, pf1 = {};
        uint32_t pfo0 = 0, pfo1 = 0;
        const bool pfc = (uint64_t)(c + 1) * CH < Ef;
        const uint4 *nsrc = src4 + (size_t)(c + 1) * nv;
        if (pfc && tid < nv) pf0 = nsrc[tid];
        if (pfc && tid + LV_NT < nv) pf1 = nsrc[tid + LV_NT];
        const bool pfr = c + 1 < R;
        if (pfr && r1 + tid <= r2) pfo0 = foff[r1 + tid];
        if (pfr && r1 + tid + LV_NT <= r2) pfo1 = foff[r1 + tid + LV_NT];
        const uint32_t r3 = c + 3 <= R ? rstart[c + 3] : n;
        const uint32_t p0 = r0, p1 = r1;
        const uint32_t *fo = fb[c & 1];
        // list entries of this round: chunk c (slot c % 3) and chunk c - 1 (slot (c + 2) % 3) are resident; a list
        // longer than a chunk may start before them and reads those entries from HBM
        const uint32_t cur0 = c * CH, prv0 = c == 0 ? 0u : (c - 1) * CH;
        const uint16_t *scur = slots + (size_t)(c % 3) * CH, *sprv = slots + (size_t)((c + 2) % 3) * CH;
#ifdef ACC_LV_PROF
        const unsigned long long t_a = clock64();
#endif
        constexpr uint32_t GPW = 64 / LV_G;   // positions per wave
        for (uint32_t base = p0 + GPW * (tid >> 6); base < p1; base += LV_NT / LV_G) {
            // wave w holds positions base + {0 .. GPW - 1}; the waves stride by LV_NT / LV_G positions (a static
            // split measured faster than claiming positions through an LDS counter)
            const uint32_t i = base + gi;
            const bool valid = i < p1;
            uint32_t a = 0, b = 0;
            if (valid) {
                const uint32_t k = i - p0;
                if (k + 1 < LV_FB) { a = fo[k]; b = fo[k + 1]; }
                else { a = foff[i]; b = foff[i + 1]; }
            }
            bool done = !valid;
            // first pass: every entry once (four LDS loads in flight per lane); deps still unpublished are kept in
            // registers (up to LV_PEND per lane) and later passes re-read only those, so a dependency hop costs one
            // LDS round trip, not a re-scan of the list
            uint32_t m = 0, np = 0, pend[LV_PEND];
            bool ovf = false, scanned = false;
#pragma unroll
            for (int q = 0; q < LV_PEND; ++q) pend[q] = 0;
            while (true) {
                if (!done) {   // group-uniform
                    if (!scanned || ovf) {
                        m = 0; np = 0; ovf = false;
                        for (uint32_t e0 = a + sub; e0 < b; e0 += 4 * LV_G) {
                            uint32_t p[4], v[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                const uint32_t e = e0 + (uint32_t)u * LV_G;
                                p[u] = 0;
                                if (e < b) p[u] = e >= cur0 ? scur[e - cur0] : e >= prv0 ? sprv[e - prv0] : (uint32_t)fdep[e];
                            }
                            // the first pass uses plain loads (batched by the compiler; a stale 0 only marks the dep
                            // pending), every re-read is volatile
#pragma unroll
                            for (int u = 0; u < 4; ++u)
                                v[u] = e0 + (uint32_t)u * LV_G >= b ? 0u : scanned ? lv_lds_ld(&lvl[p[u]]) : (uint32_t)lvl[p[u]];
                            bool z = false;
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                if (e0 + (uint32_t)u * LV_G >= b) continue;
                                m = max(m, v[u]);
                                z |= v[u] == 0;
                            }
                            if (z) {   // rare: keep the unpublished deps for the retries
#pragma unroll
                                for (int u = 0; u < 4; ++u) {
                                    if (e0 + (uint32_t)u * LV_G >= b || v[u]) continue;
#pragma unroll
                                    for (int q = 0; q < LV_PEND; ++q) if ((uint32_t)q == np) pend[q] = p[u];
                                    if (np < LV_PEND) ++np; else ovf = true;
                                }
                            }
                        }
                        scanned = true;
                    } else if (np) {
                        uint32_t keep[LV_PEND], nk = 0;
#pragma unroll
                        for (int q = 0; q < LV_PEND; ++q) keep[q] = (uint32_t)q < np ? lv_lds_ld(&lvl[pend[q]]) : 0u;
#pragma unroll
                        for (int q = 0; q < LV_PEND; ++q) {
                            if ((uint32_t)q >= np) continue;
                            if (keep[q]) { m = max(m, keep[q]); continue; }
#pragma unroll
                            for (int r = 0; r < LV_PEND; ++r) if ((uint32_t)r == nk) pend[r] = pend[q];
                            ++nk;
                        }
                        np = nk;
                    }
                    // group (= one 16-lane DPP row) max of the levels, pending flag in bit 16
                    uint32_t mm = (m & 0xFFFFu) | ((np || ovf) ? 0x10000u : 0u);
                    if constexpr (LV_G == 16) mm = row_max16(mm);
                    else {
#pragma unroll
                        for (int d = 1; d < LV_G; d <<= 1) mm = max(mm, (uint32_t)__shfl_xor(mm, d, 64));
                    }
                    const uint32_t pd = mm >> 16;
                    mm &= 0xFFFFu;
                    if (!pd) {
                        if (sub == 0) *(volatile uint16_t *)&lvl[i] = (uint16_t)(mm + 1);
                        my_max = max(my_max, mm);
                        done = true;
                    }
                }
#ifdef ACC_LV_PROF
                ++prof_pass;
#endif
                if (__all(done)) break;
            }
        }
#ifdef ACC_LV_PROF
        const unsigned long long t_b = clock64();
#endif
        uint4 *ndst = dst4 + (size_t)((c + 1) % 3) * nv;
        if (pfc && tid < nv) ndst[tid] = pf0;
        if (pfc && tid + LV_NT < nv) ndst[tid + LV_NT] = pf1;
        if (pfr && r1 + tid <= r2) fb[(c + 1) & 1][tid] = pfo0;
        if (pfr && r1 + tid + LV_NT <= r2) fb[(c + 1) & 1][tid + LV_NT] = pfo1;
        r0 = r1; r1 = r2; r2 = r3;
        __syncthreads();
#ifdef ACC_LV_PROF
        if (lane == 0) {
            prof_walk += t_b - t_a;
            prof_wait += clock64() - t_b;
        }
#endif
    }
#ifdef ACC_LV_PROF
    const uint32_t wave = tid >> 6;
    if (lane == 0) { g_lv_prof[3 * wave] = prof_walk; g_lv_prof[3 * wave + 1] = prof_wait; g_lv_prof[3 * wave + 2] = prof_pass; }
#endif
    for (uint32_t i = tid; i < n; i += LV_NT) level[order_exec[i]] = (uint32_t)lvl[i] - 1u;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) my_max = max(my_max, (uint32_t)__shfl_xor(my_max, d, 64));
    if (lane == 0 && my_max) atomicMax(max_level, my_max);
}

// ---- windowed tier (default): the exec order cut into windows of LW positions. A dep of position i is "far" when it
// lies two or more windows back, "prev" when it lies in the window before i's, "cur" in i's own window. One launch per
// window w: block 0 walks window w with one lane per position, the window's levels and its cur lists (u16 window
// offsets) in LDS, so a dependency hop inside the window is an LDS round trip; the prev deps are final in HBM and read
// once; meanwhile blocks 1.. reduce the far deps of window w + 1 (all in windows <= w - 1, final before this launch)
// to one max per position on the rest of the GPU. The single-CU walk thus reads only the cur deps from LDS (config 5:
// ~13% of the 2.5M filtered edges) instead of every list. Published levels are level + 1 (0 = unpublished); the walk
// of a window ends when every lane has published, which always happens: the smallest unfinished position's cur deps
// are all earlier positions, already published.
constexpr uint32_t LW = 1024;          // positions per window = walker threads
constexpr uint32_t LW_GW = LW / 64;    // gatherer waves per 1024-thread block (one wave per position)
constexpr uint32_t LW_CL = 61440;      // cur-list entries of a window held in LDS (u16; beyond: read from HBM)

// per position: far / prev / cur dep counts (waiting deps only: exec rank below its own, Commands.java:804-810); also
// the graph validation (err |= 1 decreasing offsets, 2 a dep >= n)
__global__ __launch_bounds__(BLOCK) void k_lw_count(uint32_t n, const uint32_t *__restrict__ order_exec,
                                                    const uint64_t *__restrict__ off, const uint32_t *__restrict__ dep,
                                                    const uint32_t *__restrict__ exec_rank, const uint32_t *__restrict__ pos,
                                                    uint64_t *__restrict__ cnt_far, uint64_t *__restrict__ cnt_prev,
                                                    uint64_t *__restrict__ cnt_cur, uint32_t *__restrict__ err)
{
    const uint32_t i = blockIdx.x * WAVES + (threadIdx.x >> 6), lane = lane_id();
    if (i >= n) return;
    const uint32_t t = order_exec[i], er = exec_rank[t], wi = i / LW;
    const uint64_t a = off[t], b = off[t + 1];
    if (b < a && lane == 0) atomicOr(err, 1u);
    uint32_t cf = 0, cp = 0, cc = 0;
    for (uint64_t e = a + lane; e < b; e += 64) {
        const uint32_t d = dep[e];
        if (d >= n) { atomicOr(err, 2u); continue; }
        if (exec_rank[d] >= er) continue;
        const uint32_t wd = pos[d] / LW;
        if (wd == wi) ++cc; else if (wd + 1 == wi) ++cp; else ++cf;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        cf += __shfl_xor(cf, d, 64); cp += __shfl_xor(cp, d, 64); cc += __shfl_xor(cc, d, 64);
    }
    if (lane == 0) { cnt_far[i] = cf; cnt_prev[i] = cp; cnt_cur[i] = cc; }
}

// the far and prev lists (exec-order positions, u32) and the cur lists (offsets in the window, u16), in exec order
__global__ __launch_bounds__(BLOCK) void k_lw_write(uint32_t n, const uint32_t *__restrict__ order_exec,
                                                    const uint64_t *__restrict__ off, const uint32_t *__restrict__ dep,
                                                    const uint32_t *__restrict__ exec_rank, const uint32_t *__restrict__ pos,
                                                    const uint64_t *__restrict__ foff, const uint64_t *__restrict__ poff,
                                                    const uint64_t *__restrict__ coff, uint32_t *__restrict__ far,
                                                    uint32_t *__restrict__ prev, uint16_t *__restrict__ cur,
                                                    const uint32_t *__restrict__ err)
{
    const uint32_t i = blockIdx.x * WAVES + (threadIdx.x >> 6), lane = lane_id();
    if (i >= n || *err) return;   // an invalid graph (k_lw_count): its counts may exceed the lists, write nothing
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const uint32_t t = order_exec[i], er = exec_rank[t], wi = i / LW;
    const uint64_t a = off[t], b = off[t + 1];
    uint64_t wf = foff[i], wp = poff[i], wc = coff[i];
    for (uint64_t c0 = a; c0 < b; c0 += 64) {
        const uint64_t e = c0 + lane;
        uint32_t p = 0, wd = 0;
        bool keep = false;
        if (e < b) {
            const uint32_t d = dep[e];
            if (d < n && exec_rank[d] < er) { p = pos[d]; wd = p / LW; keep = true; }
        }
        const bool kc = keep && wd == wi, kp = keep && wd + 1 == wi, kf = keep && !kc && !kp;
        const uint64_t bf = __ballot(kf), bp = __ballot(kp), bc = __ballot(kc);
        if (kf) far[wf + (uint64_t)__popcll(bf & lt)] = p;
        if (kp) prev[wp + (uint64_t)__popcll(bp & lt)] = p;
        if (kc) cur[wc + (uint64_t)__popcll(bc & lt)] = (uint16_t)(p - wi * LW);
        wf += (uint64_t)__popcll(bf); wp += (uint64_t)__popcll(bp); wc += (uint64_t)__popcll(bc);
    }
}


struct LwLists {
    const uint64_t *foff, *poff, *coff;
    const uint32_t *far, *prev;
    const uint16_t *cur;
};

// The in-window walk with a pending set (both windowed walks, many deps per position): a lane scans its cur list 8
// entries per round once, folding the published levels and keeping up to LW_PEND unpublished entries in registers, then
// polls only the first pending entry (one LDS load per round) until it is published. A wave spinning on a chain thus
// issues one LDS load per round instead of re-reading a batch (the sliding cursor: 16 LDS loads per lane and round,
// which made the LDS the bottleneck of every hop). More than LW_PEND unpublished entries in a batch: the scan stops at
// the first one that does not fit and resumes there once the pending set is drained.
constexpr int LW_PEND = 4;
template <typename LT, typename CurAt>
__device__ __forceinline__ void lw_walk_pend(bool valid, uint64_t ca, uint64_t cb, uint32_t &m, LT *Lw, uint32_t slot,
                                             CurAt cur_at)
{
    constexpr int B = 8;
    uint64_t e = ca;
    uint32_t pend[LW_PEND];
    uint32_t np = 0;
#pragma unroll
    for (int q = 0; q < LW_PEND; ++q) pend[q] = 0;
    bool done = !valid;
    while (true) {
        if (!done) {
            if (np) {
                const uint32_t v = *(const volatile LT *)&Lw[pend[0]];
                if (v) {
                    m = max(m, v);
#pragma unroll
                    for (int q = 0; q + 1 < LW_PEND; ++q) pend[q] = pend[q + 1];
                    --np;
                }
            } else {
                uint32_t p[B], v[B];
#pragma unroll
                for (int q = 0; q < B; ++q) p[q] = e + q < cb ? cur_at(e + q) : 0xFFFFFFFFu;
#pragma unroll
                for (int q = 0; q < B; ++q) v[q] = p[q] == 0xFFFFFFFFu ? 1u : (uint32_t)*(const volatile LT *)&Lw[p[q]];
                uint32_t adv = 0;
                bool stop = false;
#pragma unroll
                for (int q = 0; q < B; ++q) {
                    if (stop || p[q] == 0xFFFFFFFFu) continue;
                    if (v[q]) { m = max(m, v[q]); ++adv; continue; }
                    if (np == LW_PEND) { stop = true; continue; }
#pragma unroll
                    for (int r = 0; r < LW_PEND; ++r) if ((uint32_t)r == np) pend[r] = p[q];
                    ++np;
                    ++adv;
                }
                e += adv;
            }
            if (!np && e >= cb) { *(volatile LT *)&Lw[slot] = (LT)(m + 1); done = true; }
        }
        if (__all(done)) break;
    }
}

// one window step (launch w): block 0 walks window w (the pending-set walk), blocks 1.. gather the far maxima of
// window w + 1
__global__ __launch_bounds__(LW) void k_lw_step(uint32_t n, uint32_t w, LwLists g, uint32_t *__restrict__ base,
                                                uint32_t *__restrict__ lvlp, const uint32_t *__restrict__ order_exec,
                                                uint32_t *__restrict__ level, uint32_t *__restrict__ max_level,
                                                const uint32_t *__restrict__ err)
{
    const uint32_t tid = threadIdx.x, lane = lane_id();
    if (*err) return;   // invalid graph: the lists were not written (the host fails after the walk)
    if (blockIdx.x > 0) {
        // gatherer: a wave per position of window w + 1, max of the far deps' published levels (0 = no far dep)
        const uint32_t j = (w + 1) * LW + (blockIdx.x - 1) * LW_GW + (tid >> 6);
        if (j >= n || w + 1 < 2) return;
        const uint64_t a = g.foff[j], b = g.foff[j + 1];
        uint32_t m = 0;
        for (uint64_t e = a + lane; e < b; e += 4 * 64) {
            uint32_t v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) { const uint64_t q = e + (uint64_t)u * 64; v[u] = q < b ? lvlp[g.far[q]] : 0u; }
#pragma unroll
            for (int u = 0; u < 4; ++u) m = max(m, v[u]);
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) m = max(m, (uint32_t)__shfl_xor(m, d, 64));
        if (lane == 0) base[j] = m;
        return;
    }
    __shared__ uint32_t L[LW];
    __shared__ uint16_t CL[LW_CL];
    __shared__ uint32_t red[LW / 64];
#ifdef ACC_LV_PROF
    const unsigned long long t_0 = clock64();
#endif
    const uint32_t w0 = w * LW, wend = min(n, w0 + LW), i = w0 + tid;
    const bool valid = i < n;
    // the window's cur lists (contiguous in exec order) into LDS
    const uint64_t cbase = g.coff[w0], ctot = g.coff[wend] - cbase;
    const uint32_t cin = (uint32_t)min<uint64_t>(ctot, LW_CL);
    for (uint32_t e = tid; e < cin; e += LW) CL[e] = g.cur[cbase + e];
    L[tid] = 0;
    // prev deps: final in HBM, eight loads in flight
    uint32_t m = (valid && w >= 2) ? base[i] : 0u;
    if (valid) {
        const uint64_t a = g.poff[i], b = g.poff[i + 1];
        for (uint64_t e0 = a; e0 < b; e0 += 8) {
            uint32_t p[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) p[u] = e0 + u < b ? g.prev[e0 + u] : 0xFFFFFFFFu;
#pragma unroll
            for (int u = 0; u < 8; ++u) if (p[u] != 0xFFFFFFFFu) m = max(m, lvlp[p[u]]);
        }
    }
    __syncthreads();
#ifdef ACC_LV_PROF
    const unsigned long long t_1 = clock64();
#endif
    uint64_t ca = 0, cb = 0;
    if (valid) { ca = g.coff[i] - cbase; cb = g.coff[i + 1] - cbase; }
    auto cur_at = [&](uint64_t e) -> uint32_t { return e < cin ? (uint32_t)CL[e] : (uint32_t)g.cur[cbase + e]; };
    lw_walk_pend(valid, ca, cb, m, L, tid, cur_at);
    uint32_t my = m;
#ifdef ACC_LV_PROF
    const unsigned long long t_2 = clock64();
#endif
    if (valid) {
        lvlp[i] = m + 1;
        level[order_exec[i]] = m;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) my = max(my, (uint32_t)__shfl_xor(my, d, 64));
    if (lane == 0) red[tid >> 6] = my;
    __syncthreads();
#ifdef ACC_LV_PROF
    if (tid == 0) {   // per window: list load + prev fold, walk, (unused)
        g_lv_prof[3 * w] = t_1 - t_0; g_lv_prof[3 * w + 1] = t_2 - t_1; g_lv_prof[3 * w + 2] = ctot;
    }
#endif
    if (tid == 0) {
        uint32_t mx = 0;
        for (uint32_t q = 0; q < LW / 64; ++q) mx = max(mx, red[q]);
        if (mx) atomicMax(max_level, mx);
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
    // tier: the whole graph's levels in one workgroup's LDS when they fit (chunk size CH: a power of two, three
    // chunk slots beside the levels; acc_opts.lv_chunk caps it)
    const uint32_t npad = (n + 7u) & ~7u;
    uint32_t ch = 0;
    // tiers: the whole-graph LDS walk (n <= 65535: config 5 0.89 ms, the windowed walk 1.07), the windowed walk beyond
    // (the 1M-txn chain graph: 0.264 us per level); acc_opts.lv_tier forces one (ACC_LV_WAVES: the persistent-wave walk)
    const uint32_t tier = ctx->opts.lv_tier;
    if (tier > ACC_LV_WAVES) fail(ACC_E_ARG, "acc_opts.lv_tier: unknown levelise tier");
    const bool windowed = tier == ACC_LV_WINDOWED || (tier == ACC_LV_AUTO && n > LV_LDS_MAX_N);
    if (!windowed && n <= LV_LDS_MAX_N && E < 0xFFFFFFFFull && tier != ACC_LV_WAVES) {
        const uint32_t room = ((uint32_t)LV_LDS - npad) / 3u;
        uint32_t cap = std::min<uint32_t>(room, LV_CH_MAX);
        if (ctx->opts.lv_chunk) cap = std::min<uint32_t>(cap, ctx->opts.lv_chunk);
        ch = cap >= 64 ? 1u << (31 - __builtin_clz(cap)) : 0u;   // largest power of two <= cap
    }
    if (!ch && !windowed) launch(ctx, "lv_check", k_lv_check, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, off, dep, err);
    uint64_t *key = ctx->get<uint64_t>("lv_key", n);
    launch(ctx, "lv_keys", k_lv_keys, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, exec_rank, key);
    Sorted se = radix_sort(ctx, "lv_rs_exec", key, nullptr, n, 32);
    uint32_t *order_exec = ctx->get<uint32_t>("lv_order_exec", n);
    ACC_HIP(hipMemcpyAsync(order_exec, se.vals, (size_t)n * 4, hipMemcpyDeviceToDevice, st));
    uint32_t *pos = ctx->get<uint32_t>("lv_pos", n);
    launch(ctx, "lv_pos", k_lv_pos, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint32_t *)order_exec, pos);
    auto check_err = [&](uint32_t e0) {
        if (e0 & 1) fail(ACC_E_ARG, "graph offsets must be non-decreasing");
        if (e0 & 2) fail(ACC_E_ARG, "dependency index out of range");
    };
    uint32_t *level = ctx->get<uint32_t>("lv_level", n);
    uint32_t *maxl = ctx->get<uint32_t>("lv_max", 4);   // [0] max level, [1] ticket counter
    ACC_HIP(hipMemsetAsync(maxl, 0, 16, st));
    if (windowed) {
        uint64_t *cf = ctx->get<uint64_t>("lw_cf", n), *cp = ctx->get<uint64_t>("lw_cp", n), *cc = ctx->get<uint64_t>("lw_cc", n);
        const unsigned gw = (n + WAVES - 1) / WAVES;
        launch(ctx, "lv_fcount", k_lw_count, dim3(gw), dim3(BLOCK), 0, n, (const uint32_t *)order_exec, off, dep, exec_rank,
               (const uint32_t *)pos, cf, cp, cc, err);
        LwLists ls;
        uint64_t *foff = ctx->get<uint64_t>("lw_foff", (size_t)n + 1), *poff = ctx->get<uint64_t>("lw_poff", (size_t)n + 1);
        uint64_t *coff = ctx->get<uint64_t>("lw_coff", (size_t)n + 1);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, cf, foff, n, true, foff + n);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, cp, poff, n, true, poff + n);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, cc, coff, n, true, coff + n);
        // the lists sized by the unfiltered E (their sums stay on the device): with non-decreasing offsets and
        // off[n] = E every txn's range lies in [0, E) and the ranges are disjoint, so the filtered counts sum to <= E.
        // An invalid graph (flagged by the count pass: decreasing offsets, a dep >= n) writes and walks nothing (the
        // later kernels read the flag first) and fails at the end
        const uint64_t cap = std::max<uint64_t>(E, 1);
        uint32_t *far = ctx->get<uint32_t>("lw_far", cap), *prev = ctx->get<uint32_t>("lw_prev", cap);
        uint16_t *cur = ctx->get<uint16_t>("lw_cur", cap);
        launch(ctx, "lv_fwrite", k_lw_write, dim3(gw), dim3(BLOCK), 0, n, (const uint32_t *)order_exec, off, dep, exec_rank,
               (const uint32_t *)pos, (const uint64_t *)foff, (const uint64_t *)poff, (const uint64_t *)coff, far, prev, cur,
               (const uint32_t *)err);
        ls.foff = foff; ls.poff = poff; ls.coff = coff; ls.far = far; ls.prev = prev; ls.cur = cur;
        uint32_t *base = ctx->get<uint32_t>("lw_base", n), *lvlp = ctx->get<uint32_t>("lw_lvlp", n);
        const uint32_t nw = (n + LW - 1) / LW;
#ifdef ACC_LV_PROF
        {
            unsigned long long *pb = ctx->get<unsigned long long>("lv_prof", 3 * (size_t)nw);
            ACC_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_lv_prof), &pb, sizeof pb, 0, hipMemcpyHostToDevice, st));
        }
#endif
        for (uint32_t w = 0; w < nw; ++w) {
            // gatherers only when window w + 1 exists and has far deps (w + 1 >= 2)
            const uint32_t nxt = (w + 2 <= nw && w + 1 >= 2) ? std::min<uint32_t>(LW, n - (w + 1) * LW) : 0u;
            const unsigned gb = 1 + (nxt + LW_GW - 1) / LW_GW;
            launch(ctx, "lv_walk_win", k_lw_step, dim3(gb), dim3(LW), 0, n, w, ls, base, lvlp, (const uint32_t *)order_exec,
                   level, maxl, (const uint32_t *)err);
        }
        ctx->stat("levelise.lds_tier", 2);
#ifdef ACC_LV_PROF
        {
            std::vector<unsigned long long> h(3 * (size_t)nw);
            unsigned long long *pb = ctx->get<unsigned long long>("lv_prof", 3 * (size_t)nw);
            ACC_HIP(hipMemcpyAsync(h.data(), pb, h.size() * 8, hipMemcpyDeviceToHost, st));
            ACC_HIP(hipStreamSynchronize(st));
            double a = 0, b = 0, c = 0;
            for (uint32_t q = 0; q < nw; ++q) { a += h[3 * q]; b += h[3 * q + 1]; c += h[3 * q + 2]; }
            fprintf(stderr, "[lw_prof] step windows=%u avg cycles per window: lists+fold %.0f walk %.0f | cur entries %.0f\n", nw,
                    a / nw, b / nw, c / nw);
        }
#endif
    } else if (ch) {
        uint32_t *fcnt = ctx->get<uint32_t>("lv_fcnt", n);
        uint32_t *foff = ctx->get<uint32_t>("lv_foff", (size_t)n + 1);
        const unsigned gw = (n + WAVES - 1) / WAVES;
        launch(ctx, "lv_fcount", k_lv_fcount, dim3(gw), dim3(BLOCK), 0, n, (const uint32_t *)order_exec, off, dep, exec_rank, fcnt,
               err);
        scan<uint32_t, OpAdd<uint32_t>>(ctx, fcnt, foff, n, true, foff + n);
        // sized by the unfiltered E (>= the filtered count, which stays on the device) + one chunk of padding for
        // whole-chunk reads; an invalid graph (flagged by k_lv_fcount) writes and walks nothing (the later kernels read
        // the flag first) and fails at the end
        uint16_t *fdep = ctx->get<uint16_t>("lv_fdep", (size_t)E + ch);
        launch(ctx, "lv_fwrite", k_lv_fwrite, dim3(gw), dim3(BLOCK), 0, n, (const uint32_t *)order_exec, off, dep, exec_rank,
               (const uint32_t *)pos, (const uint32_t *)foff, fdep, (const uint32_t *)err);
        const int ch_shift = 31 - __builtin_clz(ch);
        uint32_t *rstart = ctx->get<uint32_t>("lv_rstart", (size_t)(E >> ch_shift) + 3);
        launch(ctx, "lv_rounds", k_lv_rounds, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, ch_shift, (const uint32_t *)foff, rstart,
               (const uint32_t *)err);
#ifdef ACC_LV_PROF
        {
            unsigned long long *pb = ctx->get<unsigned long long>("lv_prof", 3 * 16);
            ACC_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_lv_prof), &pb, sizeof pb, 0, hipMemcpyHostToDevice, st));
        }
#endif
        launch(ctx, "lv_walk_lds", k_lv_lds, dim3(1), dim3(LV_NT), 0, n, npad, ch_shift, (const uint32_t *)foff,
               (const uint16_t *)fdep, (const uint32_t *)rstart, (const uint32_t *)order_exec, level, maxl,
               (const uint32_t *)err);
        ctx->stat("levelise.lds_tier", 1);
#ifdef ACC_LV_PROF
        {
            unsigned long long *pb = ctx->get<unsigned long long>("lv_prof", 3 * 16);
            std::vector<unsigned long long> h(48);
            ACC_HIP(hipMemcpyAsync(h.data(), pb, 48 * 8, hipMemcpyDeviceToHost, st));
            ACC_HIP(hipStreamSynchronize(st));
            double w = 0, q = 0, np = 0;
            for (int i = 0; i < 16; ++i) { w += h[3 * i]; q += h[3 * i + 1]; np += h[3 * i + 2]; }
            fprintf(stderr, "[lv_prof] per wave avg: walk %.0f cycles, round-barrier wait %.0f cycles, passes %.0f\n", w / 16, q / 16, np / 16);
        }
#endif
    } else {
        ACC_HIP(hipMemcpyAsync(ctx->pinned, err, 4, hipMemcpyDeviceToHost, st));
        ctx->sync();
        uint32_t e0;
        memcpy(&e0, ctx->pinned, 4);
        check_err(e0);
        ACC_HIP(hipMemsetAsync(level, 0, (size_t)n * 4, st));
        // a persistent grid of up to 4096 waves (16 per CU): enough txns in flight to cover the memory round trips
        const uint32_t waves = std::min<uint32_t>(n, 4096u);
        launch(ctx, "lv_walk_waves", k_lv_waves, dim3((waves + WAVES - 1) / WAVES), dim3(BLOCK), 0, n, (const uint32_t *)order_exec, off, dep,
               exec_rank, level, maxl + 1, maxl);
        launch(ctx, "lv_unbias", k_lv_unbias, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, level);
        ctx->stat("levelise.lds_tier", 0);
    }
    const int pbits = bits_for(n - 1);
    launch(ctx, "lv_order_keys", k_lv_order_keys, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, (const uint32_t *)level,
           (const uint32_t *)pos, pbits, key);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, maxl, 4, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, err, 4, hipMemcpyDeviceToHost, st));
    ctx->sync();
    uint32_t ml, e1;
    memcpy(&ml, ctx->pinned, 4);
    memcpy(&e1, ctx->pinned + 1, 4);
    check_err(e1);
    Sorted so = radix_sort(ctx, "lv_rs_order", key, nullptr, n, pbits + bits_for(ml));
    hipMemcpyKind kind = in->mem == ACC_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    ACC_HIP(hipMemcpyAsync(level_out, level, (size_t)n * 4, kind, st));
    ACC_HIP(hipMemcpyAsync(order_out, so.vals, (size_t)n * 4, kind, st));
    ctx->sync();
    if (n_levels) *n_levels = ml + 1;
}

}  // namespace acc
