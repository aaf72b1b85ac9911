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
                                                    const uint32_t *__restrict__ err, uint16_t *__restrict__ prev16,
                                                    uint16_t *__restrict__ far16)
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
        if (kf) {   // far16 (the LDS windowed walk, n <= 65535): u16 positions
            if (far16) far16[wf + (uint64_t)__popcll(bf & lt)] = (uint16_t)p;
            else far[wf + (uint64_t)__popcll(bf & lt)] = p;
        }
        if (kp) {   // prev16 (the LDS windowed walk): the offset in the previous window; else the position
            if (prev16) prev16[wp + (uint64_t)__popcll(bp & lt)] = (uint16_t)(p - (wi - 1) * LW);
            else prev[wp + (uint64_t)__popcll(bp & lt)] = p;
        }
        if (kc) cur[wc + (uint64_t)__popcll(bc & lt)] = (uint16_t)(p - wi * LW);
        wf += (uint64_t)__popcll(bf); wp += (uint64_t)__popcll(bp); wc += (uint64_t)__popcll(bc);
    }
}

__device__ __forceinline__ uint32_t lw_lds_ld(const uint32_t *p) { return *(const volatile uint32_t *)p; }

struct LwLists {
    const uint64_t *foff, *poff, *coff;
    const uint32_t *far, *prev;
    const uint16_t *cur;
    const uint16_t *prev16;   // the LDS windowed walk's prev lists (offsets in the previous window)
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

// one window step (launch w): block 0 walks window w, blocks 1.. gather the far maxima of window w + 1.
// POLL = 1: the batch walk for long chains (a blocked lane re-reads one entry per round); else the sliding walk
template <int POLL>
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
    constexpr int LW_B = 8;
    bool done = !valid;
    uint32_t my = 0;
    if (POLL != 1) {   // graphs with many in-window deps per position: the pending-set walk
        lw_walk_pend(valid, ca, cb, m, L, tid, cur_at);
        my = m;
        done = true;
    } else {
        // few deps per position (long chains): batches of LW_B entries held in registers (read from LDS once per
        // batch); a "full" round loads the levels of every entry left in the batch and consumes up to the first
        // unpublished one, then the blocked lane polls that one entry only (one LDS load per round, so the waves
        // spinning behind the chain leave the LDS to the wave advancing it) and goes back to a full round once it is
        // published: a hop costs about two short rounds
        uint64_t e = ca;             // first entry of the batch
        uint32_t p[LW_B];
        uint32_t np = 0, k = 0;      // batch size, entries consumed
        bool full = true;
        while (true) {
            if (!done) {
                if (k == np) {
                    e += np;
                    np = (uint32_t)min<uint64_t>(LW_B, cb - e);
#pragma unroll
                    for (int u = 0; u < LW_B; ++u) p[u] = (uint32_t)u < np ? cur_at(e + u) : 0u;
                    k = 0;
                    full = true;
                }
                if (full) {
                    uint32_t v[LW_B];
#pragma unroll
                    for (int u = 0; u < LW_B; ++u) v[u] = ((uint32_t)u >= k && (uint32_t)u < np) ? lw_lds_ld(&L[p[u]]) : 1u;
                    bool blocked = false;
#pragma unroll
                    for (int u = 0; u < LW_B; ++u) {
                        if (blocked || (uint32_t)u < k || (uint32_t)u >= np) continue;
                        if (!v[u]) { blocked = true; continue; }
                        m = max(m, v[u]);
                        ++k;
                    }
                    full = !blocked;
                } else {
                    uint32_t pk = p[0];
#pragma unroll
                    for (int u = 1; u < LW_B; ++u) if ((uint32_t)u == k) pk = p[u];
                    const uint32_t v = lw_lds_ld(&L[pk]);
                    if (v) { m = max(m, v); ++k; full = true; }
                }
                if (k == np && e + np >= cb) {
                    *(volatile uint32_t *)&L[tid] = m + 1;
                    my = m;
                    done = true;
                }
            }
            if (__all(done)) break;
        }
    }
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

// ---- LDS windowed walk (tier 3, n <= LV_W1_MAX_N; tuning tier, ACC_LV_W1): the windowed tier's split inside ONE
// workgroup, every level in LDS (u16, level + 1, 0 = unpublished). Window u (LW positions, a lane per position):
//   1. fold: each lane folds its position's deps in earlier windows (far: absolute u16 positions, prev: offsets in window
//      u - 1), all published, reading its lists as aligned 16-B pieces, eight in flight;
//   2. the window's in-window (cur) edges transposed in LDS (successor lists by counting sort: LDS atomics);
//   3. push walk: a lane waits for its own pending-dependency counter to reach zero (one LDS word polled), then publishes
//      its level and pushes level + 1 to its successors (atomic max) and decrements their counters. A hop costs one
//      LDS atomic and one poll, however many deps a position has; a window whose cur edges exceed the successor buffer
//      takes the pending-set walk instead.
// Termination: the cur edges of a window form a DAG (earlier positions only), so some pending lane always has a zero
// counter. Measured (config 5): the single-CU fold costs ~60K cycles per window, so this tier stays behind the
// whole-graph LDS walk there (§7); kept as a tuning tier.
constexpr uint32_t LV_W1_MAX_N = 32768;
constexpr uint32_t LV_W1_SU = 36864;   // successor-list entries of a window in LDS (u16)
constexpr uint32_t LV_W1_MIN = 0xFFFFFFFFu;   // not a default tier (see above)

// max over list entries [a, b) of LV[base + entry] (level + 1, all published), the list read as aligned uint4 pieces
// (the list buffers are padded by a piece), eight pieces per round
__device__ __forceinline__ uint32_t lv_fold16(const uint16_t *__restrict__ list, uint64_t a, uint64_t b, const uint16_t *LV,
                                              uint32_t base)
{
    uint32_t m = 0;
    const uint4 *l4 = reinterpret_cast<const uint4 *>(list);
    for (uint64_t c = a & ~7ull; c < b; c += 64) {
        uint4 v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = c + 8u * q < b ? l4[(c >> 3) + q] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint32_t w[4] = { v[q].x, v[q].y, v[q].z, v[q].w };
#pragma unroll
            for (int h = 0; h < 8; ++h) {
                const uint64_t e = c + 8u * q + h;
                if (e >= a && e < b) m = max(m, (uint32_t)LV[base + ((w[h >> 1] >> (16 * (h & 1))) & 0xFFFFu)]);
            }
        }
    }
    return m;
}

__global__ __launch_bounds__(LW) void k_lv_win1(uint32_t n, LwLists g, const uint16_t *__restrict__ far16,
                                                const uint32_t *__restrict__ order_exec, uint32_t *__restrict__ level,
                                                uint32_t *__restrict__ max_level, const uint32_t *__restrict__ err)
{
    if (*err) return;   // invalid graph: the lists were not written (the host fails after the walk)
    __shared__ __attribute__((aligned(16))) uint16_t LV[LV_W1_MAX_N];
    __shared__ uint16_t SU[LV_W1_SU];
    __shared__ uint32_t Mw[LW], dg[LW], so[LW + 1], fc[LW];
    __shared__ uint32_t red[LW / 64];
    const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    for (uint32_t i = tid; i < n; i += LW) LV[i] = 0;
    const uint32_t nw = (n + LW - 1) / LW;
    uint32_t my = 0;
    __syncthreads();
    for (uint32_t u = 0; u < nw; ++u) {
        const uint32_t w0 = u * LW, wend = min(n, w0 + LW), i = w0 + tid;
        const bool valid = i < wend;
        const uint64_t cbase = g.coff[w0], ctot = g.coff[wend] - cbase;
#ifdef ACC_LV_PROF
        const unsigned long long t_0 = clock64();
#endif
        uint32_t m = 0;
        if (valid && u >= 1) {
            m = lv_fold16(far16, u >= 2 ? g.foff[i] : 0, u >= 2 ? g.foff[i + 1] : 0, LV, 0u);
            m = max(m, lv_fold16(g.prev16, g.poff[i], g.poff[i + 1], LV, (u - 1) * LW));
        }
        uint64_t ca = 0, cb = 0;
        if (valid) { ca = g.coff[i] - cbase; cb = g.coff[i + 1] - cbase; }
        uint16_t *Lw = LV + w0;
        const bool push = ctot <= LV_W1_SU;   // block-uniform
        if (push) {
            Mw[tid] = m;
            dg[tid] = (uint32_t)(cb - ca);
            fc[tid] = 0;
            __syncthreads();
            for (uint64_t e = ca; e < cb; e += 8) {   // eight list loads in flight, then their counter adds
                uint32_t d[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) d[q] = e + q < cb ? (uint32_t)g.cur[cbase + e + q] : 0xFFFFFFFFu;
#pragma unroll
                for (int q = 0; q < 8; ++q) if (d[q] != 0xFFFFFFFFu) atomicAdd(&fc[d[q]], 1u);
            }
            __syncthreads();
            {   // exclusive scan of the successor counts -> so (and the fill cursors)
                const uint32_t c = fc[tid];
                uint32_t x = c;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
                    if (lane >= (uint32_t)d) x += y;
                }
                if (lane == 63) red[wave] = x;
                __syncthreads();
                uint32_t pre = 0;
                for (uint32_t q = 0; q < wave; ++q) pre += red[q];
                so[tid] = pre + x - c;
                if (tid == LW - 1) so[LW] = pre + x;
                __syncthreads();
                fc[tid] = so[tid];
            }
            __syncthreads();
            for (uint64_t e = ca; e < cb; e += 8) {
                uint32_t d[8], slot[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) d[q] = e + q < cb ? (uint32_t)g.cur[cbase + e + q] : 0xFFFFFFFFu;
#pragma unroll
                for (int q = 0; q < 8; ++q) slot[q] = d[q] != 0xFFFFFFFFu ? atomicAdd(&fc[d[q]], 1u) : 0u;
#pragma unroll
                for (int q = 0; q < 8; ++q) if (d[q] != 0xFFFFFFFFu) SU[slot[q]] = (uint16_t)tid;
            }
            __syncthreads();
        } else {
            __syncthreads();
        }
#ifdef ACC_LV_PROF
        const unsigned long long t_1 = clock64();
#endif
#ifdef ACC_LV_PROF
        uint32_t rounds = 0;
#endif
        if (push) {
            bool done = !valid;
            while (true) {
#ifdef ACC_LV_PROF
                ++rounds;
#endif
                if (!done && *(volatile uint32_t *)&dg[tid] == 0) {
                    const uint32_t lv = *(volatile uint32_t *)&Mw[tid];
                    *(volatile uint16_t *)&Lw[tid] = (uint16_t)(lv + 1);
                    m = lv;
                    // the successor ids eight at a time, then their updates back to back (no-return LDS atomics,
                    // executed in order per lane: a successor's max lands before its counter reaches zero)
                    const uint32_t k1 = so[tid + 1];
                    for (uint32_t k = so[tid]; k < k1; k += 8) {
                        uint32_t sc[8];
#pragma unroll
                        for (int q = 0; q < 8; ++q) sc[q] = k + q < k1 ? (uint32_t)SU[k + q] : 0xFFFFFFFFu;
#pragma unroll
                        for (int q = 0; q < 8; ++q)
                            if (sc[q] != 0xFFFFFFFFu) { atomicMax(&Mw[sc[q]], lv + 1); atomicSub(&dg[sc[q]], 1u); }
                    }
                    done = true;
                }
                if (__all(done)) break;
            }
        } else {
            auto cur_at = [&](uint64_t e) -> uint32_t { return (uint32_t)g.cur[cbase + e]; };
            lw_walk_pend(valid, ca, cb, m, Lw, tid, cur_at);
        }
        if (valid) {
            level[order_exec[i]] = m;
            my = max(my, m);
        }
        __syncthreads();   // window u published before window u + 1 folds it
#ifdef ACC_LV_PROF
        {   // rounds of the slowest wave and the window's level span
            uint32_t lo = valid ? m : 0xFFFFFFFFu, hi = valid ? m : 0u, r = rounds;
            for (int d = 32; d >= 1; d >>= 1) {
                lo = min(lo, (uint32_t)__shfl_xor(lo, d, 64)); hi = max(hi, (uint32_t)__shfl_xor(hi, d, 64));
                r = max(r, (uint32_t)__shfl_xor(r, d, 64));
            }
            if (lane == 0) { Mw[wave] = lo; dg[wave] = hi; fc[wave] = r; }
            __syncthreads();
            if (tid == 0) {
                uint32_t a = 0xFFFFFFFFu, b = 0, rr = 0;
                for (uint32_t q = 0; q < LW / 64; ++q) { a = min(a, Mw[q]); b = max(b, dg[q]); rr = max(rr, fc[q]); }
                g_lv_prof[3 * u] = t_1 - t_0; g_lv_prof[3 * u + 1] = clock64() - t_1;
                g_lv_prof[3 * u + 2] = ((unsigned long long)rr << 32) | (b - a);
            }
            __syncthreads();
        }
#endif
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) my = max(my, (uint32_t)__shfl_xor(my, d, 64));
    if (lane == 0) red[tid >> 6] = my;
    __syncthreads();
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
    // chunk slots beside the levels; ACC_LV_CH caps it, ACC_LV_WAVES forces the persistent-wave walk)
    const uint32_t npad = (n + 7u) & ~7u;
    uint32_t ch = 0;
    // tiers: the whole-graph LDS walk (n <= 65535: config 5 0.89 ms, the windowed walk 1.07), the windowed walk beyond
    // (ACC_LV_WIN forces it; the 1M-txn chain graph: 0.54 us per level, the persistent-wave walk 0.75); ACC_LV_WAVES:
    // the persistent-wave walk
    // tier 3 (tuning, ACC_LV_W1, n <= LV_W1_MAX_N): the LDS windowed walk in one workgroup; ACC_LV_LDS / ACC_LV_WIN /
    // ACC_LV_WAVES select the other tiers
    const bool w1 = n <= LV_W1_MAX_N && (n >= LV_W1_MIN || getenv("ACC_LV_W1")) && !getenv("ACC_LV_LDS") &&
                    !getenv("ACC_LV_WIN") && !getenv("ACC_LV_WAVES");
    const bool windowed = (n > LV_LDS_MAX_N || getenv("ACC_LV_WIN") || w1) && !getenv("ACC_LV_LDS") && !getenv("ACC_LV_WAVES");
    if (!windowed && n <= LV_LDS_MAX_N && E < 0xFFFFFFFFull && !getenv("ACC_LV_WAVES")) {
        const uint32_t room = ((uint32_t)LV_LDS - npad) / 3u;
        uint32_t cap = std::min<uint32_t>(room, LV_CH_MAX);
        if (const char *ce = getenv("ACC_LV_CH")) cap = std::min<uint32_t>(cap, (uint32_t)std::max(1, atoi(ce)));
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
        uint32_t *far = w1 ? nullptr : ctx->get<uint32_t>("lw_far", cap), *prev = w1 ? nullptr : ctx->get<uint32_t>("lw_prev", cap);
        uint16_t *cur = ctx->get<uint16_t>("lw_cur", cap), *prev16 = w1 ? ctx->get<uint16_t>("lw_prev16", cap + 8) : nullptr;
        uint16_t *far16 = w1 ? ctx->get<uint16_t>("lw_far16", cap + 8) : nullptr;   // + a 16-B piece (k_lv_win1 reads)
        launch(ctx, "lv_fwrite", k_lw_write, dim3(gw), dim3(BLOCK), 0, n, (const uint32_t *)order_exec, off, dep, exec_rank,
               (const uint32_t *)pos, (const uint64_t *)foff, (const uint64_t *)poff, (const uint64_t *)coff, far, prev, cur,
               (const uint32_t *)err, prev16, far16);
        ls.foff = foff; ls.poff = poff; ls.coff = coff; ls.far = far; ls.prev = prev; ls.cur = cur; ls.prev16 = prev16;
        uint32_t *base = ctx->get<uint32_t>("lw_base", n), *lvlp = ctx->get<uint32_t>("lw_lvlp", n);
        const uint32_t nw = (n + LW - 1) / LW;
#ifdef ACC_LV_PROF
        {
            unsigned long long *pb = ctx->get<unsigned long long>("lv_prof", 3 * (size_t)nw);
            ACC_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_lv_prof), &pb, sizeof pb, 0, hipMemcpyHostToDevice, st));
        }
#endif
        // the pending-set walk (the 1M-txn test graph: 0.264 us per level; the batch walk, ACC_LV_POLL=1: 0.543)
        int poll = 8;
        if (const char *pe = getenv("ACC_LV_POLL")) poll = atoi(pe) == 1 ? 1 : 8;   // tuning switch
        ctx->stat("levelise.poll", (uint64_t)poll);
        if (w1)
            launch(ctx, "lv_walk_w1", k_lv_win1, dim3(1), dim3(LW), 0, n, ls, (const uint16_t *)far16,
                   (const uint32_t *)order_exec, level, maxl, (const uint32_t *)err);
        for (uint32_t w = 0; !w1 && w < nw; ++w) {
            // gatherers only when window w + 1 exists and has far deps (w + 1 >= 2)
            const uint32_t nxt = (w + 2 <= nw && w + 1 >= 2) ? std::min<uint32_t>(LW, n - (w + 1) * LW) : 0u;
            const unsigned gb = 1 + (nxt + LW_GW - 1) / LW_GW;
            if (poll == 1)
                launch(ctx, "lv_walk_win", k_lw_step<1>, dim3(gb), dim3(LW), 0, n, w, ls, base, lvlp, (const uint32_t *)order_exec,
                       level, maxl, (const uint32_t *)err);
            else
                launch(ctx, "lv_walk_win", k_lw_step<8>, dim3(gb), dim3(LW), 0, n, w, ls, base, lvlp, (const uint32_t *)order_exec,
                       level, maxl, (const uint32_t *)err);
        }
        ctx->stat("levelise.lds_tier", w1 ? 3 : 2);
#ifdef ACC_LV_PROF
        {
            std::vector<unsigned long long> h(3 * (size_t)nw);
            unsigned long long *pb = ctx->get<unsigned long long>("lv_prof", 3 * (size_t)nw);
            ACC_HIP(hipMemcpyAsync(h.data(), pb, h.size() * 8, hipMemcpyDeviceToHost, st));
            ACC_HIP(hipStreamSynchronize(st));
            double a = 0, b = 0, c = 0;
            for (uint32_t q = 0; q < nw; ++q) { a += h[3 * q]; b += h[3 * q + 1]; c += w1 ? (h[3 * q + 2] & 0xFFFFFFFFu) : h[3 * q + 2]; }
            if (w1) {
                double r = 0;
                for (uint32_t q = 0; q < nw; ++q) r += (double)(h[3 * q + 2] >> 32);
                fprintf(stderr, "[lw_prof] w1: avg rounds of the slowest wave per window %.0f (level span in cur-entries slot)\n", r / nw);
            }
            fprintf(stderr, "[lw_prof] %s windows=%u avg cycles per window: lists+fold %.0f walk %.0f | cur entries %.0f\n", w1 ? "w1" : "step", nw,
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
