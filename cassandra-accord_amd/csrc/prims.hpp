// prims.hpp — wave64 building blocks for the dependency path: block/device scans (add / max),
// order-preserving bit compaction (pext over a run plan) and a stable LSD radix sort of
// (u64 key, u32 value) pairs with 8-bit digits. Integer work only: HBM-bound, no MFMA.
#pragma once

#include "ctx.hpp"

#include <algorithm>

namespace acc {

constexpr int BLOCK = 256;
constexpr int WAVES = BLOCK / 64;

// ---------------------------------------------------------------- wave helpers

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

template <class T>
__device__ __forceinline__ T shfl_up(T v, unsigned d)
{
    if constexpr (sizeof(T) == 8) {
        uint64_t u = (uint64_t)v;
        uint32_t lo = __shfl_up((uint32_t)u, d, 64), hi = __shfl_up((uint32_t)(u >> 32), d, 64);
        return (T)(((uint64_t)hi << 32) | lo);
    } else {
        return (T)__shfl_up((uint32_t)v, d, 64);
    }
}

template <class T>
__device__ __forceinline__ T shfl_idx(T v, int src)
{
    if constexpr (sizeof(T) == 8) {
        uint64_t u = (uint64_t)v;
        uint32_t lo = __shfl((uint32_t)u, src, 64), hi = __shfl((uint32_t)(u >> 32), src, 64);
        return (T)(((uint64_t)hi << 32) | lo);
    } else {
        return (T)__shfl((uint32_t)v, src, 64);
    }
}

template <class T>
__device__ __forceinline__ T shfl_xor(T v, int m)
{
    if constexpr (sizeof(T) == 8) {
        uint64_t u = (uint64_t)v;
        uint32_t lo = __shfl_xor((uint32_t)u, m, 64), hi = __shfl_xor((uint32_t)(u >> 32), m, 64);
        return (T)(((uint64_t)hi << 32) | lo);
    } else {
        return (T)__shfl_xor((uint32_t)v, m, 64);
    }
}

// The value of lane (lane ^ m), m a power of two below 64 known at compile time (unrolled loops), without the LDS
// round trip of ds_bpermute: xor 1 / 2 are quad permutes, xor 4 / 8 a row (half-)mirror followed by a quad or
// half-mirror permute (i ^ 7 ^ 3 = i ^ 4, i ^ 15 ^ 7 = i ^ 8), xor 16 / 32 gfx950's v_permlane16/32_swap (each lane
// takes the half the swap moved across). Every lane of the wave must be active: a DPP read of a disabled lane leaves
// the `old` operand (0) instead of the value.
__device__ __forceinline__ uint32_t xor_lanes_u32(uint32_t x, int m)
{
    switch (m) {
    case 1: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    case 2: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    case 4: {
        const int y = __builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false);           // row_half_mirror
        return (uint32_t)__builtin_amdgcn_update_dpp(0, y, 0x1B, 0xF, 0xF, false);              // quad_perm [3,2,1,0]
    }
    case 8: {
        const int y = __builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false);           // row_mirror
        return (uint32_t)__builtin_amdgcn_update_dpp(0, y, 0x141, 0xF, 0xF, false);             // row_half_mirror
    }
    case 16: {
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return (threadIdx.x & 16u) ? r[0] : r[1];
    }
    default: {
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (threadIdx.x & 32u) ? r[0] : r[1];
    }
    }
}

template <class T>
__device__ __forceinline__ T xor_lanes(T v, int m)
{
    if constexpr (sizeof(T) == 8) {
        const uint64_t u = (uint64_t)v;
        const uint32_t lo = xor_lanes_u32((uint32_t)u, m), hi = xor_lanes_u32((uint32_t)(u >> 32), m);
        return (T)(((uint64_t)hi << 32) | lo);
    } else {
        return (T)xor_lanes_u32((uint32_t)v, m);
    }
}

template <class T>
struct OpAdd {
    __device__ __forceinline__ T operator()(T a, T b) const { return a + b; }
    static __device__ __forceinline__ T identity() { return (T)0; }
};

// max over unsigned values; identity 0
template <class T>
struct OpMax {
    __device__ __forceinline__ T operator()(T a, T b) const { return a > b ? a : b; }
    static __device__ __forceinline__ T identity() { return (T)0; }
};

template <class T, class Op>
__device__ __forceinline__ T wave_inclusive(T v, Op op)
{
    const uint32_t lane = lane_id();
#pragma unroll
    for (unsigned d = 1; d < 64; d <<= 1) {
        T u = shfl_up(v, d);
        if (lane >= d) v = op(u, v);
    }
    return v;
}

// Block-wide exclusive scan of per-thread values; returns the exclusive prefix of this thread and
// the block total. `lds` holds NWV elements; NWV = the block's wave count (blockDim.x / 64).
template <class T, class Op, int NWV = WAVES>
__device__ __forceinline__ T block_exclusive(T v, Op op, T *lds, T &total)
{
    const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
    T incl = wave_inclusive(v, op);
    if (lane == 63) lds[wave] = incl;
    __syncthreads();
    T wave_prefix = Op::identity();
    T tot = Op::identity();
#pragma unroll
    for (int w = 0; w < NWV; ++w) {
        T x = lds[w];
        if (w < (int)wave) wave_prefix = op(wave_prefix, x);
        tot = op(tot, x);
    }
    __syncthreads();
    T excl = shfl_up(incl, 1);
    if (lane == 0) excl = Op::identity();
    total = tot;
    return op(wave_prefix, excl);
}

// Owner map of one chunk of a workgroup's output range: own[p] = the index k < nt of the run [off[k], off[k + 1]) holding
// position c0 + p, for p < PT * BLOCK (off ascending, in LDS or registers' reach; carry = the owner of position c0,
// updated to the owner of the chunk's last position). Each run starting in the chunk marks its start (LDS max: of the
// runs starting at one position the last, the only non-empty one, wins), then a block max-scan spreads the marks:
// copies that follow read their run from own[] instead of searching the offsets per element. Whole block, uniform.
template <int PT>
__device__ __forceinline__ void chunk_owners(uint32_t nt, const uint64_t *off, uint64_t c0, uint32_t *own, uint32_t *red,
                                             uint32_t &carry)
{
    constexpr uint32_t CH = (uint32_t)PT * BLOCK;
    const uint32_t tid = threadIdx.x;
    __syncthreads();   // the previous chunk's reads of own[] are done
    for (uint32_t p = tid; p < CH; p += BLOCK) own[p] = 0;
    if (tid == 0) own[0] = carry;   // (thread 0 zeroed own[0]; before the barrier: no race with a run starting at c0)
    __syncthreads();
    if (tid < nt && off[tid] < off[tid + 1] && off[tid] >= c0 && off[tid] < c0 + CH) atomicMax(&own[off[tid] - c0], tid);
    __syncthreads();
    uint32_t v[PT], m = 0;
#pragma unroll
    for (int u = 0; u < PT; ++u) { m = max(m, own[tid * PT + u]); v[u] = m; }
    uint32_t tot;
    const uint32_t pre = block_exclusive(m, OpMax<uint32_t>(), red, tot);
#pragma unroll
    for (int u = 0; u < PT; ++u) own[tid * PT + u] = max(pre, v[u]);
    __syncthreads();
    carry = tot;
}

// ---------------------------------------------------------------- sorting networks

// ascending bitonic sort of one value per lane across the 64 lanes of a wave
template <class T>
__device__ __forceinline__ T bitonic_reg(T x)
{
    const uint32_t lane = lane_id();
#pragma unroll
    for (uint32_t k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
            const T y = xor_lanes(x, (int)jj);   // (callers run the whole wave)
            const bool up = (lane & k) == 0, lower = (lane & jj) == 0;
            const T mn = x < y ? x : y, mx = x < y ? y : x;
            x = (lower == up) ? mn : mx;
        }
    }
    return x;
}

// ascending bitonic sort of n2 (power of two) values in LDS or global memory by a whole workgroup of BLOCK threads
template <class T, int NT = BLOCK>
__device__ void block_bitonic(T *a, uint32_t n2)
{
    for (uint32_t k = 2; k <= n2; k <<= 1) {
        for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
            for (uint32_t i = threadIdx.x; i < n2; i += NT) {
                const uint32_t l = i ^ jj;
                if (l > i) {
                    const T x = a[i], y = a[l];
                    const bool up = (i & k) == 0;
                    if ((x > y) == up) { a[i] = y; a[l] = x; }
                }
            }
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------- device-wide scan
//
// Single-pass scan with decoupled look-back: tiles take tickets in launch order, publish their aggregate,
// then the nearest inclusive prefix found looking back over the previous tiles' status words. A status word is
// one naturally aligned 8-B granule {value | flag << 62} written by ONE agent-scope (sc1) store and polled with
// agent-scope loads (MI355X_MICROARCH.md, inter-workgroup hand-off: per-XCD L2s are not coherent). Values must
// stay below 2^62 (every scan here: counts, offsets, (segment << 32 | value) maxima with < 2^30 segments).
// Loads and stores go through LDS so every global access is coalesced.

constexpr uint64_t SCAN_AGG = 1ull << 62, SCAN_INC = 2ull << 62, SCAN_VAL = (1ull << 62) - 1;

__device__ __forceinline__ void scan_status_store(uint64_t *p, uint64_t w)
{
    __hip_atomic_store(p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t scan_status_load(const uint64_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Up to SCAN_MAXA independent arrays per launch (one launch instead of one per array): tickets run over the arrays'
// tiles in order, so every tile's look-back finds only tiles of its own array that took lower tickets.
constexpr int SCAN_MAXA = 4;
template <class T>
struct ScanArgs {
    const T *in[SCAN_MAXA];
    T *out[SCAN_MAXA];
    T *total[SCAN_MAXA];
    uint64_t n[SCAN_MAXA];
    uint32_t cum[SCAN_MAXA + 1];   // first ticket of each array; cum[k] = all tiles
    int k;
};

template <class T, class Op, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_scan_1p(ScanArgs<T> a, int exclusive, uint32_t *__restrict__ ticket,
                                                 uint64_t *__restrict__ status, uint64_t *__restrict__ other, uint32_t other_n)
{
    constexpr int TILE = BLOCK * ITEMS;
    __shared__ T tile[TILE + TILE / 32];
    __shared__ T lds[WAVES];
    __shared__ uint32_t s_b;
    __shared__ T s_prefix;
    const uint32_t tid = threadIdx.x, lane = lane_id();
    if (other_n) {   // reset the other status buffer for the next scan (it is not read by this one)
        const uint32_t chunk = (other_n + gridDim.x - 1) / gridDim.x;
        const uint32_t lo = blockIdx.x * chunk, hi = min(other_n, lo + chunk);
        for (uint32_t i = lo + tid; i < hi; i += BLOCK) other[i] = 0;
    }
    if (tid == 0) s_b = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t tk = s_b;
    int ai = 0;
#pragma unroll
    for (int q = 1; q < SCAN_MAXA; ++q) ai += (q < a.k && tk >= a.cum[q]) ? 1 : 0;
    const uint32_t b = tk - a.cum[ai];
    const T *__restrict__ in = a.in[ai];
    T *__restrict__ out = a.out[ai];
    T *__restrict__ total_out = a.total[ai];
    const size_t n = a.n[ai];
    uint64_t *const st = status + a.cum[ai];
    const size_t base = (size_t)b * TILE;
    Op op;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t li = i * BLOCK + tid;
        const size_t g = base + li;
        tile[li + li / 32] = g < n ? in[g] : Op::identity();
    }
    __syncthreads();
    T v[ITEMS];
    T acc = Op::identity();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t li = tid * ITEMS + i;
        v[i] = tile[li + li / 32];
        acc = op(acc, v[i]);
    }
    T total;
    T run = block_exclusive(acc, op, lds, total);
    if (b == 0) {
        if (tid == 0) scan_status_store(&st[0], (uint64_t)total | SCAN_INC);
    } else {
        if (tid == 0) scan_status_store(&st[b], (uint64_t)total | SCAN_AGG);
        if (tid < 64) {
            T pre = Op::identity();
            int64_t j = (int64_t)b - 1;
            while (true) {
                const int64_t idx = j - (int64_t)lane;
                uint64_t w = (uint64_t)Op::identity() | SCAN_INC;
                if (idx >= 0) {
                    w = scan_status_load(&st[idx]);
                    while ((w >> 62) == 0) {
                        __builtin_amdgcn_s_sleep(1);
                        w = scan_status_load(&st[idx]);
                    }
                }
                const uint64_t inc = __ballot((w >> 62) == 2);
                const uint32_t stop = inc ? (uint32_t)__builtin_ctzll(inc) : 63u;
                T x = lane <= stop ? (T)(w & SCAN_VAL) : Op::identity();
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) x = op(x, shfl_xor(x, d));
                pre = op(pre, x);
                if (inc) break;
                j -= 64;
            }
            if (tid == 0) {
                scan_status_store(&st[b], (uint64_t)op(pre, total) | SCAN_INC);
                s_prefix = pre;
            }
        }
        __syncthreads();
        run = op(s_prefix, run);
    }
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t li = tid * ITEMS + i;
        const T incl = op(run, v[i]);
        tile[li + li / 32] = exclusive ? run : incl;
        if (total_out && base + li == n - 1) *total_out = incl;
        run = incl;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t li = i * BLOCK + tid;
        const size_t g = base + li;
        if (g < n) out[g] = tile[li + li / 32];
    }
}

// k arrays (k <= SCAN_MAXA) scanned by one launch; in[i] / out[i] / n[i] / total_out[i] as scan() below
template <class T, class Op>
void scan_multi(acc_ctx *ctx, int k, const T *const *in, T *const *out, const size_t *n, bool exclusive, T *const *total_out)
{
    constexpr int ITEMS = sizeof(T) == 8 ? 16 : 32;   // 4096 / 8192-element tiles: fewer look-back hops
    constexpr size_t TILE = (size_t)BLOCK * ITEMS;
    if (k < 1 || k > SCAN_MAXA) fail(ACC_E_STATE, "internal: scan_multi array count");
    ScanArgs<T> a{};
    size_t nb = 0;
    int m = 0;
    for (int i = 0; i < k; ++i) {
        if (n[i] == 0) {   // nothing to scan: the total is the identity of the sum (0)
            if (total_out && total_out[i]) ACC_HIP(hipMemsetAsync(total_out[i], 0, sizeof(T), ctx->stream));
            continue;
        }
        a.in[m] = in[i]; a.out[m] = out[i]; a.total[m] = total_out ? total_out[i] : nullptr; a.n[m] = n[i];
        a.cum[m] = (uint32_t)nb;
        nb += (n[i] + TILE - 1) / TILE;
        if (nb > 0xFFFFFFF0ull) fail(ACC_E_CAP, "scan too large");
        ++m;
    }
    if (m == 0) return;
    a.k = m;
    for (int i = m; i <= SCAN_MAXA; ++i) a.cum[i] = (uint32_t)nb;
    // stream order is what makes the double-buffered status safe: every scan runs on the context stream
    if (ctx->launch_stream) fail(ACC_E_STATE, "internal: scan launched on a side stream");
    const size_t need = nb + 1;
    uint64_t *buf[2];
    if (need > ctx->scan_cap) {
        for (int i = 0; i < 2; ++i) {
            buf[i] = ctx->get_raw<uint64_t>(i ? "scan_status1" : "scan_status0", need);
            ACC_HIP(hipMemsetAsync(buf[i], 0, need * sizeof(uint64_t), ctx->stream));
        }
        ctx->scan_cap = need;
        ctx->scan_dirty[0] = ctx->scan_dirty[1] = 0;
    } else {
        for (int i = 0; i < 2; ++i) buf[i] = ctx->get_raw<uint64_t>(i ? "scan_status1" : "scan_status0", need);
    }
    const int p = ctx->scan_par;
    uint64_t *status = buf[p];
    uint32_t *ticket = reinterpret_cast<uint32_t *>(status + nb);
    launch(ctx, "scan", k_scan_1p<T, Op, ITEMS>, dim3((unsigned)nb), dim3(BLOCK), 0, a, (int)exclusive, ticket, status,
           buf[p ^ 1], (uint32_t)ctx->scan_dirty[p ^ 1]);
    ctx->scan_dirty[p] = need;
    ctx->scan_dirty[p ^ 1] = 0;
    ctx->scan_par = p ^ 1;
}

template <class T, class Op>
void scan(acc_ctx *ctx, const T *in, T *out, size_t n, bool exclusive, T *total_out = nullptr)
{
    T *const tot[1] = { total_out };
    scan_multi<T, Op>(ctx, 1, &in, &out, &n, exclusive, tot);
}

// u64 total of a u32 array (one atomic per block): the guard beside a u32 scan whose total may pass 2^32 - 1
static __global__ __launch_bounds__(BLOCK) void k_sum_u32(const uint32_t *__restrict__ in, size_t n, uint64_t *__restrict__ out)
{
    __shared__ uint64_t lds[WAVES];
    uint64_t x = 0;
    for (size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (size_t)gridDim.x * BLOCK) x += in[i];
    uint64_t total;
    block_exclusive(x, OpAdd<uint64_t>(), lds, total);
    if (threadIdx.x == 0 && total) atomicAdd((unsigned long long *)out, (unsigned long long)total);
}

// enqueues the u64 total of in[0, n) into *out (zeroed first); the caller reads it at its next sync
inline void sum_u32(acc_ctx *ctx, const uint32_t *in, size_t n, uint64_t *out)
{
    ACC_HIP(hipMemsetAsync(out, 0, 8, ctx->stream));
    if (n) launch(ctx, "sum_u32", k_sum_u32, dim3((unsigned)std::min<size_t>(1024, (n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0,
                  in, n, out);
}

// ---------------------------------------------------------------- bit compaction plan

// pext(w, mask) as a list of contiguous runs; masks with more than MAX_RUNS runs fall back to the
// hull [lowest set bit, highest set bit] (a superset: still order preserving, a few more bits).
struct Runs {
    static constexpr int MAX_RUNS = 12;
    int n = 0;
    int bits = 0;
    uint8_t lo[MAX_RUNS] = {}, len[MAX_RUNS] = {}, dst[MAX_RUNS] = {};
};

inline Runs make_runs(uint64_t mask)
{
    Runs r;
    int b = 0;
    int count = 0;
    for (int i = 0; i < 64;) {
        if (!((mask >> i) & 1)) { ++i; continue; }
        int j = i;
        while (j < 64 && ((mask >> j) & 1)) ++j;
        ++count;
        i = j;
    }
    if (count > Runs::MAX_RUNS) {
        int lo = __builtin_ctzll(mask), hi = 63 - __builtin_clzll(mask);
        r.n = 1; r.lo[0] = (uint8_t)lo; r.len[0] = (uint8_t)(hi - lo + 1); r.dst[0] = 0; r.bits = hi - lo + 1;
        return r;
    }
    for (int i = 0; i < 64;) {
        if (!((mask >> i) & 1)) { ++i; continue; }
        int j = i;
        while (j < 64 && ((mask >> j) & 1)) ++j;
        r.lo[r.n] = (uint8_t)i; r.len[r.n] = (uint8_t)(j - i); r.dst[r.n] = (uint8_t)b;
        b += j - i; ++r.n;
        i = j;
    }
    r.bits = b;
    return r;
}

__device__ __forceinline__ uint64_t pext_runs(uint64_t w, const Runs &r)
{
    uint64_t o = 0;
    for (int i = 0; i < r.n; ++i) {
        uint64_t m = r.len[i] >= 64 ? ~0ull : ((1ull << r.len[i]) - 1);
        o |= ((w >> r.lo[i]) & m) << r.dst[i];
    }
    return o;
}

// ---------------------------------------------------------------- LSD radix sort

constexpr int RS_ITEMS = 16;
constexpr int RS_TILE = BLOCK * RS_ITEMS;
constexpr int RS_ITEMS_S = 4;                      // one-sweep tiles of mid-size sorts
constexpr int RS_TILE_S = BLOCK * RS_ITEMS_S;
constexpr size_t rs_small_n() { return (size_t)256 << 10; }   // below: the one-sweep sort's 1,024-element tiles

static __global__ __launch_bounds__(BLOCK) void k_rs_hist(const uint64_t *__restrict__ keys, size_t n, int shift,
                                                   uint32_t *__restrict__ hist, uint32_t ntiles)
{
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * RS_TILE;
#pragma unroll 4
    for (int k = 0; k < RS_ITEMS; ++k) {
        size_t e = base + (size_t)k * BLOCK + threadIdx.x;
        if (e < n) atomicAdd(&h[(keys[e] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[(size_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// One workgroup per digit: the digit's per-tile counts (a column of hist) become its exclusive prefix over the tiles,
// in place, and total[digit] the column sum. The digits' bases (an exclusive scan of 256 totals) are formed by every
// scatter block itself, so a pass needs no device-wide look-back scan over 256 x tiles counters.
static __global__ __launch_bounds__(BLOCK) void k_rs_colscan(uint32_t *__restrict__ hist, uint32_t ntiles,
                                                      uint32_t *__restrict__ total)
{
    __shared__ uint32_t red[WAVES];
    uint32_t *col = hist + (size_t)blockIdx.x * ntiles;
    constexpr uint32_t PER = 8;
    uint32_t carry = 0;
    for (uint32_t base = 0; base < ntiles; base += BLOCK * PER) {
        const uint32_t i0 = base + threadIdx.x * PER;
        uint32_t v[PER], sum = 0;
#pragma unroll
        for (uint32_t j = 0; j < PER; ++j) { v[j] = i0 + j < ntiles ? col[i0 + j] : 0u; sum += v[j]; }
        uint32_t tot;
        uint32_t run = carry + block_exclusive(sum, OpAdd<uint32_t>(), red, tot);
#pragma unroll
        for (uint32_t j = 0; j < PER; ++j) if (i0 + j < ntiles) { col[i0 + j] = run; run += v[j]; }
        carry += tot;
    }
    if (threadIdx.x == 0) total[blockIdx.x] = carry;
}

// Stable scatter: element order inside a tile is (k, wave, lane); ranks come from 8 ballots per
// wave (peer mask of equal digits) plus a per-digit running count across waves and k steps. The tile is first
// reordered by digit in LDS (48 KiB: keys + values), then written out digit run by digit run, so neighbouring
// lanes store to neighbouring addresses (~16 elements per digit per tile) instead of one element per digit.
static __global__ __launch_bounds__(BLOCK) void k_rs_scatter(const uint64_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                      uint64_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                      size_t n, int shift, const uint32_t *__restrict__ colpre,
                                                      const uint32_t *__restrict__ dtotal, uint32_t ntiles, int iota_vals)
{
    __shared__ uint64_t sk[RS_TILE];
    __shared__ uint32_t sv[RS_TILE];
    __shared__ uint32_t cnt[WAVES][256];
    __shared__ uint32_t wpre[WAVES][256];
    __shared__ uint32_t run[256], lbase[256], gbase[256];
    __shared__ uint32_t red[WAVES];
    const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const uint64_t lt_mask = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
    // this tile's count of digit tid = difference of neighbouring entries of the digit's tile prefix; the digit's
    // global base = the exclusive scan of the digit totals (256 values, one per thread)
    const size_t hi = (size_t)tid * ntiles + blockIdx.x;
    const uint32_t dt = dtotal[tid];
    const uint32_t c0 = colpre[hi];
    const uint32_t c1 = blockIdx.x + 1 < ntiles ? colpre[hi + 1] : dt;
    uint32_t all;
    const uint32_t dbase = block_exclusive(dt, OpAdd<uint32_t>(), red, all);
    const uint32_t g0 = dbase + c0;
    uint32_t tile_total;
    const uint32_t lb = block_exclusive(c1 - c0, OpAdd<uint32_t>(), red, tile_total);
    lbase[tid] = lb;
    gbase[tid] = g0;
    run[tid] = lb;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) cnt[w][tid] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * RS_TILE;
    for (int k = 0; k < RS_ITEMS; ++k) {
        size_t e = base + (size_t)k * BLOCK + tid;
        bool valid = e < n;
        uint64_t key = valid ? kin[e] : 0;
        uint32_t val = valid ? (iota_vals ? (uint32_t)e : vin[e]) : 0;
        uint32_t d = (uint32_t)(key >> shift) & 255u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            uint64_t bal = __ballot((d >> b) & 1u);
            peers &= ((d >> b) & 1u) ? bal : ~bal;
        }
        uint32_t rank = (uint32_t)__popcll(peers & lt_mask);
        if (valid && rank == 0) cnt[wave][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        {
            uint32_t r = run[tid];
#pragma unroll
            for (int w = 0; w < WAVES; ++w) {
                wpre[w][tid] = r;
                r += cnt[w][tid];
                cnt[w][tid] = 0;
            }
            run[tid] = r;
        }
        __syncthreads();
        if (valid) {
            uint32_t dst = wpre[wave][d] + rank;
            sk[dst] = key;
            sv[dst] = val;
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < tile_total; i += BLOCK) {
        const uint64_t key = sk[i];
        const uint32_t d = (uint32_t)(key >> shift) & 255u;
        const uint32_t dst = gbase[d] + (i - lbase[d]);
        kout[dst] = key;
        vout[dst] = sv[i];
    }
}

// ---- one-sweep LSD radix sort: the digit histograms of every pass in one read of the keys, then ONE launch per pass
// whose tiles find their digits' global offsets by a decoupled look-back over the earlier tiles (tickets in launch
// order; a status word per (tile, digit) = count | flag << 30, agent-scope stores and polls: per-XCD L2s are not
// coherent). Three launches per pass (tile histograms, column scans, scatter) become one, and the per-pass histogram
// read of the keys goes. Counts must stay below 2^30.
constexpr uint32_t OS_AGG = 1u << 30, OS_INC = 2u << 30, OS_VAL = (1u << 30) - 1;
constexpr int OS_MAXP = 8;

static __global__ __launch_bounds__(BLOCK) void k_rs_ghist(const uint64_t *__restrict__ keys, size_t n, int lo, int passes,
                                                    uint32_t *__restrict__ ghist, uint32_t *__restrict__ other, uint32_t other_n)
{
    __shared__ uint32_t h[WAVES][OS_MAXP][256];
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = lane_id();
    // reset the other status buffer of this sort tag for its next sort (this sort does not read it)
    for (uint32_t i = blockIdx.x * BLOCK + tid; i < other_n; i += gridDim.x * BLOCK) other[i] = 0;
    for (uint32_t i = tid; i < WAVES * OS_MAXP * 256; i += BLOCK) (&h[0][0][0])[i] = 0;
    __syncthreads();
    // tiles of RS_TILE keys (all of a tile's loads issued up front), blocks striding over them: the block's counts go to
    // the global histogram once (every block adding to the same passes x 256 counters serialises at the L2)
    for (size_t base = (size_t)blockIdx.x * RS_TILE; base < n; base += (size_t)gridDim.x * RS_TILE) {
    uint64_t key[RS_ITEMS];
#pragma unroll
    for (int k = 0; k < RS_ITEMS; ++k) {
        const size_t e = base + (size_t)k * BLOCK + tid;
        key[k] = e < n ? keys[e] : 0;
    }
    for (int p = 0; p < passes; ++p) {
#pragma unroll
        for (int k = 0; k < RS_ITEMS; ++k) {
            // a per-wave LDS histogram, one atomic add per element; a digit shared by the whole wave (a hot key's
            // byte) takes one add instead of 64 serialised ones
            const bool valid = base + (size_t)k * BLOCK + tid < n;
            const uint32_t d = (uint32_t)(key[k] >> (lo + 8 * p)) & 255u;
            const uint32_t d0 = (uint32_t)__shfl((int)d, 0, 64);
            const uint64_t vb = __ballot(valid);
            if (__ballot(valid && d == d0) == vb) {
                if (lane == 0) h[wave][p][d0] += (uint32_t)__popcll(vb);
            } else if (valid) {
                atomicAdd(&h[wave][p][d], 1u);
            }
        }
    }
    }
    __syncthreads();
    for (uint32_t i = tid; i < (uint32_t)passes * 256; i += BLOCK) {
        uint32_t s = 0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) s += h[w][i >> 8][i & 255];
        if (s) atomicAdd(&ghist[i], s);
    }
}

__device__ __forceinline__ void os_store(uint32_t *p, uint32_t w) { __hip_atomic_store(p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ uint32_t os_load(const uint32_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// KO: keys only (no value arrays; e.g. (key << 32 | index) packed into the key): half the LDS, 8 B per element moved
// ITEMS: keys per thread (tile = BLOCK x ITEMS); 4 for small sorts (< rs_small_n() elements: four times the tiles, so a
// pass of a few tiles is not bound by their serial rank / scatter work; config 5: 0.063 -> 0.037 ms), 16 otherwise
template <bool KO, int ITEMS>
static __global__ __launch_bounds__(BLOCK) void k_rs_onesweep(const uint64_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                       uint64_t *__restrict__ kout, uint32_t *__restrict__ vout, size_t n,
                                                       int shift, const uint32_t *__restrict__ dtotal,
                                                       uint32_t *__restrict__ status, uint32_t *__restrict__ ticket,
                                                       int iota_vals)
{
    __shared__ uint64_t sk[(BLOCK * ITEMS)];
    __shared__ uint32_t sv[KO ? 1 : (BLOCK * ITEMS)];
    __shared__ uint32_t cnt[WAVES][256];
    __shared__ uint32_t wpre[WAVES][256];
    __shared__ uint32_t run[256], lbase[256], gbase[256];
    __shared__ uint32_t red[WAVES];
    __shared__ uint32_t s_b;
    const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const uint64_t lt_mask = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
    if (tid == 0) s_b = atomicAdd(ticket, 1u);
    run[tid] = 0;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) cnt[w][tid] = 0;
    __syncthreads();
    const uint32_t b = s_b;
    const size_t base = (size_t)b * (BLOCK * ITEMS);
    // the tile in registers
    uint64_t key[ITEMS];
    uint32_t val[ITEMS], lr[ITEMS], pk[ITEMS];
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const size_t e = base + (size_t)k * BLOCK + tid;
        const bool valid = e < n;
        key[k] = valid ? kin[e] : 0;
        if constexpr (!KO) val[k] = valid ? (iota_vals ? (uint32_t)e : vin[e]) : 0;
    }
    // the tile's digit counts first (one LDS add per distinct digit of a wave), published at once so later tiles'
    // look-backs find them early; each element's peer rank in its wave is kept for the stable ranking below
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const bool valid = base + (size_t)k * BLOCK + tid < n;
        const uint32_t d = (uint32_t)(key[k] >> shift) & 255u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int bb = 0; bb < 8; ++bb) {
            const uint64_t bal = __ballot((d >> bb) & 1u);
            peers &= ((d >> bb) & 1u) ? bal : ~bal;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & lt_mask);
        pk[k] = rank | ((uint32_t)__popcll(peers) << 16);
        if (valid && rank == 0) atomicAdd(&run[d], (uint32_t)__popcll(peers));
    }
    __syncthreads();
    const uint32_t c = run[tid];
    uint32_t *st = status + (size_t)b * 256;
    os_store(&st[tid], b == 0 ? (c | OS_INC) : (c | OS_AGG));
    uint32_t tile_total;
    const uint32_t lb = block_exclusive(c, OpAdd<uint32_t>(), red, tile_total);
    run[tid] = 0;
    lbase[tid] = lb;
    __syncthreads();
    // stable rank of each element among the tile's elements of its digit: order (k, wave, lane)
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const bool valid = base + (size_t)k * BLOCK + tid < n;
        const uint32_t d = (uint32_t)(key[k] >> shift) & 255u;
        const uint32_t rank = pk[k] & 0xFFFFu;
        if (valid && rank == 0) cnt[wave][d] = pk[k] >> 16;
        __syncthreads();
        {
            uint32_t r = run[tid];
#pragma unroll
            for (int w = 0; w < WAVES; ++w) {
                wpre[w][tid] = r;
                r += cnt[w][tid];
                cnt[w][tid] = 0;
            }
            run[tid] = r;
        }
        __syncthreads();
        lr[k] = wpre[wave][d] + rank;
    }
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const size_t e = base + (size_t)k * BLOCK + tid;
        if (e < n) {
            const uint32_t d = (uint32_t)(key[k] >> shift) & 255u;
            const uint32_t dst = lbase[d] + lr[k];
            sk[dst] = key[k];
            if constexpr (!KO) sv[dst] = val[k];
        }
    }
    // the digit's global base = exclusive scan of the digit totals + the earlier tiles' counts (look-back, eight
    // status words in flight per step)
    uint32_t all;
    const uint32_t dbase = block_exclusive(dtotal[tid], OpAdd<uint32_t>(), red, all);
    uint32_t pre = 0;
    if (b > 0) {
#ifndef ACC_OS_LB
#define ACC_OS_LB 8
#endif
        constexpr int LB = ACC_OS_LB;
        for (int64_t j = (int64_t)b - 1;; j -= LB) {
            uint32_t w[LB];
#pragma unroll
            for (int u = 0; u < LB; ++u) w[u] = j - u >= 0 ? os_load(&status[(size_t)(j - u) * 256 + tid]) : OS_INC;
            bool done = false;
#pragma unroll
            for (int u = 0; u < LB; ++u) {
                if (done) continue;
                while ((w[u] >> 30) == 0) {
                    __builtin_amdgcn_s_sleep(1);
                    w[u] = os_load(&status[(size_t)(j - u) * 256 + tid]);
                }
                pre += w[u] & OS_VAL;
                done = (w[u] >> 30) == 2;
            }
            if (done) break;
        }
        os_store(&st[tid], (pre + c) | OS_INC);
    }
    gbase[tid] = dbase + pre;
    __syncthreads();
    for (uint32_t i = tid; i < tile_total; i += BLOCK) {
        const uint64_t k2 = sk[i];
        const uint32_t d = (uint32_t)(k2 >> shift) & 255u;
        const uint32_t dst = gbase[d] + (i - lbase[d]);
        kout[dst] = k2;
        if constexpr (!KO) vout[dst] = sv[i];
    }
}

static __global__ void k_iota(uint32_t *__restrict__ out, size_t n)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (uint32_t)i;
}

struct Sorted {
    uint64_t *keys;
    uint32_t *vals;
};

// The one-sweep words of a sort tag: [passes x 256 digit totals][passes tickets][passes x ntiles x 256 status words].
// Two buffers per tag alternate: the histogram kernel of a sort zeroes the words the previous sort dirtied in the other
// buffer, so no memset precedes a sort (both are zeroed once when they grow). Sorts run on the context stream only.
struct OsWords {
    uint32_t *cur, *other;
    uint32_t other_n;
    acc_ctx::OsState *st;
    size_t words;
    void commit() const   // after the histogram launch: cur is dirty, other is clean
    {
        st->dirty[st->par] = words;
        st->dirty[st->par ^ 1] = 0;
        st->par ^= 1;
    }
};
static inline OsWords os_words(acc_ctx *ctx, const char *tag, size_t words)
{
    if (ctx->launch_stream) fail(ACC_E_STATE, "internal: radix sort launched on a side stream");
    if (words >= 0xFFFFFFFFull) fail(ACC_E_CAP, "internal: radix sort status beyond 2^32 words");
    acc_ctx::OsState &s = ctx->os_state[ctx->ns + tag];
    char n0[56], n1[56];
    snprintf(n0, sizeof n0, "%s_os0", tag);
    snprintf(n1, sizeof n1, "%s_os1", tag);
    uint32_t *b[2] = { ctx->get<uint32_t>(n0, std::max(words, s.cap)), ctx->get<uint32_t>(n1, std::max(words, s.cap)) };
    if (words > s.cap) {
        for (int i = 0; i < 2; ++i) ACC_HIP(hipMemsetAsync(b[i], 0, words * sizeof(uint32_t), ctx->stream));
        s.cap = words;
        s.dirty[0] = s.dirty[1] = 0;
    }
    return OsWords{ b[s.par], b[s.par ^ 1], (uint32_t)s.dirty[s.par ^ 1], &s, words };
}

// Stable sort of n (key, value) pairs by the low `bits` bits of key (higher bits must be zero).
// vals == nullptr sorts with values = index. Results live in context buffers "<tag>_k?/_v?" and stay
// valid until the next sort with the same tag.
static inline Sorted radix_sort(acc_ctx *ctx, const char *tag, const uint64_t *keys, const uint32_t *vals, size_t n, int bits)
{
    char nk0[40], nk1[40], nv0[40], nv1[40], nh[40], th[48], ts[48];
    snprintf(th, sizeof th, "%s.hist", tag);
    snprintf(ts, sizeof ts, "%s.scatter", tag);
    snprintf(nk0, sizeof nk0, "%s_k0", tag); snprintf(nk1, sizeof nk1, "%s_k1", tag);
    snprintf(nv0, sizeof nv0, "%s_v0", tag); snprintf(nv1, sizeof nv1, "%s_v1", tag);
    snprintf(nh, sizeof nh, "%s_hist", tag);
    uint64_t *k[2] = { ctx->get<uint64_t>(nk0, n), ctx->get<uint64_t>(nk1, n) };
    uint32_t *v[2] = { ctx->get<uint32_t>(nv0, n), ctx->get<uint32_t>(nv1, n) };
    int passes = (bits + 7) / 8;
    if (n == 0) return { k[0], v[0] };
    if (passes == 0) {
        ACC_HIP(hipMemcpyAsync(k[0], keys, n * sizeof(uint64_t), hipMemcpyDeviceToDevice, ctx->stream));
        if (vals) ACC_HIP(hipMemcpyAsync(v[0], vals, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, ctx->stream));
        else launch(ctx, "iota", k_iota, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, v[0], n);
        return { k[0], v[0] };
    }
    if (n < (size_t)OS_VAL && passes <= OS_MAXP) {   // else (very large sorts): three launches per pass below
        const bool small = n < rs_small_n();
        const uint32_t ntiles = (uint32_t)((n + (small ? RS_TILE_S : RS_TILE) - 1) / (small ? RS_TILE_S : RS_TILE));
        const size_t words = (size_t)passes * 256 + passes + (size_t)passes * ntiles * 256;
        const OsWords ow = os_words(ctx, tag, words);
        uint32_t *ghist = ow.cur, *tickets = ow.cur + (size_t)passes * 256, *status = tickets + passes;
        snprintf(th, sizeof th, "%s.ghist", tag);
        launch(ctx, th, k_rs_ghist, dim3(std::min<unsigned>(ntiles, 1024u)), dim3(BLOCK), 0, keys, n, 0, passes, ghist, ow.other,
               ow.other_n);
        ow.commit();
        const uint64_t *kin = keys;
        const uint32_t *vin = vals;
        int cur = 0;
        for (int p = 0; p < passes; ++p) {
            if (small)
                launch(ctx, ts, k_rs_onesweep<false, RS_ITEMS_S>, dim3(ntiles), dim3(BLOCK), 0, kin, vin, k[cur], v[cur], n, 8 * p,
                       (const uint32_t *)(ghist + (size_t)p * 256), status + (size_t)p * ntiles * 256, tickets + p,
                       (p == 0 && !vals) ? 1 : 0);
            else
                launch(ctx, ts, k_rs_onesweep<false, RS_ITEMS>, dim3(ntiles), dim3(BLOCK), 0, kin, vin, k[cur], v[cur], n, 8 * p,
                       (const uint32_t *)(ghist + (size_t)p * 256), status + (size_t)p * ntiles * 256, tickets + p,
                       (p == 0 && !vals) ? 1 : 0);
            kin = k[cur];
            vin = v[cur];
            cur ^= 1;
        }
        return { (uint64_t *)kin, (uint32_t *)vin };
    }
    const uint32_t ntiles = (uint32_t)((n + RS_TILE - 1) / RS_TILE);
    uint32_t *hist = ctx->get<uint32_t>(nh, (size_t)256 * ntiles);
    char nt[48];
    snprintf(nt, sizeof nt, "%s_dtot", tag);
    uint32_t *dtot = ctx->get<uint32_t>(nt, 256);
    const uint64_t *kin = keys;
    const uint32_t *vin = vals;
    int cur = 0;
    for (int p = 0; p < passes; ++p) {
        int shift = 8 * p;
        launch(ctx, th, k_rs_hist, dim3(ntiles), dim3(BLOCK), 0, kin, n, shift, hist, ntiles);
        launch(ctx, "rs_colscan", k_rs_colscan, dim3(256), dim3(BLOCK), 0, hist, ntiles, dtot);
        launch(ctx, ts, k_rs_scatter, dim3(ntiles), dim3(BLOCK), 0, kin, vin, k[cur], v[cur], n, shift,
               (const uint32_t *)hist, (const uint32_t *)dtot, ntiles, (p == 0 && !vals) ? 1 : 0);
        kin = k[cur];
        vin = v[cur];
        cur ^= 1;
    }
    return { (uint64_t *)kin, (uint32_t *)vin };
}

// Stable sort of n u64 keys by bits [lo, lo + bits) (bits above must be zero; bits below ride along, e.g. an index packed
// under the key). One-sweep only: n < 2^30. The result lives in the context buffers "<tag>_k?".
static inline uint64_t *radix_sort_keys(acc_ctx *ctx, const char *tag, const uint64_t *keys, size_t n, int lo, int bits)
{
    char nk0[40], nk1[40], th[48], ts[48];
    snprintf(nk0, sizeof nk0, "%s_k0", tag); snprintf(nk1, sizeof nk1, "%s_k1", tag);
    snprintf(th, sizeof th, "%s.ghist", tag);
    snprintf(ts, sizeof ts, "%s.scatter", tag);
    uint64_t *k[2] = { ctx->get<uint64_t>(nk0, n), ctx->get<uint64_t>(nk1, n) };
    const int passes = (bits + 7) / 8;
    if (n >= (size_t)OS_VAL || passes > OS_MAXP) fail(ACC_E_CAP, "internal: keys-only radix sort beyond its limits");
    if (n == 0 || passes == 0) {
        if (n) ACC_HIP(hipMemcpyAsync(k[0], keys, n * sizeof(uint64_t), hipMemcpyDeviceToDevice, ctx->cur()));
        return k[0];
    }
    const bool small = n < rs_small_n();
    const uint32_t ntiles = (uint32_t)((n + (small ? RS_TILE_S : RS_TILE) - 1) / (small ? RS_TILE_S : RS_TILE));
    const size_t words = (size_t)passes * 256 + passes + (size_t)passes * ntiles * 256;
    const OsWords ow = os_words(ctx, tag, words);
    uint32_t *ghist = ow.cur, *tickets = ow.cur + (size_t)passes * 256, *status = tickets + passes;
    launch(ctx, th, k_rs_ghist, dim3(std::min<unsigned>(ntiles, 1024u)), dim3(BLOCK), 0, keys, n, lo, passes, ghist, ow.other,
           ow.other_n);
    ow.commit();
    const uint64_t *kin = keys;
    int cur = 0;
    for (int p = 0; p < passes; ++p) {
        if (small)
            launch(ctx, ts, k_rs_onesweep<true, RS_ITEMS_S>, dim3(ntiles), dim3(BLOCK), 0, kin, (const uint32_t *)nullptr, k[cur],
                   (uint32_t *)nullptr, n, lo + 8 * p, (const uint32_t *)(ghist + (size_t)p * 256),
                   status + (size_t)p * ntiles * 256, tickets + p, 0);
        else
            launch(ctx, ts, k_rs_onesweep<true, RS_ITEMS>, dim3(ntiles), dim3(BLOCK), 0, kin, (const uint32_t *)nullptr, k[cur],
                   (uint32_t *)nullptr, n, lo + 8 * p, (const uint32_t *)(ghist + (size_t)p * 256),
                   status + (size_t)p * ntiles * 256, tickets + p, 0);
        kin = k[cur];
        cur ^= 1;
    }
    return (uint64_t *)kin;
}

inline int bits_for(uint64_t max_value)
{
    return max_value == 0 ? 0 : 64 - __builtin_clzll(max_value);
}

}  // namespace acc
