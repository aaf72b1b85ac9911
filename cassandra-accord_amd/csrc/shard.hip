// shard.hip — CommandStore shards across GPUs: the per-node reduce of per-shard PartialDeps
// (PreAccept.reduce, messages/PreAccept.java:141-156; CommandStores.mapReduce fold in shard order,
// local/CommandStores.java:575-592).
//
// Each GPU is one CommandStore owning a contiguous key range (ShardDistributor.EvenSplit,
// local/ShardDistributor.java:106-156). After its acc_keydeps_batch:
//   pack   — every txn with a non-empty shard KeyDeps becomes one fragment for its home rank (t mod world):
//            a header (t, nk, nv, no), its key codes, its TxnIds (batch indices) and its Java keysToTxnIds, in four
//            destination-major streams ready for an all-to-all(v) (RCCL over xGMI, driven by the host);
//   merge  — the home rank orders the received fragments by txn (stable: source rank = shard order within a txn),
//            lays them out as acc_merge_in replies and runs the batched KeyDeps.merge (merge.hip), which is
//            PartialDeps.with folded over the shards (KeyDeps.with = linearUnion, primitives/KeyDeps.java:238-253).
#include "prims.hpp"

#include <vector>

namespace acc {
void keydeps_merge(acc_ctx *ctx, const acc_merge_in *in, acc_merge_view *view);
void deps_merge(acc_ctx *ctx, const acc_deps_merge_in *in, acc_deps_merge_view *view);

namespace sh {

// dest-major position of txn t: dest d = t mod world, slot t / world within the dest's G = ceil(n / world) slots
__device__ __forceinline__ uint32_t dm_index(uint32_t t, uint32_t world, uint32_t G) { return (t % world) * G + t / world; }

// counts at the dest-major slot of every batch txn (slots of global txns not in this batch stay zero)
__global__ __launch_bounds__(BLOCK) void k_sh_sizes(uint32_t n, uint32_t world, uint32_t G, const uint32_t *__restrict__ gidx,
                                                    const uint64_t *__restrict__ kd_off, const uint64_t *__restrict__ u_off,
                                                    const uint64_t *__restrict__ arena_off, uint64_t *__restrict__ c_frag,
                                                    uint64_t *__restrict__ c_key, uint64_t *__restrict__ c_val,
                                                    uint64_t *__restrict__ c_k2v)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= n) return;
    const uint32_t i = dm_index(gidx ? gidx[t] : t, world, G);
    const uint64_t nk = kd_off[t + 1] - kd_off[t];   // KeyDeps.isEmpty <=> no keys (keys without deps are dropped)
    c_frag[i] = nk ? 1 : 0;
    c_key[i] = nk;
    c_val[i] = nk ? u_off[t + 1] - u_off[t] : 0;
    c_k2v[i] = nk ? arena_off[t + 1] - arena_off[t] : 0;
}

// one wave per txn with a fragment: header + key codes + TxnIds + keysToTxnIds at the stream offsets
__global__ __launch_bounds__(BLOCK) void k_sh_pack(uint32_t n, uint32_t world, uint32_t G, const uint32_t *__restrict__ key_off,
                                                   const uint64_t *__restrict__ key_code, const uint64_t *__restrict__ kd_off,
                                                   const uint32_t *__restrict__ key_idx, const uint64_t *__restrict__ u_off,
                                                   const uint32_t *__restrict__ dep_txn, const uint64_t *__restrict__ arena_off,
                                                   const int32_t *__restrict__ arena, const uint64_t *__restrict__ kd_key,
                                                   const uint32_t *__restrict__ gidx,
                                                   const uint64_t *__restrict__ o_frag,
                                                   const uint64_t *__restrict__ o_key, const uint64_t *__restrict__ o_val,
                                                   const uint64_t *__restrict__ o_k2v, uint32_t *__restrict__ hdr,
                                                   uint64_t *__restrict__ keys, uint32_t *__restrict__ vals,
                                                   int32_t *__restrict__ k2v)
{
    const uint32_t t = blockIdx.x * WAVES + (threadIdx.x >> 6), lane = lane_id();
    if (t >= n) return;
    const uint64_t k0 = kd_off[t], nk = kd_off[t + 1] - k0;
    if (nk == 0) return;
    const uint32_t tg = gidx ? gidx[t] : t;
    const uint32_t i = dm_index(tg, world, G);
    const uint64_t v0 = u_off[t], nv = u_off[t + 1] - v0, a0 = arena_off[t], no = arena_off[t + 1] - a0;
    const uint64_t f = o_frag[i], ok = o_key[i], ov = o_val[i], oo = o_k2v[i];
    if (lane < 4) hdr[4 * f + lane] = lane == 0 ? tg : lane == 1 ? (uint32_t)nk : lane == 2 ? (uint32_t)nv : (uint32_t)no;
    const uint32_t kb = key_off[t];
    // kd_key (acc_keydeps_mixed / acc_partial_deps_batch): the KeyDeps keys as codes (a range txn's keys are not its own)
    for (uint64_t j = lane; j < nk; j += 64) keys[ok + j] = kd_key ? kd_key[k0 + j] : key_code[kb + key_idx[k0 + j]];
    // the global map is increasing (a store's txns are a TxnId-ordered subsequence), so lists stay sorted
    for (uint64_t j = lane; j < nv; j += 64) vals[ov + j] = gidx ? gidx[dep_txn[v0 + j]] : dep_txn[v0 + j];
    for (uint64_t j = lane; j < no; j += 64) k2v[oo + j] = arena[a0 + j];
}

// received fragments (source-major): sizes, group (= home-local txn slot t / world) and the sort key
__global__ __launch_bounds__(BLOCK) void k_sh_frag(uint64_t F, uint32_t world, uint32_t n_groups, const uint32_t *__restrict__ hdr,
                                                   uint64_t *__restrict__ f_key, uint64_t *__restrict__ f_val,
                                                   uint64_t *__restrict__ f_k2v, uint64_t *__restrict__ gkey,
                                                   uint64_t *__restrict__ err)
{
    const uint64_t f = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (f >= F) return;
    const uint32_t t = hdr[4 * f], g = t / world;
    f_key[f] = hdr[4 * f + 1];
    f_val[f] = hdr[4 * f + 2];
    f_k2v[f] = hdr[4 * f + 3];
    gkey[f] = g;
    if (g >= n_groups) atomicOr((unsigned long long *)err, 1ull);
}

__global__ __launch_bounds__(BLOCK) void k_sh_group_hist(uint64_t F, const uint64_t *__restrict__ gkey, uint64_t *__restrict__ gcnt)
{
    const uint64_t f = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (f < F) atomicAdd((unsigned long long *)&gcnt[gkey[f]], 1ull);
}

// reply r = sorted fragment perm[r]: its sizes in reply order
__global__ __launch_bounds__(BLOCK) void k_sh_reply_sizes(uint64_t F, const uint32_t *__restrict__ perm, const uint64_t *__restrict__ f_key,
                                                          const uint64_t *__restrict__ f_val, const uint64_t *__restrict__ f_k2v,
                                                          uint64_t *__restrict__ r_key, uint64_t *__restrict__ r_val,
                                                          uint64_t *__restrict__ r_k2v)
{
    const uint64_t r = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (r >= F) return;
    const uint32_t f = perm[r];
    r_key[r] = f_key[f];
    r_val[r] = f_val[f];
    r_k2v[r] = f_k2v[f];
}

// one wave per reply: copy its three segments from the received streams into the merge layout
__global__ __launch_bounds__(BLOCK) void k_sh_gather(uint64_t F, const uint32_t *__restrict__ perm,
                                                     const uint64_t *__restrict__ sk, const uint64_t *__restrict__ sv,
                                                     const uint64_t *__restrict__ so, const uint64_t *__restrict__ rk,
                                                     const uint64_t *__restrict__ rv, const uint64_t *__restrict__ ro,
                                                     const uint64_t *__restrict__ keys, const uint32_t *__restrict__ vals,
                                                     const int32_t *__restrict__ k2v, uint64_t *__restrict__ m_keys,
                                                     uint32_t *__restrict__ m_vals, int32_t *__restrict__ m_k2v)
{
    const uint64_t r = (uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    const uint32_t lane = lane_id();
    if (r >= F) return;
    const uint32_t f = perm[r];
    const uint64_t nk = rk[r + 1] - rk[r], nv = rv[r + 1] - rv[r], no = ro[r + 1] - ro[r];
    for (uint64_t j = lane; j < nk; j += 64) m_keys[rk[r] + j] = keys[sk[f] + j];
    for (uint64_t j = lane; j < nv; j += 64) m_vals[rv[r] + j] = vals[sv[f] + j];
    for (uint64_t j = lane; j < no; j += 64) m_k2v[ro[r] + j] = k2v[so[f] + j];
}

// ---------------------------------------------------------------- fused reduce (disjoint, shard-ordered keys)
//
// Replies of one home txn come from different shards in shard order, and shards own ascending disjoint key ranges,
// so PartialDeps.with over them (linearUnion of KeyDeps) is: keys = concatenation, txnIds = sorted union of the
// replies' txnIds, each keysToTxnIds entry re-indexed into that union, header = running entry counts. The order
// assumption is checked (err) and the general batched merge runs instead when it does not hold.

constexpr uint32_t FUSE_WAVE = 64;     // raw TxnIds per txn for the wave tier
constexpr uint32_t FUSE_BLOCK = 8192;  // workgroup tier (LDS)
constexpr uint32_t FUSE_BIG = 32768;   // 1024-thread workgroup tier (128 KiB of LDS)

struct Fuse {
    uint32_t ng;
    const uint64_t *grp_off, *rk, *rv, *ro;        // replies (gathered layout)
    const uint64_t *keys;
    const uint32_t *vals;
    const int32_t *k2v;
    uint64_t *c_nk, *c_nu, *c_no;                  // sizes per group
    const uint64_t *key_out, *val_out, *k2v_out;   // offsets (write pass)
    uint64_t *m_keys;
    uint32_t *m_vals;
    int32_t *m_k2v;
    uint32_t *blk_list, *glb_list, *big_list;
    uint64_t *gstat;                               // [0] block groups, [1] global groups, [2] scratch u32, [3] order err,
                                                   // [4] big groups
    const uint64_t *glb_off;
    uint32_t *scratch;
};

__device__ __forceinline__ uint32_t lb_u32(const uint32_t *a, uint32_t n, uint32_t v)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// copy keys + re-index keysToTxnIds of group g given its union u[0..U) (LDS or global); `tid`/`nth` = this thread's
// index among the cooperating threads (a wave or a workgroup)
__device__ __forceinline__ void fuse_emit(const Fuse &f, uint32_t g, const uint32_t *u, uint32_t U, uint32_t tid, uint32_t nth)
{
    const uint64_t r0 = f.grp_off[g], r1 = f.grp_off[g + 1];
    const uint64_t kb0 = f.rk[r0], NK = f.rk[r1] - kb0, ob0 = f.ro[r0];
    const uint64_t ko = f.key_out[g], oo = f.k2v_out[g];
    for (uint64_t j = tid; j < NK; j += nth) f.m_keys[ko + j] = f.keys[kb0 + j];
    for (uint64_t r = r0; r < r1; ++r) {
        const uint64_t nk = f.rk[r + 1] - f.rk[r], no = f.ro[r + 1] - f.ro[r];
        const uint64_t kb = f.rk[r] - kb0, eb = (f.ro[r] - ob0) - kb;   // keys / entries of earlier replies
        const int32_t *src = f.k2v + f.ro[r];
        const uint32_t *vals = f.vals + f.rv[r];
        for (uint64_t j = tid; j < nk; j += nth) f.m_k2v[oo + kb + j] = (int32_t)(NK + eb + ((uint64_t)src[j] - nk));
        for (uint64_t i = tid; i < no - nk; i += nth)
            f.m_k2v[oo + NK + eb + i] = (int32_t)lb_u32(u, U, vals[src[nk + i]]);
    }
}

// key order check of group g (disjoint ascending across its replies) by the cooperating threads
__device__ __forceinline__ bool fuse_keys_ordered(const Fuse &f, uint32_t g, uint32_t tid, uint32_t nth)
{
    const uint64_t r0 = f.grp_off[g], r1 = f.grp_off[g + 1];
    bool ok = true;
    for (uint64_t r = r0 + 1 + tid; r < r1; r += nth)
        if (f.rk[r] > f.rk[r - 1] && f.rk[r + 1] > f.rk[r] && f.keys[f.rk[r] - 1] >= f.keys[f.rk[r]]) ok = false;
    return ok;
}

template <bool WRITE>
__global__ __launch_bounds__(BLOCK) void k_fuse_wave(Fuse f)
{
    __shared__ uint32_t su[WAVES][64];
    const uint32_t wave = threadIdx.x >> 6, lane = lane_id();
    const uint32_t g = blockIdx.x * WAVES + wave;
    if (g >= f.ng) return;
    const uint64_t r0 = f.grp_off[g], r1 = f.grp_off[g + 1];
    const uint64_t nraw = f.rv[r1] - f.rv[r0];
    if (!WRITE) {
        const bool ok = __all(fuse_keys_ordered(f, g, lane, 64));
        if (!ok && lane == 0) atomicOr((unsigned long long *)&f.gstat[3], 1ull);
    }
    if (nraw > FUSE_WAVE) {
        if (!WRITE && lane == 0) {
            if (nraw <= FUSE_BLOCK) f.blk_list[atomicAdd((unsigned long long *)&f.gstat[0], 1ull)] = g;
            else if (nraw <= FUSE_BIG) f.big_list[atomicAdd((unsigned long long *)&f.gstat[4], 1ull)] = g;
            else {
                f.glb_list[atomicAdd((unsigned long long *)&f.gstat[1], 1ull)] = g;
                uint64_t n2 = 64; while (n2 < nraw) n2 <<= 1;
                atomicAdd((unsigned long long *)&f.gstat[2], 2 * n2);
            }
        }
        return;
    }
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    uint32_t x = lane < nraw ? f.vals[f.rv[r0] + lane] : 0xFFFFFFFFu;
    x = bitonic_reg(x);
    const uint32_t prev = shfl_up(x, 1);
    const bool nw = lane < nraw && (lane == 0 || x != prev);
    const uint64_t nb = __ballot(nw);
    const uint32_t U = (uint32_t)__popcll(nb);
    if (!WRITE) {
        if (lane == 0) {
            f.c_nk[g] = f.rk[r1] - f.rk[r0];
            f.c_nu[g] = U;
            f.c_no[g] = f.ro[r1] - f.ro[r0];
        }
        return;
    }
    const uint32_t pos = (uint32_t)__popcll(nb & lt);
    if (nw) { su[wave][pos] = x; f.m_vals[f.val_out[g] + pos] = x; }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    fuse_emit(f, g, su[wave], U, lane, 64);
}

// one workgroup per group: sort the raw TxnIds (A), compact the union (B), re-index
template <bool WRITE>
__device__ void fuse_block(const Fuse &f, uint32_t g, uint32_t *A, uint32_t *B, uint32_t *red)
{
    const uint32_t tid = threadIdx.x;
    const uint64_t r0 = f.grp_off[g], r1 = f.grp_off[g + 1];
    const uint32_t nraw = (uint32_t)(f.rv[r1] - f.rv[r0]);
    uint32_t n2 = 64;
    while (n2 < nraw) n2 <<= 1;
    for (uint32_t i = tid; i < n2; i += BLOCK) A[i] = i < nraw ? f.vals[f.rv[r0] + i] : 0xFFFFFFFFu;
    __syncthreads();
    block_bitonic(A, n2);
    const uint32_t per = (n2 + BLOCK - 1) / BLOCK;
    const uint32_t lo = tid * per, hi = min(lo + per, n2);
    uint32_t c = 0;
    for (uint32_t i = lo; i < hi; ++i) c += (i < nraw && (i == 0 || A[i] != A[i - 1])) ? 1u : 0u;
    uint32_t U;
    uint32_t p = block_exclusive(c, OpAdd<uint32_t>(), red, U);
    if (!WRITE) {
        if (tid == 0) { f.c_nk[g] = f.rk[r1] - f.rk[r0]; f.c_nu[g] = U; f.c_no[g] = f.ro[r1] - f.ro[r0]; }
        return;
    }
    for (uint32_t i = lo; i < hi; ++i)
        if (i < nraw && (i == 0 || A[i] != A[i - 1])) { B[p] = A[i]; f.m_vals[f.val_out[g] + p] = A[i]; ++p; }
    __syncthreads();
    fuse_emit(f, g, B, U, tid, BLOCK);
}

template <bool WRITE>
__global__ __launch_bounds__(BLOCK) void k_fuse_block(Fuse f)
{
    __shared__ uint32_t A[FUSE_BLOCK], B[FUSE_BLOCK];
    __shared__ uint32_t red[WAVES];
    fuse_block<WRITE>(f, f.blk_list[blockIdx.x], A, B, red);
}

// 1024-thread workgroup per group (FUSE_BLOCK < raw TxnIds <= FUSE_BIG): sort in LDS, union compacted in place
template <bool WRITE>
__global__ __launch_bounds__(1024) void k_fuse_big(Fuse f)
{
    constexpr int NT = 1024, NW = NT / 64, PER = FUSE_BIG / NT;
    __shared__ uint32_t A[FUSE_BIG];
    __shared__ uint32_t red[NW];
    const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const uint32_t g = f.big_list[blockIdx.x];
    const uint64_t r0 = f.grp_off[g], r1 = f.grp_off[g + 1];
    const uint32_t nraw = (uint32_t)(f.rv[r1] - f.rv[r0]);
    uint32_t n2 = NT;
    while (n2 < nraw) n2 <<= 1;
    for (uint32_t i = tid; i < n2; i += NT) A[i] = i < nraw ? f.vals[f.rv[r0] + i] : 0xFFFFFFFFu;
    __syncthreads();
    block_bitonic<uint32_t, NT>(A, n2);
    const uint32_t per = n2 / NT, lo = tid * per;
    uint32_t x[PER];
    uint32_t fl = 0, c = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q)
        if ((uint32_t)q < per) {
            const uint32_t i = lo + q;
            x[q] = A[i];
            const bool nw = i < nraw && (i == 0 || A[i - 1] != x[q]);
            fl |= (uint32_t)nw << q;
            c += nw;
        }
    // block exclusive scan over 16 waves
    uint32_t incl = c;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) { const uint32_t u = __shfl_up(incl, d, 64); if (lane >= d) incl += u; }
    if (lane == 63) red[wave] = incl;
    __syncthreads();
    uint32_t p = incl - c, U = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) { const uint32_t r = red[w]; if (w < (int)wave) p += r; U += r; }
    if (!WRITE) {
        if (tid == 0) { f.c_nk[g] = f.rk[r1] - f.rk[r0]; f.c_nu[g] = U; f.c_no[g] = f.ro[r1] - f.ro[r0]; }
        return;
    }
#pragma unroll
    for (int q = 0; q < PER; ++q)
        if ((uint32_t)q < per && ((fl >> q) & 1u)) { A[p] = x[q]; f.m_vals[f.val_out[g] + p] = x[q]; ++p; }
    __syncthreads();
    fuse_emit(f, g, A, U, tid, NT);
}

template <bool WRITE>
__global__ __launch_bounds__(BLOCK) void k_fuse_global(Fuse f)
{
    __shared__ uint32_t red[WAVES];
    const uint32_t g = f.glb_list[blockIdx.x];
    const uint64_t nraw = f.rv[f.grp_off[g + 1]] - f.rv[f.grp_off[g]];
    uint64_t n2 = 64;
    while (n2 < nraw) n2 <<= 1;
    uint32_t *A = f.scratch + f.glb_off[blockIdx.x];
    fuse_block<WRITE>(f, g, A, A + n2, red);
}

__global__ __launch_bounds__(BLOCK) void k_fuse_glb_sizes(uint32_t ng, Fuse f, uint64_t *__restrict__ sz)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= ng) return;
    const uint32_t g = f.glb_list[i];
    const uint64_t nraw = f.rv[f.grp_off[g + 1]] - f.rv[f.grp_off[g]];
    uint64_t n2 = 64;
    while (n2 < nraw) n2 <<= 1;
    sz[i] = 2 * n2;
}

// ---- the RangeDeps half: a fragment per txn with a non-empty store RangeDeps = header (t, nr, nv, no), its ranges
// as (start, end) codes, its TxnIds raw (msb, lsb, node: the home rank holds no other store's batch), its Java
// rangesToTxnIds ints
__global__ __launch_bounds__(BLOCK) void k_shr_sizes(uint32_t n, uint32_t world, uint32_t G, const uint32_t *__restrict__ gidx,
                                                     const uint64_t *__restrict__ rd_off, const uint64_t *__restrict__ u_off,
                                                     const uint64_t *__restrict__ arena_off, uint64_t *__restrict__ c_frag,
                                                     uint64_t *__restrict__ c_rng, uint64_t *__restrict__ c_val,
                                                     uint64_t *__restrict__ c_k2v)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= n) return;
    const uint32_t i = dm_index(gidx ? gidx[t] : t, world, G);
    const uint64_t nr = rd_off[t + 1] - rd_off[t];   // RangeDeps.isEmpty <=> no ranges
    c_frag[i] = nr ? 1 : 0;
    c_rng[i] = nr;
    c_val[i] = nr ? u_off[t + 1] - u_off[t] : 0;
    c_k2v[i] = nr ? arena_off[t + 1] - arena_off[t] : 0;
}

__global__ __launch_bounds__(BLOCK) void k_shr_pack(uint32_t n, uint32_t world, uint32_t G, acc_rangedeps_view v,
                                                    const uint64_t *__restrict__ tm, const uint64_t *__restrict__ tl,
                                                    const int32_t *__restrict__ tn, const uint32_t *__restrict__ gidx,
                                                    const uint64_t *__restrict__ o_frag, const uint64_t *__restrict__ o_rng,
                                                    const uint64_t *__restrict__ o_val, const uint64_t *__restrict__ o_k2v,
                                                    uint32_t *__restrict__ hdr, uint64_t *__restrict__ rng,
                                                    uint64_t *__restrict__ txn, int32_t *__restrict__ k2v)
{
    const uint32_t t = blockIdx.x * WAVES + (threadIdx.x >> 6), lane = lane_id();
    if (t >= n) return;
    const uint64_t r0 = v.rd_off[t], nr = v.rd_off[t + 1] - r0;
    if (nr == 0) return;
    const uint32_t tg = gidx ? gidx[t] : t;
    const uint32_t i = dm_index(tg, world, G);
    const uint64_t v0 = v.u_off[t], nv = v.u_off[t + 1] - v0, a0 = v.arena_off[t], no = v.arena_off[t + 1] - a0;
    const uint64_t f = o_frag[i], orr = o_rng[i], ov = o_val[i], oo = o_k2v[i];
    if (lane < 4) hdr[4 * f + lane] = lane == 0 ? tg : lane == 1 ? (uint32_t)nr : lane == 2 ? (uint32_t)nv : (uint32_t)no;
    for (uint64_t j = lane; j < nr; j += 64) {
        const uint32_t id = v.range_id[r0 + j];
        rng[2 * (orr + j)] = v.rng_start[id];
        rng[2 * (orr + j) + 1] = v.rng_end[id];
    }
    for (uint64_t j = lane; j < nv; j += 64) {
        const uint32_t d = v.dep_txn[v0 + j];
        txn[3 * (ov + j)] = tm[d];
        txn[3 * (ov + j) + 1] = tl[d];
        txn[3 * (ov + j) + 2] = (uint64_t)(uint32_t)tn[d];
    }
    for (uint64_t j = lane; j < no; j += 64) k2v[oo + j] = v.arena[a0 + j];
}

// one wave per reply: its ranges, raw TxnIds and ints from the received streams into the Deps.merge input layout
__global__ __launch_bounds__(BLOCK) void k_shr_gather(uint64_t F, const uint32_t *__restrict__ perm,
                                                      const uint64_t *__restrict__ sk, const uint64_t *__restrict__ sv,
                                                      const uint64_t *__restrict__ so, const uint64_t *__restrict__ rk,
                                                      const uint64_t *__restrict__ rv, const uint64_t *__restrict__ ro,
                                                      const uint64_t *__restrict__ rng, const uint64_t *__restrict__ txn,
                                                      const int32_t *__restrict__ k2v, uint64_t *__restrict__ ka,
                                                      uint64_t *__restrict__ kb, uint64_t *__restrict__ msb,
                                                      uint64_t *__restrict__ lsb, int32_t *__restrict__ node,
                                                      int32_t *__restrict__ m_k2v)
{
    const uint64_t r = (uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    const uint32_t lane = lane_id();
    if (r >= F) return;
    const uint32_t f = perm[r];
    const uint64_t nk = rk[r + 1] - rk[r], nv = rv[r + 1] - rv[r], no = ro[r + 1] - ro[r];
    for (uint64_t j = lane; j < nk; j += 64) {
        ka[rk[r] + j] = rng[2 * (sk[f] + j)];
        kb[rk[r] + j] = rng[2 * (sk[f] + j) + 1];
    }
    for (uint64_t j = lane; j < nv; j += 64) {
        const uint64_t x = 3 * (sv[f] + j);
        msb[rv[r] + j] = txn[x];
        lsb[rv[r] + j] = txn[x + 1];
        node[rv[r] + j] = (int32_t)(uint32_t)txn[x + 2];
    }
    for (uint64_t j = lane; j < no; j += 64) m_k2v[ro[r] + j] = k2v[so[f] + j];
}

}  // namespace sh

using namespace sh;

// ctx_alloc: the four streams are allocated from the context (device) once their sizes are known and returned in
// out->hdr/keys/vals/k2v (acc_shard_reduce); otherwise they are the caller's (two-call sizing).
void shard_pack(acc_ctx *ctx, const acc_batch_in *in, acc_frag_streams *out, bool ctx_alloc)
{
    if (!in || !out) fail(ACC_E_ARG, "null argument");
    const uint32_t world = out->world;
    if (world == 0) fail(ACC_E_ARG, "world must be >= 1");
    if (!out->frag_off || !out->key_off || !out->val_off || !out->k2v_off) fail(ACC_E_ARG, "null offset arrays");
    if (!ctx->kd_valid) fail(ACC_E_STATE, "no keydeps result on this context");
    const acc_keydeps_view &v = ctx->kd_view;
    const uint32_t n = v.n_txn;
    if (in->n_txn != n) fail(ACC_E_ARG, "batch does not match the last keydeps result");
    hipStream_t st = ctx->stream;
    const size_t P = (size_t)in->n_pairs;
    const uint32_t *key_off = stage_in(ctx, "in_key_off", in->key_off, (size_t)n + 1, in->mem);
    const uint64_t *key_code = stage_in(ctx, "in_key_code", in->key_code, P, in->mem);
    const uint32_t *gidx = out->txn_global ? stage_in(ctx, "sh_gidx", out->txn_global, n, in->mem) : nullptr;
    uint32_t n_global = n;
    if (gidx && n) {
        uint32_t last = 0;
        ACC_HIP(hipMemcpyAsync(ctx->pinned, gidx + (n - 1), 4, hipMemcpyDeviceToHost, st));
        ctx->sync();
        memcpy(&last, ctx->pinned, 4);
        n_global = last + 1;
    }
    const uint32_t G = (n_global + world - 1) / world;
    const size_t M = (size_t)world * G;
    uint64_t *c[4], *o[4];
    const char *cn[4] = { "sh_c_frag", "sh_c_key", "sh_c_val", "sh_c_k2v" };
    const char *on[4] = { "sh_o_frag", "sh_o_key", "sh_o_val", "sh_o_k2v" };
    for (int q = 0; q < 4; ++q) {
        c[q] = ctx->get<uint64_t>(cn[q], M);
        o[q] = ctx->get<uint64_t>(on[q], M + 1);
        ACC_HIP(hipMemsetAsync(c[q], 0, M * sizeof(uint64_t), st));
    }
    launch(ctx, "sh_sizes", k_sh_sizes, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, world, G, gidx, v.kd_off, v.u_off,
           v.arena_off, c[0], c[1], c[2], c[3]);
    for (int q = 0; q < 4; ++q) scan<uint64_t, OpAdd<uint64_t>>(ctx, c[q], o[q], M, true, o[q] + M);
    // per-destination boundaries (slot d * G of each stream's offsets) -> host
    uint64_t *bounds = ctx->get<uint64_t>("sh_bounds", 4 * ((size_t)world + 1));
    for (int q = 0; q < 4; ++q)
        for (uint32_t d = 0; d <= world; ++d)
            ACC_HIP(hipMemcpyAsync(bounds + q * (world + 1) + d, o[q] + std::min((size_t)d * G, M), 8,
                                   hipMemcpyDeviceToDevice, st));
    std::vector<uint64_t> hb(4 * ((size_t)world + 1));
    ACC_HIP(hipMemcpyAsync(hb.data(), bounds, hb.size() * 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    uint64_t *dst[4] = { out->frag_off, out->key_off, out->val_off, out->k2v_off };
    for (int q = 0; q < 4; ++q) memcpy(dst[q], hb.data() + q * (world + 1), (world + 1) * sizeof(uint64_t));
    const uint64_t F = hb[world], NK = hb[(world + 1) + world], NV = hb[2 * (world + 1) + world],
                   NO = hb[3 * (world + 1) + world];
    if (ctx_alloc) {
        out->mem = ACC_MEM_DEVICE;
        out->hdr = ctx->get<uint32_t>("cm_s_hdr", 4 * F);
        out->keys = ctx->get<uint64_t>("cm_s_keys", NK);
        out->vals = ctx->get<uint32_t>("cm_s_vals", NV);
        out->k2v = ctx->get<int32_t>("cm_s_k2v", NO);
        out->cap_frag = F; out->cap_keys = NK; out->cap_vals = NV; out->cap_k2v = NO;
    }
    if (out->cap_frag < F || out->cap_keys < NK || out->cap_vals < NV || out->cap_k2v < NO || (F && !out->hdr) ||
        (NK && !out->keys) || (NV && !out->vals) || (NO && !out->k2v))
        fail(ACC_E_CAP, "fragment stream capacity too small (offsets written)");
    if (out->mem != ACC_MEM_DEVICE && out->mem != ACC_MEM_HOST) fail(ACC_E_ARG, "bad mem");
    uint32_t *hdr = out->hdr;
    uint64_t *keys = out->keys;
    uint32_t *vals = out->vals;
    int32_t *k2v = out->k2v;
    if (out->mem == ACC_MEM_HOST) {
        hdr = ctx->get<uint32_t>("sh_hdr", 4 * F);
        keys = ctx->get<uint64_t>("sh_keys", NK);
        vals = ctx->get<uint32_t>("sh_vals", NV);
        k2v = ctx->get<int32_t>("sh_k2v", NO);
    }
    launch(ctx, "sh_pack", k_sh_pack, dim3((n + WAVES - 1) / WAVES), dim3(BLOCK), 0, n, world, G, key_off, key_code, v.kd_off,
           v.key_idx, v.u_off, v.dep_txn, v.arena_off, v.arena, v.kd_key, gidx, (const uint64_t *)o[0], (const uint64_t *)o[1],
           (const uint64_t *)o[2], (const uint64_t *)o[3], hdr, keys, vals, k2v);
    if (out->mem == ACC_MEM_HOST) {
        if (F) ACC_HIP(hipMemcpyAsync(out->hdr, hdr, 16 * F, hipMemcpyDeviceToHost, st));
        if (NK) ACC_HIP(hipMemcpyAsync(out->keys, keys, 8 * NK, hipMemcpyDeviceToHost, st));
        if (NV) ACC_HIP(hipMemcpyAsync(out->vals, vals, 4 * NV, hipMemcpyDeviceToHost, st));
        if (NO) ACC_HIP(hipMemcpyAsync(out->k2v, k2v, 4 * NO, hipMemcpyDeviceToHost, st));
    }
    ctx->sync();
}

void shard_merge(acc_ctx *ctx, const acc_frag_recv *in, acc_merge_view *view)
{
    if (!in || !view) fail(ACC_E_ARG, "null argument");
    const uint32_t world = in->world, home = in->rank, n = in->n_txn;
    if (world == 0 || home >= world) fail(ACC_E_ARG, "rank must be below world");
    hipStream_t st = ctx->stream;
    ctx->merge_valid = false;   // a failing call must not leave the previous result readable as if current
    const uint32_t n_groups = n > home ? (n - home + world - 1) / world : 0;   // home txns t = home, home + world, ...
    uint64_t F = 0, NK = 0, NV = 0, NO = 0;
    for (uint32_t s = 0; s < world; ++s) {
        F += in->n_frag[s]; NK += in->n_keys[s]; NV += in->n_vals[s]; NO += in->n_k2v[s];
    }
    const uint32_t *hdr = stage_in(ctx, "shr_hdr", in->hdr, 4 * F, in->mem);
    const uint64_t *keys = stage_in(ctx, "shr_keys", in->keys, NK, in->mem);
    const uint32_t *vals = stage_in(ctx, "shr_vals", in->vals, NV, in->mem);
    const int32_t *k2v = stage_in(ctx, "shr_k2v", in->k2v, NO, in->mem);
    uint64_t *f_key = ctx->get<uint64_t>("shr_f_key", F), *f_val = ctx->get<uint64_t>("shr_f_val", F);
    uint64_t *f_k2v = ctx->get<uint64_t>("shr_f_k2v", F), *gkey = ctx->get<uint64_t>("shr_gkey", F);
    uint64_t *err = ctx->get<uint64_t>("shr_err", 1);
    ACC_HIP(hipMemsetAsync(err, 0, 8, st));
    launch(ctx, "shr_frag", k_sh_frag, dim3(grid_for(F, BLOCK)), dim3(BLOCK), 0, F, world, n_groups, hdr, f_key, f_val, f_k2v,
           gkey, err);
    // stream offsets of each received fragment (received order)
    uint64_t *sk = ctx->get<uint64_t>("shr_sk", F + 1), *sv = ctx->get<uint64_t>("shr_sv", F + 1), *so = ctx->get<uint64_t>("shr_so", F + 1);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, f_key, sk, F, true, sk + F);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, f_val, sv, F, true, sv + F);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, f_k2v, so, F, true, so + F);
    // replies grouped by home txn, source (shard) order kept within a txn: stable sort by group
    Sorted fs = radix_sort(ctx, "rs_shr", gkey, nullptr, F, bits_for(n_groups ? n_groups - 1 : 0));
    uint64_t *r_key = ctx->get<uint64_t>("shr_r_key", F), *r_val = ctx->get<uint64_t>("shr_r_val", F);
    uint64_t *r_k2v = ctx->get<uint64_t>("shr_r_k2v", F);
    launch(ctx, "shr_reply_sizes", k_sh_reply_sizes, dim3(grid_for(F, BLOCK)), dim3(BLOCK), 0, F, (const uint32_t *)fs.vals,
           (const uint64_t *)f_key, (const uint64_t *)f_val, (const uint64_t *)f_k2v, r_key, r_val, r_k2v);
    uint64_t *rk = ctx->get<uint64_t>("shr_rk", F + 1), *rv = ctx->get<uint64_t>("shr_rv", F + 1), *ro = ctx->get<uint64_t>("shr_ro", F + 1);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, r_key, rk, F, true, rk + F);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, r_val, rv, F, true, rv + F);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, r_k2v, ro, F, true, ro + F);
    uint64_t *gcnt = ctx->get<uint64_t>("shr_gcnt", (size_t)n_groups + 1);
    uint64_t *grp_off = ctx->get<uint64_t>("shr_grp_off", (size_t)n_groups + 1);
    ACC_HIP(hipMemsetAsync(gcnt, 0, ((size_t)n_groups + 1) * 8, st));
    launch(ctx, "shr_group_hist", k_sh_group_hist, dim3(grid_for(F, BLOCK)), dim3(BLOCK), 0, F, (const uint64_t *)gkey, gcnt);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, gcnt, grp_off, n_groups, true, grp_off + n_groups);
    uint64_t *m_keys = ctx->get<uint64_t>("shr_m_keys", NK);
    uint32_t *m_vals = ctx->get<uint32_t>("shr_m_vals", NV);
    int32_t *m_k2v = ctx->get<int32_t>("shr_m_k2v", NO);
    launch(ctx, "shr_gather", k_sh_gather, dim3((unsigned)((F + WAVES - 1) / WAVES)), dim3(BLOCK), 0, F, (const uint32_t *)fs.vals,
           (const uint64_t *)sk, (const uint64_t *)sv, (const uint64_t *)so, (const uint64_t *)rk, (const uint64_t *)rv,
           (const uint64_t *)ro, keys, vals, k2v, m_keys, m_vals, m_k2v);
    // ---- fused reduce: sizes (and the key-order check), offsets, writes
    Fuse fz{};
    fz.ng = n_groups; fz.grp_off = grp_off; fz.rk = rk; fz.rv = rv; fz.ro = ro; fz.keys = m_keys; fz.vals = m_vals;
    fz.k2v = m_k2v;
    fz.c_nk = ctx->get<uint64_t>("shm_c_nk", n_groups);
    fz.c_nu = ctx->get<uint64_t>("shm_c_nu", n_groups);
    fz.c_no = ctx->get<uint64_t>("shm_c_no", n_groups);
    fz.blk_list = ctx->get<uint32_t>("shm_blk", n_groups);
    fz.glb_list = ctx->get<uint32_t>("shm_glb", n_groups);
    fz.big_list = ctx->get<uint32_t>("shm_big", n_groups);
    fz.gstat = ctx->get<uint64_t>("shm_gstat", 5);
    ACC_HIP(hipMemsetAsync(fz.gstat, 0, 5 * 8, st));
    const unsigned gw = (n_groups + WAVES - 1) / WAVES;
    launch(ctx, "shm_fuse_wave_sizes", k_fuse_wave<false>, dim3(gw), dim3(BLOCK), 0, fz);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, err, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, fz.gstat, 5 * 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    if (ctx->pinned[0]) fail(ACC_E_ARG, "received a fragment for a txn that is not homed on this rank");
    const uint64_t nblk = ctx->pinned[1], nglb = ctx->pinned[2], glb_elems = ctx->pinned[3], nbig = ctx->pinned[5];
    ctx->stat("shard.big_groups", nbig);
    ctx->stat("shard.global_groups", nglb);
    if (ctx->pinned[4]) {
        // replies of a txn are not in ascending disjoint key order (not a key-range split): general merge
        ctx->stat("shard.general_merge", 1);
        acc_merge_in mi{ ACC_MEM_DEVICE, n_groups, F, grp_off, rk, m_keys, rv, m_vals, ro, m_k2v };
        keydeps_merge(ctx, &mi, view);
        return;
    }
    ctx->stat("shard.general_merge", 0);
    if (nblk) launch(ctx, "shm_fuse_block_sizes", k_fuse_block<false>, dim3((unsigned)nblk), dim3(BLOCK), 0, fz);
    if (nbig) launch(ctx, "shm_fuse_big_sizes", k_fuse_big<false>, dim3((unsigned)nbig), dim3(1024), 0, fz);
    if (nglb) {
        uint64_t *gsz = ctx->get<uint64_t>("shm_glb_sz", nglb);
        uint64_t *goff = ctx->get<uint64_t>("shm_glb_off", nglb + 1);
        launch(ctx, "shm_glb_sizes", k_fuse_glb_sizes, dim3(grid_for(nglb, BLOCK)), dim3(BLOCK), 0, (uint32_t)nglb, fz, gsz);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, gsz, goff, nglb, true, goff + nglb);
        fz.glb_off = goff;
        fz.scratch = ctx->get<uint32_t>("shm_scratch", glb_elems);
        launch(ctx, "shm_fuse_global_sizes", k_fuse_global<false>, dim3((unsigned)nglb), dim3(BLOCK), 0, fz);
    }
    uint64_t *key_out = ctx->get<uint64_t>("shm_key_off", (size_t)n_groups + 1);
    uint64_t *val_out = ctx->get<uint64_t>("shm_val_off", (size_t)n_groups + 1);
    uint64_t *k2v_out = ctx->get<uint64_t>("shm_k2v_off", (size_t)n_groups + 1);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, fz.c_nk, key_out, n_groups, true, key_out + n_groups);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, fz.c_nu, val_out, n_groups, true, val_out + n_groups);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, fz.c_no, k2v_out, n_groups, true, k2v_out + n_groups);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, val_out + n_groups, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t NU = ctx->pinned[0];
    fz.key_out = key_out; fz.val_out = val_out; fz.k2v_out = k2v_out;
    fz.m_keys = ctx->get<uint64_t>("shm_keys", NK);
    fz.m_vals = ctx->get<uint32_t>("shm_vals", NU);
    fz.m_k2v = ctx->get<int32_t>("shm_k2v", NO);
    launch(ctx, "shm_fuse_wave", k_fuse_wave<true>, dim3(gw), dim3(BLOCK), 0, fz);
    if (nblk) launch(ctx, "shm_fuse_block", k_fuse_block<true>, dim3((unsigned)nblk), dim3(BLOCK), 0, fz);
    if (nbig) launch(ctx, "shm_fuse_big", k_fuse_big<true>, dim3((unsigned)nbig), dim3(1024), 0, fz);
    if (nglb) launch(ctx, "shm_fuse_global", k_fuse_global<true>, dim3((unsigned)nglb), dim3(BLOCK), 0, fz);
    ctx->sync();
    *view = acc_merge_view{ n_groups, NK, NU, NO, NO, key_out, fz.m_keys, val_out, fz.m_vals, k2v_out, fz.m_k2v };
    ctx->merge_view = *view;
    ctx->merge_valid = true;
}


// The RangeDeps fragments of the last acc_rangedeps_batch / acc_partial_deps_batch on ctx for the txns' home ranks, in
// four destination-major context-owned streams (header, ranges, raw TxnIds, ints); off[q] = host [world+1] element
// offsets.
void range_pack(acc_ctx *ctx, const acc_range_batch_in *in, const uint32_t *txn_global, uint32_t world, uint32_t n_global,
                void *send[4], std::vector<uint64_t> off[4])
{
    if (!in) fail(ACC_E_ARG, "null argument");
    if (!ctx->rd_valid) fail(ACC_E_STATE, "no rangedeps result on this context");
    const acc_rangedeps_view &v = ctx->rd_view;
    const uint32_t n = v.n_txn;
    if (in->n_txn != n) fail(ACC_E_ARG, "batch does not match the last rangedeps result");
    hipStream_t st = ctx->stream;
    const uint64_t *tm = stage_in(ctx, "shr_in_tm", in->txn_id.msb, n, in->mem);
    const uint64_t *tl = stage_in(ctx, "shr_in_tl", in->txn_id.lsb, n, in->mem);
    const int32_t *tn = stage_in(ctx, "shr_in_tn", in->txn_id.node, n, in->mem);
    const uint32_t *gidx = txn_global ? stage_in(ctx, "shr_gidx", txn_global, n, in->mem) : nullptr;
    if (!txn_global) n_global = std::max(n_global, n);
    const uint32_t G = (n_global + world - 1) / world;
    const size_t M = (size_t)world * G;
    uint64_t *c[4], *o[4];
    const char *cn[4] = { "shr_c_frag", "shr_c_rng", "shr_c_val", "shr_c_k2v" };
    const char *on[4] = { "shr_o_frag", "shr_o_rng", "shr_o_val", "shr_o_k2v" };
    for (int q = 0; q < 4; ++q) {
        c[q] = ctx->get<uint64_t>(cn[q], M);
        o[q] = ctx->get<uint64_t>(on[q], M + 1);
        ACC_HIP(hipMemsetAsync(c[q], 0, M * sizeof(uint64_t), st));
    }
    launch(ctx, "shr_sizes", k_shr_sizes, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, n, world, G, gidx, v.rd_off, v.u_off,
           v.arena_off, c[0], c[1], c[2], c[3]);
    for (int q = 0; q < 4; ++q) scan<uint64_t, OpAdd<uint64_t>>(ctx, c[q], o[q], M, true, o[q] + M);
    uint64_t *bounds = ctx->get<uint64_t>("shr_bounds", 4 * ((size_t)world + 1));
    for (int q = 0; q < 4; ++q)
        for (uint32_t d = 0; d <= world; ++d)
            ACC_HIP(hipMemcpyAsync(bounds + q * (world + 1) + d, o[q] + std::min((size_t)d * G, M), 8,
                                   hipMemcpyDeviceToDevice, st));
    std::vector<uint64_t> hb(4 * ((size_t)world + 1));
    ACC_HIP(hipMemcpyAsync(hb.data(), bounds, hb.size() * 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    for (int q = 0; q < 4; ++q) off[q].assign(hb.begin() + q * (world + 1), hb.begin() + (q + 1) * (world + 1));
    const uint64_t F = off[0][world], NR = off[1][world], NV = off[2][world], NO = off[3][world];
    uint32_t *hdr = ctx->get<uint32_t>("shr_s_hdr", 4 * F);
    uint64_t *rng = ctx->get<uint64_t>("shr_s_rng", 2 * NR);
    uint64_t *txn = ctx->get<uint64_t>("shr_s_txn", 3 * NV);
    int32_t *k2v = ctx->get<int32_t>("shr_s_k2v", NO);
    launch(ctx, "shr_pack", k_shr_pack, dim3((n + WAVES - 1) / WAVES), dim3(BLOCK), 0, n, world, G, v, tm, tl, tn, gidx,
           (const uint64_t *)o[0], (const uint64_t *)o[1], (const uint64_t *)o[2], (const uint64_t *)o[3], hdr, rng, txn, k2v);
    send[0] = hdr; send[1] = rng; send[2] = txn; send[3] = k2v;
}

// What the home rank received of the RangeDeps half (streams source-major, per-source element counts): the fragments
// grouped by home txn in source (= store) order, RangeDeps.with folded over them = the batched Deps.merge of the range
// half over raw TxnIds (depsmerge.hip; RelationMultiMap.linearUnion over Range::compare, primitives/RangeDeps.java:
// 567-582). Group g = home txn rank + g * world.
void range_merge(acc_ctx *ctx, uint32_t world, uint32_t rank, uint32_t n_global, const std::vector<uint64_t> n_src[4],
                 void *const recv[4], acc_deps_merge_view *view)
{
    NsScope scope(ctx, "prr.");
    hipStream_t st = ctx->stream;
    const uint32_t n_groups = n_global > rank ? (n_global - rank + world - 1) / world : 0;
    uint64_t F = 0;
    for (uint32_t s = 0; s < world; ++s) F += n_src[0][s];
    const uint32_t *hdr = static_cast<const uint32_t *>(recv[0]);
    uint64_t *f_key = ctx->get<uint64_t>("f_key", F), *f_val = ctx->get<uint64_t>("f_val", F);
    uint64_t *f_k2v = ctx->get<uint64_t>("f_k2v", F), *gkey = ctx->get<uint64_t>("gkey", F);
    uint64_t *err = ctx->get<uint64_t>("err", 1);
    ACC_HIP(hipMemsetAsync(err, 0, 8, st));
    launch(ctx, "shr_frag", k_sh_frag, dim3(grid_for(F, BLOCK)), dim3(BLOCK), 0, F, world, n_groups, hdr, f_key, f_val, f_k2v,
           gkey, err);
    uint64_t *sk = ctx->get<uint64_t>("sk", F + 1), *sv = ctx->get<uint64_t>("sv", F + 1), *so = ctx->get<uint64_t>("so", F + 1);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, f_key, sk, F, true, sk + F);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, f_val, sv, F, true, sv + F);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, f_k2v, so, F, true, so + F);
    Sorted fs = radix_sort(ctx, "rs", gkey, nullptr, F, bits_for(n_groups ? n_groups - 1 : 0));
    uint64_t *r_key = ctx->get<uint64_t>("r_key", F), *r_val = ctx->get<uint64_t>("r_val", F), *r_k2v = ctx->get<uint64_t>("r_k2v", F);
    launch(ctx, "shr_reply_sizes", k_sh_reply_sizes, dim3(grid_for(F, BLOCK)), dim3(BLOCK), 0, F, (const uint32_t *)fs.vals,
           (const uint64_t *)f_key, (const uint64_t *)f_val, (const uint64_t *)f_k2v, r_key, r_val, r_k2v);
    uint64_t *rk = ctx->get<uint64_t>("rk", F + 1), *rv = ctx->get<uint64_t>("rv", F + 1), *ro = ctx->get<uint64_t>("ro", F + 1);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, r_key, rk, F, true, rk + F);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, r_val, rv, F, true, rv + F);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, r_k2v, ro, F, true, ro + F);
    uint64_t *gcnt = ctx->get<uint64_t>("gcnt", (size_t)n_groups + 1), *grp_off = ctx->get<uint64_t>("grp_off", (size_t)n_groups + 1);
    ACC_HIP(hipMemsetAsync(gcnt, 0, ((size_t)n_groups + 1) * 8, st));
    launch(ctx, "shr_group_hist", k_sh_group_hist, dim3(grid_for(F, BLOCK)), dim3(BLOCK), 0, F, (const uint64_t *)gkey, gcnt);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, gcnt, grp_off, n_groups, true, grp_off + n_groups);
    uint64_t NR = 0, NV = 0, NO = 0;
    for (uint32_t s = 0; s < world; ++s) { NR += n_src[1][s]; NV += n_src[2][s]; NO += n_src[3][s]; }
    uint64_t *ka = ctx->get<uint64_t>("ka", NR + 1), *kb = ctx->get<uint64_t>("kb", NR + 1);
    uint64_t *msb = ctx->get<uint64_t>("msb", NV + 1), *lsb = ctx->get<uint64_t>("lsb", NV + 1);
    int32_t *node = ctx->get<int32_t>("node", NV + 1), *mk2v = ctx->get<int32_t>("k2v", NO + 1);
    launch(ctx, "shr_gather", k_shr_gather, dim3((unsigned)((F + WAVES - 1) / WAVES)), dim3(BLOCK), 0, F,
           (const uint32_t *)fs.vals, (const uint64_t *)sk, (const uint64_t *)sv, (const uint64_t *)so, (const uint64_t *)rk,
           (const uint64_t *)rv, (const uint64_t *)ro, static_cast<const uint64_t *>(recv[1]),
           static_cast<const uint64_t *>(recv[2]), static_cast<const int32_t *>(recv[3]), ka, kb, msb, lsb, node, mk2v);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, err, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    if (ctx->pinned[0]) fail(ACC_E_ARG, "received a RangeDeps fragment for a txn that is not homed on this rank");
    acc_rmm_in none{};
    acc_rmm_in rh{ rk, ka, kb, rv, acc_ts_cols{ msb, lsb, node }, ro, mk2v };
    acc_deps_merge_in dmi{ ACC_MEM_DEVICE, n_groups, F, grp_off, none, rh };
    const bool kvalid = ctx->merge_valid;
    const acc_merge_view kview = ctx->merge_view;
    deps_merge(ctx, &dmi, view);
    ctx->merge_view = kview;   // the KeyDeps half's view (shard_merge) stays the context's current merge view
    ctx->merge_valid = kvalid;
}
}  // namespace acc
