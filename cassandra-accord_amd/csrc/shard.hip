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

namespace acc {
void keydeps_merge(acc_ctx *ctx, const acc_merge_in *in, acc_merge_view *view);

namespace sh {

// dest-major position of txn t: dest d = t mod world, slot t / world within the dest's G = ceil(n / world) slots
__device__ __forceinline__ uint32_t dm_index(uint32_t t, uint32_t world, uint32_t G) { return (t % world) * G + t / world; }

__global__ __launch_bounds__(BLOCK) void k_sh_sizes(uint32_t n, uint32_t world, uint32_t G, const uint64_t *__restrict__ kd_off,
                                                    const uint64_t *__restrict__ u_off, const uint64_t *__restrict__ arena_off,
                                                    uint64_t *__restrict__ c_frag, uint64_t *__restrict__ c_key,
                                                    uint64_t *__restrict__ c_val, uint64_t *__restrict__ c_k2v)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;   // dest-major index
    if (i >= world * G) return;
    const uint32_t d = i / G, s = i % G;
    const uint64_t t = (uint64_t)s * world + d;
    uint64_t nk = 0, nv = 0, no = 0;
    if (t < n) {
        nk = kd_off[t + 1] - kd_off[t];         // KeyDeps.isEmpty <=> no keys (keys without deps are dropped)
        if (nk) { nv = u_off[t + 1] - u_off[t]; no = arena_off[t + 1] - arena_off[t]; }
    }
    c_frag[i] = nk ? 1 : 0;
    c_key[i] = nk;
    c_val[i] = nv;
    c_k2v[i] = no;
}

// one wave per txn with a fragment: header + key codes + TxnIds + keysToTxnIds at the stream offsets
__global__ __launch_bounds__(BLOCK) void k_sh_pack(uint32_t n, uint32_t world, uint32_t G, const uint32_t *__restrict__ key_off,
                                                   const uint64_t *__restrict__ key_code, const uint64_t *__restrict__ kd_off,
                                                   const uint32_t *__restrict__ key_idx, const uint64_t *__restrict__ u_off,
                                                   const uint32_t *__restrict__ dep_txn, const uint64_t *__restrict__ arena_off,
                                                   const int32_t *__restrict__ arena, const uint64_t *__restrict__ o_frag,
                                                   const uint64_t *__restrict__ o_key, const uint64_t *__restrict__ o_val,
                                                   const uint64_t *__restrict__ o_k2v, uint32_t *__restrict__ hdr,
                                                   uint64_t *__restrict__ keys, uint32_t *__restrict__ vals,
                                                   int32_t *__restrict__ k2v)
{
    const uint32_t t = blockIdx.x * WAVES + (threadIdx.x >> 6), lane = lane_id();
    if (t >= n) return;
    const uint64_t k0 = kd_off[t], nk = kd_off[t + 1] - k0;
    if (nk == 0) return;
    const uint32_t i = dm_index(t, world, G);
    const uint64_t v0 = u_off[t], nv = u_off[t + 1] - v0, a0 = arena_off[t], no = arena_off[t + 1] - a0;
    const uint64_t f = o_frag[i], ok = o_key[i], ov = o_val[i], oo = o_k2v[i];
    if (lane < 4) hdr[4 * f + lane] = lane == 0 ? t : lane == 1 ? (uint32_t)nk : lane == 2 ? (uint32_t)nv : (uint32_t)no;
    const uint32_t kb = key_off[t];
    for (uint64_t j = lane; j < nk; j += 64) keys[ok + j] = key_code[kb + key_idx[k0 + j]];
    for (uint64_t j = lane; j < nv; j += 64) vals[ov + j] = dep_txn[v0 + j];
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

}  // namespace sh

using namespace sh;

void shard_pack(acc_ctx *ctx, const acc_batch_in *in, acc_frag_streams *out)
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
    const uint32_t G = (n + world - 1) / world;
    const size_t M = (size_t)world * G;
    uint64_t *c[4], *o[4];
    const char *cn[4] = { "sh_c_frag", "sh_c_key", "sh_c_val", "sh_c_k2v" };
    const char *on[4] = { "sh_o_frag", "sh_o_key", "sh_o_val", "sh_o_k2v" };
    for (int q = 0; q < 4; ++q) { c[q] = ctx->get<uint64_t>(cn[q], M); o[q] = ctx->get<uint64_t>(on[q], M + 1); }
    launch(ctx, "sh_sizes", k_sh_sizes, dim3(grid_for(M, BLOCK)), dim3(BLOCK), 0, n, world, G, v.kd_off, v.u_off, v.arena_off,
           c[0], c[1], c[2], c[3]);
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
           v.key_idx, v.u_off, v.dep_txn, v.arena_off, v.arena, (const uint64_t *)o[0], (const uint64_t *)o[1],
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
    ACC_HIP(hipMemcpyAsync(ctx->pinned, err, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    if (ctx->pinned[0]) fail(ACC_E_ARG, "received a fragment for a txn that is not homed on this rank");
    acc_merge_in mi{ ACC_MEM_DEVICE, n_groups, F, grp_off, rk, m_keys, rv, m_vals, ro, m_k2v };
    keydeps_merge(ctx, &mi, view);
}

}  // namespace acc
