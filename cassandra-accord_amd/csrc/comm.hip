// comm.hip — the node's CommandStore exchange behind the C ABI: acc_comm (an RCCL communicator, or a caller-supplied
// host all-to-all(v) transport) and acc_shard_reduce = PreAccept.reduce of the per-store KeyDeps
// (messages/PreAccept.java:141-156, PartialDeps.with): pack the fragments of the last acc_keydeps_batch for their home
// ranks, one size exchange, one all-to-all(v) of the four fragment streams, and the KeyDeps.with fold on the home rank.
//
// RCCL is resolved at run time (dlopen of librccl.so.1, the copy the process may already have loaded through torch), so
// the library links and runs without it; only acc_comm_init_rccl needs it. Over xGMI every rank talks to every other
// point to point, which is what the grouped ncclSend/ncclRecv pairs below express (no ring collective is needed for an
// all-to-all(v) of skewed sizes).
#include "prims.hpp"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <vector>

namespace acc {
void shard_pack(acc_ctx *ctx, const acc_batch_in *in, acc_frag_streams *out, bool ctx_alloc);
void shard_merge(acc_ctx *ctx, const acc_frag_recv *in, acc_merge_view *view);

struct Rccl {
    bool ok = false;
    std::string why;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
};

static Rccl &rccl()
{
    static Rccl r;
    static bool tried = false;
    if (tried) return r;
    tried = true;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) { r.why = std::string("librccl not loadable: ") + dlerror(); return r; }
    auto sym = [&](const char *name) { return dlsym(h, name); };
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(sym("ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(sym("ncclCommDestroy"));
    r.send = reinterpret_cast<decltype(r.send)>(sym("ncclSend"));
    r.recv = reinterpret_cast<decltype(r.recv)>(sym("ncclRecv"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(sym("ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(sym("ncclGroupEnd"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
    r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.send && r.recv && r.group_start && r.group_end &&
           r.error_string;
    if (!r.ok) r.why = "librccl lacks a required symbol";
    return r;
}

#define ACC_NCCL(expr)                                                                                           \
    do {                                                                                                         \
        ncclResult_t r_ = (expr);                                                                                \
        if (r_ != ncclSuccess) ::acc::fail(ACC_E_DEVICE, std::string(#expr) + ": " + ::acc::rccl().error_string(r_)); \
    } while (0)

}  // namespace acc

struct acc_comm {
    acc_ctx *ctx = nullptr;
    uint32_t world = 1, rank = 0;
    ncclComm_t nc = nullptr;            // RCCL transport
    acc_alltoallv_fn fn = nullptr;      // host transport
    void *user = nullptr;
};

namespace acc {

// all-to-all(v) of one byte stream: send[off_s[d] .. off_s[d+1]) to rank d, receive rank s's bytes into
// recv[off_r[s] .. off_r[s+1]); device buffers (the RCCL transport moves them directly, the host transport stages).
static void exchange(acc_comm *c, const uint8_t *send, const std::vector<uint64_t> &off_s, uint8_t *recv,
                     const std::vector<uint64_t> &off_r)
{
    acc_ctx *ctx = c->ctx;
    const uint32_t W = c->world;
    if (c->nc) {
        Rccl &r = rccl();
        ACC_NCCL(r.group_start());
        for (uint32_t p = 0; p < W; ++p) {
            const uint64_t ns = off_s[p + 1] - off_s[p], nr = off_r[p + 1] - off_r[p];
            if (ns) ACC_NCCL(r.send(send + off_s[p], ns, ncclUint8, (int)p, c->nc, ctx->stream));
            if (nr) ACC_NCCL(r.recv(recv + off_r[p], nr, ncclUint8, (int)p, c->nc, ctx->stream));
        }
        ACC_NCCL(r.group_end());
        return;
    }
    std::vector<uint8_t> hs(off_s[W]), hr(off_r[W]);
    std::vector<uint64_t> bs(W), br(W);
    for (uint32_t p = 0; p < W; ++p) { bs[p] = off_s[p + 1] - off_s[p]; br[p] = off_r[p + 1] - off_r[p]; }
    if (off_s[W]) ACC_HIP(hipMemcpyAsync(hs.data(), send, off_s[W], hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
    const int rc = c->fn(c->user, hs.data(), bs.data(), hr.data(), br.data());
    if (rc != 0) fail(ACC_E_STATE, "host transport all-to-all failed (" + std::to_string(rc) + ")");
    if (off_r[W]) ACC_HIP(hipMemcpyAsync(recv, hr.data(), off_r[W], hipMemcpyHostToDevice, ctx->stream));
    ctx->sync();
}

void shard_reduce(acc_ctx *ctx, acc_comm *c, const acc_batch_in *in, const uint32_t *txn_global, uint32_t n_global,
                  acc_merge_view *view)
{
    if (!c || !in || !view) fail(ACC_E_ARG, "null argument");
    if (c->ctx != ctx) fail(ACC_E_ARG, "communicator belongs to another context");
    const uint32_t W = c->world;
    // ---- pack (destination-major streams, context-owned)
    std::vector<uint64_t> off[4];
    for (auto &o : off) o.assign(W + 1, 0);
    acc_frag_streams fs{};
    fs.world = W;
    fs.mem = ACC_MEM_DEVICE;
    fs.frag_off = off[0].data(); fs.key_off = off[1].data(); fs.val_off = off[2].data(); fs.k2v_off = off[3].data();
    fs.txn_global = txn_global;
    shard_pack(ctx, in, &fs, true);
    const uint64_t esz[4] = { 16, 8, 4, 4 };   // bytes per element: header (4 x u32), key code, TxnId index, int
    // ---- one size exchange: element counts per stream for every peer
    uint64_t *cnt_s = ctx->get<uint64_t>("cm_cnt_s", 4 * (size_t)W), *cnt_r = ctx->get<uint64_t>("cm_cnt_r", 4 * (size_t)W);
    std::vector<uint64_t> hcs(4 * (size_t)W), hcr(4 * (size_t)W);
    for (uint32_t d = 0; d < W; ++d)
        for (int q = 0; q < 4; ++q) hcs[4 * d + q] = off[q][d + 1] - off[q][d];
    ACC_HIP(hipMemcpyAsync(cnt_s, hcs.data(), hcs.size() * 8, hipMemcpyHostToDevice, ctx->stream));
    std::vector<uint64_t> cs(W + 1), cr(W + 1);
    for (uint32_t d = 0; d <= W; ++d) cs[d] = cr[d] = 32ull * d;
    exchange(c, reinterpret_cast<const uint8_t *>(cnt_s), cs, reinterpret_cast<uint8_t *>(cnt_r), cr);
    ACC_HIP(hipMemcpyAsync(hcr.data(), cnt_r, hcr.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
    // ---- the four streams
    std::vector<uint64_t> n_src[4];
    void *recv[4];
    const char *rn[4] = { "cm_r_hdr", "cm_r_keys", "cm_r_vals", "cm_r_k2v" };
    const void *send[4] = { fs.hdr, fs.keys, fs.vals, fs.k2v };
    for (int q = 0; q < 4; ++q) {
        std::vector<uint64_t> os(W + 1), orr(W + 1);
        n_src[q].assign(W, 0);
        for (uint32_t p = 0; p < W; ++p) {
            os[p + 1] = os[p] + (off[q][p + 1] - off[q][p]) * esz[q];
            n_src[q][p] = hcr[4 * p + q];
            orr[p + 1] = orr[p] + hcr[4 * p + q] * esz[q];
        }
        recv[q] = ctx->get<uint8_t>(rn[q], orr[W]);
        exchange(c, static_cast<const uint8_t *>(send[q]) + off[q][0] * esz[q], os, static_cast<uint8_t *>(recv[q]), orr);
    }
    // ---- KeyDeps.with fold of every home txn (stream order makes the merge wait for the receives)
    acc_frag_recv fr{ ACC_MEM_DEVICE, W, c->rank, n_global, n_src[0].data(), n_src[1].data(), n_src[2].data(),
                      n_src[3].data(), static_cast<const uint32_t *>(recv[0]), static_cast<const uint64_t *>(recv[1]),
                      static_cast<const uint32_t *>(recv[2]), static_cast<const int32_t *>(recv[3]) };
    shard_merge(ctx, &fr, view);
}

}  // namespace acc

extern "C" {

int acc_comm_unique_id(uint8_t *id_out)
{
    if (!id_out) return ACC_E_ARG;
    acc::Rccl &r = acc::rccl();
    if (!r.ok) return ACC_E_DEVICE;
    ncclUniqueId id;
    if (r.get_unique_id(&id) != ncclSuccess) return ACC_E_DEVICE;
    static_assert(sizeof(ncclUniqueId) == ACC_COMM_ID_BYTES, "RCCL unique id size");
    memcpy(id_out, &id, sizeof id);
    return ACC_OK;
}

int acc_comm_init_rccl(acc_ctx *ctx, uint32_t world, uint32_t rank, const uint8_t *id, acc_comm **out)
{
    if (!ctx || !id || !out || world == 0 || rank >= world) return ACC_E_ARG;
    *out = nullptr;
    acc_comm *c = new (std::nothrow) acc_comm();
    if (!c) return ACC_E_NOMEM;
    int rc = acc_guard(ctx, [&] {
        acc::Rccl &r = acc::rccl();
        if (!r.ok) acc::fail(ACC_E_DEVICE, r.why);
        ACC_HIP(hipSetDevice(ctx->device));
        ncclUniqueId uid;
        memcpy(&uid, id, sizeof uid);
        c->ctx = ctx; c->world = world; c->rank = rank;
        ACC_NCCL(r.comm_init_rank(&c->nc, (int)world, uid, (int)rank));
    });
    if (rc != ACC_OK) { delete c; return rc; }
    *out = c;
    return ACC_OK;
}

int acc_comm_init_host(acc_ctx *ctx, uint32_t world, uint32_t rank, acc_alltoallv_fn fn, void *user, acc_comm **out)
{
    if (!ctx || !fn || !out || world == 0 || rank >= world) return ACC_E_ARG;
    acc_comm *c = new (std::nothrow) acc_comm();
    if (!c) return ACC_E_NOMEM;
    c->ctx = ctx; c->world = world; c->rank = rank; c->fn = fn; c->user = user;
    *out = c;
    return ACC_OK;
}

void acc_comm_destroy(acc_comm *c)
{
    if (!c) return;
    if (c->nc) {
        if (c->ctx && c->ctx->stream) (void)hipStreamSynchronize(c->ctx->stream);
        (void)acc::rccl().comm_destroy(c->nc);
    }
    delete c;
}

int acc_shard_reduce(acc_ctx *ctx, acc_comm *comm, const acc_batch_in *in, const uint32_t *txn_global, uint32_t n_global,
                     acc_merge_view *out_view)
{
    return acc_guard(ctx, [&] { acc::shard_reduce(ctx, comm, in, txn_global, n_global, out_view); });
}

}  // extern "C"
