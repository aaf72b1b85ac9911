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
uint8_t *frag_encode(acc_ctx *ctx, uint32_t W, const uint64_t *fo, const uint64_t *ko_h, const uint64_t *vo_h,
                     const uint64_t *oo_h, const uint32_t *hdr, const uint64_t *keys, const uint32_t *vals,
                     const int32_t *k2v, uint32_t G, std::vector<uint64_t> &boff);
void frag_decode(acc_ctx *ctx, uint32_t W, uint32_t rank, uint32_t n_global, const uint8_t *recv,
                 const std::vector<uint64_t> &nb, acc_frag_recv &fr, std::vector<uint64_t> cnt[4]);
void partial_deps_reduce(acc_ctx *ctx, acc_comm *c, const acc_range_batch_in *in, const uint32_t *txn_global,
                         uint32_t n_global, const acc_rlist *covering, acc_merge_view *key_view,
                         acc_deps_merge_view *range_view, acc_covering_view *covering_view);

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

// Fragment streams of one exchange: stream q = elements of esz[q] bytes, destination-major (destination d owns
// elements [off[q][d], off[q][d+1]) of send[q]). After exchange_streams: recv[q] = what the sources sent, concatenated in
// source-rank order, n_src[q][s] elements from source s.
constexpr int MAX_STREAMS = 10;
struct Streams {
    int ns = 0;
    const void *send[MAX_STREAMS] = {};
    std::vector<uint64_t> off[MAX_STREAMS];
    uint64_t esz[MAX_STREAMS] = {};
    void *recv[MAX_STREAMS] = {};
    std::vector<uint64_t> n_src[MAX_STREAMS];
};

// ONE size exchange (every stream's element count per peer) and ONE grouped all-to-all(v) carrying every stream: the
// RCCL transport issues all streams' point-to-point sends / receives inside one ncclGroupStart / End; the host transport
// hands the caller one byte block per peer (the peer's slice of every stream, concatenated) in a single call.
static void exchange_streams(acc_comm *c, Streams &S)
{
    acc_ctx *ctx = c->ctx;
    const uint32_t W = c->world;
    const int ns = S.ns;
    hipStream_t st = ctx->stream;
    // ---- sizes
    uint64_t *cnt_s = ctx->get<uint64_t>("cm_cnt_s", (size_t)ns * W), *cnt_r = ctx->get<uint64_t>("cm_cnt_r", (size_t)ns * W);
    std::vector<uint64_t> hcs((size_t)ns * W), hcr((size_t)ns * W);
    for (uint32_t d = 0; d < W; ++d)
        for (int q = 0; q < ns; ++q) hcs[(size_t)ns * d + q] = S.off[q][d + 1] - S.off[q][d];
    ACC_HIP(hipMemcpyAsync(cnt_s, hcs.data(), hcs.size() * 8, hipMemcpyHostToDevice, st));
    std::vector<uint64_t> cs(W + 1), cr(W + 1);
    for (uint32_t d = 0; d <= W; ++d) cs[d] = cr[d] = 8ull * ns * d;
    exchange(c, reinterpret_cast<const uint8_t *>(cnt_s), cs, reinterpret_cast<uint8_t *>(cnt_r), cr);
    ACC_HIP(hipMemcpyAsync(hcr.data(), cnt_r, hcr.size() * 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    // ---- receive buffers (source-major per stream)
    static const char *rn[MAX_STREAMS] = { "cm_r0", "cm_r1", "cm_r2", "cm_r3", "cm_r4", "cm_r5", "cm_r6", "cm_r7", "cm_r8",
                                           "cm_r9" };
    std::vector<uint64_t> rb[MAX_STREAMS];   // byte offsets per source
    for (int q = 0; q < ns; ++q) {
        S.n_src[q].assign(W, 0);
        rb[q].assign(W + 1, 0);
        for (uint32_t p = 0; p < W; ++p) {
            S.n_src[q][p] = hcr[(size_t)ns * p + q];
            rb[q][p + 1] = rb[q][p] + S.n_src[q][p] * S.esz[q];
        }
        S.recv[q] = ctx->get<uint8_t>(rn[q], rb[q][W]);
    }
    auto sptr = [&](int q, uint32_t p) {
        return static_cast<const uint8_t *>(S.send[q]) + (S.off[q][p] - S.off[q][0]) * S.esz[q];
    };
    uint64_t sent = 0, got = 0;
    for (int q = 0; q < ns; ++q) {
        sent += (S.off[q][W] - S.off[q][0] - (S.off[q][c->rank + 1] - S.off[q][c->rank])) * S.esz[q];
        got += rb[q][W] - (rb[q][c->rank + 1] - rb[q][c->rank]);
    }
    ctx->stat("exchange.bytes_sent", sent);       // to other ranks (the self slice stays on the GPU's own links)
    ctx->stat("exchange.bytes_received", got);
    if (c->nc) {
        Rccl &r = rccl();
        ACC_NCCL(r.group_start());
        for (uint32_t p = 0; p < W; ++p)
            for (int q = 0; q < ns; ++q) {
                const uint64_t nsb = (S.off[q][p + 1] - S.off[q][p]) * S.esz[q], nrb = rb[q][p + 1] - rb[q][p];
                if (nsb) ACC_NCCL(r.send(sptr(q, p), nsb, ncclUint8, (int)p, c->nc, st));
                if (nrb) ACC_NCCL(r.recv(static_cast<uint8_t *>(S.recv[q]) + rb[q][p], nrb, ncclUint8, (int)p, c->nc, st));
            }
        ACC_NCCL(r.group_end());
        return;
    }
    // host transport: every stream to the host once, per-peer blocks assembled, one call, scattered back per stream
    std::vector<std::vector<uint8_t>> hs(ns);
    for (int q = 0; q < ns; ++q) {
        const uint64_t nb = (S.off[q][W] - S.off[q][0]) * S.esz[q];
        hs[q].resize(nb);
        if (nb) ACC_HIP(hipMemcpyAsync(hs[q].data(), sptr(q, 0), nb, hipMemcpyDeviceToHost, st));
    }
    ctx->sync();
    std::vector<uint64_t> bs(W, 0), br(W, 0);
    for (uint32_t p = 0; p < W; ++p)
        for (int q = 0; q < ns; ++q) {
            bs[p] += (S.off[q][p + 1] - S.off[q][p]) * S.esz[q];
            br[p] += rb[q][p + 1] - rb[q][p];
        }
    uint64_t ts = 0, tr = 0;
    for (uint32_t p = 0; p < W; ++p) { ts += bs[p]; tr += br[p]; }
    std::vector<uint8_t> send(ts), recv(tr);
    uint64_t w = 0;
    for (uint32_t p = 0; p < W; ++p)
        for (int q = 0; q < ns; ++q) {
            const uint64_t a0 = (S.off[q][p] - S.off[q][0]) * S.esz[q], nb = (S.off[q][p + 1] - S.off[q][p]) * S.esz[q];
            if (nb) memcpy(send.data() + w, hs[q].data() + a0, nb);
            w += nb;
        }
    const int rc = c->fn(c->user, send.data(), bs.data(), recv.data(), br.data());
    if (rc != 0) fail(ACC_E_STATE, "host transport all-to-all failed (" + std::to_string(rc) + ")");
    std::vector<std::vector<uint8_t>> hr(ns);
    for (int q = 0; q < ns; ++q) hr[q].resize(rb[q][W]);
    uint64_t x = 0;
    for (uint32_t p = 0; p < W; ++p)
        for (int q = 0; q < ns; ++q) {
            const uint64_t nb = rb[q][p + 1] - rb[q][p];
            if (nb) memcpy(hr[q].data() + rb[q][p], recv.data() + x, nb);
            x += nb;
        }
    for (int q = 0; q < ns; ++q)
        if (rb[q][W]) ACC_HIP(hipMemcpyAsync(S.recv[q], hr[q].data(), rb[q][W], hipMemcpyHostToDevice, st));
    ctx->sync();
}

// the KeyDeps fragments of the last KeyDeps result on ctx (acc_shard_pack's four streams, on the device) in their
// compact wire form (fragwire.hip): one byte stream, slot 0 of S
static void add_key_streams(acc_ctx *ctx, const acc_batch_in *in, const uint32_t *txn_global, uint32_t W, uint32_t n_global,
                            Streams &S)
{
    std::vector<uint64_t> fo(W + 1), ko(W + 1), vo(W + 1), oo(W + 1);
    acc_frag_streams fs{};
    fs.world = W;
    fs.mem = ACC_MEM_DEVICE;
    fs.frag_off = fo.data(); fs.key_off = ko.data(); fs.val_off = vo.data(); fs.k2v_off = oo.data();
    fs.txn_global = txn_global;
    shard_pack(ctx, in, &fs, true);
    const uint32_t G = (std::max(n_global, 1u) + W - 1) / W;
    S.off[0].clear();
    S.send[0] = frag_encode(ctx, W, fo.data(), ko.data(), vo.data(), oo.data(), fs.hdr, fs.keys, fs.vals, fs.k2v, G, S.off[0]);
    S.esz[0] = 1;
    S.ns = 1;
}

static void merge_key_streams(acc_ctx *ctx, acc_comm *c, uint32_t n_global, const Streams &S, acc_merge_view *view)
{
    acc_frag_recv fr{};
    std::vector<uint64_t> cnt[4];
    frag_decode(ctx, c->world, c->rank, n_global, static_cast<const uint8_t *>(S.recv[0]), S.n_src[0], fr, cnt);
    shard_merge(ctx, &fr, view);
}

void shard_reduce(acc_ctx *ctx, acc_comm *c, const acc_batch_in *in, const uint32_t *txn_global, uint32_t n_global,
                  acc_merge_view *view)
{
    if (!c || !in || !view) fail(ACC_E_ARG, "null argument");
    if (c->ctx != ctx) fail(ACC_E_ARG, "communicator belongs to another context");
    if (!txn_global && n_global < in->n_txn) fail(ACC_E_ARG, "n_global must be >= n_txn when txn_global is null");
    Streams S;
    add_key_streams(ctx, in, txn_global, c->world, n_global, S);
    exchange_streams(c, S);
    // KeyDeps.with fold of every home txn (stream order makes the merge wait for the receives)
    merge_key_streams(ctx, c, n_global, S, view);
}

void range_pack(acc_ctx *ctx, const acc_range_batch_in *in, const uint32_t *txn_global, uint32_t world, uint32_t n_global,
                void *send[4], std::vector<uint64_t> off[4]);
void range_merge(acc_ctx *ctx, uint32_t world, uint32_t rank, uint32_t n_global, const std::vector<uint64_t> n_src[4],
                 void *const recv[4], acc_deps_merge_view *view);
void partial_deps_covering(acc_ctx *ctx, const acc_rlist *covering, uint32_t end_inclusive);
void covering_pack(acc_ctx *ctx, const acc_rlist *covering, const uint32_t *txn_global_dev, uint32_t n_store, uint32_t world,
                   void *send[2], std::vector<uint64_t> off[2]);
void covering_merge(acc_ctx *ctx, uint32_t world, uint32_t rank, uint32_t n_global, uint32_t end_inclusive,
                    const std::vector<uint64_t> &n_part, const void *recv_part, const std::vector<uint64_t> &n_cov,
                    const void *recv_cov, const acc_merge_view *kv, const acc_deps_merge_view *rv, acc_covering_view *out);

// PreAccept.reduce of a store's whole PartialDeps: both halves' fragments in one exchange (8 streams), then KeyDeps.with
// (shard_merge) and RangeDeps.with in store order (range_merge) on the home rank
void partial_deps_reduce(acc_ctx *ctx, acc_comm *c, const acc_range_batch_in *in, const uint32_t *txn_global,
                         uint32_t n_global, const acc_rlist *covering, acc_merge_view *key_view,
                         acc_deps_merge_view *range_view, acc_covering_view *covering_view)
{
    if (!c || !in || !key_view || !range_view || (covering && !covering_view)) fail(ACC_E_ARG, "null argument");
    if (c->ctx != ctx) fail(ACC_E_ARG, "communicator belongs to another context");
    // without a placement the batch index is the global index: one check for every call form (with or without a
    // covering), so the key / range results never depend on whether a covering is passed
    if (!txn_global && n_global < in->n_txn) fail(ACC_E_ARG, "n_global must be >= n_txn when txn_global is null");
    const acc_batch_in kin{ in->n_txn, in->mem, in->n_pairs, in->txn_id, in->execute_at, in->status, in->key_off, in->key_code };
    Streams S;
    add_key_streams(ctx, &kin, txn_global, c->world, n_global, S);
    void *rs[4];
    std::vector<uint64_t> ro[4];
    range_pack(ctx, in, txn_global, c->world, n_global, rs, ro);
    const uint64_t resz[4] = { 16, 16, 24, 4 };   // header (4 x u32), Range (start, end), raw TxnId (msb, lsb, node), int
    for (int q = 0; q < 4; ++q) { S.send[1 + q] = rs[q]; S.off[1 + q] = ro[q]; S.esz[1 + q] = resz[q]; }
    S.ns = 5;
    if (covering) {   // the store's txns (u32 global indices) by home rank and its covering ((start, end) pairs)
        const uint32_t n = in->n_txn;
        const uint32_t *gidx = nullptr;
        if (txn_global) gidx = stage_in(ctx, "cov_gidx", txn_global, n, in->mem);
        else {
            uint32_t *io = ctx->get<uint32_t>("cov_iota", std::max<uint32_t>(n, 1));
            if (n) launch(ctx, "iota", k_iota, dim3(grid_for(n, BLOCK)), dim3(BLOCK), 0, io, (size_t)n);
            gidx = io;
        }
        void *cs[2];
        std::vector<uint64_t> co[2];
        covering_pack(ctx, covering, gidx, n, c->world, cs, co);
        S.send[5] = cs[0]; S.off[5] = co[0]; S.esz[5] = 4;
        S.send[6] = cs[1]; S.off[6] = co[1]; S.esz[6] = 16;
        S.ns = 7;
    }
    exchange_streams(c, S);
    merge_key_streams(ctx, c, n_global, S, key_view);
    std::vector<uint64_t> rn[4];
    void *rr[4];
    for (int q = 0; q < 4; ++q) { rn[q] = S.n_src[1 + q]; rr[q] = S.recv[1 + q]; }
    range_merge(ctx, c->world, c->rank, n_global, rn, rr, range_view);
    if (covering)
        covering_merge(ctx, c->world, c->rank, n_global, in->end_inclusive, S.n_src[5], S.recv[5], S.n_src[6], S.recv[6],
                       key_view, range_view, covering_view);
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
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::shard_reduce(ctx, comm, in, txn_global, n_global, out_view);
    });
}

int acc_partial_deps_reduce(acc_ctx *ctx, acc_comm *comm, const acc_range_batch_in *in, const uint32_t *txn_global,
                            uint32_t n_global, const acc_rlist *covering, acc_merge_view *key_view,
                            acc_deps_merge_view *range_view, acc_covering_view *covering_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::partial_deps_reduce(ctx, comm, in, txn_global, n_global, covering, key_view, range_view, covering_view);
    });
}

int acc_partial_deps_covering(acc_ctx *ctx, const acc_range_batch_in *in, const acc_rlist *covering)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        if (!in) acc::fail(ACC_E_ARG, "null argument");
        acc::partial_deps_covering(ctx, covering, in->end_inclusive);
    });
}

}  // extern "C"
