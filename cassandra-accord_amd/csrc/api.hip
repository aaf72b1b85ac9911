// api.hip — the extern "C" surface of include/accord_amd.h: context lifecycle, error text, result
// copy-out with two-call sizing, and kernel timing read-out.
#include "dict.hpp"
#include <exception>
#include <thread>

namespace acc {
void keydeps_batch(acc_ctx *ctx, const acc_batch_in *in, acc_keydeps_view *view);
void keydeps_mixed(acc_ctx *ctx, const acc_range_batch_in *in, acc_keydeps_view *view, SharedDict *shared = nullptr);
void keydeps_merge(acc_ctx *ctx, const acc_merge_in *in, acc_merge_view *view);
void levelise(acc_ctx *ctx, const acc_graph_in *in, uint32_t *level, uint32_t *order, uint32_t *n_levels);
void rangedeps_batch(acc_ctx *ctx, const acc_range_batch_in *in, acc_rangedeps_view *view, const SharedDict *shared = nullptr);
void shard_pack(acc_ctx *ctx, const acc_batch_in *in, acc_frag_streams *out, bool ctx_alloc);
void shard_merge(acc_ctx *ctx, const acc_frag_recv *in, acc_merge_view *view);
void deps_merge(acc_ctx *ctx, const acc_deps_merge_in *in, acc_deps_merge_view *view);
void rmm_invert(acc_ctx *ctx, const acc_rmm_batch *in, acc_csr_view *out);
void rmm_slice(acc_ctx *ctx, const acc_rmm_batch *in, const acc_ranges_in *select, acc_slice_view *out);
void rangedeps_stab(acc_ctx *ctx, const acc_rmm_batch *rd, const acc_stab_in *q, acc_stab_view *out);
void rmm_without(acc_ctx *ctx, const acc_rmm_batch *in, const acc_ts_cols *txn, const acc_txn_sets *set_a,
                 const acc_txn_sets *set_b, acc_without_view *out);
void recovery_deps_reduce(acc_ctx *ctx, const acc_deps_merge_in *cw, const acc_deps_merge_in *anw, acc_recovery_deps_view *view);
void map_reduce_full(acc_ctx *ctx, const acc_batch_in *in, const acc_recovery_in *q, acc_keydeps_view *view);
void map_reduce_full_ranges(acc_ctx *ctx, const acc_range_cmds_in *c, const acc_recovery_ranges_in *q, acc_rangedeps_view *view);
void latest_deps_merge(acc_ctx *ctx, const acc_latest_in *in, acc_latest_view *view);
void deps_from_json(acc_ctx *ctx, const acc_json_in *in, acc_json_deps_view *view);
void deps_to_json(acc_ctx *ctx, const acc_json_out_in *in, acc_json_out *out);
void cfk_update(acc_ctx *ctx, acc_cfk *cfk, const acc_batch_in *in);
void cfk_apply(acc_ctx *ctx, const acc_cfk_snap *in, const acc_cfk_updates *up, acc_cfk_snap_view *view);
void cfk_snap_to_batch(acc_ctx *ctx, const acc_cfk_snap *in, acc_cfk_batch_view *view, bool trusted = false);
void max_conflicts(acc_ctx *ctx, const acc_conflicts_in *u, const acc_preaccept_in *q, acc_preaccept_out *out);
acc_maxconflicts *mc_new(int device, uint32_t end_inclusive);
void mc_free(acc_maxconflicts *m);
uint64_t mc_size(const acc_maxconflicts *m);
void mc_update(acc_ctx *ctx, acc_maxconflicts *m, const acc_conflicts_in *u);
void mc_get(acc_ctx *ctx, const acc_maxconflicts *m, const acc_preaccept_in *q, acc_preaccept_out *out);
void cfk_view(acc_cfk *cfk, acc_batch_in *out);
void cfk_apply_deps(acc_ctx *ctx, acc_cfk *cfk, const acc_cfk_updates *up);
void cfk_state(acc_cfk *cfk, acc_cfk_snap *out);
void cfk_missing(acc_cfk *cfk, acc_cfk_batch_view *out);
void cfk_free(acc_cfk *cfk);
acc_cfk *cfk_new(int device);
}  // namespace acc

namespace {
// Internal entry points behind acc_create / acc_destroy: the library never calls its own exported names (an
// acc_create exported by another loaded library, e.g. libgomp's OpenACC acc_create(void *, size_t), would
// interpose on a PLT call from inside this library).
int ctx_create(int device, const acc_opts *opts, acc_ctx **out_ctx);
void ctx_destroy(acc_ctx *ctx);
}  // namespace

extern "C" {

const char *acc_version(void) { return "accord_amd 0.1 (gfx950)"; }

int acc_create(int device, const acc_opts *opts, acc_ctx **out_ctx) { return ctx_create(device, opts, out_ctx); }

void acc_destroy(acc_ctx *ctx) { ctx_destroy(ctx); }

}  // extern "C"

namespace {

int ctx_create(int device, const acc_opts *opts, acc_ctx **out_ctx)
{
    if (!out_ctx) return ACC_E_ARG;
    *out_ctx = nullptr;
    acc_ctx *ctx = new (std::nothrow) acc_ctx();
    if (!ctx) return ACC_E_NOMEM;
    int rc = acc_guard(ctx, [&] {
        int count = 0;
        ACC_HIP(hipGetDeviceCount(&count));
        if (device < 0 || device >= count) acc::fail(ACC_E_ARG, "no such HIP device");
        ACC_HIP(hipSetDevice(device));
        ctx->device = device;
        if (opts) ctx->opts = *opts;
        ctx->flags = ctx->opts.flags;
        ACC_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
        ACC_HIP(hipHostMalloc((void **)&ctx->pinned, acc_ctx::PINNED_WORDS * sizeof(uint64_t), hipHostMallocDefault));
    });
    if (rc != ACC_OK) {
        ctx_destroy(ctx);
        return rc;
    }
    *out_ctx = ctx;
    return ACC_OK;
}

void ctx_destroy(acc_ctx *ctx)
{
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (auto &kv : ctx->bufs)
        if (kv.second.ptr) (void)hipFree(kv.second.ptr);
    for (void *p : ctx->graveyard) (void)hipFree(p);
    for (auto &p : ctx->pending) { (void)hipEventDestroy(p.start); (void)hipEventDestroy(p.stop); }
    for (auto e : ctx->event_pool) (void)hipEventDestroy(e);
    for (int i = 0; i < acc_ctx::NAUX; ++i) {
        if (ctx->aux[i]) { (void)hipStreamSynchronize(ctx->aux[i]); (void)hipStreamDestroy(ctx->aux[i]); }
        if (ctx->join_ev[i]) (void)hipEventDestroy(ctx->join_ev[i]);
    }
    if (ctx->fork_ev) (void)hipEventDestroy(ctx->fork_ev);
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    acc_ctx *child = ctx->child;
    delete ctx;
    ctx_destroy(child);
}

}  // namespace

extern "C" {

const char *acc_last_error(const acc_ctx *ctx) { return ctx ? ctx->last_error.c_str() : "null context"; }

int acc_sync(acc_ctx *ctx)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] { ctx->sync(); });
}

void *acc_stream(acc_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int acc_keydeps_batch(acc_ctx *ctx, const acc_batch_in *in, acc_keydeps_view *out_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::keydeps_batch(ctx, in, out_view);
    });
}

int acc_keydeps_mixed(acc_ctx *ctx, const acc_range_batch_in *in, acc_keydeps_view *out_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::keydeps_mixed(ctx, in, out_view);
    });
}

int acc_map_reduce_full(acc_ctx *ctx, const acc_batch_in *snapshot, const acc_recovery_in *q, acc_keydeps_view *out_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::map_reduce_full(ctx, snapshot, q, out_view);
    });
}

int acc_map_reduce_full_ranges(acc_ctx *ctx, const acc_range_cmds_in *cmds, const acc_recovery_ranges_in *q,
                               acc_rangedeps_view *out_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::map_reduce_full_ranges(ctx, cmds, q, out_view);
    });
}

int acc_latest_deps_merge(acc_ctx *ctx, const acc_latest_in *in, acc_latest_view *out_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::latest_deps_merge(ctx, in, out_view);
    });
}

int acc_partial_deps_batch(acc_ctx *ctx, const acc_range_batch_in *in, acc_keydeps_view *key_view,
                           acc_rangedeps_view *range_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        if (!key_view || !range_view) acc::fail(ACC_E_ARG, "null argument");
        const bool serial = (ctx->flags & ACC_OPT_PD_SERIAL) != 0;   // both halves in order on this context
        if (!ctx->child && !serial) {
            const acc_opts o = ctx->opts;
            const int rc = ctx_create(ctx->device, &o, &ctx->child);
            if (rc != ACC_OK) acc::fail(rc, "cannot create the RangeDeps half's context");
        }
        acc_ctx *const child = serial ? nullptr : ctx->child;
        // the RangeDeps half starts on the child context (own stream, own host thread) as soon as the KeyDeps half's
        // dictionary is enqueued: its stream waits for that point of this context's stream, and it reads the
        // dictionary in place (not written again by the KeyDeps half)
        acc::SharedDict sd;
        std::thread th;
        int rrc = ACC_OK;
        hipEvent_t ev = nullptr;
        struct Join {
            std::thread &t;
            hipEvent_t &e;
            ~Join() { if (t.joinable()) t.join(); if (e) (void)hipEventDestroy(e); }
        } join{ th, ev };
        if (child) {
            child->opts = ctx->opts;              // the options and the timing filter as the parent's
            child->flags = ctx->flags;
            child->time_only = ctx->time_only;
            sd.ready = [&](const acc::SharedDict &d) {
                ACC_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
                ACC_HIP(hipEventRecord(ev, ctx->stream));
                th = std::thread([&rrc, child, in, range_view, ev, d] {
                    rrc = acc_guard(child, [&] {
                        ACC_HIP(hipSetDevice(child->device));
                        ACC_HIP(hipStreamWaitEvent(child->stream, ev, 0));
                        acc::rangedeps_batch(child, in, range_view, &d);
                        child->sync();
                    });
                });
            };
        }
        acc::keydeps_mixed(ctx, in, key_view, &sd);
        if (th.joinable()) {
            th.join();
            if (rrc != ACC_OK) acc::fail(rrc, child->last_error.c_str());
            ctx->rd_view = child->rd_view;   // child buffers, valid until the next acc_partial_deps_batch on ctx
            ctx->rd_valid = child->rd_valid;
            ctx->rd_ent_hint = child->rd_ent_hint;
            for (const auto &kv : child->stats) ctx->stat(kv.first.c_str(), kv.second);
            // the RangeDeps half's kernel timings (resolved by the child's sync) join this context's, under their own
            // launch tags: acc_timing readers see both halves of the call
            for (auto &sl : child->slots) {
                if (!sl.launches) continue;
                acc::TimingSlot &d = ctx->slots[ctx->slot(sl.name.c_str())];
                d.total_ms += sl.total_ms;
                d.launches += sl.launches;
                sl.total_ms = 0;
                sl.launches = 0;
            }
        } else {
            acc::rangedeps_batch(ctx, in, range_view, &sd);   // no key pairs (no dictionary to share), or serial
        }
        ctx->kd_valid = true;   // both views stay readable (distinct buffers)
    });
}

int acc_deps_from_json(acc_ctx *ctx, const acc_json_in *in, acc_json_deps_view *out_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::deps_from_json(ctx, in, out_view);
    });
}

int acc_deps_to_json(acc_ctx *ctx, const acc_json_out_in *in, acc_json_out *out)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::deps_to_json(ctx, in, out);
    });
}

int acc_cfk_create(acc_ctx *ctx, acc_cfk **out)
{
    if (!ctx || !out) return ACC_E_ARG;
    *out = nullptr;
    return acc_guard(ctx, [&] { *out = acc::cfk_new(ctx->device); });
}

void acc_cfk_destroy(acc_cfk *cfk) { acc::cfk_free(cfk); }

int acc_cfk_update(acc_ctx *ctx, acc_cfk *cfk, const acc_batch_in *delta)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::cfk_update(ctx, cfk, delta);
    });
}

int acc_cfk_view(acc_ctx *ctx, acc_cfk *cfk, acc_batch_in *out)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::cfk_view(cfk, out);
    });
}

int acc_cfk_apply_deps(acc_ctx *ctx, acc_cfk *cfk, const acc_cfk_updates *updates)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::cfk_apply_deps(ctx, cfk, updates);
    });
}

int acc_cfk_state(acc_ctx *ctx, acc_cfk *cfk, acc_cfk_snap *out)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] { acc::cfk_state(cfk, out); });
}

int acc_cfk_missing(acc_ctx *ctx, acc_cfk *cfk, acc_cfk_batch_view *out)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] { acc::cfk_missing(cfk, out); });
}

int acc_keydeps_copy_out(acc_ctx *ctx, acc_keydeps_out *out)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        if (!out) acc::fail(ACC_E_ARG, "null output");
        if (!ctx->kd_valid) acc::fail(ACC_E_STATE, "no keydeps result on this context");
        const acc_keydeps_view &v = ctx->kd_view;
        out->need_arena = v.total_arena;
        out->need_keys = v.total_keys;
        out->need_deps = v.total_deps;
        if (!out->arena_off || !out->kd_off || !out->u_off)   // sizing call
            acc::fail(ACC_E_CAP, "sizing call (null offset arrays); required sizes written to need_*");
        if (out->cap_arena < v.total_arena || out->cap_keys < v.total_keys || out->cap_deps < v.total_deps)
            acc::fail(ACC_E_CAP, "output capacity too small; required sizes written to need_*");
        hipMemcpyKind kind = out->mem == ACC_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
        size_t n1 = (size_t)v.n_txn + 1;
        ACC_HIP(hipMemcpyAsync(out->arena_off, v.arena_off, n1 * 8, kind, ctx->stream));
        ACC_HIP(hipMemcpyAsync(out->kd_off, v.kd_off, n1 * 8, kind, ctx->stream));
        ACC_HIP(hipMemcpyAsync(out->u_off, v.u_off, n1 * 8, kind, ctx->stream));
        if (v.total_arena) ACC_HIP(hipMemcpyAsync(out->arena, v.arena, v.total_arena * 4, kind, ctx->stream));
        if (v.total_keys) ACC_HIP(hipMemcpyAsync(out->key_idx, v.key_idx, v.total_keys * 4, kind, ctx->stream));
        if (v.total_deps) ACC_HIP(hipMemcpyAsync(out->dep_txn, v.dep_txn, v.total_deps * 4, kind, ctx->stream));
        if (out->kd_key && v.kd_key && v.total_keys)
            ACC_HIP(hipMemcpyAsync(out->kd_key, v.kd_key, v.total_keys * 8, kind, ctx->stream));
        ctx->sync();
    });
}

int acc_rangedeps_batch(acc_ctx *ctx, const acc_range_batch_in *in, acc_rangedeps_view *out_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::rangedeps_batch(ctx, in, out_view);
    });
}

int acc_rangedeps_copy_out(acc_ctx *ctx, acc_rangedeps_out *out)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        if (!out) acc::fail(ACC_E_ARG, "null argument");
        if (!ctx->rd_valid) acc::fail(ACC_E_STATE, "no rangedeps result on this context");
        const acc_rangedeps_view &v = ctx->rd_view;
        out->need_arena = v.total_arena;
        out->need_ranges = v.total_ranges;
        out->need_deps = v.total_deps;
        out->need_dict = v.n_ranges;
        if (!out->arena_off || !out->rd_off || !out->u_off || out->cap_arena < v.total_arena ||
            out->cap_ranges < v.total_ranges || out->cap_deps < v.total_deps || out->cap_dict < v.n_ranges)
            acc::fail(ACC_E_CAP, "output capacity too small (required sizes written)");
        if (out->mem != ACC_MEM_HOST && out->mem != ACC_MEM_DEVICE) acc::fail(ACC_E_ARG, "bad mem");
        const hipMemcpyKind k = out->mem == ACC_MEM_HOST ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
        const size_t n1 = (size_t)v.n_txn + 1;
        ACC_HIP(hipMemcpyAsync(out->arena_off, v.arena_off, n1 * 8, k, ctx->stream));
        ACC_HIP(hipMemcpyAsync(out->rd_off, v.rd_off, n1 * 8, k, ctx->stream));
        ACC_HIP(hipMemcpyAsync(out->u_off, v.u_off, n1 * 8, k, ctx->stream));
        if (v.total_arena) ACC_HIP(hipMemcpyAsync(out->arena, v.arena, v.total_arena * 4, k, ctx->stream));
        if (v.total_ranges) ACC_HIP(hipMemcpyAsync(out->range_id, v.range_id, v.total_ranges * 4, k, ctx->stream));
        if (v.total_deps) ACC_HIP(hipMemcpyAsync(out->dep_txn, v.dep_txn, v.total_deps * 4, k, ctx->stream));
        if (v.n_ranges) {
            ACC_HIP(hipMemcpyAsync(out->rng_start, v.rng_start, (size_t)v.n_ranges * 8, k, ctx->stream));
            ACC_HIP(hipMemcpyAsync(out->rng_end, v.rng_end, (size_t)v.n_ranges * 8, k, ctx->stream));
        }
        ctx->sync();
    });
}

int acc_shard_pack(acc_ctx *ctx, const acc_batch_in *in, acc_frag_streams *out)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::shard_pack(ctx, in, out, false);
    });
}

int acc_shard_merge(acc_ctx *ctx, const acc_frag_recv *in, acc_merge_view *out_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::shard_merge(ctx, in, out_view);
        ctx->merge_view = *out_view;
        ctx->merge_valid = true;
    });
}

int acc_keydeps_merge(acc_ctx *ctx, const acc_merge_in *in, acc_merge_view *out_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::keydeps_merge(ctx, in, out_view);
    });
}

int acc_merge_copy_out(acc_ctx *ctx, acc_merge_out *out)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        if (!out) acc::fail(ACC_E_ARG, "null output");
        if (!ctx->merge_valid) acc::fail(ACC_E_STATE, "no merge result on this context");
        const acc_merge_view &v = ctx->merge_view;
        out->need_keys = v.total_keys;
        out->need_vals = v.total_vals;
        out->need_k2v = v.total_k2v;
        if (!out->key_off || !out->val_off || !out->k2v_off)
            acc::fail(ACC_E_CAP, "sizing call (null offset arrays); required sizes written to need_*");
        if (out->cap_keys < v.total_keys || out->cap_vals < v.total_vals || out->cap_k2v < v.total_k2v)
            acc::fail(ACC_E_CAP, "output capacity too small; required sizes written to need_*");
        hipMemcpyKind kind = out->mem == ACC_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
        size_t n1 = (size_t)v.n_groups + 1;
        ACC_HIP(hipMemcpyAsync(out->key_off, v.key_off, n1 * 8, kind, ctx->stream));
        ACC_HIP(hipMemcpyAsync(out->val_off, v.val_off, n1 * 8, kind, ctx->stream));
        ACC_HIP(hipMemcpyAsync(out->k2v_off, v.k2v_off, n1 * 8, kind, ctx->stream));
        if (v.total_keys) ACC_HIP(hipMemcpyAsync(out->key_code, v.key_code, v.total_keys * 8, kind, ctx->stream));
        if (v.total_vals) ACC_HIP(hipMemcpyAsync(out->txn_rank, v.txn_rank, v.total_vals * 4, kind, ctx->stream));
        if (v.total_k2v) ACC_HIP(hipMemcpyAsync(out->k2v, v.k2v, v.total_k2v * 4, kind, ctx->stream));
        ctx->sync();
    });
}

int acc_deps_merge(acc_ctx *ctx, const acc_deps_merge_in *in, acc_deps_merge_view *out_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::deps_merge(ctx, in, out_view);
    });
}

int acc_rmm_copy_out(acc_ctx *ctx, uint32_t n_groups, const acc_rmm_view *v, acc_rmm_out *out)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        if (!out || !v) acc::fail(ACC_E_ARG, "null argument");
        if (out->mem != ACC_MEM_HOST && out->mem != ACC_MEM_DEVICE) acc::fail(ACC_E_ARG, "bad mem");
        out->need_keys = v->total_keys;
        out->need_vals = v->total_vals;
        out->need_k2v = v->total_k2v;
        if (!out->key_off || !out->val_off || !out->k2v_off)
            acc::fail(ACC_E_CAP, "sizing call (null offset arrays); required sizes written to need_*");
        if (out->cap_keys < v->total_keys || out->cap_vals < v->total_vals || out->cap_k2v < v->total_k2v)
            acc::fail(ACC_E_CAP, "output capacity too small; required sizes written to need_*");
        const hipMemcpyKind k = out->mem == ACC_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
        const size_t n1 = (size_t)n_groups + 1;
        hipStream_t st = ctx->stream;
        ACC_HIP(hipMemcpyAsync(out->key_off, v->key_off, n1 * 8, k, st));
        ACC_HIP(hipMemcpyAsync(out->val_off, v->val_off, n1 * 8, k, st));
        ACC_HIP(hipMemcpyAsync(out->k2v_off, v->k2v_off, n1 * 8, k, st));
        if (v->total_keys) {
            if (out->key_a) ACC_HIP(hipMemcpyAsync(out->key_a, v->key_a, v->total_keys * 8, k, st));
            if (out->key_b && v->key_b) ACC_HIP(hipMemcpyAsync(out->key_b, v->key_b, v->total_keys * 8, k, st));
        }
        if (v->total_vals) {
            if (out->txn_msb) ACC_HIP(hipMemcpyAsync(out->txn_msb, v->txn_msb, v->total_vals * 8, k, st));
            if (out->txn_lsb) ACC_HIP(hipMemcpyAsync(out->txn_lsb, v->txn_lsb, v->total_vals * 8, k, st));
            if (out->txn_node) ACC_HIP(hipMemcpyAsync(out->txn_node, v->txn_node, v->total_vals * 4, k, st));
            if (out->txn_src && v->txn_src) ACC_HIP(hipMemcpyAsync(out->txn_src, v->txn_src, v->total_vals * 4, k, st));
        }
        if (v->total_k2v && out->k2v) ACC_HIP(hipMemcpyAsync(out->k2v, v->k2v, v->total_k2v * 4, k, st));
        ctx->sync();
    });
}

int acc_rmm_invert(acc_ctx *ctx, const acc_rmm_batch *in, acc_csr_view *out_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::rmm_invert(ctx, in, out_view);
    });
}

int acc_rmm_slice(acc_ctx *ctx, const acc_rmm_batch *in, const acc_ranges_in *select, acc_slice_view *out_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::rmm_slice(ctx, in, select, out_view);
    });
}

int acc_rmm_without(acc_ctx *ctx, const acc_rmm_batch *in, const acc_ts_cols *txn, const acc_txn_sets *set_a,
                    const acc_txn_sets *set_b, acc_without_view *out_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::rmm_without(ctx, in, txn, set_a, set_b, out_view);
    });
}

int acc_recovery_deps_reduce(acc_ctx *ctx, const acc_deps_merge_in *committed_witness,
                             const acc_deps_merge_in *accepted_no_witness, acc_recovery_deps_view *out_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::recovery_deps_reduce(ctx, committed_witness, accepted_no_witness, out_view);
    });
}

int acc_rangedeps_stab(acc_ctx *ctx, const acc_rmm_batch *range_deps, const acc_stab_in *queries, acc_stab_view *out_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::rangedeps_stab(ctx, range_deps, queries, out_view);
    });
}

int acc_copy_out(acc_ctx *ctx, void *dst, const void *src_device, size_t bytes, uint32_t mem)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        if (mem != ACC_MEM_HOST && mem != ACC_MEM_DEVICE) acc::fail(ACC_E_ARG, "bad mem");
        if (!bytes) return;
        if (!dst || !src_device) acc::fail(ACC_E_ARG, "null pointer");
        ACC_HIP(hipMemcpyAsync(dst, src_device, bytes, mem == ACC_MEM_HOST ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice,
                               ctx->stream));
        ctx->sync();
    });
}

int acc_levelise(acc_ctx *ctx, const acc_graph_in *in, uint32_t *level, uint32_t *order, uint32_t *n_levels)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::levelise(ctx, in, level, order, n_levels);
    });
}

int acc_timing_count(acc_ctx *ctx)
{
    if (!ctx) return 0;
    int rc = acc_guard(ctx, [&] { ctx->sync(); });
    return rc == ACC_OK ? (int)ctx->slots.size() : rc;
}

int acc_timing_get(acc_ctx *ctx, int i, const char **name, double *total_ms, uint64_t *launches)
{
    if (!ctx || i < 0 || i >= (int)ctx->slots.size()) return ACC_E_ARG;
    if (name) *name = ctx->slots[i].name.c_str();
    if (total_ms) *total_ms = ctx->slots[i].total_ms;
    if (launches) *launches = ctx->slots[i].launches;
    return ACC_OK;
}

void acc_timing_reset(acc_ctx *ctx)
{
    if (!ctx) return;
    acc_guard(ctx, [&] { ctx->sync(); });
    for (auto &s : ctx->slots) { s.total_ms = 0; s.launches = 0; }
}

int acc_timing_filter(acc_ctx *ctx, const char *tags_csv)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ctx->time_only.clear();
        if (!tags_csv) return;
        std::string cur;
        for (const char *c = tags_csv;; ++c) {
            if (*c == ',' || *c == 0) {
                if (!cur.empty()) ctx->time_only.push_back(cur);
                cur.clear();
                if (!*c) break;
            } else {
                cur.push_back(*c);
            }
        }
    });
}

int acc_stats_count(acc_ctx *ctx) { return ctx ? (int)ctx->stats.size() : 0; }

int acc_stats_get(acc_ctx *ctx, int i, const char **name, uint64_t *value)
{
    if (!ctx || i < 0 || i >= (int)ctx->stats.size()) return ACC_E_ARG;
    if (name) *name = ctx->stats[i].first.c_str();
    if (value) *value = ctx->stats[i].second;
    return ACC_OK;
}

int acc_cfk_apply(acc_ctx *ctx, const acc_cfk_snap *snap, const acc_cfk_updates *updates, acc_cfk_snap_view *out_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::cfk_apply(ctx, snap, updates, out_view);
    });
}

int acc_cfk_snap_to_batch(acc_ctx *ctx, const acc_cfk_snap *snap, acc_cfk_batch_view *out_view)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::cfk_snap_to_batch(ctx, snap, out_view);
    });
}

int acc_max_conflicts(acc_ctx *ctx, const acc_conflicts_in *updates, const acc_preaccept_in *queries, acc_preaccept_out *out)
{
    if (!ctx) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::max_conflicts(ctx, updates, queries, out);
    });
}


int acc_maxconflicts_create(acc_ctx *ctx, uint32_t end_inclusive, acc_maxconflicts **out)
{
    if (!ctx || !out) return ACC_E_ARG;
    *out = nullptr;
    return acc_guard(ctx, [&] { *out = acc::mc_new(ctx->device, end_inclusive); });
}

void acc_maxconflicts_destroy(acc_maxconflicts *map) { acc::mc_free(map); }

int acc_maxconflicts_update(acc_ctx *ctx, acc_maxconflicts *map, const acc_conflicts_in *updates)
{
    if (!ctx || !map) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::mc_update(ctx, map, updates);
    });
}

int acc_maxconflicts_get(acc_ctx *ctx, acc_maxconflicts *map, const acc_preaccept_in *queries, acc_preaccept_out *out)
{
    if (!ctx || !map) return ACC_E_ARG;
    return acc_guard(ctx, [&] {
        ACC_HIP(hipSetDevice(ctx->device));
        acc::mc_get(ctx, map, queries, out);
    });
}

uint64_t acc_maxconflicts_size(const acc_maxconflicts *map) { return acc::mc_size(map); }

}  // extern "C"
