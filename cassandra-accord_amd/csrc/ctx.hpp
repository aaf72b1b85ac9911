// ctx.hpp — acc_ctx: one HIP stream, a grow-only device arena keyed by buffer name, per-kernel
// HIP-event timing, and the exception -> error-code plumbing behind the C ABI (include/accord_amd.h).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/accord_amd.h"

namespace acc {

// Internal failure: carried to the C boundary and mapped to an ACC_E_* code.
struct Error {
    int code;
    std::string msg;
};

[[noreturn]] inline void fail(int code, const std::string &msg) { throw Error{code, msg}; }

#define ACC_HIP(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            ::acc::fail(e_ == hipErrorOutOfMemory ? ACC_E_NOMEM : ACC_E_DEVICE,                \
                        std::string(#expr ": ") + hipGetErrorString(e_));                      \
    } while (0)

struct Buf {
    void *ptr = nullptr;
    size_t bytes = 0;
};

struct TimingSlot {
    std::string name;
    double total_ms = 0;
    uint64_t launches = 0;
};

struct PendingEvent {
    int slot;
    hipEvent_t start, stop;
};

}  // namespace acc

struct acc_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // side streams for independent launches (the KeyDeps write tiers): forked from / joined into `stream`
    static constexpr int NAUX = 3;
    hipStream_t aux[NAUX] = {};
    hipEvent_t fork_ev = nullptr, join_ev[NAUX] = {};
    hipStream_t launch_stream = nullptr;   // where acc::launch enqueues (nullptr = `stream`)
    // decoupled look-back scan status, double buffered: each scan zeroes the words the previous scan dirtied in
    // the other buffer, so no memset launch precedes a scan (acc::scan, prims.hpp)
    size_t scan_cap = 0, scan_dirty[2] = {0, 0};
    int scan_par = 0;
    // one-sweep radix status words per sort tag, double buffered the same way (acc::radix_sort, prims.hpp)
    struct OsState {
        size_t cap = 0, dirty[2] = {0, 0};
        int par = 0;
    };
    std::unordered_map<std::string, OsState> os_state;
    uint32_t flags = 0;
    acc_opts opts{};   // as given to acc_create (flags == opts.flags)
    std::string last_error;
    // a second context on the same device (own stream, buffers, pinned staging), created on first use: the RangeDeps
    // half of acc_partial_deps_batch runs on it from a second host thread, concurrently with the KeyDeps half
    acc_ctx *child = nullptr;
    std::unordered_map<std::string, acc::Buf> bufs;
    // buffers replaced by a larger allocation while kernels may still read them: freed at the next sync
    std::vector<void *> graveyard;
    // pinned host staging for small read-backs (sizes, flags); words [PINNED_SLOTS, +512) hold slotted partials
    static constexpr size_t PINNED_WORDS = 1024, PINNED_SLOTS = 512;
    uint64_t *pinned = nullptr;
    // timing
    std::vector<acc::TimingSlot> slots;
    std::unordered_map<std::string, int> slot_index;
    std::vector<acc::PendingEvent> pending;
    std::vector<hipEvent_t> event_pool;
    std::vector<std::string> time_only;   // non-empty: only these launch tags are timed (acc_timing_filter)
    bool timed(const char *name) const
    {
        if (!(flags & ACC_OPT_TIMING)) return false;
        if (time_only.empty()) return true;
        for (const auto &t : time_only)
            if (t == name) return true;
        return false;
    }
    // counters of the last call (name -> value), exposed by acc_stats_*
    std::vector<std::pair<std::string, uint64_t>> stats;
    void stat(const char *name, uint64_t value)
    {
        for (auto &kv : stats)
            if (kv.first == name) { kv.second = value; return; }
        stats.emplace_back(name, value);
    }
    // last results
    acc_keydeps_view kd_view{};
    acc_merge_view merge_view{};
    acc_rangedeps_view rd_view{};
    acc_deps_merge_view dm_view{};
    bool dm_valid = false;
    uint64_t rd_ent_hint = 0;   // RangeDeps raw pairs of the last batch (output capacity of the stabbing pass)
    bool rd_valid = false;
    bool kd_valid = false;
    bool merge_valid = false;
    // sufficientFor of the last acc_latest_deps_merge (host)
    std::vector<uint64_t> latest_suff_off, latest_suff_s, latest_suff_e;

    // buffer-name namespace (NsScope): lets one call run a sub-pipeline twice (e.g. the KeyDeps and RangeDeps halves
    // of Deps.merge) without the second run overwriting the first one's results
    std::string ns;

    // Grow-only named device buffer. Contents are NOT preserved across growth.
    template <class T>
    T *get(const char *name, size_t count)
    {
        return get_raw<T>(ns.empty() ? std::string(name) : ns + name, count);
    }
    // the same, outside any namespace (state shared by every sub-pipeline: the scan status buffers)
    template <class T>
    T *get_raw(const std::string &name, size_t count)
    {
        size_t bytes = count * sizeof(T);
        if (bytes == 0) bytes = 16;
        acc::Buf &b = bufs[name];
        if (b.bytes < bytes) {
            if (b.ptr) graveyard.push_back(b.ptr);
            b.ptr = nullptr;
            // headroom for the next, larger batch (a store that grows batch by batch would otherwise reallocate its
            // working buffers every other call: each hipMalloc / deferred hipFree stalls the stream); 1/8 past 4 GiB
            size_t want = bytes + (bytes < (4ull << 30) ? bytes / 2 : bytes / 8);
            ACC_HIP(hipMalloc(&b.ptr, want));
            b.bytes = want;
        }
        return static_cast<T *>(b.ptr);
    }

    // Exchange the named buffer with (ptr, bytes): the caller takes the buffer (and its contents), the context keeps the
    // caller's allocation under that name (grown by a later get as usual). Lets a store adopt a call's result arrays
    // instead of copying them.
    void swap_buf(const char *name, void *&ptr, size_t &bytes)
    {
        acc::Buf &b = bufs[ns.empty() ? std::string(name) : ns + name];
        std::swap(b.ptr, ptr);
        std::swap(b.bytes, bytes);
    }

    // the named buffer's current allocation (nullptr if none)
    const void *buf_ptr(const char *name) const
    {
        auto it = bufs.find(ns.empty() ? std::string(name) : ns + name);
        return it == bufs.end() ? nullptr : it->second.ptr;
    }

    hipEvent_t take_event()
    {
        if (!event_pool.empty()) {
            hipEvent_t e = event_pool.back();
            event_pool.pop_back();
            return e;
        }
        hipEvent_t e;
        ACC_HIP(hipEventCreate(&e));
        return e;
    }

    int slot(const char *name)
    {
        auto it = slot_index.find(name);
        if (it != slot_index.end()) return it->second;
        int i = (int)slots.size();
        slots.push_back({name, 0, 0});
        slot_index[name] = i;
        return i;
    }

    // Resolve recorded kernel intervals (requires the stream to be idle).
    void resolve_timing()
    {
        for (auto &p : pending) {
            float ms = 0;
            ACC_HIP(hipEventElapsedTime(&ms, p.start, p.stop));
            slots[p.slot].total_ms += ms;
            slots[p.slot].launches += 1;
            event_pool.push_back(p.start);
            event_pool.push_back(p.stop);
        }
        pending.clear();
    }

    hipStream_t cur() const { return launch_stream ? launch_stream : stream; }

    // aux streams 0..k-1 wait for everything enqueued on the main stream so far
    void fork(int k)
    {
        if (!fork_ev) {
            ACC_HIP(hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming));
            for (int i = 0; i < NAUX; ++i) {
                ACC_HIP(hipStreamCreateWithFlags(&aux[i], hipStreamNonBlocking));
                ACC_HIP(hipEventCreateWithFlags(&join_ev[i], hipEventDisableTiming));
            }
        }
        ACC_HIP(hipEventRecord(fork_ev, stream));
        for (int i = 0; i < k; ++i) ACC_HIP(hipStreamWaitEvent(aux[i], fork_ev, 0));
    }
    // the main stream waits for aux streams 0..k-1
    void join(int k)
    {
        for (int i = 0; i < k; ++i) {
            ACC_HIP(hipEventRecord(join_ev[i], aux[i]));
            ACC_HIP(hipStreamWaitEvent(stream, join_ev[i], 0));
        }
        launch_stream = nullptr;
    }

    // after a failure inside a call: no launch is left pointing at a side stream, and every stream is drained before
    // the next call (or a sync) frees graveyard buffers a side-stream kernel may still read. Errors are ignored here:
    // the failure being reported is the first one.
    void recover() noexcept
    {
        launch_stream = nullptr;
        for (int i = 0; i < NAUX; ++i)
            if (aux[i]) (void)hipStreamSynchronize(aux[i]);
        if (stream) (void)hipStreamSynchronize(stream);
    }

    void sync()
    {
        ACC_HIP(hipStreamSynchronize(stream));
        for (void *p : graveyard) ACC_HIP(hipFree(p));
        graveyard.clear();
        if (!pending.empty()) resolve_timing();
    }
};

namespace acc {

// Scoped buffer-name namespace on a context (see acc_ctx::ns).
struct NsScope {
    acc_ctx *ctx;
    std::string saved;
    NsScope(acc_ctx *c, const char *prefix) : ctx(c), saved(c->ns) { ctx->ns = saved + prefix; }
    ~NsScope() { ctx->ns = saved; }
};

// Launch a kernel on the context stream (or the side stream selected by launch_stream); with ACC_OPT_TIMING, bracket it with HIP events recorded on
// that same stream (so the interval is the kernel's own device time).
template <class K, class... Args>
inline void launch(acc_ctx *ctx, const char *name, K kernel, dim3 grid, dim3 block, size_t shmem, Args... args)
{
    if (grid.x == 0 || grid.y == 0 || grid.z == 0) return;
    PendingEvent pe{};
    const bool timed = ctx->timed(name);
    if (timed) {
        pe.slot = ctx->slot(name);
        pe.start = ctx->take_event();
        pe.stop = ctx->take_event();
        ACC_HIP(hipEventRecord(pe.start, ctx->cur()));
    }
    hipLaunchKernelGGL(kernel, grid, block, shmem, ctx->cur(), args...);
    ACC_HIP(hipGetLastError());
    if (timed) {
        ACC_HIP(hipEventRecord(pe.stop, ctx->cur()));
        ctx->pending.push_back(pe);
    }
}

inline unsigned grid_for(size_t n, unsigned per_block)
{
    size_t g = (n + per_block - 1) / per_block;
    return (unsigned)(g ? g : 1);
}

// Copy caller input (host or device) into a device buffer owned by the context.
template <class T>
inline const T *stage_in(acc_ctx *ctx, const char *name, const T *src, size_t count, uint32_t mem)
{
    if (count == 0) return ctx->get<T>(name, 1);
    if (!src) fail(ACC_E_ARG, std::string("null input array: ") + name);
    if (mem == ACC_MEM_DEVICE) return src;
    T *d = ctx->get<T>(name, count);
    ACC_HIP(hipMemcpyAsync(d, src, count * sizeof(T), hipMemcpyHostToDevice, ctx->stream));
    return d;
}

}  // namespace acc

// Run `body` and translate failures into the C error model.
template <class F>
inline int acc_guard(acc_ctx *ctx, F &&body)
{
    try {
        body();
        if (ctx) ctx->last_error.clear();
        return ACC_OK;
    } catch (const acc::Error &e) {
        if (ctx) { ctx->recover(); ctx->last_error = e.msg; }
        return e.code;
    } catch (const std::bad_alloc &) {
        if (ctx) { ctx->recover(); ctx->last_error = "host allocation failed"; }
        return ACC_E_NOMEM;
    } catch (...) {
        if (ctx) { ctx->recover(); ctx->last_error = "unknown failure"; }
        return ACC_E_STATE;
    }
}
