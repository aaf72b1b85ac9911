// fragwire.hip — the compact wire form of the KeyDeps fragments that acc_shard_reduce / acc_partial_deps_reduce send
// to each txn's home rank (PreAccept.reduce over the stores' replies, messages/PreAccept.java:141-156;
// CommandStores.mapReduce, local/CommandStores.java:575-592).
//
// acc_shard_pack's fragment (the explicit ABI form, kept as it is) spends 16 B of header, 8 B per key code and 4 B per
// keysToTxnIds int. On the wire, everything the home rank can derive is dropped:
//   * the txn: home(t) = t mod world is the destination, so a fragment is its slot g = t / world, and the slots a
//     source sends to one home are one bitmap of G bits (or a u32 list when sparser than 1 in 32);
//   * sizes: (nk, nv, vb) as u16 (u32 when a message needs it); no = nk + entries, and the entries are counted on
//     arrival;
//   * keys: a store's keys lie in its own key range, so each is a u32 offset from the message's smallest key (u64
//     codes when a message spans 2^32 or more);
//   * TxnIds: the fragment's sorted global indices as LEB128 varints, the first relative to t (zigzag), the others
//     as gaps minus one;
//   * keysToTxnIds: which of the nv TxnIds each key lists is an nk x nv bit matrix (a KeyDeps key's list is a sorted
//     subset of the txn's TxnIds, RelationMultiMap), omitted for one key (its list is every TxnId).
// A message (one per destination) = a 64-B header, then the sections slots / counts / keys / TxnIds / key bits, each
// 8-B aligned. The receiver rebuilds acc_shard_pack's four streams in source order and runs acc_shard_merge on them.
#include "prims.hpp"

#include <vector>

namespace acc {

namespace fw {

constexpr uint32_t MAGIC = 0x4B464341u;   // "ACFK"
enum : uint32_t { F_SLOT_LIST = 1, F_WIDE_CNT = 2, F_WIDE_KEY = 4 };
constexpr uint32_t HDR_WORDS = 16;

struct Msg {                  // one message's layout (sender: per destination; receiver: per source)
    uint64_t base;            // byte offset of the message in the send / receive buffer
    uint64_t slot, cnt, key, val, kbm, end;   // section byte offsets from base (end = message size)
    uint64_t kbase;
    uint32_t flags, nfrag, G, pad;
    uint64_t f0;              // index of the message's first fragment (sender: dest-major; receiver: source-major)
    uint64_t k0, vb0, kb0;    // sender: its first key / TxnId byte / key-bit byte among all fragments' (prefix values)
    uint64_t w0;              // receiver: its first bitmap word among all bitmap words
};

__host__ __device__ inline uint64_t al8(uint64_t x) { return (x + 7) & ~7ull; }

__device__ __forceinline__ uint32_t vlen(uint64_t x)
{
    uint32_t n = 1;
    while (x >= 0x80) { x >>= 7; ++n; }
    return n;
}
__device__ __forceinline__ uint64_t zigzag(int64_t d) { return ((uint64_t)d << 1) ^ (uint64_t)(d >> 63); }
__device__ __forceinline__ int64_t unzigzag(uint64_t z) { return (int64_t)(z >> 1) ^ -(int64_t)(z & 1); }

// the varint of TxnId j of a fragment (vals sorted ascending): j = 0 relative to t, else the gap minus one
__device__ __forceinline__ uint64_t val_code(const uint32_t *v, uint64_t j, uint32_t t)
{
    return j == 0 ? zigzag((int64_t)v[0] - (int64_t)t) : (uint64_t)(v[j] - v[j - 1] - 1u);
}

// ---------------------------------------------------------------- sender
// per fragment (one wave): the varint bytes of its TxnIds, its key-bit bytes, its key span and largest count
__global__ __launch_bounds__(BLOCK) void k_fe_meas(uint64_t F, const uint32_t *__restrict__ hdr,
                                                   const uint64_t *__restrict__ ko, const uint64_t *__restrict__ vo,
                                                   const uint64_t *__restrict__ keys, const uint32_t *__restrict__ vals,
                                                   uint64_t *__restrict__ vb, uint64_t *__restrict__ kb,
                                                   uint64_t *__restrict__ fmin, uint64_t *__restrict__ fmax,
                                                   uint32_t *__restrict__ fcm)
{
    const uint64_t f = (uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    const uint32_t lane = lane_id();
    if (f >= F) return;
    const uint32_t t = hdr[4 * f], nk = hdr[4 * f + 1], nv = hdr[4 * f + 2];
    const uint64_t k0 = ko[f], v0 = vo[f];
    uint64_t mn = ~0ull, mx = 0, bytes = 0;
    for (uint64_t j = lane; j < nk; j += 64) { const uint64_t k = keys[k0 + j]; mn = min(mn, k); mx = max(mx, k); }
    for (uint64_t j = lane; j < nv; j += 64) bytes += vlen(val_code(vals + v0, j, t));
    bytes = wave_inclusive(bytes, OpAdd<uint64_t>());
    mx = wave_inclusive(mx, OpMax<uint64_t>());
    mn = ~wave_inclusive(~mn, OpMax<uint64_t>());   // (min as the max of complements)
    if (lane == 63) {
        vb[f] = bytes;
        kb[f] = nk >= 2 ? ((uint64_t)nk * nv + 7) / 8 : 0;
        fmin[f] = mn; fmax[f] = mx;
        fcm[f] = max(max(nk, nv), (uint32_t)min<uint64_t>(bytes, 0xFFFFFFFFull));
    }
}

// per destination d (blocks d * FE_DB .. + FE_DB): key span and largest count over its fragments [fo[d], fo[d+1]),
// one atomic per block
constexpr uint32_t FE_DB = 32;
__global__ __launch_bounds__(BLOCK) void k_fe_dest(const uint64_t *__restrict__ fo, const uint64_t *__restrict__ fmin,
                                                   const uint64_t *__restrict__ fmax, const uint32_t *__restrict__ fcm,
                                                   uint64_t *__restrict__ kmin, uint64_t *__restrict__ kmax,
                                                   uint32_t *__restrict__ cmax)
{
    const uint32_t d = blockIdx.x / FE_DB, c = blockIdx.x % FE_DB;
    uint64_t mn = ~0ull, mx = 0, cm = 0;
    for (uint64_t f = fo[d] + (uint64_t)c * BLOCK + threadIdx.x; f < fo[d + 1]; f += (uint64_t)FE_DB * BLOCK) {
        mn = min(mn, fmin[f]); mx = max(mx, fmax[f]); cm = max(cm, (uint64_t)fcm[f]);
    }
    __shared__ uint64_t lds[WAVES];
    uint64_t tot;
    block_exclusive(mx, OpMax<uint64_t>(), lds, tot);
    mx = tot;
    __syncthreads();
    block_exclusive(~mn, OpMax<uint64_t>(), lds, tot);
    mn = ~tot;
    __syncthreads();
    block_exclusive(cm, OpMax<uint64_t>(), lds, tot);
    if (threadIdx.x == 0) {
        if (mn <= mx) {
            atomicMin((unsigned long long *)&kmin[d], (unsigned long long)mn);
            atomicMax((unsigned long long *)&kmax[d], (unsigned long long)mx);
        }
        atomicMax(&cmax[d], (uint32_t)min<uint64_t>(tot, 0xFFFFFFFFull));
    }
}

__device__ __forceinline__ void put_bit(uint8_t *buf, uint64_t byte0, uint64_t bit)
{
    const uint64_t b = byte0 * 8 + bit;   // byte0: 4-B aligned section start + byte offset
    atomicOr(reinterpret_cast<uint32_t *>(buf) + (b >> 5), 1u << (b & 31));
}

// per fragment (one wave): slot bit, counts, keys, TxnId varints, key bits into its destination's message (zeroed)
__global__ __launch_bounds__(BLOCK) void k_fe_write(uint64_t F, uint32_t W, const Msg *__restrict__ msg,
                                                    const uint32_t *__restrict__ hdr, const uint64_t *__restrict__ ko,
                                                    const uint64_t *__restrict__ vo, const uint64_t *__restrict__ oo,
                                                    const uint64_t *__restrict__ keys, const uint32_t *__restrict__ vals,
                                                    const int32_t *__restrict__ k2v, const uint64_t *__restrict__ vbo,
                                                    const uint64_t *__restrict__ kbo, uint8_t *__restrict__ buf)
{
    const uint64_t f = (uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    const uint32_t lane = lane_id();
    if (f >= F) return;
    const uint32_t t = hdr[4 * f], nk = hdr[4 * f + 1], nv = hdr[4 * f + 2];
    const Msg m = msg[t % W];
    uint8_t *mb = buf + m.base;
    const uint64_t i = f - m.f0;   // index within the message
    const uint32_t g = t / W;
    if (lane == 0) {
        if (m.flags & F_SLOT_LIST) reinterpret_cast<uint32_t *>(mb + m.slot)[i] = g;
        else put_bit(mb, m.slot, g);
        const uint32_t vbytes = (uint32_t)(vbo[f + 1] - vbo[f]);
        if (m.flags & F_WIDE_CNT) {
            uint32_t *c = reinterpret_cast<uint32_t *>(mb + m.cnt) + 3 * i;
            c[0] = nk; c[1] = nv; c[2] = vbytes;
        } else {
            uint16_t *c = reinterpret_cast<uint16_t *>(mb + m.cnt) + 3 * i;
            c[0] = (uint16_t)nk; c[1] = (uint16_t)nv; c[2] = (uint16_t)vbytes;
        }
    }
    const uint64_t k0 = ko[f], kd = k0 - m.k0;
    for (uint64_t j = lane; j < nk; j += 64) {
        const uint64_t k = keys[k0 + j];
        if (m.flags & F_WIDE_KEY) reinterpret_cast<uint64_t *>(mb + m.key)[kd + j] = k;
        else reinterpret_cast<uint32_t *>(mb + m.key)[kd + j] = (uint32_t)(k - m.kbase);
    }
    // TxnId varints: 64 at a time, byte positions by a wave prefix of their lengths
    const uint32_t *v = vals + vo[f];
    uint8_t *vp = mb + m.val + (vbo[f] - m.vb0);
    uint64_t pos = 0;
    for (uint64_t c0 = 0; c0 < nv; c0 += 64) {
        const uint64_t j = c0 + lane;
        uint64_t x = j < nv ? val_code(v, j, t) : 0;
        const uint64_t len = j < nv ? vlen(x) : 0;
        const uint64_t incl = wave_inclusive(len, OpAdd<uint64_t>());
        uint64_t p = pos + incl - len;
        for (uint64_t q = 0; q < len; ++q) {
            vp[p++] = (uint8_t)((x & 0x7F) | (q + 1 < len ? 0x80 : 0));
            x >>= 7;
        }
        pos += __shfl(incl, 63, 64);
    }
    // key bits: entry e of key k (an index into the TxnIds) -> bit k * nv + e
    if (nk >= 2) {
        const int32_t *a = k2v + oo[f];
        const uint64_t kbyte = m.kbm + (kbo[f] - m.kb0);
        const uint32_t no = (uint32_t)(oo[f + 1] - oo[f]);
        for (uint32_t j = nk + lane; j < no; j += 64) {
            uint32_t lo = 0, hi = nk;   // key of entry position j: first k with end[k] > j
            while (lo < hi) { const uint32_t mid = (lo + hi) >> 1; if ((uint32_t)a[mid] > j) hi = mid; else lo = mid + 1; }
            put_bit(mb, kbyte, (uint64_t)lo * nv + (uint32_t)a[j]);
        }
    }
}

// per-fragment sizes from the headers, for the stream offsets (dest-major, the order of acc_shard_pack's streams)
__global__ __launch_bounds__(BLOCK) void k_fe_sizes(uint64_t F, const uint32_t *__restrict__ hdr, uint64_t *__restrict__ nk,
                                                    uint64_t *__restrict__ nv, uint64_t *__restrict__ no)
{
    const uint64_t f = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (f >= F) return;
    nk[f] = hdr[4 * f + 1]; nv[f] = hdr[4 * f + 2]; no[f] = hdr[4 * f + 3];
}

// ---------------------------------------------------------------- receiver
__device__ __forceinline__ uint32_t src_of(const Msg *m, uint32_t W, uint64_t f)
{
    uint32_t s = 0;
    while (s + 1 < W && m[s + 1].f0 <= f) ++s;
    return s;
}
__device__ __forceinline__ uint32_t src_of_word(const Msg *m, uint32_t W, uint64_t w)
{
    uint32_t s = 0;
    while (s + 1 < W && m[s + 1].w0 <= w) ++s;
    return s;
}

// bitmap words of every bitmap-form message, concatenated: their popcounts
__global__ __launch_bounds__(BLOCK) void k_fd_popc(uint64_t NW, uint32_t W, const Msg *__restrict__ msg,
                                                   const uint8_t *__restrict__ buf, uint32_t *__restrict__ pc)
{
    const uint64_t w = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (w >= NW) return;
    const Msg &m = msg[src_of_word(msg, W, w)];
    pc[w] = __popc(reinterpret_cast<const uint32_t *>(buf + m.base + m.slot)[w - m.w0]);
}

// set bits -> fragment txns (t = rank + slot * world), in slot order per source
__global__ __launch_bounds__(BLOCK) void k_fd_bits(uint64_t NW, uint32_t W, uint32_t rank, const Msg *__restrict__ msg,
                                                   const uint8_t *__restrict__ buf, const uint32_t *__restrict__ pco,
                                                   uint32_t *__restrict__ hdr, uint64_t *__restrict__ err)
{
    const uint64_t w = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (w >= NW) return;
    const uint32_t s = src_of_word(msg, W, w);
    const Msg &m = msg[s];
    uint32_t bits = reinterpret_cast<const uint32_t *>(buf + m.base + m.slot)[w - m.w0];
    uint64_t i = m.f0 + (pco[w] - pco[m.w0]);
    const uint32_t g0 = (uint32_t)(w - m.w0) * 32;
    if (bits && (g0 + 32 - __clz(bits)) > m.G) atomicOr((unsigned long long *)err, 1ull);   // a bit past G
    while (bits) {
        const uint32_t b = __ffs(bits) - 1;
        bits &= bits - 1;
        hdr[4 * i++] = rank + (g0 + b) * W;
    }
}

// per fragment: txn (list form), counts, and the per-fragment sizes to scan
__global__ __launch_bounds__(BLOCK) void k_fd_counts(uint64_t F, uint32_t W, uint32_t rank, const Msg *__restrict__ msg,
                                                     const uint8_t *__restrict__ buf, uint32_t *__restrict__ hdr,
                                                     uint64_t *__restrict__ a_nk, uint64_t *__restrict__ a_nv,
                                                     uint64_t *__restrict__ a_vb, uint64_t *__restrict__ a_kb)
{
    const uint64_t f = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (f >= F) return;
    const Msg &m = msg[src_of(msg, W, f)];
    const uint8_t *mb = buf + m.base;
    const uint64_t i = f - m.f0;
    if (m.flags & F_SLOT_LIST) hdr[4 * f] = rank + reinterpret_cast<const uint32_t *>(mb + m.slot)[i] * W;
    uint32_t nk, nv, vb;
    if (m.flags & F_WIDE_CNT) {
        const uint32_t *c = reinterpret_cast<const uint32_t *>(mb + m.cnt) + 3 * i;
        nk = c[0]; nv = c[1]; vb = c[2];
    } else {
        const uint16_t *c = reinterpret_cast<const uint16_t *>(mb + m.cnt) + 3 * i;
        nk = c[0]; nv = c[1]; vb = c[2];
    }
    hdr[4 * f + 1] = nk; hdr[4 * f + 2] = nv;
    a_nk[f] = nk; a_nv[f] = nv; a_vb[f] = vb;
    a_kb[f] = nk >= 2 ? ((uint64_t)nk * nv + 7) / 8 : 0;
}

// per fragment (one wave): entries = set key bits (every TxnId for one key) -> no = nk + entries
__global__ __launch_bounds__(BLOCK) void k_fd_no(uint64_t F, uint32_t W, const Msg *__restrict__ msg,
                                                 const uint8_t *__restrict__ buf, uint32_t *__restrict__ hdr,
                                                 const uint64_t *__restrict__ kbo, uint64_t *__restrict__ a_no)
{
    const uint64_t f = (uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    const uint32_t lane = lane_id();
    if (f >= F) return;
    const uint32_t nk = hdr[4 * f + 1], nv = hdr[4 * f + 2];
    uint64_t e = 0;
    if (nk >= 2) {
        const Msg &m = msg[src_of(msg, W, f)];
        const uint8_t *kp = buf + m.base + m.kbm + (kbo[f] - kbo[m.f0]);
        const uint64_t nb = ((uint64_t)nk * nv + 7) / 8;
        for (uint64_t j = lane; j < nb; j += 64) e += __popc(kp[j]);
        e = wave_inclusive(e, OpAdd<uint64_t>());
        e = __shfl(e, 63, 64);
    } else {
        e = nk ? nv : 0;
    }
    if (lane == 0) { hdr[4 * f + 3] = nk + (uint32_t)e; a_no[f] = nk + e; }
}

__device__ __forceinline__ bool kbit(const uint8_t *kp, uint64_t b) { return (kp[b >> 3] >> (b & 7)) & 1u; }

// per fragment (one wave): keys, TxnIds (varints decoded 64 bytes at a time), keysToTxnIds from the key bits
__global__ __launch_bounds__(BLOCK) void k_fd_unpack(uint64_t F, uint32_t W, const Msg *__restrict__ msg,
                                                     const uint8_t *__restrict__ buf, const uint32_t *__restrict__ hdr,
                                                     const uint64_t *__restrict__ sk, const uint64_t *__restrict__ sv,
                                                     const uint64_t *__restrict__ svb, const uint64_t *__restrict__ skb,
                                                     const uint64_t *__restrict__ so, uint64_t *__restrict__ keys,
                                                     uint32_t *__restrict__ vals, int32_t *__restrict__ k2v,
                                                     uint64_t *__restrict__ err)
{
    const uint64_t f = (uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    const uint32_t lane = lane_id();
    if (f >= F) return;
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const Msg m = msg[src_of(msg, W, f)];
    const uint8_t *mb = buf + m.base;
    const uint32_t t = hdr[4 * f], nk = hdr[4 * f + 1], nv = hdr[4 * f + 2], no = hdr[4 * f + 3];
    const uint64_t kd = sk[f] - sk[m.f0];
    for (uint64_t j = lane; j < nk; j += 64)
        keys[sk[f] + j] = (m.flags & F_WIDE_KEY) ? reinterpret_cast<const uint64_t *>(mb + m.key)[kd + j]
                                                 : m.kbase + reinterpret_cast<const uint32_t *>(mb + m.key)[kd + j];
    // TxnIds: a byte with the top bit clear ends a varint; the wave finds the ends 64 bytes at a time, each ending lane
    // decodes its value from its start (the previous end + 1), and a prefix sum of the decoded gaps gives the indices
    const uint8_t *vp = mb + m.val + (svb[f] - svb[m.f0]);
    const uint64_t VB = svb[f + 1] - svb[f];
    uint32_t *vo = vals + sv[f];
    uint64_t done = 0, start = 0;   // values written; byte where the next varint starts
    int64_t run = 0;                // the last decoded index (before the first: t)
    for (uint64_t c0 = 0; c0 < VB; c0 += 64) {
        const uint64_t p = c0 + lane;
        const uint8_t by = p < VB ? vp[p] : 0x80;
        const uint64_t ends = __ballot(p < VB && !(by & 0x80));
        const bool mine = (ends >> lane) & 1ull;
        int64_t val = 0;
        if (mine) {
            const uint64_t below = ends & lt;
            const uint64_t s0 = below ? c0 + 63 - __clzll(below) + 1 : start;
            uint64_t x = 0;
            for (uint64_t q = s0, sh = 0; q <= p && sh < 64; ++q, sh += 7) x |= (uint64_t)(vp[q] & 0x7F) << sh;
            const uint64_t idx = done + __popcll(below);
            val = idx == 0 ? (int64_t)t + unzigzag(x) : (int64_t)x + 1;
        }
        int64_t incl = wave_inclusive(val, OpAdd<int64_t>());
        if (mine) {
            const uint64_t idx = done + __popcll(ends & lt);
            const int64_t v = run + incl;
            if (idx < nv && v >= 0 && v <= 0xFFFFFFFFll) vo[idx] = (uint32_t)v;
            else atomicOr((unsigned long long *)err, 2ull);
        }
        run += __shfl(incl, 63, 64);
        done += __popcll(ends);
        if (ends) start = c0 + 63 - __clzll(ends) + 1;
    }
    if (lane == 0 && done != nv) atomicOr((unsigned long long *)err, 2ull);
    // keysToTxnIds: [end of each key's list (from nk)] then each key's TxnId indices, ascending
    int32_t *a = k2v + so[f];
    if (nk == 1) {
        if (lane == 0) a[0] = (int32_t)(1 + nv);
        for (uint32_t j = lane; j < nv; j += 64) a[1 + j] = (int32_t)j;
    } else if (nk >= 2) {
        const uint8_t *kp = mb + m.kbm + (skb[f] - skb[m.f0]);
        const uint64_t NB = (uint64_t)nk * nv;
        uint64_t cnt = 0;
        for (uint64_t c0 = 0; c0 < NB; c0 += 64) {
            const uint64_t b = c0 + lane;
            const bool set = b < NB && kbit(kp, b);
            const uint64_t bal = __ballot(set);
            const uint64_t at = cnt + __popcll(bal & lt) + (set ? 1 : 0);   // entries up to and including this bit
            const uint32_t k = (uint32_t)(b / nv), e = (uint32_t)(b % nv);
            if (set && nk + at - 1 < no) a[nk + at - 1] = (int32_t)e;
            if (b < NB && e == nv - 1) a[k] = (int32_t)(nk + at);   // the key's last bit: its list ends here
            cnt += __popcll(bal);
        }
    }
}

}  // namespace fw

using namespace fw;

// Encode acc_shard_pack's dest-major streams (device; host offsets fo/ko/vo/oo of W+1 entries) into one message per
// destination. Returns the device buffer (owned by ctx) and the per-destination byte offsets (W+1).
uint8_t *frag_encode(acc_ctx *ctx, uint32_t W, const uint64_t *fo, const uint64_t *ko_h, const uint64_t *vo_h,
                     const uint64_t *oo_h, const uint32_t *hdr, const uint64_t *keys, const uint32_t *vals,
                     const int32_t *k2v, uint32_t G, std::vector<uint64_t> &boff)
{
    hipStream_t st = ctx->stream;
    const uint64_t F = fo[W];
    uint64_t *nk = ctx->get<uint64_t>("fe_nk", F), *nv = ctx->get<uint64_t>("fe_nv", F), *no = ctx->get<uint64_t>("fe_no", F);
    uint64_t *ko = ctx->get<uint64_t>("fe_ko", F + 1), *vo = ctx->get<uint64_t>("fe_vo", F + 1), *oo = ctx->get<uint64_t>("fe_oo", F + 1);
    uint64_t *vb = ctx->get<uint64_t>("fe_vb", F), *kb = ctx->get<uint64_t>("fe_kb", F);
    uint64_t *vbo = ctx->get<uint64_t>("fe_vbo", F + 1), *kbo = ctx->get<uint64_t>("fe_kbo", F + 1);
    uint64_t *kmin = ctx->get<uint64_t>("fe_kmin", W), *kmax = ctx->get<uint64_t>("fe_kmax", W);
    uint32_t *cmax = ctx->get<uint32_t>("fe_cmax", W);
    ACC_HIP(hipMemsetAsync(kmin, 0xFF, 8 * W, st));
    ACC_HIP(hipMemsetAsync(kmax, 0, 8 * W, st));
    ACC_HIP(hipMemsetAsync(cmax, 0, 4 * W, st));
    if (F) {
        launch(ctx, "fe_sizes", k_fe_sizes, dim3(grid_for(F, BLOCK)), dim3(BLOCK), 0, F, hdr, nk, nv, no);
        const uint64_t *si[3] = { nk, nv, no };
        uint64_t *so[3] = { ko, vo, oo }, *stot[3] = { ko + F, vo + F, oo + F };
        const size_t sn[3] = { F, F, F };
        scan_multi<uint64_t, OpAdd<uint64_t>>(ctx, 3, si, so, sn, true, stot);
        uint64_t *fmin = ctx->get<uint64_t>("fe_fmin", F), *fmax = ctx->get<uint64_t>("fe_fmax", F);
        uint32_t *fcm = ctx->get<uint32_t>("fe_fcm", F);
        launch(ctx, "fe_meas", k_fe_meas, dim3((unsigned)((F + WAVES - 1) / WAVES)), dim3(BLOCK), 0, F, hdr,
               (const uint64_t *)ko, (const uint64_t *)vo, keys, vals, vb, kb, fmin, fmax, fcm);
        uint64_t *fo_d = ctx->get<uint64_t>("fe_fo", (size_t)W + 1);
        ACC_HIP(hipMemcpyAsync(fo_d, fo, 8 * ((size_t)W + 1), hipMemcpyHostToDevice, st));
        launch(ctx, "fe_dest", k_fe_dest, dim3(W * FE_DB), dim3(BLOCK), 0, (const uint64_t *)fo_d, (const uint64_t *)fmin,
               (const uint64_t *)fmax, (const uint32_t *)fcm, kmin, kmax, cmax);
        const uint64_t *si2[2] = { vb, kb };
        uint64_t *so2[2] = { vbo, kbo }, *stot2[2] = { vbo + F, kbo + F };
        const size_t sn2[2] = { F, F };
        scan_multi<uint64_t, OpAdd<uint64_t>>(ctx, 2, si2, so2, sn2, true, stot2);
    } else {
        ACC_HIP(hipMemsetAsync(vbo, 0, 8, st));
        ACC_HIP(hipMemsetAsync(kbo, 0, 8, st));
    }
    // per destination: prefix values at its first fragment, key span, largest count -> host
    std::vector<uint64_t> h(4 * ((size_t)W + 1) + 3 * (size_t)W);
    uint64_t *dv = ctx->get<uint64_t>("fe_bounds", h.size());
    for (uint32_t d = 0; d <= W; ++d) {
        ACC_HIP(hipMemcpyAsync(dv + d, vbo + fo[d], 8, hipMemcpyDeviceToDevice, st));
        ACC_HIP(hipMemcpyAsync(dv + (W + 1) + d, kbo + fo[d], 8, hipMemcpyDeviceToDevice, st));
    }
    ACC_HIP(hipMemcpyAsync(h.data(), dv, 2 * (W + 1) * 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(h.data() + 4 * (W + 1), kmin, 8 * W, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(h.data() + 4 * (W + 1) + W, kmax, 8 * W, hipMemcpyDeviceToHost, st));
    std::vector<uint32_t> hc(W);
    ACC_HIP(hipMemcpyAsync(hc.data(), cmax, 4 * W, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t *hvb = h.data(), *hkb = h.data() + (W + 1), *hmin = h.data() + 4 * (W + 1), *hmax = hmin + W;
    std::vector<Msg> msg(W);
    boff.assign(W + 1, 0);
    std::vector<uint32_t> head((size_t)W * HDR_WORDS, 0);
    for (uint32_t d = 0; d < W; ++d) {
        Msg &m = msg[d];
        m.nfrag = (uint32_t)(fo[d + 1] - fo[d]);
        m.G = G;
        m.f0 = fo[d]; m.k0 = ko_h[d]; m.vb0 = hvb[d]; m.kb0 = hkb[d];
        const uint64_t NKd = ko_h[d + 1] - ko_h[d];
        const uint64_t bitmap = 4ull * ((G + 31) / 32), list = 4ull * m.nfrag;
        m.flags = (list < bitmap ? F_SLOT_LIST : 0u) | (hc[d] > 0xFFFFu ? F_WIDE_CNT : 0u) |
                  (NKd && hmax[d] - hmin[d] > 0xFFFFFFFFull ? F_WIDE_KEY : 0u);
        m.kbase = NKd ? hmin[d] : 0;
        m.base = boff[d];
        uint64_t o = HDR_WORDS * 4;
        m.slot = o; o = al8(o + (m.nfrag ? ((m.flags & F_SLOT_LIST) ? list : bitmap) : 0));
        m.cnt = o; o = al8(o + (uint64_t)m.nfrag * ((m.flags & F_WIDE_CNT) ? 12 : 6));
        m.key = o; o = al8(o + NKd * ((m.flags & F_WIDE_KEY) ? 8 : 4));
        m.val = o; o = al8(o + (hvb[d + 1] - hvb[d]));
        m.kbm = o; o = al8(o + (hkb[d + 1] - hkb[d]));
        m.end = o;
        boff[d + 1] = boff[d] + o;
        uint32_t *hw = head.data() + (size_t)d * HDR_WORDS;
        const uint64_t sz[5] = { m.cnt - m.slot, m.key - m.cnt, m.val - m.key, m.kbm - m.val, m.end - m.kbm };
        hw[0] = MAGIC; hw[1] = m.flags; hw[2] = m.nfrag; hw[3] = G;
        hw[4] = (uint32_t)m.kbase; hw[5] = (uint32_t)(m.kbase >> 32);
        for (int q = 0; q < 5; ++q) { hw[6 + 2 * q] = (uint32_t)sz[q]; hw[7 + 2 * q] = (uint32_t)(sz[q] >> 32); }
    }
    uint8_t *buf = ctx->get<uint8_t>("fe_buf", boff[W]);
    ACC_HIP(hipMemsetAsync(buf, 0, boff[W], st));
    Msg *dm = ctx->get<Msg>("fe_msg", W);
    ACC_HIP(hipMemcpyAsync(dm, msg.data(), W * sizeof(Msg), hipMemcpyHostToDevice, st));
    for (uint32_t d = 0; d < W; ++d)
        ACC_HIP(hipMemcpyAsync(buf + boff[d], head.data() + (size_t)d * HDR_WORDS, HDR_WORDS * 4, hipMemcpyHostToDevice, st));
    if (F)
        launch(ctx, "fe_write", k_fe_write, dim3((unsigned)((F + WAVES - 1) / WAVES)), dim3(BLOCK), 0, F, W,
               (const Msg *)dm, hdr, (const uint64_t *)ko, (const uint64_t *)vo, (const uint64_t *)oo, keys, vals, k2v,
               (const uint64_t *)vbo, (const uint64_t *)kbo, buf);
    // (the host vectors the copies read stay alive until the stream drains)
    ctx->sync();
    uint64_t raw = 16 * F + 8 * ko_h[W] + 4 * vo_h[W] + 4 * oo_h[W];
    ctx->stat("exchange.frag_raw_bytes", raw);
    ctx->stat("exchange.frag_wire_bytes", boff[W]);
    return buf;
}

// Decode the messages received from every source (recv: source-major, nb[s] bytes from source s) into acc_shard_pack's
// four streams in source order (device, owned by ctx) and fill `fr` (its count arrays point into cnt[4]).
void frag_decode(acc_ctx *ctx, uint32_t W, uint32_t rank, uint32_t n_global, const uint8_t *recv,
                 const std::vector<uint64_t> &nb, acc_frag_recv &fr, std::vector<uint64_t> cnt[4])
{
    hipStream_t st = ctx->stream;
    std::vector<uint64_t> rb(W + 1, 0);
    for (uint32_t s = 0; s < W; ++s) rb[s + 1] = rb[s] + nb[s];
    if ((size_t)W * HDR_WORDS * 4 > (acc_ctx::PINNED_SLOTS) * 8) fail(ACC_E_CAP, "world too large for the header read-back");
    uint32_t *ph = reinterpret_cast<uint32_t *>(ctx->pinned);
    for (uint32_t s = 0; s < W; ++s) {
        if (nb[s] < HDR_WORDS * 4) fail(ACC_E_STATE, "fragment message shorter than its header");
        ACC_HIP(hipMemcpyAsync(ph + (size_t)s * HDR_WORDS, recv + rb[s], HDR_WORDS * 4, hipMemcpyDeviceToHost, st));
    }
    ctx->sync();
    std::vector<Msg> msg(W);
    uint64_t F = 0, NW = 0;
    for (uint32_t s = 0; s < W; ++s) {
        const uint32_t *hw = ph + (size_t)s * HDR_WORDS;
        if (hw[0] != MAGIC) fail(ACC_E_STATE, "not a fragment message");
        Msg &m = msg[s];
        m.flags = hw[1]; m.nfrag = hw[2]; m.G = hw[3];
        m.kbase = hw[4] | ((uint64_t)hw[5] << 32);
        uint64_t sz[5];
        for (int q = 0; q < 5; ++q) sz[q] = hw[6 + 2 * q] | ((uint64_t)hw[7 + 2 * q] << 32);
        m.base = rb[s];
        m.slot = HDR_WORDS * 4; m.cnt = m.slot + sz[0]; m.key = m.cnt + sz[1]; m.val = m.key + sz[2]; m.kbm = m.val + sz[3];
        m.end = m.kbm + sz[4];
        if (m.end != nb[s]) fail(ACC_E_STATE, "fragment message size does not match its header");
        m.f0 = F;
        m.w0 = NW;
        F += m.nfrag;
        if (!(m.flags & F_SLOT_LIST) && m.nfrag) NW += (m.G + 31) / 32;
    }
    for (uint32_t s = 0; s < W; ++s) {   // (bitmap words of a message without fragments are not read)
        Msg &m = msg[s];
        if ((m.flags & F_SLOT_LIST) || !m.nfrag) m.w0 = s + 1 < W ? msg[s + 1].w0 : NW;
    }
    Msg *dm = ctx->get<Msg>("fd_msg", W);
    ACC_HIP(hipMemcpyAsync(dm, msg.data(), W * sizeof(Msg), hipMemcpyHostToDevice, st));
    uint32_t *hdr = ctx->get<uint32_t>("fd_hdr", 4 * F);
    uint64_t *err = ctx->get<uint64_t>("fd_err", 1);
    ACC_HIP(hipMemsetAsync(err, 0, 8, st));
    if (NW) {
        uint32_t *pc = ctx->get<uint32_t>("fd_pc", NW), *pco = ctx->get<uint32_t>("fd_pco", NW + 1);
        launch(ctx, "fd_popc", k_fd_popc, dim3(grid_for(NW, BLOCK)), dim3(BLOCK), 0, NW, W, (const Msg *)dm, recv, pc);
        scan<uint32_t, OpAdd<uint32_t>>(ctx, pc, pco, NW, true, pco + NW);
        launch(ctx, "fd_bits", k_fd_bits, dim3(grid_for(NW, BLOCK)), dim3(BLOCK), 0, NW, W, rank, (const Msg *)dm, recv,
               (const uint32_t *)pco, hdr, err);
    }
    uint64_t *a[5], *o[5];
    const char *an[5] = { "fd_nk", "fd_nv", "fd_vb", "fd_kb", "fd_no" }, *on[5] = { "fd_sk", "fd_sv", "fd_svb", "fd_skb", "fd_so" };
    for (int q = 0; q < 5; ++q) { a[q] = ctx->get<uint64_t>(an[q], F); o[q] = ctx->get<uint64_t>(on[q], F + 1); }
    if (F) {
        launch(ctx, "fd_counts", k_fd_counts, dim3(grid_for(F, BLOCK)), dim3(BLOCK), 0, F, W, rank, (const Msg *)dm, recv,
               hdr, a[0], a[1], a[2], a[3]);
        const uint64_t *si[4] = { a[0], a[1], a[2], a[3] };
        uint64_t *so[4] = { o[0], o[1], o[2], o[3] }, *stot[4] = { o[0] + F, o[1] + F, o[2] + F, o[3] + F };
        const size_t sn[4] = { F, F, F, F };
        scan_multi<uint64_t, OpAdd<uint64_t>>(ctx, 4, si, so, sn, true, stot);
        launch(ctx, "fd_no", k_fd_no, dim3((unsigned)((F + WAVES - 1) / WAVES)), dim3(BLOCK), 0, F, W, (const Msg *)dm,
               recv, hdr, (const uint64_t *)o[3], a[4]);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, a[4], o[4], F, true, o[4] + F);
    } else {
        for (int q = 0; q < 5; ++q) ACC_HIP(hipMemsetAsync(o[q], 0, 8, st));
    }
    // per-source totals (prefix values at the sources' first fragments) -> host; every message's own bases into the table
    std::vector<uint64_t> hb(5 * ((size_t)W + 1));
    uint64_t *bd = ctx->get<uint64_t>("fd_bounds", hb.size());
    for (int q = 0; q < 5; ++q)
        for (uint32_t s = 0; s <= W; ++s)
            ACC_HIP(hipMemcpyAsync(bd + q * (W + 1) + s, o[q] + (s < W ? msg[s].f0 : F), 8, hipMemcpyDeviceToDevice, st));
    ACC_HIP(hipMemcpyAsync(hb.data(), bd, hb.size() * 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned, err, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    if (ctx->pinned[0]) fail(ACC_E_STATE, "malformed fragment message");
    for (int q = 0; q < 4; ++q) cnt[q].assign(W, 0);
    const int qi[4] = { -1, 0, 1, 4 };   // frag, keys, vals, k2v
    for (uint32_t s = 0; s < W; ++s) {
        cnt[0][s] = msg[s].nfrag;
        for (int q = 1; q < 4; ++q) cnt[q][s] = hb[qi[q] * (W + 1) + s + 1] - hb[qi[q] * (W + 1) + s];
    }
    const uint64_t NK = hb[W], NV = hb[(W + 1) + W], NO = hb[4 * (W + 1) + W];
    uint64_t *keys = ctx->get<uint64_t>("fd_keys", NK);
    uint32_t *vals = ctx->get<uint32_t>("fd_vals", NV);
    int32_t *k2v = ctx->get<int32_t>("fd_k2v", NO);
    if (F)
        launch(ctx, "fd_unpack", k_fd_unpack, dim3((unsigned)((F + WAVES - 1) / WAVES)), dim3(BLOCK), 0, F, W,
               (const Msg *)dm, recv, (const uint32_t *)hdr, (const uint64_t *)o[0], (const uint64_t *)o[1],
               (const uint64_t *)o[2], (const uint64_t *)o[3], (const uint64_t *)o[4], keys, vals, k2v, err);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, err, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    if (ctx->pinned[0]) fail(ACC_E_STATE, "malformed fragment message");
    fr = acc_frag_recv{ ACC_MEM_DEVICE, W, rank, n_global, cnt[0].data(), cnt[1].data(), cnt[2].data(), cnt[3].data(),
                        hdr, keys, vals, k2v };
}

}  // namespace acc
