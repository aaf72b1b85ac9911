// wire.hip — Deps wire format <-> device: the Maelstrom JSON of Deps
// (accord-maelstrom Json.DEPS_ADAPTER, mael/Json.java:316-398) parsed and written on device.
//
// Ingest (acc_deps_from_json): a batch of JSON documents in one buffer, one thread per document (two passes over its
// bytes: count, then emit) -> per entry a Datum (MaelstromKey, mael/Datum.java) and a TxnId (Json.TXNID_ADAPTER :153-166:
// [msb, lsb, node], node = null | "n<id>" | "c<id>", Json.parseId :80-90). Datum order (Datum.compareTo :172-186,
// COMPARE_BY_HASH): hash(value) (CRC32 of value.hashCode(), :188-200; a Hash's own hash; null = Integer.MAX_VALUE), then
// Kind, then null last, then the value; the batch's datums are dense-ranked in that order (dictionary.hip), so key codes
// are exact order-preserving codes. Each document's entries then go through the KeyDeps / RangeDeps Builder
// (Json.java:356-392): every entry a one-key reply, the document's replies merged by the batched Deps.merge
// (depsmerge.hip), which equals AbstractBuilder.build here (sorted unique keys and TxnIds, first instance kept).
// Egress (acc_deps_to_json): the inverse, one thread per deps object, two passes (sizes, bytes) over the Java
// iteration order (keys ascending, then each key's TxnIds), Gson's compact form.
// Datum kinds on this path: LONG (integer literals) and HASH; STRING and DOUBLE datums are rejected with ACC_E_ARG.
#include "dict.hpp"

namespace acc {

void deps_merge(acc_ctx *ctx, const acc_deps_merge_in *in, acc_deps_merge_view *view);

namespace wire {

enum : uint32_t { K_STRING = 0, K_LONG = 1, K_DOUBLE = 2, K_HASH = 3 };   // Datum.Kind ordinals (Datum.java:69)
enum : uint64_t {
    E_SYNTAX = 1, E_KIND = 2, E_FIELD = 4, E_NULL_TXN = 8, E_NODE = 16, E_DUP = 32, E_RANGE = 64, E_UNSUPPORTED = 128,
};

struct Datum { uint32_t kind, null; uint64_t value; int32_t hash; };

// java.util.zip.CRC32 over the low bytes of i, i >> 8, i >> 16, i >> 24 (Datum.hash, Datum.java:188-200)
__device__ __forceinline__ int32_t crc32_int(int32_t i)
{
    uint32_t c = 0xFFFFFFFFu;
    for (int b = 0; b < 4; ++b) {
        c ^= (uint32_t)(i >> (8 * b)) & 0xFFu;
#pragma unroll
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    }
    return (int32_t)(c ^ 0xFFFFFFFFu);
}

__device__ __forceinline__ int32_t datum_hash(const Datum &d)
{
    if (d.null) return 0x7FFFFFFF;                                  // hash(null) = Integer.MAX_VALUE
    if (d.kind == K_HASH) return (int32_t)(uint32_t)d.value;         // Hash.hash
    const uint64_t v = d.value;                                      // Long.hashCode
    return crc32_int((int32_t)(uint32_t)(v ^ (v >> 32)));
}

struct Cur {
    const uint8_t *p;
    uint64_t i, n;
    uint64_t err;
    __device__ void ws() { while (i < n && (p[i] == ' ' || p[i] == '\n' || p[i] == '\r' || p[i] == '\t')) ++i; }
    __device__ int peek() { ws(); return i < n ? p[i] : -1; }
    __device__ bool eat(uint8_t c) { if (peek() == c) { ++i; return true; } return false; }
    __device__ void expect(uint8_t c) { if (!eat(c)) err |= E_SYNTAX; }
    // a JSON integer literal (JsonReader.nextLong on an integral token); fractions / exponents are not accepted here
    __device__ int64_t integer()
    {
        ws();
        bool neg = false;
        if (i < n && p[i] == '-') { neg = true; ++i; }
        uint64_t v = 0;
        uint64_t d0 = i;
        while (i < n && p[i] >= '0' && p[i] <= '9') {
            const uint64_t nv = v * 10 + (p[i] - '0');
            if (nv / 10 != v) err |= E_SYNTAX;
            v = nv;
            ++i;
        }
        if (i == d0) err |= E_SYNTAX;
        if (i < n && (p[i] == '.' || p[i] == 'e' || p[i] == 'E')) err |= E_UNSUPPORTED;   // DOUBLE datums
        if (v > (neg ? (1ull << 63) : (1ull << 63) - 1)) err |= E_SYNTAX;
        return neg ? (int64_t)(0 - v) : (int64_t)v;
    }
    // a string's [begin, end) (no escapes in this format)
    __device__ void str(uint64_t &b, uint64_t &e)
    {
        b = e = i;
        if (peek() != '"') { err |= E_SYNTAX; return; }
        ++i;
        b = i;
        while (i < n && p[i] != '"') { if (p[i] == '\\') err |= E_UNSUPPORTED; ++i; }
        e = i;
        if (i < n) ++i; else err |= E_SYNTAX;
    }
    __device__ bool str_is(uint64_t b, uint64_t e, const char *lit)
    {
        uint64_t k = 0;
        for (; lit[k]; ++k) if (b + k >= e || p[b + k] != (uint8_t)lit[k]) return false;
        return b + k == e;
    }
    __device__ bool word(const char *lit)
    {
        ws();
        uint64_t k = 0;
        for (; lit[k]; ++k) if (i + k >= n || p[i + k] != (uint8_t)lit[k]) return false;
        i += k;
        return true;
    }
};

// Datum.read (Datum.java:229-255)
__device__ Datum read_datum(Cur &c)
{
    Datum d{ K_LONG, 0, 0, 0 };
    const int t = c.peek();
    if (t == '[') {
        ++c.i;
        uint64_t b, e;
        c.str(b, e);
        if (c.str_is(b, e, "HASH")) d.kind = K_HASH;
        else if (c.str_is(b, e, "LONG")) d.kind = K_LONG;
        else if (c.str_is(b, e, "DOUBLE")) d.kind = K_DOUBLE;
        else if (c.str_is(b, e, "STRING")) d.kind = K_STRING;
        else c.err |= E_KIND;
        d.null = 1;
        if (d.kind == K_HASH) {
            c.expect(',');
            if (c.word("true")) { c.expect(','); d.value = (uint64_t)(uint32_t)(int32_t)c.integer(); d.null = 0; }
            else if (!c.word("false")) c.err |= E_SYNTAX;
        }
        c.expect(']');
    } else if (t == '"') {
        c.err |= E_UNSUPPORTED;   // STRING datum
        uint64_t b, e;
        c.str(b, e);
    } else {
        d.value = (uint64_t)c.integer();
    }
    d.hash = datum_hash(d);
    return d;
}

struct Txn { uint64_t msb, lsb; int32_t node; };

// Json.readTimestamp (:124-137) with ID_ADAPTER (:58-78) / parseId (:80-90)
__device__ Txn read_txn(Cur &c)
{
    Txn t{ 0, 0, 0 };
    if (c.word("null")) { c.err |= E_NULL_TXN; return t; }
    c.expect('[');
    t.msb = (uint64_t)c.integer();
    c.expect(',');
    t.lsb = (uint64_t)c.integer();
    c.expect(',');
    if (!c.word("null")) {
        uint64_t b, e;
        c.str(b, e);
        if (e - b < 2 || (c.p[b] != 'n' && c.p[b] != 'c')) c.err |= E_NODE;
        Cur s{ c.p, b + 1, e, 0 };
        t.node = (int32_t)s.integer();
        if (s.err || s.i != e) c.err |= E_NODE;
    }
    c.expect(']');
    return t;
}

struct Out {   // emit pass targets (global entry / datum slots)
    Datum *kd;          // key entries' datums
    Txn *kt;            // key entries' TxnIds
    Datum *rs, *re;     // range entries' start / end datums
    Txn *rt;
};

// one document: {"keyDeps":[[datum, txnId], ...], "rangeDeps":[[start, end, txnId], ...]} (either field optional)
template <bool EMIT>
__device__ uint64_t parse_doc(const uint8_t *p, uint64_t b, uint64_t e, uint32_t &nk, uint32_t &nr, const Out &o,
                              uint64_t kbase, uint64_t rbase)
{
    Cur c{ p, b, e, 0 };
    nk = nr = 0;
    bool seen_k = false, seen_r = false;
    c.expect('{');
    if (!c.eat('}')) {
        while (!c.err) {
            uint64_t nb, ne;
            c.str(nb, ne);
            c.expect(':');
            const bool isk = c.str_is(nb, ne, "keyDeps"), isr = c.str_is(nb, ne, "rangeDeps");
            if (!isk && !isr) { c.err |= E_FIELD; break; }   // "Unknown name" (AssertionError)
            if ((isk && seen_k) || (isr && seen_r)) { c.err |= E_DUP; break; }
            seen_k |= isk; seen_r |= isr;
            c.expect('[');
            if (!c.eat(']')) {
                while (!c.err) {
                    c.expect('[');
                    const Datum d0 = read_datum(c);
                    c.expect(',');
                    Datum d1{};
                    if (isr) { d1 = read_datum(c); c.expect(','); }
                    const Txn t = read_txn(c);
                    c.expect(']');
                    if (EMIT && !c.err) {
                        if (isk) { o.kd[kbase + nk] = d0; o.kt[kbase + nk] = t; }
                        else { o.rs[rbase + nr] = d0; o.re[rbase + nr] = d1; o.rt[rbase + nr] = t; }
                    }
                    if (isk) ++nk; else ++nr;
                    if (!c.eat(',')) break;
                }
                c.expect(']');
            }
            if (!c.eat(',')) break;
        }
        c.expect('}');
    }
    if (c.peek() != -1) c.err |= E_SYNTAX;   // trailing bytes
    return c.err;
}

}  // namespace wire

using namespace wire;

__global__ __launch_bounds__(BLOCK) void k_json_count(uint32_t nd, const uint8_t *__restrict__ bytes, const uint64_t *__restrict__ doc_off,
                                                      uint64_t *__restrict__ nk, uint64_t *__restrict__ nr, uint64_t *__restrict__ nrep,
                                                      uint64_t *__restrict__ errs)
{
    const uint32_t d = blockIdx.x * BLOCK + threadIdx.x;
    if (d >= nd) return;
    uint32_t a = 0, r = 0;
    const uint64_t e = parse_doc<false>(bytes, doc_off[d], doc_off[d + 1], a, r, Out{}, 0, 0);
    nk[d] = a; nr[d] = r; nrep[d] = a > r ? a : r;
    if (e) atomicOr((unsigned long long *)errs, (unsigned long long)e);
}

__global__ __launch_bounds__(BLOCK) void k_json_emit(uint32_t nd, const uint8_t *__restrict__ bytes, const uint64_t *__restrict__ doc_off,
                                                     const uint64_t *__restrict__ kb, const uint64_t *__restrict__ rb, Out o)
{
    const uint32_t d = blockIdx.x * BLOCK + threadIdx.x;
    if (d >= nd) return;
    uint32_t a, r;
    parse_doc<true>(bytes, doc_off[d], doc_off[d + 1], a, r, o, kb[d], rb[d]);
}

// Datum.compareTo as two u64 words: (hash ^ sign, kind, null last), then the value (LONG signed order; HASH = hash)
__global__ __launch_bounds__(BLOCK) void k_json_words(uint64_t n, const Datum *__restrict__ dat, uint64_t *__restrict__ w0,
                                                      uint64_t *__restrict__ w1)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const Datum d = dat[i];
    w0[i] = ((uint64_t)((uint32_t)d.hash ^ 0x80000000u) << 32) | ((uint64_t)d.kind << 1) | d.null;
    w1[i] = d.null ? 0ull : (d.kind == K_LONG ? d.value ^ (1ull << 63) : d.value);
}

struct Sing {   // per-reply singleton layout (reply r of document d = key entry q and / or range entry q)
    const uint64_t *rep_off, *kb, *rb, *nk, *nr;
    uint32_t nd;
};

__global__ __launch_bounds__(BLOCK) void k_json_reply_offs(uint64_t R, Sing s, uint64_t *__restrict__ koff, uint64_t *__restrict__ roff)
{
    const uint64_t r = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (r > R) return;
    if (r == R) { koff[r] = s.kb[s.nd]; roff[r] = s.rb[s.nd]; return; }
    uint32_t lo = 0, hi = s.nd;   // document d: rep_off[d] <= r < rep_off[d + 1]
    while (hi - lo > 1) { const uint32_t m = (lo + hi) >> 1; if (s.rep_off[m] <= r) lo = m; else hi = m; }
    const uint64_t q = r - s.rep_off[lo];
    koff[r] = s.kb[lo] + min(q, s.nk[lo]);
    roff[r] = s.rb[lo] + min(q, s.nr[lo]);
}

// singleton halves: entry i = one key (its datum rank), one TxnId, keysToTxnIds [2, 0]
__global__ __launch_bounds__(BLOCK) void k_json_singletons(uint64_t NK, uint64_t NR, const uint32_t *__restrict__ rank,
                                                           const Txn *__restrict__ kt, const Txn *__restrict__ rt,
                                                           uint64_t *__restrict__ kkey, uint64_t *__restrict__ km,
                                                           uint64_t *__restrict__ kl, int32_t *__restrict__ kn, int32_t *__restrict__ kk2v,
                                                           uint64_t *__restrict__ rka, uint64_t *__restrict__ rkb,
                                                           uint64_t *__restrict__ rm, uint64_t *__restrict__ rl, int32_t *__restrict__ rn,
                                                           int32_t *__restrict__ rk2v)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < NK) {
        kkey[i] = rank[i];
        const Txn t = kt[i];
        km[i] = t.msb; kl[i] = t.lsb; kn[i] = t.node;
        kk2v[2 * i] = 2; kk2v[2 * i + 1] = 0;
    }
    if (i < NR) {
        rka[i] = rank[NK + i];
        rkb[i] = rank[NK + NR + i];
        const Txn t = rt[i];
        rm[i] = t.msb; rl[i] = t.lsb; rn[i] = t.node;
        rk2v[2 * i] = 2; rk2v[2 * i + 1] = 0;
    }
}

__global__ __launch_bounds__(BLOCK) void k_json_double(uint64_t *__restrict__ a, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) a[i] *= 2;
}

__global__ __launch_bounds__(BLOCK) void k_json_dict(uint64_t nranks, const uint32_t *__restrict__ first, const Datum *__restrict__ dat,
                                                     uint8_t *__restrict__ kind, uint8_t *__restrict__ nul, uint64_t *__restrict__ val,
                                                     int32_t *__restrict__ hash)
{
    const uint64_t r = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (r >= nranks) return;
    const Datum d = dat[first[r]];
    kind[r] = (uint8_t)d.kind; nul[r] = (uint8_t)d.null; val[r] = d.value; hash[r] = d.hash;
}

static void check_json(uint64_t e)
{
    if (e & E_UNSUPPORTED) fail(ACC_E_ARG, "STRING / DOUBLE datums (or escaped strings) are not supported on the device JSON path");
    if (e & E_FIELD) fail(ACC_E_STATE, "Unknown name in Deps JSON (AssertionError, Json.java:392)");
    if (e & E_KIND) fail(ACC_E_ARG, "unknown Datum.Kind name (Kind.valueOf)");
    if (e & E_NULL_TXN) fail(ACC_E_ARG, "null TxnId in a Deps entry");
    if (e & E_NODE) fail(ACC_E_ARG, "malformed node id (Json.parseId)");
    if (e & E_DUP) fail(ACC_E_ARG, "keyDeps / rangeDeps given twice in one document");
    if (e & E_SYNTAX) fail(ACC_E_ARG, "malformed Deps JSON");
}

void deps_from_json(acc_ctx *ctx, const acc_json_in *in, acc_json_deps_view *view)
{
    if (!in || !view) fail(ACC_E_ARG, "null argument");
    if (in->mem != ACC_MEM_HOST && in->mem != ACC_MEM_DEVICE) fail(ACC_E_ARG, "mem must be ACC_MEM_HOST or ACC_MEM_DEVICE");
    hipStream_t st = ctx->stream;
    const uint32_t nd = in->n_docs;
    const uint64_t *doc_off = stage_in(ctx, "js_doc_off", in->doc_off, (size_t)nd + 1, in->mem);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, doc_off + nd, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t nbytes = ctx->pinned[0];
    const uint8_t *bytes = stage_in(ctx, "js_bytes", in->bytes, nbytes, in->mem);
    uint64_t *nk = ctx->get<uint64_t>("js_nk", nd), *nr = ctx->get<uint64_t>("js_nr", nd), *nrep = ctx->get<uint64_t>("js_nrep", nd);
    uint64_t *kb = ctx->get<uint64_t>("js_kb", (size_t)nd + 1), *rb = ctx->get<uint64_t>("js_rb", (size_t)nd + 1);
    uint64_t *rep_off = ctx->get<uint64_t>("js_rep_off", (size_t)nd + 1);
    uint64_t *errs = ctx->get<uint64_t>("js_errs", 1);
    ACC_HIP(hipMemsetAsync(errs, 0, 8, st));
    if (nd) launch(ctx, "json_count", k_json_count, dim3(grid_for(nd, BLOCK)), dim3(BLOCK), 0, nd, bytes, doc_off, nk, nr, nrep, errs);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, nk, kb, nd, true, kb + nd);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, nr, rb, nd, true, rb + nd);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, nrep, rep_off, nd, true, rep_off + nd);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, errs, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, kb + nd, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 2, rb + nd, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 3, rep_off + nd, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    check_json(ctx->pinned[0]);
    const uint64_t NK = ctx->pinned[1], NR = ctx->pinned[2], R = ctx->pinned[3];
    const uint64_t ND = NK + 2 * NR;
    if (ND >= 0xFFFFFFFFull) fail(ACC_E_CAP, "too many Deps entries in one JSON batch");
    Datum *dat = ctx->get<Datum>("js_datum", ND + 1);
    Txn *kt = ctx->get<Txn>("js_kt", NK + 1), *rt = ctx->get<Txn>("js_rt", NR + 1);
    Out o{ dat, kt, dat + NK, dat + NK + NR, rt };
    if (nd) launch(ctx, "json_emit", k_json_emit, dim3(grid_for(nd, BLOCK)), dim3(BLOCK), 0, nd, bytes, doc_off,
                   (const uint64_t *)kb, (const uint64_t *)rb, o);
    // ---- dense ranks of every datum in Datum.compareTo order = the batch's key codes
    uint64_t *w0 = ctx->get<uint64_t>("js_w0", ND + 1), *w1 = ctx->get<uint64_t>("js_w1", ND + 1);
    if (ND) launch(ctx, "json_words", k_json_words, dim3(grid_for(ND, BLOCK)), dim3(BLOCK), 0, ND, (const Datum *)dat, w0, w1);
    const uint64_t *words[2] = { w0, w1 };
    DenseRank dr = dense_rank(ctx, "js_dr", ND, 2, words, nullptr, nullptr, true);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, dr.count_dev, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t NDICT = ND ? ctx->pinned[0] : 0;
    uint8_t *dk = ctx->get<uint8_t>("js_dict_kind", NDICT + 1), *dn = ctx->get<uint8_t>("js_dict_null", NDICT + 1);
    uint64_t *dv = ctx->get<uint64_t>("js_dict_value", NDICT + 1);
    int32_t *dh = ctx->get<int32_t>("js_dict_hash", NDICT + 1);
    if (NDICT) launch(ctx, "json_dict", k_json_dict, dim3(grid_for(NDICT, BLOCK)), dim3(BLOCK), 0, NDICT, (const uint32_t *)dr.first,
                      (const Datum *)dat, dk, dn, dv, dh);
    // ---- the Builder: one singleton reply per entry, Deps.merge per document
    uint64_t *koff = ctx->get<uint64_t>("js_koff", R + 1), *roff = ctx->get<uint64_t>("js_roff", R + 1);
    uint64_t *kk2o = ctx->get<uint64_t>("js_kk2o", R + 1), *rk2o = ctx->get<uint64_t>("js_rk2o", R + 1);
    Sing sg{ rep_off, kb, rb, nk, nr, nd };
    launch(ctx, "json_reply_offs", k_json_reply_offs, dim3(grid_for(R + 1, BLOCK)), dim3(BLOCK), 0, R, sg, koff, roff);
    ACC_HIP(hipMemcpyAsync(kk2o, koff, (R + 1) * 8, hipMemcpyDeviceToDevice, st));
    ACC_HIP(hipMemcpyAsync(rk2o, roff, (R + 1) * 8, hipMemcpyDeviceToDevice, st));
    launch(ctx, "json_double", k_json_double, dim3(grid_for(R + 1, BLOCK)), dim3(BLOCK), 0, kk2o, R + 1);
    launch(ctx, "json_double", k_json_double, dim3(grid_for(R + 1, BLOCK)), dim3(BLOCK), 0, rk2o, R + 1);
    uint64_t *kkey = ctx->get<uint64_t>("js_kkey", NK + 1), *km = ctx->get<uint64_t>("js_km", NK + 1), *kl = ctx->get<uint64_t>("js_kl", NK + 1);
    int32_t *kn = ctx->get<int32_t>("js_kn", NK + 1), *kk2v = ctx->get<int32_t>("js_kk2v", 2 * NK + 1);
    uint64_t *rka = ctx->get<uint64_t>("js_rka", NR + 1), *rkb = ctx->get<uint64_t>("js_rkb", NR + 1);
    uint64_t *rm = ctx->get<uint64_t>("js_rm", NR + 1), *rl = ctx->get<uint64_t>("js_rl", NR + 1);
    int32_t *rn = ctx->get<int32_t>("js_rn", NR + 1), *rk2v = ctx->get<int32_t>("js_rk2v", 2 * NR + 1);
    if (NK || NR)
        launch(ctx, "json_singletons", k_json_singletons, dim3(grid_for(NK > NR ? NK : NR, BLOCK)), dim3(BLOCK), 0, NK, NR,
               (const uint32_t *)dr.rank, (const Txn *)kt, (const Txn *)rt, kkey, km, kl, kn, kk2v, rka, rkb, rm, rl, rn, rk2v);
    acc_rmm_in kh{ koff, kkey, nullptr, koff, acc_ts_cols{ km, kl, kn }, kk2o, kk2v };
    acc_rmm_in rh{ roff, rka, rkb, roff, acc_ts_cols{ rm, rl, rn }, rk2o, rk2v };
    acc_deps_merge_in dmi{ ACC_MEM_DEVICE, nd, R, rep_off, kh, rh };
    acc_deps_merge_view dv2{};
    deps_merge(ctx, &dmi, &dv2);
    ctx->stat("json.key_entries", NK);
    ctx->stat("json.range_entries", NR);
    *view = acc_json_deps_view{ nd, dv2, NDICT, dk, dn, dv, dh };
}

// ---------------------------------------------------------------- egress

namespace wire {

__device__ __forceinline__ uint32_t dec_len(int64_t v)
{
    uint64_t u = v < 0 ? 0 - (uint64_t)v : (uint64_t)v;
    uint32_t n = v < 0 ? 2 : 1;
    while (u >= 10) { u /= 10; ++n; }
    return n;
}

struct Sink {
    uint8_t *out;   // null: size only
    uint64_t n;
    __device__ void c(uint8_t x) { if (out) out[n] = x; ++n; }
    __device__ void s(const char *lit) { for (uint32_t k = 0; lit[k]; ++k) c((uint8_t)lit[k]); }
    __device__ void dec(int64_t v)
    {
        const uint32_t len = dec_len(v);
        if (out) {
            uint64_t u = v < 0 ? 0 - (uint64_t)v : (uint64_t)v;
            uint64_t q = n + len;
            do { out[--q] = (uint8_t)('0' + u % 10); u /= 10; } while (u);
            if (v < 0) out[n] = '-';
        }
        n += len;
    }
};

struct Dict { const uint8_t *kind, *null; const uint64_t *value; uint64_t n; };

// Datum.write (Datum.java:209-226); returns false for kinds this path does not write
__device__ bool write_datum(Sink &k, const Dict &d, uint64_t code)
{
    if (code >= d.n) return false;
    const uint32_t kind = d.kind[code];
    if (d.null[code]) {
        k.s(kind == K_HASH ? "[\"HASH\",false]" : kind == K_LONG ? "[\"LONG\"]" : kind == K_DOUBLE ? "[\"DOUBLE\"]" : "[\"STRING\"]");
        return true;
    }
    if (kind == K_HASH) { k.s("[\"HASH\",true,"); k.dec((int32_t)(uint32_t)d.value[code]); k.c(']'); return true; }
    if (kind == K_LONG) { k.dec((int64_t)d.value[code]); return true; }
    return false;
}

// Json.writeTimestamp (:139-151) with ID_ADAPTER.write / toString(Id) (:61-65, 92-96)
__device__ void write_txn(Sink &k, uint64_t msb, uint64_t lsb, int32_t node)
{
    k.c('['); k.dec((int64_t)msb); k.c(','); k.dec((int64_t)lsb); k.c(',');
    if (node == 0) k.s("null");
    else { k.c('"'); k.c(node < 0 ? 'c' : 'n'); k.dec(node); k.c('"'); }
    k.c(']');
}

struct Obj {   // one half of the deps objects being written
    const uint64_t *key_off, *key_a, *key_b, *val_off, *msb, *lsb, *k2v_off;
    const int32_t *node, *k2v;
};

__device__ bool write_half(Sink &k, const Obj &h, uint32_t g, const Dict &d, bool is_range)
{
    bool ok = true, first = true;
    if (!h.key_off) return true;
    const uint64_t k0 = h.key_off[g], nk = h.key_off[g + 1] - k0, v0 = h.val_off[g], o0 = h.k2v_off[g];
    uint64_t prev = nk;
    for (uint64_t i = 0; i < nk; ++i) {
        const uint64_t end = (uint64_t)h.k2v[o0 + i];
        for (uint64_t x = prev; x < end; ++x) {
            const uint64_t v = v0 + (uint64_t)h.k2v[o0 + x];
            if (!first) k.c(',');
            first = false;
            k.c('[');
            ok = ok && write_datum(k, d, h.key_a[k0 + i]);
            if (is_range) { k.c(','); ok = ok && write_datum(k, d, h.key_b[k0 + i]); }
            k.c(',');
            write_txn(k, h.msb[v], h.lsb[v], h.node[v]);
            k.c(']');
        }
        prev = end;
    }
    return ok;
}

}  // namespace wire

// Json.DEPS_ADAPTER.write (:318-344) of deps object g
__global__ __launch_bounds__(BLOCK) void k_json_write(uint32_t ng, Obj kh, Obj rh, Dict d, const uint64_t *__restrict__ off,
                                                      uint8_t *__restrict__ out, uint64_t *__restrict__ len, uint64_t *__restrict__ errs)
{
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g >= ng) return;
    Sink k{ out ? out + off[g] : nullptr, 0 };
    k.s("{\"keyDeps\":[");
    bool ok = write_half(k, kh, g, d, false);
    k.s("],\"rangeDeps\":[");
    ok = write_half(k, rh, g, d, true) && ok;
    k.s("]}");
    if (len) len[g] = k.n;
    if (!ok) atomicOr((unsigned long long *)errs, (unsigned long long)E_UNSUPPORTED);
}

void deps_to_json(acc_ctx *ctx, const acc_json_out_in *in, acc_json_out *out)
{
    if (!in || !out) fail(ACC_E_ARG, "null argument");
    hipStream_t st = ctx->stream;
    const uint32_t ng = in->n_groups;
    Obj kh{ in->key_deps.key_off, in->key_deps.key_a, nullptr, in->key_deps.val_off, in->key_deps.txn_msb,
            in->key_deps.txn_lsb, in->key_deps.k2v_off, in->key_deps.txn_node, in->key_deps.k2v };
    Obj rh{ in->range_deps.key_off, in->range_deps.key_a, in->range_deps.key_b, in->range_deps.val_off, in->range_deps.txn_msb,
            in->range_deps.txn_lsb, in->range_deps.k2v_off, in->range_deps.txn_node, in->range_deps.k2v };
    Dict d{ in->dict_kind, in->dict_null, in->dict_value, in->n_dict };
    uint64_t *len = ctx->get<uint64_t>("jw_len", ng), *off = ctx->get<uint64_t>("jw_off", (size_t)ng + 1);
    uint64_t *errs = ctx->get<uint64_t>("jw_errs", 1);
    ACC_HIP(hipMemsetAsync(errs, 0, 8, st));
    if (ng) launch(ctx, "json_size", k_json_write, dim3(grid_for(ng, BLOCK)), dim3(BLOCK), 0, ng, kh, rh, d, (const uint64_t *)nullptr,
                   (uint8_t *)nullptr, len, errs);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, len, off, ng, true, off + ng);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, errs, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, off + ng, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    if (ctx->pinned[0]) fail(ACC_E_ARG, "a key is no LONG / HASH datum of the dictionary (device JSON writer)");
    const uint64_t total = ctx->pinned[1];
    out->need_bytes = total;
    if (!out->bytes || !out->doc_off || out->cap_bytes < total)
        fail(ACC_E_CAP, "sizing call (null buffers or capacity below need_bytes); need_bytes written");
    uint8_t *dst = out->mem == ACC_MEM_DEVICE ? out->bytes : ctx->get<uint8_t>("jw_bytes", total + 1);
    if (ng) launch(ctx, "json_write", k_json_write, dim3(grid_for(ng, BLOCK)), dim3(BLOCK), 0, ng, kh, rh, d, (const uint64_t *)off,
                   dst, (uint64_t *)nullptr, errs);
    const hipMemcpyKind kind = out->mem == ACC_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    ACC_HIP(hipMemcpyAsync(out->doc_off, off, ((size_t)ng + 1) * 8, kind, st));
    if (out->mem != ACC_MEM_DEVICE && total) ACC_HIP(hipMemcpyAsync(out->bytes, dst, total, hipMemcpyDeviceToHost, st));
    ctx->sync();
}

}  // namespace acc
