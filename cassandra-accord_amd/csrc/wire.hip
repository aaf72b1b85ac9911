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
// Datum kinds: every kind (Datum.read :229-255). STRING: ASCII text, JSON escapes of ASCII characters resolved;
// ordered by hash, then String.compareTo through its first 16 bytes (ties beyond them are detected and rejected, never
// mis-ordered). Numbers as Gson reads them (JsonReader.nextLong, else nextDouble): integer literals that fit a long are
// LONG; other literals go through Double.parseDouble and are LONG when (long) d == d, else DOUBLE -- the decimal ->
// double conversion is the exactly rounded fast path (<= 19 significant digits, mantissa <= 2^53, |exponent| <= 22
// (+15)); literals outside it are rejected. DOUBLE egress is Double.toString: the shortest decimal that rounds back to
// the value, closest on ties (JDK >= 19; JDK-4511638 changed a few outputs of older JDKs), with Java's layout rules.
#include "dict.hpp"

namespace acc {

void deps_merge(acc_ctx *ctx, const acc_deps_merge_in *in, acc_deps_merge_view *view);

namespace wire {

enum : uint32_t { K_STRING = 0, K_LONG = 1, K_DOUBLE = 2, K_HASH = 3 };   // Datum.Kind ordinals (Datum.java:69)
enum : uint64_t {
    E_SYNTAX = 1, E_KIND = 2, E_FIELD = 4, E_NULL_TXN = 8, E_NODE = 16, E_DUP = 32, E_RANGE = 64, E_UNSUPPORTED = 128,
    E_OFF = 256,
};

// value: LONG the long; HASH the hash (u32); DOUBLE Double.doubleToLongBits; STRING byte offset of the unescaped text in
// the batch's string pool, len its length
struct Datum { uint32_t kind, null; uint64_t value; int32_t hash; uint32_t len; };

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

// String.hashCode of ASCII text (one UTF-16 unit per byte)
__device__ __forceinline__ int32_t string_hash(const uint8_t *p, uint32_t n)
{
    uint32_t h = 0;
    for (uint32_t i = 0; i < n; ++i) h = 31u * h + p[i];
    return (int32_t)h;
}

__device__ __forceinline__ int32_t datum_hash(const Datum &d, const uint8_t *pool)
{
    if (d.null) return 0x7FFFFFFF;                                  // hash(null) = Integer.MAX_VALUE
    if (d.kind == K_HASH) return (int32_t)(uint32_t)d.value;         // Hash.hash
    if (d.kind == K_STRING) return crc32_int(string_hash(pool + d.value, d.len));
    const uint64_t v = d.value;                                      // Long.hashCode / Double.hashCode (of the bits)
    return crc32_int((int32_t)(uint32_t)(v ^ (v >> 32)));
}

// exact powers of ten as doubles (10^22 is the largest exactly representable one)
__device__ __forceinline__ double pow10_exact(int e)
{
    double r = 1.0;
    for (int i = 0; i < e; ++i) r *= 10.0;   // every partial product is exact for e <= 22
    return r;
}

struct Big {
    static constexpr int L = 44;   // 1408 bits: 10^342 * 2^64 and 2^1128 * 10 both fit
    uint32_t w[L];
    __device__ void set(uint64_t v) { for (int i = 0; i < L; ++i) w[i] = 0; w[0] = (uint32_t)v; w[1] = (uint32_t)(v >> 32); }
    __device__ void mul(uint32_t m)
    {
        uint64_t c = 0;
        for (int i = 0; i < L; ++i) { const uint64_t x = (uint64_t)w[i] * m + c; w[i] = (uint32_t)x; c = x >> 32; }
    }
    __device__ void shl(int b) { while (b >= 16) { mul(1u << 16); b -= 16; } if (b) mul(1u << b); }
    __device__ void pow10(int e) { while (e >= 9) { mul(1000000000u); e -= 9; } while (e-- > 0) mul(10u); }
    __device__ void add(const Big &o)
    {
        uint64_t c = 0;
        for (int i = 0; i < L; ++i) { const uint64_t x = (uint64_t)w[i] + o.w[i] + c; w[i] = (uint32_t)x; c = x >> 32; }
    }
    __device__ void sub(const Big &o)   // this >= o
    {
        int64_t br = 0;
        for (int i = 0; i < L; ++i) {
            int64_t x = (int64_t)w[i] - o.w[i] - br;
            br = x < 0;
            w[i] = (uint32_t)(x + (br << 32));
        }
    }
    __device__ int cmp(const Big &o) const
    {
        for (int i = L - 1; i >= 0; --i) if (w[i] != o.w[i]) return w[i] < o.w[i] ? -1 : 1;
        return 0;
    }
    __device__ int bitlen() const
    {
        for (int i = L - 1; i >= 0; --i) if (w[i]) return 32 * i + 32 - __builtin_clz(w[i]);
        return 0;
    }
    __device__ void shr1()
    {
        for (int i = 0; i < L; ++i) w[i] = (w[i] >> 1) | (i + 1 < L ? w[i + 1] << 31 : 0u);
    }
    __device__ bool zero() const { for (int i = 0; i < L; ++i) if (w[i]) return false; return true; }
    __device__ uint64_t low64() const { return (uint64_t)w[0] | ((uint64_t)w[1] << 32); }
    // this >> s (s < 64 * ... ) keeping the low 64 bits, and whether any shifted-out bit was set
    __device__ uint64_t shr64(int sh, bool &sticky) const
    {
        sticky = false;
        for (int b = 0; b < sh; ++b) if ((w[b >> 5] >> (b & 31)) & 1u) { sticky = true; break; }
        uint64_t r = 0;
        for (int b = 0; b < 64; ++b) {
            const int x = sh + b;
            if (x < 32 * L && ((w[x >> 5] >> (x & 31)) & 1u)) r |= 1ull << b;
        }
        return r;
    }
};

// Double.parseDouble of m * 10^e10 (m < 2^64), exactly rounded (half even), by big-integer arithmetic; false when the
// result overflows to infinity (JsonReader rejects infinities)
__device__ bool decimal_to_double(uint64_t m, int e10, bool neg, uint64_t &bits_out)
{
    const uint64_t sign = neg ? 1ull << 63 : 0ull;
    if (m == 0) { bits_out = sign; return true; }
    if (e10 > 310) return false;
    if (e10 < -343) { bits_out = sign; return true; }   // below half the smallest subnormal: rounds to zero
    Big num, den;
    num.set(m);
    den.set(1);
    if (e10 >= 0) num.pow10(e10); else den.pow10(-e10);
    // q = floor(num * 2^k / den) with bitlen(q) in [56, 57]: enough bits for any precision plus a round bit
    int k = 56 - (num.bitlen() - den.bitlen());
    if (k > 0) num.shl(k); else if (k < 0) den.shl(-k);
    uint64_t q = 0;
    Big d = den;
    d.shl(57);
    for (int i = 57; i >= 0; --i) {
        if (num.cmp(d) >= 0) { num.sub(d); q |= 1ull << i; }
        d.shr1();
    }
    const bool rem = !num.zero();
    const int bl = 64 - __builtin_clzll(q);
    const int E = bl - 1 - k;                       // v in [2^E, 2^(E+1))
    int P = E >= -1022 ? 53 : 53 - (-1022 - E);     // significant bits of the result (fewer for subnormals)
    if (P < 0) { bits_out = sign; return true; }
    const int sh = bl - P;                          // bits of q below the result's last bit
    uint64_t mant = P ? q >> sh : 0;
    const uint64_t half = 1ull << (sh - 1);
    const uint64_t low = q & ((1ull << sh) - 1);
    const bool up = low > half || (low == half && (rem || (mant & 1)));
    if (low == half && !rem && !(mant & 1)) { /* exact tie, even: down */ }
    mant += up ? 1 : 0;
    int e2 = E;
    if (E >= -1022) {
        if (mant == (1ull << 53)) { mant >>= 1; ++e2; }
        if (e2 > 1023) return false;
        bits_out = sign | ((uint64_t)(e2 + 1023) << 52) | (mant & ((1ull << 52) - 1));
    } else {
        bits_out = sign | mant;   // subnormal (a carry into 2^52 is the smallest normal, encoded the same way)
    }
    return true;
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
    // a string's raw [begin, end) (field names: no escapes)
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
    __device__ int hexv(uint8_t c) { return c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1; }
    // a string value (JsonReader.nextString): escapes resolved; ASCII only (a character >= 0x80 is rejected). Writes the
    // unescaped bytes to out (when non-null) and returns their count.
    __device__ uint32_t text(uint8_t *out)
    {
        uint32_t len = 0;
        if (peek() != '"') { err |= E_SYNTAX; return 0; }
        ++i;
        while (i < n && p[i] != '"') {
            uint32_t c = p[i++];
            if (c < 0x20) { err |= E_SYNTAX; break; }
            if (c >= 0x80) { err |= E_UNSUPPORTED; break; }
            if (c == '\\') {
                if (i >= n) { err |= E_SYNTAX; break; }
                const uint32_t x = p[i++];
                switch (x) {
                case '"': case '\\': case '/': c = x; break;
                case 'b': c = 8; break;
                case 't': c = 9; break;
                case 'n': c = 10; break;
                case 'f': c = 12; break;
                case 'r': c = 13; break;
                case 'u': {
                    uint32_t v = 0;
                    for (int k = 0; k < 4; ++k) {
                        const int h = i < n ? hexv(p[i]) : -1;
                        if (h < 0) { err |= E_SYNTAX; break; }
                        v = v * 16 + (uint32_t)h;
                        ++i;
                    }
                    if (v >= 0x80) err |= E_UNSUPPORTED;
                    c = v;
                    break;
                }
                default: err |= E_SYNTAX;
                }
            }
            if (out) out[len] = (uint8_t)c;
            ++len;
        }
        if (i < n) ++i; else err |= E_SYNTAX;
        return len;
    }
    // a JSON number as Gson's Datum.read takes it: nextLong, else nextDouble (JsonReader.peekNumber / nextLong)
    __device__ void number(Datum &d)
    {
        ws();
        const uint64_t b = i;
        bool neg = false;
        if (i < n && p[i] == '-') { neg = true; ++i; }
        uint64_t m = 0;
        int nd = 0, e10 = 0, nint = 0;
        bool inexact = false, frac = false, expo = false;
        auto digit = [&](uint32_t dg, bool fractional) {
            if (m == 0 && dg == 0) { if (fractional) --e10; return; }   // leading zeros carry no digits
            if (nd < 19) { m = m * 10 + dg; ++nd; if (fractional) --e10; }
            else { if (dg) inexact = true; if (!fractional) ++e10; }
        };
        const uint64_t i0 = i;
        while (i < n && p[i] >= '0' && p[i] <= '9') { digit(p[i] - '0', false); ++i; ++nint; }
        if (nint == 0 || (nint > 1 && p[i0] == '0')) err |= E_SYNTAX;   // JSON: no empty or leading-zero integer part
        if (i < n && p[i] == '.') {
            frac = true;
            ++i;
            const uint64_t f0 = i;
            while (i < n && p[i] >= '0' && p[i] <= '9') { digit(p[i] - '0', true); ++i; }
            if (i == f0) err |= E_SYNTAX;
        }
        if (i < n && (p[i] == 'e' || p[i] == 'E')) {
            expo = true;
            ++i;
            bool eneg = false;
            if (i < n && (p[i] == '+' || p[i] == '-')) { eneg = p[i] == '-'; ++i; }
            int ev = 0;
            const uint64_t x0 = i;
            while (i < n && p[i] >= '0' && p[i] <= '9') { if (ev < 100000) ev = ev * 10 + (p[i] - '0'); ++i; }
            if (i == x0) err |= E_SYNTAX;
            e10 += eneg ? -ev : ev;
        }
        d.null = 0;
        if (!frac && !expo && !(neg && m == 0)) {
            // PEEKED_LONG: an integer literal that fits a long is read exactly
            Cur c2{ p, b, i, 0 };
            const int64_t v = c2.integer();
            if (!c2.err) { d.kind = K_LONG; d.value = (uint64_t)v; return; }
        }
        // PEEKED_NUMBER: Double.parseDouble (exactly rounded fast path only), then (long) d == d -> LONG
        while (m && m % 10 == 0) { m /= 10; ++e10; }
        double v;
        if (inexact) { err |= E_UNSUPPORTED; return; }   // > 19 significant digits
        if (m == 0) v = 0.0;
        else if (m <= (1ull << 53) && e10 >= 0 && e10 <= 22) v = (double)m * pow10_exact(e10);   // Clinger's fast path
        else if (m <= (1ull << 53) && e10 < 0 && e10 >= -22) v = (double)m / pow10_exact(-e10);
        else {
            uint64_t bits;
            if (!decimal_to_double(m, e10, false, bits)) { err |= E_SYNTAX; return; }   // an infinity (rejected by Gson)
            v = __longlong_as_double((long long)bits);
        }
        if (neg) v = -v;
        const int64_t r = v >= 9.2233720368547758e18 ? INT64_MAX : v <= -9.2233720368547758e18 ? INT64_MIN : (int64_t)v;
        if ((double)r == v) { d.kind = K_LONG; d.value = (uint64_t)r; }
        else { d.kind = K_DOUBLE; d.value = (uint64_t)__double_as_longlong(v); }
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

// Datum.read (Datum.java:229-255). STRING text goes to pool + *pool_len (pool null: count only).
__device__ Datum read_datum(Cur &c, uint8_t *pool, uint64_t &pool_len)
{
    Datum d{ K_LONG, 0, 0, 0, 0 };
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
        d.kind = K_STRING;
        d.value = pool_len;
        d.len = c.text(pool ? pool + pool_len : nullptr);
        pool_len += d.len;
    } else {
        c.number(d);
    }
    d.hash = pool || d.kind != K_STRING ? datum_hash(d, pool) : 0;
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
        const int64_t v = s.integer();
        // Integer.parseInt: a value outside int32 throws (NumberFormatException), it does not wrap
        if (s.err || s.i != e || v < INT32_MIN || v > INT32_MAX) c.err |= E_NODE;
        t.node = (int32_t)v;
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
// STRING datums' unescaped text: pool + sbase onwards (EMIT), its byte count in ns
template <bool EMIT>
__device__ uint64_t parse_doc(const uint8_t *p, uint64_t b, uint64_t e, uint32_t &nk, uint32_t &nr, const Out &o,
                              uint64_t kbase, uint64_t rbase, uint8_t *pool, uint64_t sbase, uint64_t &ns)
{
    Cur c{ p, b, e, 0 };
    nk = nr = 0;
    uint64_t pl = sbase;
    uint8_t *const wpool = EMIT ? pool : nullptr;
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
                    const Datum d0 = read_datum(c, wpool, pl);
                    c.expect(',');
                    Datum d1{};
                    if (isr) { d1 = read_datum(c, wpool, pl); c.expect(','); }
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
    ns = pl - sbase;
    return c.err;
}

}  // namespace wire

using namespace wire;

// Also validates the document offsets against the staged byte count (doc_off[0] == 0, non-decreasing, within nbytes):
// a document with bad offsets is not parsed (its bytes would lie outside the buffer) and the batch fails with E_OFF.
__global__ __launch_bounds__(BLOCK) void k_json_count(uint32_t nd, uint64_t nbytes, const uint8_t *__restrict__ bytes,
                                                      const uint64_t *__restrict__ doc_off, uint64_t *__restrict__ nk,
                                                      uint64_t *__restrict__ nr, uint64_t *__restrict__ nrep,
                                                      uint64_t *__restrict__ nstr, uint64_t *__restrict__ errs)
{
    const uint32_t d = blockIdx.x * BLOCK + threadIdx.x;
    if (d >= nd) return;
    uint32_t a = 0, r = 0;
    const uint64_t b0 = doc_off[d], b1 = doc_off[d + 1];
    if ((d == 0 && b0 != 0) || b1 < b0 || b1 > nbytes) {
        nk[d] = 0; nr[d] = 0; nrep[d] = 0; nstr[d] = 0;
        atomicOr((unsigned long long *)errs, (unsigned long long)E_OFF);
        return;
    }
    uint64_t ns = 0;
    const uint64_t e = parse_doc<false>(bytes, b0, b1, a, r, Out{}, 0, 0, nullptr, 0, ns);
    nk[d] = a; nr[d] = r; nrep[d] = a > r ? a : r; nstr[d] = ns;
    if (e) atomicOr((unsigned long long *)errs, (unsigned long long)e);
}

__global__ __launch_bounds__(BLOCK) void k_json_emit(uint32_t nd, const uint8_t *__restrict__ bytes, const uint64_t *__restrict__ doc_off,
                                                     const uint64_t *__restrict__ kb, const uint64_t *__restrict__ rb,
                                                     const uint64_t *__restrict__ sb, uint8_t *__restrict__ pool, Out o)
{
    const uint32_t d = blockIdx.x * BLOCK + threadIdx.x;
    if (d >= nd) return;
    uint32_t a, r;
    uint64_t ns;
    parse_doc<true>(bytes, doc_off[d], doc_off[d + 1], a, r, o, kb[d], rb[d], pool, sb[d], ns);
}

// bytes [b, b + 8) of a string, big-endian, zero padded (String.compareTo order of ASCII text through 8 characters)
__device__ __forceinline__ uint64_t str_word(const uint8_t *p, uint32_t len, uint32_t b)
{
    uint64_t w = 0;
    for (uint32_t k = 0; k < 8; ++k) w = (w << 8) | (b + k < len ? p[b + k] : 0u);
    return w;
}

// Datum.compareTo as three u64 words: (hash ^ sign, kind, null last), then the value: LONG signed order, HASH the hash,
// DOUBLE Double.compare order of the bits (-0.0 < 0.0), STRING its first 16 bytes (k_json_strcheck catches ties beyond)
__global__ __launch_bounds__(BLOCK) void k_json_words(uint64_t n, const Datum *__restrict__ dat, const uint8_t *__restrict__ pool,
                                                      uint64_t *__restrict__ w0, uint64_t *__restrict__ w1, uint64_t *__restrict__ w2)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const Datum d = dat[i];
    w0[i] = ((uint64_t)((uint32_t)d.hash ^ 0x80000000u) << 32) | ((uint64_t)d.kind << 1) | d.null;
    uint64_t a = 0, b = 0;
    if (!d.null) {
        if (d.kind == K_LONG) a = d.value ^ (1ull << 63);
        else if (d.kind == K_DOUBLE) a = (d.value >> 63) ? ~d.value : d.value | (1ull << 63);
        else if (d.kind == K_STRING) { a = str_word(pool + d.value, d.len, 0); b = str_word(pool + d.value, d.len, 8); }
        else a = d.value;
    }
    w1[i] = a;
    w2[i] = b;
}

// a STRING datum ranked equal to its rank's first datum must hold the same text (ties beyond the 16 ranked bytes)
__global__ __launch_bounds__(BLOCK) void k_json_strcheck(uint64_t n, const Datum *__restrict__ dat, const uint8_t *__restrict__ pool,
                                                         const uint32_t *__restrict__ rank, const uint32_t *__restrict__ first,
                                                         uint64_t *__restrict__ errs)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const Datum d = dat[i];
    if (d.kind != K_STRING || d.null) return;
    const Datum f = dat[first[rank[i]]];
    bool same = f.len == d.len;
    for (uint32_t k = 16; same && k < d.len; ++k) same = pool[f.value + k] == pool[d.value + k];
    if (!same) atomicOr((unsigned long long *)errs, (unsigned long long)E_UNSUPPORTED);
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
                                                     int32_t *__restrict__ hash, uint32_t *__restrict__ len)
{
    const uint64_t r = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (r >= nranks) return;
    const Datum d = dat[first[r]];
    kind[r] = (uint8_t)d.kind; nul[r] = (uint8_t)d.null; val[r] = d.value; hash[r] = d.hash;
    len[r] = d.kind == K_STRING && !d.null ? d.len : 0u;
}

// the dictionary's STRING texts into its own pool (value = offset there)
__global__ __launch_bounds__(BLOCK) void k_json_dict_str(uint64_t nranks, const uint32_t *__restrict__ first, const Datum *__restrict__ dat,
                                                         const uint8_t *__restrict__ pool, const uint64_t *__restrict__ soff,
                                                         const uint8_t *__restrict__ kind, uint64_t *__restrict__ val,
                                                         uint8_t *__restrict__ dpool)
{
    const uint64_t r = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (r >= nranks || kind[r] != K_STRING) return;
    const Datum d = dat[first[r]];
    val[r] = soff[r];
    for (uint32_t k = 0; k < d.len; ++k) dpool[soff[r] + k] = pool[d.value + k];
}

__global__ __launch_bounds__(BLOCK) void k_json_widen(uint64_t n, const uint32_t *__restrict__ a, uint64_t *__restrict__ b)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) b[i] = a[i];
}

static void check_json(uint64_t e)
{
    if (e & E_OFF) fail(ACC_E_ARG, "doc_off must start at 0, be non-decreasing and end at the byte count");
    if (e & E_UNSUPPORTED)
        fail(ACC_E_ARG, "a datum outside the device path: non-ASCII STRING text, or a number needing Double.parseDouble's slow path");
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
    uint64_t *nstr = ctx->get<uint64_t>("js_nstr", nd), *sb = ctx->get<uint64_t>("js_sb", (size_t)nd + 1);
    uint64_t *errs = ctx->get<uint64_t>("js_errs", 1);
    ACC_HIP(hipMemsetAsync(errs, 0, 8, st));
    if (nd) launch(ctx, "json_count", k_json_count, dim3(grid_for(nd, BLOCK)), dim3(BLOCK), 0, nd, nbytes, bytes, doc_off, nk, nr,
                   nrep, nstr, errs);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, nk, kb, nd, true, kb + nd);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, nr, rb, nd, true, rb + nd);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, nrep, rep_off, nd, true, rep_off + nd);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, nstr, sb, nd, true, sb + nd);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, errs, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, kb + nd, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 2, rb + nd, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 3, rep_off + nd, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 4, sb + nd, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    check_json(ctx->pinned[0]);
    const uint64_t NK = ctx->pinned[1], NR = ctx->pinned[2], R = ctx->pinned[3], NS = nd ? ctx->pinned[4] : 0;
    const uint64_t ND = NK + 2 * NR;
    if (ND >= 0xFFFFFFFFull) fail(ACC_E_CAP, "too many Deps entries in one JSON batch");
    Datum *dat = ctx->get<Datum>("js_datum", ND + 1);
    Txn *kt = ctx->get<Txn>("js_kt", NK + 1), *rt = ctx->get<Txn>("js_rt", NR + 1);
    uint8_t *pool = ctx->get<uint8_t>("js_pool", NS + 1);   // every STRING datum's unescaped text
    Out o{ dat, kt, dat + NK, dat + NK + NR, rt };
    if (nd) launch(ctx, "json_emit", k_json_emit, dim3(grid_for(nd, BLOCK)), dim3(BLOCK), 0, nd, bytes, doc_off,
                   (const uint64_t *)kb, (const uint64_t *)rb, (const uint64_t *)sb, pool, o);
    // ---- dense ranks of every datum in Datum.compareTo order = the batch's key codes
    uint64_t *w0 = ctx->get<uint64_t>("js_w0", ND + 1), *w1 = ctx->get<uint64_t>("js_w1", ND + 1);
    uint64_t *w2 = ctx->get<uint64_t>("js_w2", ND + 1);
    if (ND) launch(ctx, "json_words", k_json_words, dim3(grid_for(ND, BLOCK)), dim3(BLOCK), 0, ND, (const Datum *)dat,
                   (const uint8_t *)pool, w0, w1, w2);
    const uint64_t *words[3] = { w0, w1, w2 };
    DenseRank dr = dense_rank(ctx, "js_dr", ND, 3, words, nullptr, nullptr, true);
    if (ND && NS)
        launch(ctx, "json_strcheck", k_json_strcheck, dim3(grid_for(ND, BLOCK)), dim3(BLOCK), 0, ND, (const Datum *)dat,
               (const uint8_t *)pool, (const uint32_t *)dr.rank, (const uint32_t *)dr.first, errs);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, dr.count_dev, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, errs, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    if (ctx->pinned[1] & E_UNSUPPORTED)
        fail(ACC_E_ARG, "STRING datums with equal hashes and first 16 characters but different text (device ranking limit)");
    const uint64_t NDICT = ND ? ctx->pinned[0] : 0;
    uint8_t *dk = ctx->get<uint8_t>("js_dict_kind", NDICT + 1), *dn = ctx->get<uint8_t>("js_dict_null", NDICT + 1);
    uint64_t *dv = ctx->get<uint64_t>("js_dict_value", NDICT + 1);
    int32_t *dh = ctx->get<int32_t>("js_dict_hash", NDICT + 1);
    uint32_t *dl = ctx->get<uint32_t>("js_dict_len", NDICT + 1);
    uint64_t *dlen64 = ctx->get<uint64_t>("js_dict_len64", NDICT + 1), *dso = ctx->get<uint64_t>("js_dict_soff", NDICT + 1);
    if (NDICT) launch(ctx, "json_dict", k_json_dict, dim3(grid_for(NDICT, BLOCK)), dim3(BLOCK), 0, NDICT, (const uint32_t *)dr.first,
                      (const Datum *)dat, dk, dn, dv, dh, dl);
    uint8_t *dpool = nullptr;
    if (NDICT && NS) {
        launch(ctx, "json_u32_to_u64", k_json_widen, dim3(grid_for(NDICT, BLOCK)), dim3(BLOCK), 0, NDICT, (const uint32_t *)dl, dlen64);
        scan<uint64_t, OpAdd<uint64_t>>(ctx, dlen64, dso, NDICT, true, dso + NDICT);
        dpool = ctx->get<uint8_t>("js_dict_pool", NS + 1);
        launch(ctx, "json_dict_str", k_json_dict_str, dim3(grid_for(NDICT, BLOCK)), dim3(BLOCK), 0, NDICT, (const uint32_t *)dr.first,
               (const Datum *)dat, (const uint8_t *)pool, (const uint64_t *)dso, (const uint8_t *)dk, dv, dpool);
    }
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
    *view = acc_json_deps_view{ nd, dv2, NDICT, dk, dn, dv, dh, dl, dpool ? dpool : ctx->get<uint8_t>("js_dict_pool", 1) };
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

struct Dict { const uint8_t *kind, *null; const uint64_t *value; uint64_t n; const uint32_t *len; const uint8_t *str; };

// ---- Double.toString (JDK >= 19: the shortest decimal that rounds to the double, the closest one on ties, and when the
// shortest has one digit the closest of the one- and two-digit ones), exact integer arithmetic (Burger & Dybvig's
// free-format digit generation over a 1216-bit bignum)
// digits of v = f * 2^e (f > 0) into dig[], returns their count; *k10 = decimal exponent of the first digit (v = 0.d1d2.. * 10^(k10+1))
__device__ int shortest_digits(uint64_t f, int e, bool min_e, uint8_t (&dig)[20], int &k10)
{
    const bool even = (f & 1) == 0;   // round-half-even: the interval's ends round to v when f is even
    Big r, s, mp, mm;
    const bool pow2 = f == (1ull << 52);
    if (e >= 0) {
        r.set(f); r.shl(e + (pow2 ? 2 : 1));
        s.set(pow2 ? 4 : 2);
        mp.set(1); mp.shl(e + (pow2 ? 1 : 0));
        mm.set(1); mm.shl(e);
    } else if (min_e || !pow2) {
        r.set(f); r.shl(1);
        s.set(1); s.shl(1 - e);
        mp.set(1); mm.set(1);
    } else {
        r.set(f); r.shl(2);
        s.set(1); s.shl(2 - e);
        mp.set(2); mm.set(1);
    }
    // k = ceil(log10 v) estimate from the binary exponent, corrected by the fixup below
    const int bits = 64 - __builtin_clzll(f) + e;   // v in [2^(bits-1), 2^bits)
    int k = (int)ceil((bits - 1) * 0.30102999566398119521 - 1e-10);
    if (k >= 0) s.pow10(k);
    else { r.pow10(-k); mp.pow10(-k); mm.pow10(-k); }
    Big t = r;
    t.add(mp);
    const int c0 = t.cmp(s);
    if (even ? c0 >= 0 : c0 > 0) ++k;
    else { r.mul(10); mp.mul(10); mm.mul(10); }
    // r / s in [1, 10) scaled: generate
    const Big r0 = r, mp0 = mp, mm0 = mm;
    int n = 0;
    while (true) {
        uint32_t d = 0;
        while (r.cmp(s) >= 0) { r.sub(s); ++d; }
        Big rp = r;
        rp.add(mp);
        const int cl = r.cmp(mm), ch = rp.cmp(s);
        const bool tc1 = even ? cl <= 0 : cl < 0, tc2 = even ? ch >= 0 : ch > 0;
        if (!tc1 && !tc2) { dig[n++] = (uint8_t)d; r.mul(10); mp.mul(10); mm.mul(10); continue; }
        if (tc1 && !tc2) { dig[n++] = (uint8_t)d; break; }
        if (!tc1 && tc2) { dig[n++] = (uint8_t)(d + 1); break; }
        Big r2 = r;
        r2.mul(2);
        const int cr = r2.cmp(s);
        dig[n++] = (uint8_t)(cr < 0 ? d : cr > 0 ? d + 1 : ((d & 1) ? d + 1 : d));   // closest; ties to the even digit
        break;
    }
    // a digit 10 (carry) cannot occur: the generation stops inside the rounding interval
    k10 = k - 1;
    if (n == 1) {
        // the closest two-digit decimal c/10 * 10^k10 in the interval, when closer than the one-digit one
        Big t10 = r0;   // r0 / s = v / 10^k10 in [1, 10)
        t10.mul(10);
        uint32_t c = 0;
        Big rem = t10;
        while (rem.cmp(s) >= 0) { rem.sub(s); ++c; }
        Big r2 = rem;
        r2.mul(2);
        const int cr = r2.cmp(s);
        const bool up = cr > 0 || (cr == 0 && (c & 1));
        if (up) ++c;
        if (c < 100 && c % 10 != 0) {
            // distances at the scale of t10: |c s - t10| against |10 d s - t10|, and the interval ends (10 m+ / 10 m-)
            Big cs = s, ds = s;
            cs.mul(c);
            ds.mul(10u * dig[0]);
            Big dc = cs.cmp(t10) >= 0 ? cs : t10, dd = ds.cmp(t10) >= 0 ? ds : t10;
            if (cs.cmp(t10) >= 0) dc.sub(t10); else { Big x = t10; x.sub(cs); dc = x; }
            if (ds.cmp(t10) >= 0) dd.sub(t10); else { Big x = t10; x.sub(ds); dd = x; }
            Big lim = cs.cmp(t10) >= 0 ? mp0 : mm0;   // at the scale of r0 (x 10 below)
            lim.mul(10);
            const int cin = dc.cmp(lim);
            const bool inside = even ? cin <= 0 : cin < 0;
            if (inside && dc.cmp(dd) < 0) { dig[0] = (uint8_t)(c / 10); dig[1] = (uint8_t)(c % 10); n = 2; }
        }
    }
    return n;
}

__device__ void write_double(Sink &k, uint64_t bits)
{
    const bool neg = bits >> 63;
    const uint64_t mant = bits & ((1ull << 52) - 1);
    const int ex = (int)((bits >> 52) & 0x7FF);
    if (neg) k.c('-');
    if (ex == 0 && mant == 0) { k.s("0.0"); return; }
    if (ex == 0x7FF) { k.s(mant ? "NaN" : "Infinity"); return; }
    const uint64_t f = ex ? (mant | (1ull << 52)) : mant;
    const int e = ex ? ex - 1075 : -1074;
    uint8_t dig[20];
    int k10 = 0;
    const int n = shortest_digits(f, e, ex <= 1, dig, k10);
    if (k10 >= -3 && k10 < 7) {   // 10^-3 <= |v| < 10^7: plain notation, at least one fraction digit
        if (k10 < 0) {
            k.s("0.");
            for (int z = 0; z < -k10 - 1; ++z) k.c('0');
            for (int i = 0; i < n; ++i) k.c('0' + dig[i]);
        } else {
            for (int i = 0; i <= k10; ++i) k.c(i < n ? '0' + dig[i] : '0');
            k.c('.');
            if (n > k10 + 1) for (int i = k10 + 1; i < n; ++i) k.c('0' + dig[i]);
            else k.c('0');
        }
    } else {   // computerized scientific notation
        k.c('0' + dig[0]);
        k.c('.');
        if (n > 1) for (int i = 1; i < n; ++i) k.c('0' + dig[i]);
        else k.c('0');
        k.c('E');
        k.dec(k10);
    }
}

// JsonWriter.string with Gson's default HTML-safe escaping (GsonBuilder: htmlSafe unless disableHtmlEscaping)
__device__ void write_string(Sink &k, const uint8_t *p, uint32_t n)
{
    static constexpr char hex[] = "0123456789abcdef";
    k.c('"');
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t c = p[i];
        if (c == '"') k.s("\\\"");
        else if (c == '\\') k.s("\\\\");
        else if (c == '\t') k.s("\\t");
        else if (c == '\b') k.s("\\b");
        else if (c == '\n') k.s("\\n");
        else if (c == '\r') k.s("\\r");
        else if (c == '\f') k.s("\\f");
        else if (c < 0x20 || c == '<' || c == '>' || c == '&' || c == '=' || c == '\'') {
            k.s("\\u00"); k.c(hex[c >> 4]); k.c(hex[c & 15]);
        } else k.c((uint8_t)c);
    }
    k.c('"');
}

// Datum.write (Datum.java:209-226)
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
    if (kind == K_DOUBLE) { write_double(k, d.value[code]); return true; }
    if (kind == K_STRING && d.str && d.len) { write_string(k, d.str + d.value[code], d.len[code]); return true; }
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
    Dict d{ in->dict_kind, in->dict_null, in->dict_value, in->n_dict, in->dict_len, in->dict_str };
    uint64_t *len = ctx->get<uint64_t>("jw_len", ng), *off = ctx->get<uint64_t>("jw_off", (size_t)ng + 1);
    uint64_t *errs = ctx->get<uint64_t>("jw_errs", 1);
    ACC_HIP(hipMemsetAsync(errs, 0, 8, st));
    if (ng) launch(ctx, "json_size", k_json_write, dim3(grid_for(ng, BLOCK)), dim3(BLOCK), 0, ng, kh, rh, d, (const uint64_t *)nullptr,
                   (uint8_t *)nullptr, len, errs);
    scan<uint64_t, OpAdd<uint64_t>>(ctx, len, off, ng, true, off + ng);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, errs, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, off + ng, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    if (ctx->pinned[0]) fail(ACC_E_ARG, "a key is no datum of the dictionary (or a STRING one without dict_len / dict_str)");
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
