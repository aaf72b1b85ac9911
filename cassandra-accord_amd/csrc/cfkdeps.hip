// cfkdeps.hip — CommandsForKey.update with each command's deps: missing[] maintenance and the
// TRANSITIVELY_KNOWN additions (local/CommandsForKey.java:657-1149), for a batch of command updates applied, in batch
// order, to every CommandsForKey (key) they touch.
//
// The state is key-major: per key its TxnInfos (TxnId, executeAt, InternalStatus) in TxnId order, each with its
// TxnInfoWithMissing.missing (sorted TxnIds). Keys are independent, so the batch runs as one lane per key:
//   1. the snapshot keys and every (update, key) pair are radix sorted by key code (stable: a key's snapshot first,
//      then its updates in batch order); distinct keys by a flag scan;
//   2. per key, working-space bounds (entries: snapshot + one per update + its deps, exact; missing: a linear first
//      guess below the proven bound, min(entries^2, snapshot missing + entries x (deps + 2) per update)) and one scan
//      of them give each key two ping-pong buffers in one pool;
//   3. one lane per key replays its updates: CommandsForKey.update -> insert / update, computeInfoAndAdditions,
//      insertInfoAndOneMissing, updateOrInsertWithAdditions with mergeAndFilterMissing / to / insertMissing,
//      removeMissing — each update rebuilding the key's TxnInfo array into the other buffer, as the Java builds a new
//      array;
//      a key whose missing[] outgrows its guess is flagged; the flagged keys' guesses grow 4x (up to the proven bound)
//      and the replay runs again, so a hot key with thousands of dep-carrying updates costs the space it really uses,
//      not the quadratic bound; from the third round on a flagged key takes the bound at once, so a batch replays at
//      most four times (every key replays: the pool's layout moves when the flagged keys grow);
//   4. final sizes, two scans, and a compaction into the key-major output (keys without entries dropped).
// Keys with more than acc_opts.cfk_hot (64) sorted elements skip step 3: their final state is the replay's closed form,
// computed data-parallel over the key's updates (the hot-key section below).
// Errors: a status going back (IllegalStateException "stale status", ACC_E_STATE), an addition equal to an existing
// TxnId or depsKnownBefore equal to a TxnId (the reference's checkState, ACC_E_STATE), malformed input (ACC_E_ARG).
#include "dict.hpp"

namespace acc {
namespace cd {

constexpr uint64_t IDENTITY_LSB = 0xFFFFFFFFFFFF001EULL;
constexpr uint32_t NONE_K = 0xFFFFFFFFu;
enum : uint32_t { TK = 0, PRE = 2, ACC = 3, COMMITTED = 4, APPLIED = 6, INVALID = 7 };
enum : uint64_t { E_ARG_STATUS = 1, E_ARG_SORT = 2, E_ARG_OFF = 4, E_STALE = 8, E_STATE = 16, E_CAP = 32, E_MCAP = 64 };

struct Ts {
    uint64_t m, l;
    int32_t n;
};

__device__ __forceinline__ int cmp(const Ts &a, const Ts &b)
{
    if (a.m != b.m) return a.m < b.m ? -1 : 1;
    const uint64_t a1 = a.l & IDENTITY_LSB, b1 = b.l & IDENTITY_LSB;
    if (a1 != b1) return a1 < b1 ? -1 : 1;
    if (a.n != b.n) return a.n < b.n ? -1 : 1;
    return 0;
}
__device__ __forceinline__ uint32_t kind(const Ts &t) { return (uint32_t)(t.l >> 1) & 7u; }
// Kind.witnesses() (primitives/Txn.java:221-236)
__device__ __forceinline__ uint32_t witnesses_mask(uint32_t k)
{
    switch (k) {
    case 0: case 2: return 1u << 1;
    case 1: case 3: return (1u << 0) | (1u << 1);
    case 4: return (1u << 0) | (1u << 1) | (1u << 3) | (1u << 4);
    default: return 0;
    }
}
__device__ __forceinline__ bool witnesses(const Ts &owner, const Ts &t) { return (witnesses_mask(kind(owner)) >> kind(t)) & 1u; }
__device__ __forceinline__ bool has_info(uint32_t s) { return s >= ACC && s <= APPLIED; }

struct Info {
    Ts id, ex;
    uint32_t st, self;   // self: executeAt is the TxnId (TxnInfo.create keeps the TxnId object)
    uint32_t ms, mn;     // missing[] in the buffer's missing area
};
// TxnInfo.depsKnownBefore() (:322-325, InternalStatus.depsKnownBefore :260-279): the txn itself or its executeAt
__device__ __forceinline__ bool dkb_self(const Info &x) { return x.st == PRE || x.st == ACC || x.self; }
__device__ __forceinline__ const Ts &dkb(const Info &x) { return dkb_self(x) ? x.id : x.ex; }

// The working buffers of the 64 keys of one wave are interleaved element by element (key k = lane k % 64 of wave k / 64:
// element i of its buffer at [i * CD_W + lane]), so when the lanes walk their keys' arrays side by side -- the replay
// rebuilds every array per update -- each wave-wide access is one contiguous span instead of 64 scattered lines.
constexpr long CD_W = 64;
constexpr long CD_S = CD_W;   // element stride (a per-key contiguous layout, stride 1, measured: cd_apply 5.3 -> 7.8 ms)
template <class T>
struct SP {   // a lane's strided view of an interleaved buffer
    T *p;
    __device__ T &operator[](long i) const { return p[i * CD_S]; }
    __device__ SP operator+(long k) const { return SP{ p + k * CD_S }; }
    __device__ bool operator==(const SP &o) const { return p == o.p; }
};

// the command's keyDeps.txnIds(key) read in place from the update arrays (SoA columns), no staging copy
struct DepsIn {
    const uint64_t *m, *l;
    const int32_t *n;
    __device__ Ts operator[](long i) const { return Ts{ m[i], l[i], n[i] }; }
};

// A TxnInfo as stored: 48 B (status and the executeAt-is-TxnId flag in the top bits of the missing count) instead of the
// 64-B working struct; read and written whole through a lane's strided view
struct InfoP {
    uint64_t im, il, xm, xl;
    int32_t in, xn;
    uint32_t ms, mnst;   // missing[] start; count | status << 28 | self << 31
};
static_assert(sizeof(InfoP) == 48, "48-B stored TxnInfo");
constexpr uint32_t MN_MAX = 1u << 28;
struct EP {
    InfoP *p;
    __device__ Info get(long i) const
    {
        const InfoP q = p[i * CD_S];
        Info x;
        x.id = Ts{ q.im, q.il, q.in };
        x.ex = Ts{ q.xm, q.xl, q.xn };
        x.ms = q.ms;
        x.mn = q.mnst & (MN_MAX - 1);
        x.st = (q.mnst >> 28) & 7u;
        x.self = q.mnst >> 31;
        return x;
    }
    __device__ void set(long i, const Info &x) const
    {
        p[i * CD_S] = InfoP{ x.id.m, x.id.l, x.ex.m, x.ex.l, x.id.n, x.ex.n, x.ms, x.mn | (x.st << 28) | (x.self << 31) };
    }
    __device__ EP operator+(long k) const { return EP{ p + k * CD_S }; }
};

struct Buf {
    EP e;
    SP<Ts> m;
    uint32_t n, mtop;
};

struct Work {   // one key's working space
    Buf a, b;
    uint32_t ecap, mcap;
    SP<Ts> tmiss;   // the new TxnInfo's missing[] (ecap)
    SP<Ts> adds;    // additions (dcap)
    SP<Ts> owned;   // insertMissing result (dcap + 1)
};

template <class P>
__device__ long bsearch_ts(P a, long from, long to, const Ts &k)   // Arrays.binarySearch
{
    long lo = from, hi = to - 1;
    while (lo <= hi) {
        const long mid = (long)(((unsigned long)lo + (unsigned long)hi) >> 1);
        const int c = cmp(a[mid], k);
        if (c < 0) lo = mid + 1; else if (c > 0) hi = mid - 1; else return mid;
    }
    return -(lo + 1);
}
__device__ long bsearch_info(const Buf &b, long from, long to, const Ts &k)
{
    long lo = from, hi = to - 1;
    while (lo <= hi) {
        const long mid = (long)(((unsigned long)lo + (unsigned long)hi) >> 1);
        const int c = cmp(b.e.get(mid).id, k);
        if (c < 0) lo = mid + 1; else if (c > 0) hi = mid - 1; else return mid;
    }
    return -(lo + 1);
}

struct Ctx {
    Work w;
    uint64_t err;
    __device__ __forceinline__ bool room_e(uint32_t n) { if (n > w.ecap) { err |= E_CAP; return false; } return true; }
    // missing areas: beyond the key's current guess (E_MCAP: grown and replayed by the host)
    __device__ __forceinline__ bool room_m(const Buf &b, uint32_t add) { if ((uint64_t)b.mtop + add > w.mcap) { err |= E_MCAP; return false; } return true; }
    // append an entry (its missing count must fit the stored 28 bits)
    __device__ __forceinline__ void put_e(Buf &dst, const Info &y)
    {
        if (y.mn >= MN_MAX) { err |= E_CAP; return; }
        if (room_e(dst.n + 1)) dst.e.set(dst.n++, y);
    }

    // append entry x of src with its missing[] copied (dropping `drop` when given) to dst
    __device__ __forceinline__ void put(Buf &dst, const Info &x, SP<Ts> src_m, const Ts *drop)
    {
        Info y = x;
        y.ms = dst.mtop;
        y.mn = 0;
        if (x.mn && room_m(dst, x.mn)) {
            for (uint32_t q = 0; q < x.mn; ++q) {
                const Ts &t = src_m[x.ms + q];
                if (drop && cmp(t, *drop) == 0) continue;
                dst.m[dst.mtop + y.mn++] = t;
            }
        }
        dst.mtop += y.mn;
        put_e(dst, y);
    }
    // x with `ins` inserted into its missing[] (SortedArrays.insert)
    __device__ __forceinline__ void put_with_one(Buf &dst, const Info &x, SP<Ts> src_m, const Ts &ins)
    {
        Info y = x;
        y.ms = dst.mtop;
        y.mn = 0;
        if (!room_m(dst, x.mn + 1)) return;
        bool done = false;
        for (uint32_t q = 0; q < x.mn; ++q) {
            const Ts &t = src_m[x.ms + q];
            const int c = cmp(t, ins);
            if (!done && c >= 0) { if (c > 0) dst.m[dst.mtop + y.mn++] = ins; done = true; }
            dst.m[dst.mtop + y.mn++] = t;
        }
        if (!done) dst.m[dst.mtop + y.mn++] = ins;
        dst.mtop += y.mn;
        put_e(dst, y);
    }
    // mergeAndFilterMissing (:988-1025) of additions[0, count) into x's missing[], written to dst
    __device__ __forceinline__ void put_merged(Buf &dst, const Info &x, SP<Ts> src_m, SP<Ts> add, uint32_t count)
    {
        const uint32_t kinds = witnesses_mask(kind(x.id));
        uint32_t keep = 0;
        for (uint32_t i = 0; i < count; ++i) keep += (kinds >> kind(add[i])) & 1u;
        if (!keep) { put(dst, x, src_m, nullptr); return; }
        Info y = x;
        y.ms = dst.mtop;
        y.mn = 0;
        if (!room_m(dst, x.mn + keep)) return;
        SP<Ts> o = dst.m + dst.mtop;
        uint32_t i = 0, j = 0, n = 0;
        while (i < count && j < x.mn) {
            if ((kinds >> kind(add[i])) & 1u) {
                if (cmp(add[i], src_m[x.ms + j]) < 0) o[n++] = add[i++];
                else o[n++] = src_m[x.ms + j++];
            } else ++i;
        }
        for (; i < count; ++i) if ((kinds >> kind(add[i])) & 1u) o[n++] = add[i];
        while (j < x.mn) o[n++] = src_m[x.ms + j++];
        if (n != x.mn + keep) err |= E_STATE;   // checkState(count == additionCount + current.length)
        y.mn = n;
        dst.mtop += n;
        put_e(dst, y);
    }
    // a new TxnInfo whose missing[] is in w.tmiss
    __device__ __forceinline__ void put_new(Buf &dst, const Info &x, uint32_t nm)
    {
        Info y = x;
        y.ms = dst.mtop;
        y.mn = 0;
        if (nm && room_m(dst, nm)) {
            for (uint32_t q = 0; q < nm; ++q) dst.m[dst.mtop + q] = w.tmiss[q];
            y.mn = nm;
        }
        dst.mtop += y.mn;
        put_e(dst, y);
    }
    __device__ __forceinline__ void put_tk(Buf &dst, const Ts &id)   // TxnInfo.create(txnId, TRANSITIVELY_KNOWN, txnId)
    {
        Info y;
        y.id = id; y.ex = id; y.st = TK; y.self = 1; y.ms = dst.mtop; y.mn = 0;
        put_e(dst, y);
    }

    // insert(pos, TxnInfo) (:880-897) with insertInfoAndOneMissing (:899-944); the new info's missing[] in tmiss
    __device__ __forceinline__ void insert_plain(const Buf &A, Buf &B, uint32_t pos, const Info &ins, uint32_t nm)
    {
        const bool plain = ins.st >= COMMITTED;
        for (uint32_t i = 0; i < pos; ++i) {
            const Info x = A.e.get(i);
            if (!plain && has_info(x.st) && cmp(dkb(x), ins.id) > 0 && witnesses(x.id, ins.id)) put_with_one(B, x, A.m, ins.id);
            else put(B, x, A.m, nullptr);
        }
        put_new(B, ins, nm);
        for (uint32_t i = pos; i < A.n; ++i) {
            const Info x = A.e.get(i);
            if (!plain && has_info(x.st) && witnesses(x.id, ins.id)) put_with_one(B, x, A.m, ins.id);
            else put(B, x, A.m, nullptr);
        }
    }
    // update(pos, txnId, cur, new) (:865-875): the entry replaced, removeMissing (:946-972) when it becomes committed
    __device__ __forceinline__ void update_plain(const Buf &A, Buf &B, uint32_t pos, const Info &nw, uint32_t nm)
    {
        const bool crossed = A.e.get(pos).st < COMMITTED && nw.st >= COMMITTED;
        for (uint32_t i = 0; i < A.n; ++i) {
            if (i == pos) put_new(B, nw, nm);
            else put(B, A.e.get(i), A.m, crossed ? &nw.id : nullptr);
        }
    }

    // computeInfoAndAdditions (:1057-1149): the new TxnInfo (missing[] to tmiss) and the deps this CFK lacks (adds)
    __device__ __forceinline__ Info compute_info(const Buf &A, long insert_pos, long update_pos, const Ts &id, uint32_t st, const Ts &ex_in,
                                 DepsIn deps, uint32_t nd, uint32_t &nm, uint32_t &na)
    {
        Info x;
        x.id = id; x.st = st; x.self = 1; x.ex = id; x.ms = 0; x.mn = 0;
        if (cmp(ex_in, id) != 0) { x.ex = ex_in; x.self = 0; }
        const bool self = st == PRE || st == ACC || x.self;
        long dpos = insert_pos;
        if (!self) {
            dpos = bsearch_info(A, insert_pos, (long)A.n, x.ex);
            if (dpos >= 0) err |= E_STATE;   // checkState(depsKnownBeforePos < 0)
            dpos = -1 - dpos;
        }
        nm = 0; na = 0;
        long ti = 0;
        uint32_t di = 0;
        while (ti < dpos && di < nd) {
            const Info t = A.e.get(ti);
            const Ts dd = deps[di];
            const int r = cmp(t.id, dd);
            if (r == 0) { ++ti; ++di; }
            else if (r < 0) {
                if (ti != update_pos && t.st < COMMITTED && witnesses(id, t.id)) w.tmiss[nm++] = t.id;
                ++ti;
            } else { w.adds[na++] = dd; ++di; }
        }
        for (; ti < dpos; ++ti) {
            const Info t = A.e.get(ti);
            if (ti != update_pos && t.st < COMMITTED && witnesses(id, t.id)) w.tmiss[nm++] = t.id;
        }
        while (di < nd) w.adds[na++] = deps[di++];
        return x;
    }

    // updateOrInsertWithAdditions (:772-863)
    __device__ __forceinline__ void with_additions(const Buf &A, Buf &B, long src_insert, long src_update, const Info &winfo, uint32_t nm,
                                   uint32_t na)
    {
        const SP<Ts> add = w.adds;
        long aip = bsearch_ts(add, 0, (long)na, winfo.id);
        if (aip >= 0) { err |= E_STATE; return; }
        aip = -1 - aip;
        const uint32_t target = (uint32_t)(src_insert + aip);
        SP<Ts> msrc = add;
        const bool insert_self_missing = src_update < 0 && winfo.st < COMMITTED;
        uint32_t i = 0, j = 0, mcount = 0, mlimit = na, count = 0;
        while (i < A.n) {
            if (count == target) {
                put_new(B, winfo, nm);
                if ((long)i == src_update) ++i;
                else if (insert_self_missing) ++mcount;
                ++count;
                continue;
            }
            const Info xi = A.e.get(i);
            const int r = j == na ? -1 : cmp(xi.id, add[j]);
            if (r < 0) {
                const Info &x = xi;
                if ((long)i == src_update) put_new(B, winfo, nm);
                else if (has_info(x.st)) {
                    if (insert_self_missing && msrc == add && (mcount != j || (!dkb_self(x) && cmp(dkb(x), winfo.id) > 0))) {
                        // insertMissing (:979-986)
                        for (long q = 0; q < aip; ++q) w.owned[q] = add[q];
                        w.owned[aip] = winfo.id;
                        for (uint32_t q = (uint32_t)aip; q < na; ++q) w.owned[q + 1] = add[q];
                        msrc = w.owned;
                        ++mlimit;
                    }
                    // to (:1027-1033)
                    uint32_t to = mcount;
                    if (!dkb_self(x)) {
                        long t = bsearch_ts(msrc, 0, (long)mlimit, dkb(x));
                        to = (uint32_t)(t < 0 ? -1 - t : t);
                    }
                    if (to > 0) put_merged(B, x, A.m, msrc, to);
                    else put(B, x, A.m, nullptr);
                } else put(B, x, A.m, nullptr);
                ++i;
            } else if (r > 0) {
                put_tk(B, add[j++]);
                ++mcount;
            } else {
                err |= E_STATE;   // "should be an insertion, but found match when merging with origin"
                return;
            }
            ++count;
        }
        if (j < na) {
            if (count <= target) {
                while (count < target) { put_tk(B, add[j++]); ++count; }
                put_new(B, winfo, nm);
                count = target + 1;
            }
            while (j < na) { put_tk(B, add[j++]); ++count; }
        } else if (count == target) {
            put_new(B, winfo, nm);
        }
    }

    // removeMissing over a whole buffer, in place (:946-972)
    __device__ __forceinline__ void remove_missing(Buf &B, const Ts &id)
    {
        for (uint32_t i = 0; i < B.n; ++i) {
            Info x = B.e.get(i);
            if (!x.mn) continue;
            const long j = bsearch_ts(B.m + x.ms, 0, (long)x.mn, id);
            if (j < 0) continue;
            for (uint32_t q = (uint32_t)j; q + 1 < x.mn; ++q) B.m[x.ms + q] = B.m[x.ms + q + 1];
            --x.mn;
            B.e.set(i, x);
        }
    }

    // CommandsForKey.update(prev, next) (:657-722) on this key; returns true when the state moved to B
    // fl: bit 0 = acceptedOrCommitted changed, bit 1 = next.status() == AcceptedInvalidate
    // a key's state summary for the in-place fast paths: nlow = entries below COMMITTED (the candidates of a new
    // TxnInfo's missing[]), maxdkb = an upper bound of depsKnownBefore over the entries with info (the entries
    // insertInfoAndOneMissing may touch), mlive = the missing[] entries of all entries (what removeMissing would edit)
    struct Sum {
        Ts maxdkb;
        bool any;
        uint32_t nlow, mlive;
    };
    __device__ __forceinline__ void sum_add(Sum &sm, const Info &x)
    {
        sm.nlow += x.st < COMMITTED ? 1u : 0u;
        sm.mlive += x.mn;
        if (has_info(x.st) && (!sm.any || cmp(dkb(x), sm.maxdkb) > 0)) { sm.maxdkb = dkb(x); sm.any = true; }
    }
    __device__ __forceinline__ void sum_of(const Buf &A, Sum &sm)
    {
        sm.any = false; sm.nlow = 0; sm.mlive = 0;
        for (uint32_t i = 0; i < A.n; ++i) sum_add(sm, A.e.get(i));
    }
    // every dep among the entries [0, to): computeInfoAndAdditions finds no addition. Walked from the last dep down,
    // each first tried just below where the one above it was found (a key's deps are usually its latest entries, one
    // probe each), and searched for otherwise
    __device__ __forceinline__ bool deps_present(const Buf &A, long to, DepsIn deps, uint32_t nd)
    {
        long g = to - 1;
        for (long d = (long)nd - 1; d >= 0; --d) {
            const Ts k = deps[d];
            if (g < 0 || cmp(A.e.get(g).id, k) != 0) {
                g = bsearch_info(A, 0, to, k);
                if (g < 0) return false;
            }
            --g;
        }
        return true;
    }

    // CommandsForKey.update(prev, next) (:657-722) on this key. Returns 0 when the state is unchanged, 1 when the new
    // state is in B (the Java's new arrays), 2 when A was updated in place: the fast paths below take the cases where
    // the Java's rebuild copies every other entry unchanged -- an insert at the end that adds nothing to any entry's
    // missing[] and takes no missing[] itself, or an update of one entry with nothing to remove -- so A's other entries
    // stay where they are (a replaced entry's missing[] is left behind in the missing area; the next full rebuild
    // compacts it). fl: bit 0 = acceptedOrCommitted changed, bit 1 = next.status() == AcceptedInvalidate
    __device__ __forceinline__ int apply(Buf &A, Buf &B, const Ts &id, const Ts &ex, uint32_t st, uint32_t fl, DepsIn deps,
                                         uint32_t nd, Sum &sm)
    {
        B.n = 0; B.mtop = 0;
        // a TxnId past the key's last one (the usual first update) needs no search
        long pos = A.n == 0 || cmp(A.e.get(A.n - 1).id, id) < 0 ? -1 - (long)A.n : bsearch_info(A, 0, (long)A.n, id);
        if (pos < 0) {
            pos = -1 - pos;
            Info ni;
            ni.id = id; ni.ex = id; ni.st = st; ni.self = 1; ni.ms = A.mtop; ni.mn = 0;
            if (has_info(st) && cmp(ex, id) != 0) { ni.ex = ex; ni.self = 0; }
            if (pos == (long)A.n && (st >= COMMITTED || !sm.any || cmp(sm.maxdkb, id) <= 0) &&
                (!has_info(st) || (sm.nlow == 0 && deps_present(A, (long)A.n, deps, nd))) && room_e(A.n + 1)) {
                put_e(A, ni);   // insert at the end: no entry gains a missing TxnId, the new one has none
                sum_add(sm, ni);
                return 2;
            }
            if (has_info(st)) {
                uint32_t nm, na;
                const Info nc = compute_info(A, pos, -1, id, st, ex, deps, nd, nm, na);
                if (na == 0) insert_plain(A, B, (uint32_t)pos, nc, nm);
                else with_additions(A, B, pos, -1, nc, nm, na);
            } else {
                ni.ms = 0;
                insert_plain(A, B, (uint32_t)pos, ni, 0);
            }
            return 1;
        }
        const Info cur = A.e.get(pos);
        if (st <= cur.st) {
            // Invariants.checkState(cur.status == newStatus || next.status() == AcceptedInvalidate) (:681-686)
            if (cur.st != st && !(fl & 2u)) { err |= E_STALE; return 0; }
            if (!has_info(st) || !(fl & 1u)) return 0;   // acceptedOrCommitted unchanged: this (:687-688)
        }
        {   // in place: the entry replaced, no missing[] for it, nothing to remove from the others
            Info ni;
            ni.id = id; ni.ex = id; ni.st = st; ni.self = 1; ni.ms = A.mtop; ni.mn = 0;
            if (has_info(st) && cmp(ex, id) != 0) { ni.ex = ex; ni.self = 0; }
            const bool crossed = cur.st < COMMITTED && st >= COMMITTED;
            bool ok = !crossed || sm.mlive == cur.mn;
            if (ok && has_info(st)) {
                long dpos = pos;
                if (!(st == PRE || st == ACC || ni.self)) {
                    dpos = bsearch_info(A, pos, (long)A.n, ni.ex);
                    if (dpos >= 0) ok = false;   // the general path reports it (checkState)
                    else dpos = -1 - dpos;
                }
                ok = ok && sm.nlow - (cur.st < COMMITTED ? 1u : 0u) == 0 && deps_present(A, dpos, deps, nd);
            }
            if (ok) {
                A.e.set(pos, ni);
                sm.nlow = sm.nlow - (cur.st < COMMITTED ? 1u : 0u) + (st < COMMITTED ? 1u : 0u);
                sm.mlive -= cur.mn;
                if (has_info(st) && (!sm.any || cmp(dkb(ni), sm.maxdkb) > 0)) { sm.maxdkb = dkb(ni); sm.any = true; }
                return 2;
            }
        }
        if (has_info(st)) {
            uint32_t nm, na;
            const Info ni = compute_info(A, pos, pos, id, st, ex, deps, nd, nm, na);
            if (na == 0) update_plain(A, B, (uint32_t)pos, ni, nm);
            else {
                with_additions(A, B, pos, pos, ni, nm, na);
                if (cur.st < COMMITTED && st >= COMMITTED) remove_missing(B, id);
            }
        } else {
            Info ni;
            ni.id = id; ni.ex = id; ni.st = st; ni.self = 1; ni.ms = 0; ni.mn = 0;
            update_plain(A, B, (uint32_t)pos, ni, 0);
        }
        return 1;
    }
};

struct Snap {
    const uint64_t *key;
    const uint32_t *ent_off, *miss_off;
    const uint64_t *em, *el, *xm, *xl, *mm, *ml;
    const int32_t *en, *xn, *mn;
    const uint8_t *st;
    uint32_t n_keys;
    uint64_t n_ent, n_miss;
};
struct Upd {
    const uint64_t *um, *ul, *uxm, *uxl, *key, *dm, *dl;
    const int32_t *un, *uxn, *dn;
    const uint8_t *st, *fl;
    const uint32_t *key_off, *dep_off, *owner;   // owner: update of each (update, key) pair
    uint32_t n_upd;
    uint64_t NP, ND;
};

// validation + the pair -> update map; rng (when given): the smallest and largest key code, so the key sort orders
// code - smallest on the bits the span needs
__global__ __launch_bounds__(BLOCK) void k_cd_check(Snap s, Upd u, uint32_t *__restrict__ owner, uint64_t *__restrict__ err,
                                                    uint64_t *__restrict__ rng)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    uint64_t e = 0;
    if (rng) {
        unsigned long long lo = ~0ull, hi = 0;
        if (i < s.n_keys) { lo = s.key[i]; hi = lo; }
        if (i < u.NP) {
            const unsigned long long k = u.key[i];
            lo = k < lo ? k : lo;
            hi = k > hi ? k : hi;
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const unsigned long long a = __shfl_xor(lo, d, 64), b = __shfl_xor(hi, d, 64);
            lo = a < lo ? a : lo;
            hi = b > hi ? b : hi;
        }
        if (lane_id() == 0 && lo <= hi) {   // an atomic only where this wave moves a bound (one address for every wave)
            unsigned long long *r = (unsigned long long *)rng;
            if (lo < __hip_atomic_load(&r[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(&r[0], lo);
            if (hi > __hip_atomic_load(&r[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(&r[1], hi);
        }
    }
    if (i < u.n_upd) {
        const uint32_t a = u.key_off[i], b = u.key_off[i + 1];
        if (b < a || b > u.NP || (i == 0 && a != 0) || (i + 1 == u.n_upd && b != u.NP)) e |= E_ARG_OFF;
        else {
            for (uint32_t j = a; j < b; ++j) {
                owner[j] = (uint32_t)i;
                if (j > a && u.key[j - 1] >= u.key[j]) e |= E_ARG_SORT;
            }
        }
        if (u.st[i] > INVALID && u.st[i] != 0xFF) e |= E_ARG_STATUS;
    }
    if (i < u.NP) {
        const uint32_t a = u.dep_off[i], b = u.dep_off[i + 1];
        if (b < a || b > u.ND || (i == 0 && a != 0) || (i + 1 == u.NP && b != u.ND)) e |= E_ARG_OFF;
        // (each pair's deps strictly ascending: k_cd_depchk)
    }
    if (i < s.n_keys) {
        if (i > 0 && s.key[i - 1] >= s.key[i]) e |= E_ARG_SORT;
        const uint32_t a = s.ent_off[i], b = s.ent_off[i + 1];
        if (b < a || b > s.n_ent || (i == 0 && a != 0) || (i + 1 == s.n_keys && b != s.n_ent)) e |= E_ARG_OFF;
    }
    if (i < s.n_ent) {   // a thread per entry (a hot key holds hundreds of thousands); its key by a search of the offsets
        uint32_t lo = 0, hi = s.n_keys;   // last key whose entries start at or before i
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s.ent_off[mid] <= i) lo = mid; else hi = mid;
        }
        if (s.st[i] > INVALID) e |= E_ARG_STATUS;
        if (i > s.ent_off[lo] && cmp(Ts{ s.em[i - 1], s.el[i - 1], s.en[i - 1] }, Ts{ s.em[i], s.el[i], s.en[i] }) >= 0) e |= E_ARG_SORT;
        const uint32_t m0 = s.miss_off[i], m1 = s.miss_off[i + 1];
        if (m1 < m0 || m1 > s.n_miss) e |= E_ARG_OFF;
    }
    if (e) atomicOr((unsigned long long *)err, (unsigned long long)e);
}

// each pair's deps strictly ascending. A wave takes 64 consecutive pairs and walks their deps (one contiguous range)
// side by side, so the loads coalesce; a dep is compared with the one before it unless it starts its pair's range (a
// search of the 64 starts held one per lane). The lsb / node words are read only where two msb words tie. Ranges are
// clamped to [0, n_deps): malformed offsets (k_cd_check reports them) never read out of bounds.
__global__ __launch_bounds__(BLOCK) void k_cd_depchk(Upd u, uint64_t *__restrict__ err)
{
    const uint64_t p0 = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) & ~(uint64_t)63;
    if (p0 >= u.NP) return;   // (whole waves: p0 is the wave's first pair)
    const uint32_t lane = lane_id();
    const uint64_t pl = p0 + lane < u.NP ? p0 + lane : u.NP;   // lanes past the end hold the end offset
    const uint32_t st = (uint32_t)std::min<uint64_t>(u.dep_off[pl], u.ND);
    const uint32_t lo = __shfl(st, 0, 64);
    const uint64_t pe = p0 + 64 < u.NP ? p0 + 64 : u.NP;
    const uint32_t hi = (uint32_t)std::min<uint64_t>(u.dep_off[pe], u.ND);
    bool bad = false;
    for (uint32_t base = lo; base < hi; base += 64) {   // (uniform over the wave: every lane takes part in the shuffles)
        const uint32_t j = base + lane;
        // a pair's start: some lane's st == j (st non-decreasing over lanes when the offsets are valid); branchless
        // lower bound over the 64 starts
        uint32_t pos = 0;
#pragma unroll
        for (uint32_t step = 32; step >= 1; step >>= 1)
            if (__shfl(st, (int)(pos + step - 1), 64) < j) pos += step;
        const bool start = __shfl(st, (int)pos, 64) == j;
        if (j < hi && j > 0 && !start) {
            const uint64_t pm = u.dm[j - 1], m = u.dm[j];
            if (m < pm || (m == pm && cmp(Ts{ pm, u.dl[j - 1], u.dn[j - 1] }, Ts{ m, u.dl[j], u.dn[j] }) >= 0)) bad = true;
        }
    }
    if (__ballot(bad) && lane == 0) atomicOr((unsigned long long *)err, (unsigned long long)E_ARG_SORT);
}

__global__ __launch_bounds__(BLOCK) void k_cd_keys(uint32_t nk, uint64_t NP, const uint64_t *__restrict__ skey,
                                                   const uint64_t *__restrict__ ukey, uint64_t base, uint64_t *__restrict__ all)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < nk) all[i] = skey[i] - base;
    else if (i < nk + NP) all[i] = ukey[i - nk] - base;
}

__global__ __launch_bounds__(BLOCK) void k_cd_kflag(uint64_t T, const uint64_t *__restrict__ sk, uint32_t *__restrict__ f)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < T) f[i] = (i == 0 || sk[i] != sk[i - 1]) ? 1u : 0u;
}

// per distinct key: the start of its run [kstart[k], kstart[k + 1]) of the sorted elements
__global__ __launch_bounds__(BLOCK) void k_cd_kstart(uint64_t T, const uint32_t *__restrict__ f, const uint32_t *__restrict__ fi,
                                                     uint32_t nkeys, uint32_t *__restrict__ kstart)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < T && f[i]) kstart[fi[i] - 1] = (uint32_t)i;
    if (i == 0) kstart[nkeys] = (uint32_t)T;
}
// per distinct key (a lane per key, so a wave's lanes walk adjacent runs): its working-space bounds. rec: each update
// element's record (k_cd_urec: its deps range)
// per sorted element (in order, so the loads coalesce), its share of its key's bounds: entries, snapshot missing,
// regrowth (deps + 2 per update) and the largest deps count, summed per key by a segmented scan over the wave (a key's
// elements are adjacent) and one atomic per key and wave into zeroed accumulators
struct BSum {
    uint64_t *e, *m, *g;
    uint32_t *d;
};
__global__ __launch_bounds__(BLOCK) void k_cd_bsum(uint64_t T, const uint32_t *__restrict__ kinc, const uint32_t *__restrict__ src,
                                                   const uint2 *__restrict__ rda, uint32_t nk, Snap s, BSum b)
{
    const uint64_t q = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t lane = lane_id();
    uint32_t k = NONE_K, d = 0;
    uint64_t e = 0, m = 0, g = 0;
    if (q < T) {
        k = kinc[q] - 1;
        const uint32_t v = src[q];
        if (v < nk) {
            e = s.ent_off[v + 1] - s.ent_off[v];
            m = s.miss_off[s.ent_off[v + 1]] - s.miss_off[s.ent_off[v]];
        } else {
            const uint2 r = rda[q * 8 + 7];   // the record's (da, db) words (UpdRec bytes 56..63)
            d = r.y - r.x;
            e = 1 + (uint64_t)d;
            g = (uint64_t)d + 2;
        }
    }
#pragma unroll
    for (int w = 1; w < 64; w <<= 1) {
        const uint32_t ok = __shfl_up(k, w, 64), od = __shfl_up(d, w, 64);
        const uint64_t oe = __shfl_up((unsigned long long)e, w, 64), om = __shfl_up((unsigned long long)m, w, 64);
        const uint64_t og = __shfl_up((unsigned long long)g, w, 64);
        if ((int)lane >= w && ok == k) { e += oe; m += om; g += og; d = od > d ? od : d; }
    }
    const uint32_t nxt = __shfl_down(k, 1, 64);
    if (k != NONE_K && (lane == 63 || nxt != k)) {
        atomicAdd((unsigned long long *)&b.e[k], (unsigned long long)e);
        if (m) atomicAdd((unsigned long long *)&b.m[k], (unsigned long long)m);
        if (g) atomicAdd((unsigned long long *)&b.g[k], (unsigned long long)g);
        if (d) atomicMax(&b.d[k], d);
    }
}
__global__ __launch_bounds__(BLOCK) void k_cd_bounds(uint32_t nkeys, const uint32_t *__restrict__ kstart,
                                                     const uint32_t *__restrict__ src, uint32_t nk,
                                                     const uint32_t *__restrict__ snap_ent_off, BSum b,
                                                     uint64_t *__restrict__ ecap,
                                                     uint64_t *__restrict__ mcap, uint64_t *__restrict__ mmax,
                                                     uint64_t *__restrict__ dcap, uint32_t *__restrict__ ovf,
                                                     uint32_t hot_thr, int keep_hot, uint8_t *__restrict__ hot,
                                                     uint32_t *__restrict__ nhot)
{
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k >= nkeys) return;
    // a key with more than hot_thr items (snapshot entries + update pairs) takes the hot-key path (no lane working
    // space: a lane would copy a large snapshot alone); keep_hot: flags as left by the hot-key path (its irregular keys
    // cleared)
    if (!keep_hot) {
        const uint32_t q0 = kstart[k], v = src[q0];
        const uint64_t items = (uint64_t)(kstart[k + 1] - q0) - (v < nk ? 1u : 0u) +
                               (v < nk ? snap_ent_off[v + 1] - snap_ent_off[v] : 0u);
        hot[k] = items > hot_thr ? 1 : 0;
    }
    if (hot[k]) {
        ecap[k] = 0; mcap[k] = 0; mmax[k] = 0; dcap[k] = 1; ovf[k] = 0;
        atomicAdd(nhot, 1u);
        return;
    }
    const uint64_t e = b.e[k], m = b.m[k], d = b.d[k], grow = b.g[k];
    ecap[k] = e;
    // every missing[] entry is an uncommitted TxnId of the key held by an entry with info: at most e per entry, and an
    // update adds at most its deps + 2 to each entry
    const uint64_t sq = e * e, lin = m + e * grow, bound = sq < lin ? sq : lin, guess = m + 4 * e + 64;
    mmax[k] = bound;
    mcap[k] = guess < bound ? guess : bound;
    dcap[k] = d + 1;
    ovf[k] = 0;
}

// keys whose missing[] outgrew the guess: 4x, up to the proven bound (at the bound: an internal error); from the
// CD_GROW_STEPS-th regrow round on, straight to the bound, so a batch is replayed at most CD_GROW_STEPS + 2 times
constexpr uint32_t CD_GROW_STEPS = 2;
__global__ __launch_bounds__(BLOCK) void k_cd_grow(uint32_t nkeys, uint32_t *__restrict__ ovf, uint64_t *__restrict__ mcap,
                                                   const uint64_t *__restrict__ mmax, uint64_t *__restrict__ err,
                                                   uint32_t round)
{
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k >= nkeys || !ovf[k]) return;
    ovf[k] = 0;
    if (mcap[k] >= mmax[k]) { atomicOr((unsigned long long *)err, (unsigned long long)E_CAP); return; }
    const uint64_t g = round >= CD_GROW_STEPS ? mmax[k] : 4 * mcap[k];
    mcap[k] = g < mmax[k] ? g : mmax[k];
}

struct Pool {
    InfoP *e;
    Ts *m;
    const uint64_t *ecw, *mcw, *dcw;   // per wave of 64 keys: the largest entry / missing / deps capacity of its keys
    const uint64_t *eoffw, *toffw;     // exclusive scans over waves of 2 ecw and of 2 mcw + ecw + 2 dcw (per-lane units)
    const uint32_t *perm;              // slot -> key: keys ordered by entry capacity, so a wave's keys are alike in size
    uint32_t *kslot;                   // key -> slot
};

// slot k's working space (key p.perm[k]), interleaved with its wave's slots: entries A | B (2 ecw), then its Ts
// region: the new TxnInfo's missing[] (ecw), additions (dcw), insertMissing (dcw), then the A and B missing
// areas (mcw)
__device__ __forceinline__ void key_bufs(const Pool &p, uint32_t k, Work &w)
{
    const uint32_t wv = k / (uint32_t)CD_W, l = k % (uint32_t)CD_W;
    const uint64_t ec = p.ecw[wv], mc = p.mcw[wv], dc = p.dcw[wv];
    w.ecap = (uint32_t)ec;
    w.mcap = (uint32_t)mc;
    w.a.e = EP{ p.e + p.eoffw[wv] * CD_W + l };
    w.b.e = w.a.e + (long)ec;
    const SP<Ts> R{ p.m + p.toffw[wv] * CD_W + l };
    w.tmiss = R;
    w.adds = R + (long)ec;
    w.owned = w.adds + (long)dc;
    w.a.m = w.owned + (long)dc;
    w.b.m = w.a.m + (long)mc;
}

// slots in descending capacity: the waves with the longest replays start first (the short ones fill in behind them)
__global__ __launch_bounds__(BLOCK) void k_cd_rev(uint32_t nkeys, const uint32_t *__restrict__ in, uint32_t *__restrict__ out)
{
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k < nkeys) out[k] = in[nkeys - 1 - k];
}
// per wave of 64 keys: the largest capacities of its keys and the wave's per-lane region sizes
__global__ __launch_bounds__(BLOCK) void k_cd_wcap(uint32_t nkeys, const uint32_t *__restrict__ perm, uint32_t *__restrict__ kslot,
                                                   const uint64_t *__restrict__ ecap,
                                                   const uint64_t *__restrict__ mcap, const uint64_t *__restrict__ dcap,
                                                   uint64_t *__restrict__ ecw, uint64_t *__restrict__ mcw,
                                                   uint64_t *__restrict__ dcw, uint64_t *__restrict__ esz,
                                                   uint64_t *__restrict__ tsz)
{
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;   // slot
    const uint32_t key = k < nkeys ? perm[k] : 0u;
    if (k < nkeys) kslot[key] = k;
    uint64_t e = k < nkeys ? ecap[key] : 0, m = k < nkeys ? mcap[key] : 0, d = k < nkeys ? dcap[key] : 0;
#pragma unroll
    for (int x = 32; x >= 1; x >>= 1) {
        e = max(e, (uint64_t)__shfl_xor((unsigned long long)e, x, 64));
        m = max(m, (uint64_t)__shfl_xor((unsigned long long)m, x, 64));
        d = max(d, (uint64_t)__shfl_xor((unsigned long long)d, x, 64));
    }
    const uint32_t wv = k / (uint32_t)CD_W;
    if (lane_id() == 0 && (uint64_t)wv * CD_W < nkeys) {
        ecw[wv] = e; mcw[wv] = m; dcw[wv] = d;
        esz[wv] = 2 * e;
        tsz[wv] = 2 * m + e + 2 * d;
    }
}

// Each sorted (key, update) element's update fields gathered once into a 64-B record at its sorted position (pairs
// read in pair order, records scattered whole), so the replay reads one record per update instead of a chain of
// dependent loads (element -> update -> its columns, deps range). Snapshot elements' slots stay unwritten.
struct UpdRec {
    uint64_t im, il, xm, xl;
    int32_t in, xn;
    uint32_t st_fl;   // status | flags << 8
    uint32_t pad[3];
    uint32_t da, db;  // deps range (the record's last 8 bytes: k_cd_bounds reads them alone)
};
static_assert(sizeof(UpdRec) == 64, "64-B update record");
// the sorted position of every (update, key) pair
__global__ __launch_bounds__(BLOCK) void k_cd_inv(uint64_t T, const uint32_t *__restrict__ src, uint32_t nk,
                                                  uint32_t *__restrict__ qpos)
{
    const uint64_t q = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (q >= T) return;
    const uint32_t v = src[q];
    if (v >= nk) qpos[v - nk] = (uint32_t)q;
}
// thread per pair, in pair order (the update columns read nearly contiguously), record written at its sorted position
__global__ __launch_bounds__(BLOCK) void k_cd_urec(uint64_t NP, const uint32_t *__restrict__ qpos, Upd u,
                                                   UpdRec *__restrict__ rec)
{
    const uint64_t j = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (j >= NP) return;
    const uint32_t i = u.owner[j];
    UpdRec r;
    r.im = u.um[i]; r.il = u.ul[i]; r.in = u.un[i];
    r.xm = u.uxm[i]; r.xl = u.uxl[i]; r.xn = u.uxn[i];
    r.st_fl = (uint32_t)u.st[i] | ((uint32_t)u.fl[i] << 8);
    r.da = u.dep_off[j]; r.db = u.dep_off[j + 1];
    r.pad[0] = r.pad[1] = r.pad[2] = 0;
    rec[qpos[j]] = r;
}

// one lane per key: load the snapshot, replay its updates, record the final buffer and sizes
#ifdef CD_WPE
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(CD_WPE))) void k_cd_apply(
#else
__global__ __launch_bounds__(BLOCK) void k_cd_apply(
#endif
uint32_t nkeys, const uint32_t *__restrict__ kstart,
                                                    const uint32_t *__restrict__ src, const uint64_t *__restrict__ ecap,
                                                    const uint64_t *__restrict__ mcap, uint32_t nk, Snap s, Upd u, Pool p,
                                                    uint8_t *__restrict__ final_b, uint32_t *__restrict__ fin_n,
                                                    uint32_t *__restrict__ fin_m, uint32_t *__restrict__ ovf,
                                                    uint64_t *__restrict__ err, unsigned long long *__restrict__ paths,
                                                    const UpdRec *__restrict__ urec, const uint8_t *__restrict__ hot)
{
    const uint32_t slot = blockIdx.x * BLOCK + threadIdx.x;
    uint32_t n_fast = 0, n_rebuild = 0;
    auto count_paths = [&]() {   // per wave: in-place updates, full rebuilds (stats)
        unsigned long long f = n_fast, r = n_rebuild;
        for (int d = 32; d >= 1; d >>= 1) { f += __shfl_xor(f, d, 64); r += __shfl_xor(r, d, 64); }
        if (lane_id() == 0 && (f || r)) { atomicAdd(&paths[0], f); atomicAdd(&paths[1], r); }
    };
    if (slot >= nkeys || hot[p.perm[slot]]) { count_paths(); return; }
    const uint32_t k = p.perm[slot];
    Ctx c;
    c.err = 0;
    key_bufs(p, slot, c.w);   // the capacities of the wave (>= this key's own)
    const uint64_t dk = p.dcw[slot / (uint32_t)CD_W];
    // the current state and the next one by value (a pointer swap would put both in scratch memory)
    Buf A = c.w.a, B = c.w.b;
    bool in_a = true;
    A.n = 0; A.mtop = 0;
    Ctx::Sum sm{};
    bool sum_ok = false;
    uint32_t q0 = kstart[k];
    const uint32_t q1 = kstart[k + 1];
    if (const uint32_t v = src[q0]; v < nk) {   // the snapshot of this key: the first element of its run
        ++q0;
        {
            for (uint32_t x = s.ent_off[v]; x < s.ent_off[v + 1]; ++x) {
                Info y;
                y.id = Ts{ s.em[x], s.el[x], s.en[x] };
                y.ex = Ts{ s.xm[x], s.xl[x], s.xn[x] };
                y.self = cmp(y.ex, y.id) == 0;
                if (y.self) y.ex = y.id;
                y.st = s.st[x];
                y.ms = A.mtop;
                y.mn = s.miss_off[x + 1] - s.miss_off[x];
                if (!c.room_m(A, y.mn) || !c.room_e(A.n + 1)) break;
                for (uint32_t t = 0; t < y.mn; ++t) {
                    const uint32_t z = s.miss_off[x] + t;
                    A.m[A.mtop + t] = Ts{ s.mm[z], s.ml[z], s.mn[z] };
                }
                A.mtop += y.mn;
                c.put_e(A, y);
            }
        }
    }
    for (uint32_t q = q0; q < q1 && !c.err; ++q) {   // then its updates (one record each)
        const UpdRec ur = urec[q];
        const uint32_t st = ur.st_fl & 0xFFu, fl = ur.st_fl >> 8;
        if (st == 0xFF) continue;   // InternalStatus.from(saveStatus) == null: unchanged
        const Ts id{ ur.im, ur.il, ur.in }, ex{ ur.xm, ur.xl, ur.xn };
        // the command's keyDeps.txnIds(key), read in place; computeInfoAndAdditions copies the additions out (their
        // area and the insertMissing area hold at most dk entries each)
        const uint32_t da = ur.da, db = ur.db;
        if (db - da > dk) { c.err |= E_CAP; break; }
        const DepsIn deps{ u.dm + da, u.dl + da, u.dn + da };
        if (!sum_ok) { c.sum_of(A, sm); sum_ok = true; }
        const int r = c.apply(A, B, id, ex, st, fl, deps, db - da, sm);
        n_fast += r == 2;
        n_rebuild += r == 1;
        if (r == 1) {
            const Buf t = A; A = B; B = t;
            in_a = !in_a;
            sum_ok = false;   // recomputed before the next update
        }
    }
    final_b[k] = in_a ? 0 : 1;
    fin_n[k] = A.n;
    fin_m[k] = A.mtop;
    if (c.err & E_MCAP) { ovf[k] = 1; c.err = E_MCAP; }   // anything else this key reports shows again on the replay
    if (c.err) atomicOr((unsigned long long *)err, (unsigned long long)c.err);
    count_paths();
}

// output: keys with entries, their entry counts
__global__ __launch_bounds__(BLOCK) void k_cd_out1(uint32_t nkeys, const uint32_t *__restrict__ fin_n, uint32_t *__restrict__ keep)
{
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k < nkeys) keep[k] = fin_n[k] ? 1u : 0u;
}

// the kept keys' codes and entry offsets (eall: exclusive scan of the entry counts over every key)
__global__ __launch_bounds__(BLOCK) void k_cd_out2(uint32_t nkeys, const uint32_t *__restrict__ keep, const uint32_t *__restrict__ kpos,
                                                   const uint32_t *__restrict__ kstart, const uint64_t *__restrict__ sk,
                                                   uint64_t kbase, const uint32_t *__restrict__ eall, uint64_t *__restrict__ okey,
                                                   uint32_t *__restrict__ ent_off, uint32_t nko, uint32_t ne,
                                                   uint32_t *__restrict__ kkey)
{
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k == 0) ent_off[nko] = ne;
    if (k >= nkeys || !keep[k]) return;
    okey[kpos[k]] = sk[kstart[k]] + kbase;
    ent_off[kpos[k]] = eall[k];
    kkey[kpos[k]] = k;
}

struct Out {
    uint64_t *em, *el, *xm, *xl, *mm, *ml;
    int32_t *en, *xn, *mn;
    uint8_t *st;
    uint32_t *ent_off, *mcnt, *miss_off;
};

// entries of every kept key and each entry's missing count, a thread per output entry (its key by a search of the kept
// keys' offsets): the column writes coalesce
__global__ __launch_bounds__(BLOCK) void k_cd_out3e(uint32_t ne, uint32_t nko, const uint32_t *__restrict__ kkey, Pool p,
                                                    const uint8_t *__restrict__ final_b, Out o, const uint8_t *__restrict__ hot)
{
    const uint32_t e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= ne) return;
    uint32_t lo = 0, hi = nko;   // last kept key whose entries start at or before e
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (o.ent_off[mid] <= e) lo = mid; else hi = mid;
    }
    const uint32_t k = kkey[lo];
    if (hot[k]) return;   // (k_ch_out3)
    Work w;
    key_bufs(p, p.kslot[k], w);
    const Info x = (final_b[k] ? w.b.e : w.a.e).get(e - o.ent_off[lo]);
    o.em[e] = x.id.m; o.el[e] = x.id.l; o.en[e] = x.id.n;
    o.xm[e] = x.ex.m; o.xl[e] = x.ex.l; o.xn[e] = x.ex.n;
    o.st[e] = (uint8_t)x.st;
    o.mcnt[e] = x.mn;
}

__global__ __launch_bounds__(BLOCK) void k_cd_out4(uint32_t nkeys, const uint32_t *__restrict__ keep, const uint32_t *__restrict__ kpos,
                                                   const uint64_t *__restrict__ ecap, const uint64_t *__restrict__ mcap, Pool p,
                                                   const uint8_t *__restrict__ final_b, Out o, const uint8_t *__restrict__ hot)
{
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;   // key order: a wave's lanes write adjacent output runs
    if (k >= nkeys || !keep[k] || hot[k]) return;
    Work w;
    key_bufs(p, p.kslot[k], w);
    const Buf &F = final_b[k] ? w.b : w.a;
    const uint32_t base = o.ent_off[kpos[k]], n = o.ent_off[kpos[k] + 1] - base;
    for (uint32_t i = 0; i < n; ++i) {
        const Info x = F.e.get(i);
        uint32_t dst = o.miss_off[base + i];
        for (uint32_t q = 0; q < x.mn; ++q, ++dst) {
            const Ts &t = F.m[x.ms + q];
            o.mm[dst] = t.m; o.ml[dst] = t.l; o.mn[dst] = t.n;
        }
    }
}

__global__ __launch_bounds__(BLOCK) void k_cd_widen(uint32_t n, const uint32_t *__restrict__ in, uint64_t *__restrict__ out)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) out[i] = in[i];
}

// ---- hot keys: the replay's closed form, data-parallel over a key's updates
// A key with more than acc_opts.cfk_hot (default 64) updates in the batch is not replayed by one lane: its final state is
// computed from the update stream directly. Its TxnInfos are every TxnId its snapshot, its updates or their deps name
// (a dep the key lacks becomes a TRANSITIVELY_KNOWN entry, updateOrInsertWithAdditions :772-863); each takes the status /
// executeAt of its last update that changed it (update :657-706: stale checks, unchanged returns). The missing[] of an
// entry X with info then follows from the reference's edits, which only ever add an uncommitted TxnId t below
// max(TxnId, depsKnownBefore) of X that X witnesses (computeInfoAndAdditions :1071-1150, insertInfoAndOneMissing :899-944,
// mergeAndFilterMissing :988-1025) and remove t when it commits (removeMissing :946-972):
//   X last computed in this batch, with deps D:  { t uncommitted at the end, t != X, t < bound(X), X witnesses t } \ D
//   X's info from the snapshot:  (snapshot missing[] \ TxnIds committed in this batch)
//                                u { t new in this batch, uncommitted at the end, t < bound(X), X witnesses t }
// Statuses only rise, so "uncommitted at the end" is "uncommitted whenever X looked". The shapes the closed form does not
// cover -- a status going back (AcceptedInvalidate), executeAt below its TxnId, a dep at or above depsKnownBefore or equal
// to the txn, depsKnownBefore equal to an entry, two encodings of one TxnId -- mark the key irregular: it is replayed by
// the lane path instead (which also reports the reference's errors exactly).
constexpr uint32_t NONE = 0xFFFFFFFFu;
static_assert(NONE == NONE_K, "one sentinel");
constexpr uint32_t CH_DEFAULT_HOT = 64;
enum : uint8_t { HI_SNAP = 0, HI_PAIR = 1, HI_TK = 2 };
enum : uint8_t { HF_CROSSED = 1, HF_NEW = 2 };

struct HG {   // one (key, TxnId) group: the entry it becomes
    uint64_t im, il, xm, xl;
    int32_t in, xn;
    uint32_t info_q;   // pair of the last recompute (its deps), NONE: none in this batch
    uint32_t snap_x;   // snapshot entry, NONE: new
    uint32_t h;
    uint8_t st, self, present, flags;
    uint32_t pad[2];
};
static_assert(sizeof(HG) == 64, "64-B group record");

__device__ __forceinline__ Ts hg_id(const HG &g) { return Ts{ g.im, g.il, g.in }; }
__device__ __forceinline__ Ts hg_bound(const HG &g)   // depsKnownBefore (>= the TxnId on a regular key)
{
    return (g.st == PRE || g.st == ACC || g.self) ? Ts{ g.im, g.il, g.in } : Ts{ g.xm, g.xl, g.xn };
}

// per hot key: its item count (snapshot entries + pairs) and whether its run starts with the snapshot element
__global__ __launch_bounds__(BLOCK) void k_ch_count(uint32_t nh, const uint32_t *__restrict__ hk, const uint32_t *__restrict__ kstart,
                                                    const uint32_t *__restrict__ src, uint32_t nk, Snap s,
                                                    uint32_t *__restrict__ icnt, uint32_t *__restrict__ nsnap, uint8_t *__restrict__ hsnap)
{
    const uint32_t h = blockIdx.x * BLOCK + threadIdx.x;
    if (h >= nh) return;
    const uint32_t k = hk[h], q0 = kstart[k], q1 = kstart[k + 1];
    const uint32_t v = src[q0];
    const bool sn = v < nk;
    const uint32_t ne = sn ? s.ent_off[v + 1] - s.ent_off[v] : 0u;
    nsnap[h] = ne;
    hsnap[h] = sn ? 1 : 0;
    icnt[h] = ne + (q1 - q0) - (sn ? 1u : 0u);
}

struct HItems {
    uint64_t *im, *il, *inode;   // TxnId words (node biased for the dense rank)
    uint32_t *ih, *isrc;
    uint8_t *ikind;
};

// every item of the hot keys: their snapshot entries, then their pairs in batch order
__global__ __launch_bounds__(BLOCK) void k_ch_items(uint64_t NI, uint32_t nh, const uint32_t *__restrict__ ioff,
                                                    const uint32_t *__restrict__ hk, const uint32_t *__restrict__ nsnap,
                                                    const uint8_t *__restrict__ hsnap, const uint32_t *__restrict__ kstart,
                                                    const uint32_t *__restrict__ src, Snap s, const UpdRec *__restrict__ urec,
                                                    HItems it)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= NI) return;
    uint32_t lo = 0, hi = nh;   // last h with ioff[h] <= i
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (ioff[mid] <= i) lo = mid; else hi = mid;
    }
    const uint32_t h = lo, r = (uint32_t)(i - ioff[h]), k = hk[h], q0 = kstart[k];
    uint64_t m, l;
    int32_t n;
    if (r < nsnap[h]) {
        const uint32_t x = s.ent_off[src[q0]] + r;
        m = s.em[x]; l = s.el[x]; n = s.en[x];
        it.isrc[i] = x;
        it.ikind[i] = HI_SNAP;
    } else {
        const uint32_t q = q0 + hsnap[h] + (r - nsnap[h]);
        const UpdRec &u = urec[q];
        m = u.im; l = u.il; n = u.in;
        it.isrc[i] = q;
        it.ikind[i] = HI_PAIR;
    }
    it.im[i] = m; it.il[i] = l; it.inode[i] = (uint32_t)n ^ 0x80000000u;
    it.ih[i] = h;
}

// sort keys: (hot key, TxnId rank); group starts
__global__ __launch_bounds__(BLOCK) void k_ch_skey(uint64_t NI, const uint32_t *__restrict__ ih, const uint32_t *__restrict__ rank,
                                                   int rb, uint64_t *__restrict__ key)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < NI) key[i] = ((uint64_t)ih[i] << rb) | rank[i];
}
__global__ __launch_bounds__(BLOCK) void k_ch_gflag(uint64_t NI, const uint64_t *__restrict__ sk, uint32_t *__restrict__ f)
{
    const uint64_t p = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p < NI) f[p] = (p == 0 || sk[p] != sk[p - 1]) ? 1u : 0u;
}
__global__ __launch_bounds__(BLOCK) void k_ch_gstart(uint64_t NI, const uint32_t *__restrict__ f, const uint32_t *__restrict__ fi,
                                                     uint32_t ng, uint32_t *__restrict__ gstart)
{
    const uint64_t p = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p < NI && f[p]) gstart[fi[p] - 1] = (uint32_t)p;
    if (p == 0) gstart[ng] = (uint32_t)NI;
}

// one thread per group: its items in time order through update's status rules (:657-706)
__global__ __launch_bounds__(BLOCK) void k_ch_walk(uint32_t ng, const uint32_t *__restrict__ gstart, const uint32_t *__restrict__ perm,
                                                   HItems it, Snap s, const UpdRec *__restrict__ urec, HG *__restrict__ G,
                                                   uint8_t *__restrict__ mention, uint32_t *__restrict__ irr,
                                                   uint64_t *__restrict__ err)
{
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g >= ng) return;
    const uint32_t p0 = gstart[g], p1 = gstart[g + 1];
    const uint32_t i0 = perm[p0];
    const Ts id{ it.im[i0], it.il[i0], (int32_t)(uint32_t)(it.inode[i0] ^ 0x80000000u) };
    const uint32_t h = it.ih[i0];
    bool present = false, crossed = false, isnew = true, bad = false;
    uint32_t st = TK, self = 1, info_q = NONE, snap_x = NONE;
    Ts ex = id;
    uint64_t e = 0;
    for (uint32_t p = p0; p < p1 && !e; ++p) {
        const uint32_t i = perm[p];
        mention[p] = 0;
        if (it.il[i] != id.l) bad = true;   // two encodings of one TxnId
        const uint8_t kd = it.ikind[i];
        if (kd == HI_SNAP) {
            const uint32_t x = it.isrc[i];
            present = true; isnew = false; snap_x = x;
            st = s.st[x];
            ex = Ts{ s.xm[x], s.xl[x], s.xn[x] };
            self = cmp(ex, id) == 0;
            if (self) ex = id;
        } else if (kd == HI_TK) {
            if (!present) { present = true; st = TK; ex = id; self = 1; }
        } else {
            const UpdRec u = urec[it.isrc[i]];
            const uint32_t sn = u.st_fl & 0xFFu, fl = u.st_fl >> 8;
            if (sn == 0xFF) continue;
            if (present) {
                if (sn <= st) {
                    if (st != sn && !(fl & 2u)) { e |= E_STALE; break; }
                    if (!has_info(sn) || !(fl & 1u)) continue;
                    if (sn < st) bad = true;   // AcceptedInvalidate taking the status back
                }
                if (st < COMMITTED && sn >= COMMITTED) crossed = true;
            }
            present = true;
            st = sn;
            if (has_info(sn)) {
                ex = Ts{ u.xm, u.xl, u.xn };
                self = cmp(ex, id) == 0;
                if (self) ex = id;
                info_q = it.isrc[i];
                mention[p] = 1;
            } else {
                ex = id; self = 1; info_q = NONE;
            }
        }
    }
    // executeAt below the TxnId: the reference's edits then differ by position (no depsKnownBefore test after it)
    if (present && has_info(st) && !(st == PRE || st == ACC || self) && cmp(ex, id) < 0) bad = true;
    HG r;
    r.im = id.m; r.il = id.l; r.in = id.n;
    r.xm = ex.m; r.xl = ex.l; r.xn = ex.n;
    r.info_q = info_q; r.snap_x = snap_x; r.h = h;
    r.st = (uint8_t)st; r.self = (uint8_t)self; r.present = present ? 1 : 0;
    r.flags = (crossed ? HF_CROSSED : 0) | (isnew ? HF_NEW : 0);
    r.pad[0] = r.pad[1] = 0;
    G[g] = r;
    if (bad) irr[h] = 1;
    if (e) atomicOr((unsigned long long *)err, (unsigned long long)e);
}

// each hot key's first group (groups are in hot-key order; every hot key has one)
__global__ __launch_bounds__(BLOCK) void k_ch_gofs(uint32_t ng, uint32_t nh, const HG *__restrict__ G, uint32_t *__restrict__ gofs,
                                                   uint32_t *__restrict__ pflag)
{
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g < ng) {
        if (g == 0 || G[g].h != G[g - 1].h) gofs[G[g].h] = g;
        pflag[g] = G[g].present;
    }
    if (g == 0) gofs[nh] = ng;
}
// entries (the present groups) -> group; each hot key's first entry
__global__ __launch_bounds__(BLOCK) void k_ch_entries(uint32_t ng, uint32_t nh, uint32_t ne, const HG *__restrict__ G,
                                                      const uint32_t *__restrict__ pexcl, const uint32_t *__restrict__ gofs,
                                                      uint32_t *__restrict__ eg, uint32_t *__restrict__ eoff)
{
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g < ng && G[g].present) eg[pexcl[g]] = g;
    if (g <= nh) eoff[g] = g == nh ? ne : pexcl[gofs[g]];
}
// entries still uncommitted (missing[] candidates), and each hot key's first one
// newonly: only the entries new in this batch (the TxnIds a snapshot entry's missing[] may gain)
__global__ __launch_bounds__(BLOCK) void k_ch_uflag(uint32_t ne, const uint32_t *__restrict__ eg, const HG *__restrict__ G,
                                                    int newonly, uint32_t *__restrict__ uflag)
{
    const uint32_t e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= ne) return;
    const HG &g = G[eg[e]];
    uflag[e] = g.st < COMMITTED && (!newonly || (g.flags & HF_NEW)) ? 1u : 0u;
}
struct UR {   // an uncommitted entry, as the missing[] walks read it
    uint64_t m, l;
    int32_t n;
    uint32_t flags;
};
__global__ __launch_bounds__(BLOCK) void k_ch_ulist(uint32_t ne, uint32_t nh, uint32_t nu, const uint32_t *__restrict__ uflag,
                                                    const uint32_t *__restrict__ uexcl, const uint32_t *__restrict__ eoff,
                                                    const uint32_t *__restrict__ eg, const HG *__restrict__ G,
                                                    UR *__restrict__ ulist, uint32_t *__restrict__ uoff)
{
    const uint32_t e = blockIdx.x * BLOCK + threadIdx.x;
    if (e < ne && uflag[e]) {
        const HG &g = G[eg[e]];
        ulist[uexcl[e]] = UR{ g.im, g.il, g.in, g.flags };
    }
    if (e <= nh) uoff[e] = e == nh ? nu : (eoff[e] < ne ? uexcl[eoff[e]] : nu);
}

// the first entry >= t in [lo, e1): galloping from lo (a sorted run of TxnIds looked up in order moves a few steps)
__device__ __forceinline__ uint32_t ch_lower(const uint32_t *__restrict__ eg, const HG *__restrict__ G, uint32_t lo, uint32_t e1,
                                             const Ts &t)
{
    uint32_t hi = lo, step = 1;
    while (hi < e1 && cmp(hg_id(G[eg[hi]]), t) < 0) {
        lo = hi + 1;
        hi = lo + step < e1 ? lo + step : e1;
        step <<= 1;
    }
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (cmp(hg_id(G[eg[mid]]), t) < 0) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// the first entry >= t in [e0, hi]: galloping down from hi (t a little below the entry at hi)
__device__ __forceinline__ uint32_t ch_lower_back(const uint32_t *__restrict__ eg, const HG *__restrict__ G, uint32_t e0, uint32_t hi,
                                                  const Ts &t)
{
    uint32_t lo = hi, step = 1;   // invariant: entries at and after hi are >= t (or hi is the end)
    while (lo > e0 && cmp(hg_id(G[eg[lo - 1]]), t) >= 0) {
        hi = lo - 1;
        lo = hi - e0 > step ? hi - step : e0;
        step <<= 1;
    }
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (cmp(hg_id(G[eg[mid]]), t) < 0) lo = mid + 1; else hi = mid;
    }
    return lo;
}
// every recompute's deps: a dep the key does not hold becomes a TRANSITIVELY_KNOWN item (pass 1 counts, pass 2 writes);
// the shapes outside the closed form mark the key irregular. The lookups start at the txn's own entry (its deps sit
// just below it, its executeAt just above)
__global__ __launch_bounds__(BLOCK) void k_ch_mention(uint64_t NI, const uint8_t *__restrict__ mention, const uint32_t *__restrict__ perm,
                                                     HItems it, const UpdRec *__restrict__ urec, Upd u, const uint32_t *__restrict__ eg,
                                                     const HG *__restrict__ G, const uint32_t *__restrict__ gincl,
                                                     const uint32_t *__restrict__ pexcl, const uint32_t *__restrict__ eoff,
                                                     uint32_t *__restrict__ irr, uint32_t *__restrict__ nextra, uint64_t cap,
                                                     HItems xo)
{
    const uint64_t p = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p >= NI || !mention[p]) return;
    const uint32_t i = perm[p], h = it.ih[i];
    const UpdRec r = urec[it.isrc[i]];
    const uint32_t st = r.st_fl & 0xFFu;
    const Ts id{ r.im, r.il, r.in }, ex{ r.xm, r.xl, r.xn };
    const bool self = st == PRE || st == ACC || cmp(ex, id) == 0;
    const Ts bound = self ? id : ex;
    const uint32_t e0 = eoff[h], e1 = eoff[h + 1], own = pexcl[gincl[p] - 1];
    bool bad = false;
    if (!self) {
        if (cmp(ex, id) < 0) bad = true;
        else {
            const uint32_t x = ch_lower(eg, G, own, e1, ex);
            if (x < e1 && cmp(hg_id(G[eg[x]]), ex) == 0) bad = true;
        }
    }
    // deps are sorted: the first one galloping down from the txn's entry, each next one on from the previous
    uint32_t at = r.db > r.da && !bad ? ch_lower_back(eg, G, e0, own, Ts{ u.dm[r.da], u.dl[r.da], u.dn[r.da] }) : e0;
    for (uint32_t d = r.da; d < r.db && !bad; ++d) {
        const Ts t{ u.dm[d], u.dl[d], u.dn[d] };
        if (cmp(t, bound) >= 0 || cmp(t, id) == 0) { bad = true; break; }
        at = ch_lower(eg, G, at, e1, t);
        if (at < e1 && cmp(hg_id(G[eg[at]]), t) == 0) { ++at; continue; }
        const uint32_t w = atomicAdd(nextra, 1u);
        if (w < cap) {
            xo.im[w] = t.m; xo.il[w] = t.l; xo.inode[w] = (uint32_t)t.n ^ 0x80000000u;
            xo.ih[w] = h; xo.isrc[w] = NONE; xo.ikind[w] = HI_TK;
        }
    }
    if (bad) irr[h] = 1;
}

// the closed-form missing[] of entry e (count only when out is null)
// The (hot key, TxnId) groups that crossed to committed in this batch, as an open-addressing hash set (32-B slots): a
// snapshot missing[] TxnId is dropped when its group crossed (removeMissing, CommandsForKey.java:946-972), one probe per
// element instead of a binary search over the key's entries (a hot key holds ~10^6: ~40 dependent loads)
struct XSet {
    ulonglong4 *slot;   // (msb, lsb & IDENTITY_LSB, node << 32 | hot key, used)
    uint32_t mask;      // 0: the set is empty (no lookups)
};
__device__ __forceinline__ uint32_t xs_hash(uint32_t h, uint64_t m, uint64_t l, int32_t n)
{
    uint64_t x = m * 0x9E3779B97F4A7C15ull ^ (l & IDENTITY_LSB) ^ ((uint64_t)(uint32_t)n << 40) ^ ((uint64_t)h << 20);
    x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 29; x *= 0x94D049BB133111EBull; x ^= x >> 32;
    return (uint32_t)x;
}
__global__ __launch_bounds__(BLOCK) void k_ch_xcount(uint32_t ng, const HG *__restrict__ G, uint32_t *__restrict__ cnt)
{
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    const bool x = g < ng && (G[g].flags & HF_CROSSED);
    const uint64_t b = __ballot(x);
    if (lane_id() == 0 && b) atomicAdd(cnt, (uint32_t)__popcll(b));
}
__global__ __launch_bounds__(BLOCK) void k_ch_xbuild(uint32_t ng, const HG *__restrict__ G, XSet xs)
{
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g >= ng || !(G[g].flags & HF_CROSSED)) return;
    const HG &X = G[g];
    const uint64_t l = X.il & IDENTITY_LSB;
    for (uint32_t i = xs_hash(X.h, X.im, l, X.in) & xs.mask;; i = (i + 1) & xs.mask)
        if (atomicCAS((unsigned long long *)&xs.slot[i].w, 0ull, 1ull) == 0ull) {
            xs.slot[i].x = X.im; xs.slot[i].y = l; xs.slot[i].z = ((uint64_t)(uint32_t)X.in << 32) | X.h;
            return;
        }
}
__device__ __forceinline__ bool xs_has(const XSet &xs, uint32_t h, const Ts &t)
{
    if (!xs.mask) return false;
    const uint64_t l = t.l & IDENTITY_LSB, z = ((uint64_t)(uint32_t)t.n << 32) | h;
    for (uint32_t i = xs_hash(h, t.m, l, t.n) & xs.mask;; i = (i + 1) & xs.mask) {
        const ulonglong4 e = xs.slot[i];
        if (e.w == 0) return false;
        if (e.x == t.m && e.y == l && e.z == z) return true;
    }
}

struct NewList {   // per hot key, its uncommitted entries new in this batch
    const UR *list;
    const uint32_t *off;
};
__device__ __forceinline__ uint32_t ur_lower(const UR *__restrict__ l, uint32_t lo, uint32_t hi, const Ts &t)
{
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (cmp(Ts{ l[mid].m, l[mid].l, l[mid].n }, t) < 0) lo = mid + 1; else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ uint32_t ch_missing(uint32_t e, const uint32_t *__restrict__ eg, const HG *__restrict__ G,
                                               const uint32_t *__restrict__ eoff, const UR *__restrict__ ulist,
                                               const uint32_t *__restrict__ uoff, const UpdRec *__restrict__ urec, Upd u, Snap s,
                                               const XSet &xs, const NewList &nl, uint64_t *om, uint64_t *ol, int32_t *on)
{
    const HG X = G[eg[e]];
    if (!has_info(X.st)) return 0;
    const Ts id = hg_id(X), bound = hg_bound(X);
    const uint32_t wm = witnesses_mask(kind(id));
    const uint32_t h = X.h;
    uint32_t n = 0;
    auto put = [&](const UR &t) {
        if (om) { om[n] = t.m; ol[n] = t.l; on[n] = t.n; }
        ++n;
    };
    if (X.info_q != NONE) {   // computed in this batch: the uncommitted entries below the bound, less its deps
        const uint32_t u0 = uoff[h], ub = ur_lower(ulist, u0, uoff[h + 1], bound);
        const UpdRec r = urec[X.info_q];
        uint32_t d = r.da;
        for (uint32_t k = u0; k < ub; ++k) {
            const UR t = ulist[k];
            const Ts tid{ t.m, t.l, t.n };
            if (cmp(tid, id) == 0 || !((wm >> kind(tid)) & 1u)) continue;
            while (d < r.db && cmp(Ts{ u.dm[d], u.dl[d], u.dn[d] }, tid) < 0) ++d;
            if (d < r.db && cmp(Ts{ u.dm[d], u.dl[d], u.dn[d] }, tid) == 0) continue;
            put(t);
        }
        return n;
    }
    if (X.snap_x == NONE) return 0;
    // the snapshot's missing[] (less the TxnIds committed in this batch) merged with the new uncommitted entries below
    // the bound (a list of the new ones only: walking every uncommitted entry of a hot key per snapshot entry was the
    // cost)
    const uint32_t m0 = s.miss_off[X.snap_x], m1 = s.miss_off[X.snap_x + 1];
    const uint32_t ub = ur_lower(nl.list, nl.off[h], nl.off[h + 1], bound);
    uint32_t a = m0, k = nl.off[h];
    const UR *ulist_n = nl.list;
    auto next_new = [&]() {
        while (k < ub) {
            const UR &t = ulist_n[k];
            const Ts tid{ t.m, t.l, t.n };
            if (cmp(tid, id) != 0 && ((wm >> kind(tid)) & 1u)) return;
            ++k;
        }
    };
    auto next_snap = [&]() {   // (skips the snapshot TxnIds whose group on this key crossed to committed)
        while (a < m1 && xs_has(xs, h, Ts{ s.mm[a], s.ml[a], s.mn[a] })) ++a;
    };
    next_new();
    next_snap();
    while (a < m1 || k < ub) {
        int c;
        if (a == m1) c = 1;
        else if (k == ub) c = -1;
        else c = cmp(Ts{ s.mm[a], s.ml[a], s.mn[a] }, Ts{ ulist_n[k].m, ulist_n[k].l, ulist_n[k].n });
        if (c <= 0) {
            if (om) { om[n] = s.mm[a]; ol[n] = s.ml[a]; on[n] = s.mn[a]; }
            ++n;
            ++a;
            if (c == 0) ++k;
        } else {
            put(ulist_n[k]);
            ++k;
        }
        next_new();
        next_snap();
    }
    return n;
}
// count (EMIT false) or write the missing[] of every entry. An entry computed in this batch whose uncommitted range is
// long (a hot key's late entries: thousands) is walked by the whole wave, lanes side by side over the range (a ballot
// compacts the kept TxnIds, deps looked up by search); the others by their own lane
constexpr uint32_t CH_LONG = 32;
template <bool EMIT>
__global__ __launch_bounds__(BLOCK) void k_ch_miss(uint32_t ne, const uint32_t *__restrict__ eg, const HG *__restrict__ G,
                                                   const uint32_t *__restrict__ eoff, const UR *__restrict__ ulist,
                                                   const uint32_t *__restrict__ uoff, const UpdRec *__restrict__ urec, Upd u,
                                                   Snap s, XSet xs, NewList nl, uint32_t *__restrict__ mcnt,
                                                   const uint32_t *__restrict__ moff, uint64_t *__restrict__ mm,
                                                   uint64_t *__restrict__ ml, int32_t *__restrict__ mn)
{
    const uint32_t e = blockIdx.x * BLOCK + threadIdx.x, lane = lane_id();
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    bool lng = false, lsn = false;
    uint32_t u0 = 0, ub = 0, da = 0, db = 0, wm = 0, out = 0, h = 0;
    Ts id{ 0, 0, 0 };
    if (e < ne) {
        const HG X = G[eg[e]];
        if (has_info(X.st) && X.info_q != NONE) {
            id = hg_id(X);
            const Ts bound = hg_bound(X);
            u0 = uoff[X.h];
            ub = ur_lower(ulist, u0, uoff[X.h + 1], bound);
            lng = ub - u0 >= CH_LONG;
            const UpdRec r = urec[X.info_q];
            da = r.da; db = r.db;
            wm = witnesses_mask(kind(id));
            if (EMIT) out = moff[e];
        } else if (has_info(X.st) && X.snap_x != NONE) {
            // a snapshot entry with a long missing[] and no new uncommitted TxnId below its bound (an old entry of a hot
            // key): its list less the crossed TxnIds, filtered by the whole wave
            const uint32_t m0 = s.miss_off[X.snap_x], m1 = s.miss_off[X.snap_x + 1];
            const uint32_t n0 = nl.off[X.h];
            if (m1 - m0 >= CH_LONG && ur_lower(nl.list, n0, nl.off[X.h + 1], hg_bound(X)) == n0) {
                lsn = true;
                u0 = m0; ub = m1; h = X.h;
                if (EMIT) out = moff[e];
            }
        }
        if (!lng && !lsn) {
            if (EMIT) ch_missing(e, eg, G, eoff, ulist, uoff, urec, u, s, xs, nl, mm + moff[e], ml + moff[e], mn + moff[e]);
            else mcnt[e] = ch_missing(e, eg, G, eoff, ulist, uoff, urec, u, s, xs, nl, nullptr, nullptr, nullptr);
        }
    }
    for (uint64_t todo = __ballot(lng); todo; todo &= todo - 1) {
        const int src = __builtin_ctzll(todo);
        const uint32_t a = __shfl(u0, src, 64), z = __shfl(ub, src, 64), d0 = __shfl(da, src, 64), d1 = __shfl(db, src, 64);
        const uint32_t w = __shfl(wm, src, 64), o0 = __shfl(out, src, 64);
        const Ts x{ (uint64_t)__shfl((unsigned long long)id.m, src, 64), (uint64_t)__shfl((unsigned long long)id.l, src, 64),
                    __shfl(id.n, src, 64) };
        uint32_t n = 0;
        for (uint32_t base = a; base < z; base += 64) {
            const uint32_t k = base + lane;
            bool keep = false;
            UR t{};
            if (k < z) {
                t = ulist[k];
                const Ts tid{ t.m, t.l, t.n };
                keep = cmp(tid, x) != 0 && ((w >> kind(tid)) & 1u);
                if (keep) {   // not among the deps (sorted)
                    uint32_t lo = d0, hi = d1;
                    while (lo < hi) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (cmp(Ts{ u.dm[mid], u.dl[mid], u.dn[mid] }, tid) < 0) lo = mid + 1; else hi = mid;
                    }
                    if (lo < d1 && cmp(Ts{ u.dm[lo], u.dl[lo], u.dn[lo] }, tid) == 0) keep = false;
                }
            }
            const uint64_t kb = __ballot(keep);
            if (EMIT && keep) {
                const uint32_t q = o0 + n + (uint32_t)__popcll(kb & lt);
                mm[q] = t.m; ml[q] = t.l; mn[q] = t.n;
            }
            n += (uint32_t)__popcll(kb);
        }
        if (!EMIT && lane == (uint32_t)src) mcnt[e] = n;
    }
    for (uint64_t todo = __ballot(lsn); todo; todo &= todo - 1) {
        const int src = __builtin_ctzll(todo);
        const uint32_t a = __shfl(u0, src, 64), z = __shfl(ub, src, 64), hk = __shfl(h, src, 64), o0 = __shfl(out, src, 64);
        uint32_t n = 0;
        for (uint32_t base = a; base < z; base += 64) {
            const uint32_t j = base + lane;
            bool keep = false;
            Ts t{ 0, 0, 0 };
            if (j < z) {
                t = Ts{ s.mm[j], s.ml[j], s.mn[j] };
                keep = !xs_has(xs, hk, t);
            }
            const uint64_t kb = __ballot(keep);
            if (EMIT && keep) {
                const uint32_t q = o0 + n + (uint32_t)__popcll(kb & lt);
                mm[q] = t.m; ml[q] = t.l; mn[q] = t.n;
            }
            n += (uint32_t)__popcll(kb);
        }
        if (!EMIT && lane == (uint32_t)src) mcnt[e] = n;
    }
}
// the hot keys' final entry counts (the lane path's fin_n), and the irregular ones back to the lane path
__global__ __launch_bounds__(BLOCK) void k_ch_fin(uint32_t nh, const uint32_t *__restrict__ hk, const uint32_t *__restrict__ eoff,
                                                  const uint32_t *__restrict__ irr, uint32_t *__restrict__ fin_n,
                                                  uint8_t *__restrict__ hot, uint32_t *__restrict__ nirr)
{
    const uint32_t h = blockIdx.x * BLOCK + threadIdx.x;
    if (h >= nh) return;
    if (irr[h]) { hot[hk[h]] = 0; atomicAdd(nirr, 1u); }
    else fin_n[hk[h]] = eoff[h + 1] - eoff[h];
}
// output: the hot keys' entries and missing[] into the key-major layout
__global__ __launch_bounds__(BLOCK) void k_ch_out3(uint32_t ne, const uint32_t *__restrict__ eg, const HG *__restrict__ G,
                                                   const uint32_t *__restrict__ eoff, const uint32_t *__restrict__ hk,
                                                   const uint32_t *__restrict__ kpos, const uint32_t *__restrict__ mcnt, Out o)
{
    const uint32_t e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= ne) return;
    const HG X = G[eg[e]];
    const uint32_t dst = o.ent_off[kpos[hk[X.h]]] + (e - eoff[X.h]);
    o.em[dst] = X.im; o.el[dst] = X.il; o.en[dst] = X.in;
    o.xm[dst] = X.xm; o.xl[dst] = X.xl; o.xn[dst] = X.xn;
    o.st[dst] = X.st;
    o.mcnt[dst] = mcnt[e];
}
// a thread per missing[] TxnId (its entry by a search of the offsets): the copies stay coalesced whatever the lengths
__global__ __launch_bounds__(BLOCK) void k_ch_out4(uint64_t nm, uint32_t ne, const uint32_t *__restrict__ eg, const HG *__restrict__ G,
                                                   const uint32_t *__restrict__ eoff, const uint32_t *__restrict__ hk,
                                                   const uint32_t *__restrict__ kpos, const uint32_t *__restrict__ moff,
                                                   const uint64_t *__restrict__ mm, const uint64_t *__restrict__ ml,
                                                   const int32_t *__restrict__ mn, Out o)
{
    const uint64_t q = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (q >= nm) return;
    uint32_t lo = 0, hi = ne;   // last e with moff[e] <= q
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (moff[mid] <= q) lo = mid; else hi = mid;
    }
    const uint32_t e = lo, h = G[eg[e]].h;
    const uint32_t pos = o.ent_off[kpos[hk[h]]] + (e - eoff[h]);
    const uint32_t dst = o.miss_off[pos] + (uint32_t)(q - moff[e]);
    o.mm[dst] = mm[q]; o.ml[dst] = ml[q]; o.mn[dst] = mn[q];
}

__global__ __launch_bounds__(BLOCK) void k_ch_hflag(uint32_t nkeys, const uint8_t *__restrict__ hot, uint32_t *__restrict__ f)
{
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k < nkeys) f[k] = hot[k];
}
__global__ __launch_bounds__(BLOCK) void k_ch_hk(uint32_t nkeys, const uint32_t *__restrict__ f, const uint32_t *__restrict__ fx,
                                                 uint32_t *__restrict__ hk)
{
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k < nkeys && f[k]) hk[fx[k]] = k;
}

struct HotOut {
    uint32_t nh = 0, ne = 0;
    uint64_t nm = 0;
    const uint32_t *hk = nullptr, *eg = nullptr, *eoff = nullptr, *mcnt = nullptr, *moff = nullptr;
    const HG *G = nullptr;
    const uint64_t *mm = nullptr, *ml = nullptr;
    const int32_t *mn = nullptr;
};

// The hot keys' final states (closed form above). Returns false when some hot keys turned out irregular: their hot
// flags are cleared and the caller lays the lane path out again with them.
static bool hot_keys(acc_ctx *ctx, uint32_t nkeys, uint8_t *hot, const uint32_t *kstart, const uint32_t *src, uint32_t nk,
                     const Snap &s, const Upd &u, const UpdRec *urec, uint32_t *fin_n, uint64_t *errs, HotOut &ho)
{
    hipStream_t st = ctx->stream;
    auto read32 = [&](const uint32_t *p) {
        ACC_HIP(hipMemcpyAsync(ctx->pinned, p, 4, hipMemcpyDeviceToHost, st));
        ctx->sync();
        return reinterpret_cast<uint32_t *>(ctx->pinned)[0];
    };
    ho = HotOut{};
    uint32_t *hf = ctx->get<uint32_t>("ch_hf", nkeys), *hx = ctx->get<uint32_t>("ch_hx", (size_t)nkeys + 1);
    launch(ctx, "ch_hflag", k_ch_hflag, dim3(grid_for(nkeys, BLOCK)), dim3(BLOCK), 0, nkeys, (const uint8_t *)hot, hf);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, hf, hx, nkeys, true, hx + nkeys);
    const uint32_t nh = read32(hx + nkeys);
    if (!nh) return true;
    uint32_t *hk = ctx->get<uint32_t>("ch_hk", nh);
    launch(ctx, "ch_hk", k_ch_hk, dim3(grid_for(nkeys, BLOCK)), dim3(BLOCK), 0, nkeys, (const uint32_t *)hf, (const uint32_t *)hx, hk);
    uint32_t *icnt = ctx->get<uint32_t>("ch_icnt", nh), *nsnap = ctx->get<uint32_t>("ch_nsnap", nh);
    uint32_t *ioff = ctx->get<uint32_t>("ch_ioff", (size_t)nh + 1);
    uint8_t *hsnap = ctx->get<uint8_t>("ch_hsnap", nh);
    launch(ctx, "ch_count", k_ch_count, dim3(grid_for(nh, BLOCK)), dim3(BLOCK), 0, nh, (const uint32_t *)hk, kstart, src, nk, s,
           icnt, nsnap, hsnap);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, icnt, ioff, nh, true, ioff + nh);
    const uint64_t NI0 = read32(ioff + nh);
    uint32_t *nextra = ctx->get<uint32_t>("ch_nextra", 1);
    uint32_t *irr = ctx->get<uint32_t>("ch_irr", nh);
    uint64_t NX = 0, NI = 0;
    uint32_t ng = 0, ne = 0;
    HItems it{};
    HG *G = nullptr;
    uint32_t *eg = nullptr, *eoff = nullptr;
    for (int pass = 0; pass < 2; ++pass) {
        NI = NI0 + NX;
        it = HItems{ ctx->get<uint64_t>("ch_im", NI), ctx->get<uint64_t>("ch_il", NI), ctx->get<uint64_t>("ch_inode", NI),
                     ctx->get<uint32_t>("ch_ih", NI), ctx->get<uint32_t>("ch_isrc", NI), ctx->get<uint8_t>("ch_ikind", NI) };
        launch(ctx, "ch_items", k_ch_items, dim3(grid_for(NI0, BLOCK)), dim3(BLOCK), 0, NI0, nh, (const uint32_t *)ioff,
               (const uint32_t *)hk, (const uint32_t *)nsnap, (const uint8_t *)hsnap, kstart, src, s, urec, it);
        if (NX) {   // the first pass's TRANSITIVELY_KNOWN items after the rest
            ACC_HIP(hipMemcpyAsync(it.im + NI0, ctx->get<uint64_t>("ch_xim", NX), NX * 8, hipMemcpyDeviceToDevice, st));
            ACC_HIP(hipMemcpyAsync(it.il + NI0, ctx->get<uint64_t>("ch_xil", NX), NX * 8, hipMemcpyDeviceToDevice, st));
            ACC_HIP(hipMemcpyAsync(it.inode + NI0, ctx->get<uint64_t>("ch_xinode", NX), NX * 8, hipMemcpyDeviceToDevice, st));
            ACC_HIP(hipMemcpyAsync(it.ih + NI0, ctx->get<uint32_t>("ch_xih", NX), NX * 4, hipMemcpyDeviceToDevice, st));
            ACC_HIP(hipMemcpyAsync(it.isrc + NI0, ctx->get<uint32_t>("ch_xisrc", NX), NX * 4, hipMemcpyDeviceToDevice, st));
            ACC_HIP(hipMemcpyAsync(it.ikind + NI0, ctx->get<uint8_t>("ch_xikind", NX), NX, hipMemcpyDeviceToDevice, st));
        }
        // items grouped by (hot key, TxnId), batch order kept inside a group
        const uint64_t *words[3] = { it.im, it.il, it.inode };
        const uint64_t wand[3] = { ~0ull, IDENTITY_LSB, ~0ull };
        DenseRank dr = dense_rank(ctx, "ch_dr", NI, 3, words, wand, nullptr, false);
        const int rb = std::max(1, bits_for(NI)), hb = std::max(1, bits_for(nh));
        uint64_t *key = ctx->get<uint64_t>("ch_key", NI);
        launch(ctx, "ch_skey", k_ch_skey, dim3(grid_for(NI, BLOCK)), dim3(BLOCK), 0, NI, (const uint32_t *)it.ih,
               (const uint32_t *)dr.rank, rb, key);
        Sorted so = radix_sort(ctx, "ch_rs", key, nullptr, NI, rb + hb);
        uint32_t *gf = ctx->get<uint32_t>("ch_gf", NI), *gi = ctx->get<uint32_t>("ch_gi", NI);
        launch(ctx, "ch_gflag", k_ch_gflag, dim3(grid_for(NI, BLOCK)), dim3(BLOCK), 0, NI, (const uint64_t *)so.keys, gf);
        scan<uint32_t, OpAdd<uint32_t>>(ctx, gf, gi, NI, false);
        ng = read32(gi + NI - 1);
        uint32_t *gstart = ctx->get<uint32_t>("ch_gstart", (size_t)ng + 1);
        launch(ctx, "ch_gstart", k_ch_gstart, dim3(grid_for(NI, BLOCK)), dim3(BLOCK), 0, NI, (const uint32_t *)gf, (const uint32_t *)gi,
               ng, gstart);
        G = ctx->get<HG>("ch_G", ng);
        uint8_t *mention = ctx->get<uint8_t>("ch_mention", NI);
        ACC_HIP(hipMemsetAsync(mention, 0, NI, st));
        ACC_HIP(hipMemsetAsync(irr, 0, (size_t)nh * 4, st));
        launch(ctx, "ch_walk", k_ch_walk, dim3(grid_for(ng, BLOCK)), dim3(BLOCK), 0, ng, (const uint32_t *)gstart,
               (const uint32_t *)so.vals, it, s, urec, G, mention, irr, errs);
        uint32_t *gofs = ctx->get<uint32_t>("ch_gofs", (size_t)nh + 1), *pf = ctx->get<uint32_t>("ch_pf", ng);
        uint32_t *px = ctx->get<uint32_t>("ch_px", (size_t)ng + 1);
        launch(ctx, "ch_gofs", k_ch_gofs, dim3(grid_for(ng, BLOCK)), dim3(BLOCK), 0, ng, nh, (const HG *)G, gofs, pf);
        scan<uint32_t, OpAdd<uint32_t>>(ctx, pf, px, ng, true, px + ng);
        ne = read32(px + ng);
        eg = ctx->get<uint32_t>("ch_eg", std::max<uint32_t>(ne, 1));
        eoff = ctx->get<uint32_t>("ch_eoff", (size_t)nh + 1);
        launch(ctx, "ch_entries", k_ch_entries, dim3(grid_for(std::max<uint64_t>(ng, (uint64_t)nh + 1), BLOCK)), dim3(BLOCK), 0,
               ng, nh, ne, (const HG *)G, (const uint32_t *)px, (const uint32_t *)gofs, eg, eoff);
        // the recomputes' deps: the ones no entry holds become TRANSITIVELY_KNOWN items (counted, then written)
        ACC_HIP(hipMemsetAsync(nextra, 0, 4, st));
        HItems none{};
        launch(ctx, "ch_mention", k_ch_mention, dim3(grid_for(NI, BLOCK)), dim3(BLOCK), 0, NI, (const uint8_t *)mention,
               (const uint32_t *)so.vals, it, urec, u, (const uint32_t *)eg, (const HG *)G, (const uint32_t *)gi,
               (const uint32_t *)px, (const uint32_t *)eoff, irr, nextra, (uint64_t)0, none);
        const uint32_t nx = read32(nextra);
        if (!nx) break;
        if (pass == 1) fail(ACC_E_STATE, "internal: CommandsForKey hot-key additions did not settle");
        NX = nx;
        HItems xo{ ctx->get<uint64_t>("ch_xim", NX), ctx->get<uint64_t>("ch_xil", NX), ctx->get<uint64_t>("ch_xinode", NX),
                   ctx->get<uint32_t>("ch_xih", NX), ctx->get<uint32_t>("ch_xisrc", NX), ctx->get<uint8_t>("ch_xikind", NX) };
        ACC_HIP(hipMemsetAsync(nextra, 0, 4, st));
        launch(ctx, "ch_mention", k_ch_mention, dim3(grid_for(NI, BLOCK)), dim3(BLOCK), 0, NI, (const uint8_t *)mention,
               (const uint32_t *)so.vals, it, urec, u, (const uint32_t *)eg, (const HG *)G, (const uint32_t *)gi,
               (const uint32_t *)px, (const uint32_t *)eoff, irr, nextra, NX, xo);
    }
    uint32_t *nirr = ctx->get<uint32_t>("ch_nirr", 1);
    ACC_HIP(hipMemsetAsync(nirr, 0, 4, st));
    launch(ctx, "ch_fin", k_ch_fin, dim3(grid_for(nh, BLOCK)), dim3(BLOCK), 0, nh, (const uint32_t *)hk, (const uint32_t *)eoff,
           (const uint32_t *)irr, fin_n, hot, nirr);
    const uint32_t ni = read32(nirr);
    ctx->stat("cfk.hot_irregular", ni);
    if (ni) return false;
    // the uncommitted entries per hot key, then every entry's missing[]
    uint32_t *uf = ctx->get<uint32_t>("ch_uf", std::max<uint32_t>(ne, 1)), *ux = ctx->get<uint32_t>("ch_ux", (size_t)ne + 1);
    launch(ctx, "ch_uflag", k_ch_uflag, dim3(grid_for(ne, BLOCK)), dim3(BLOCK), 0, ne, (const uint32_t *)eg, (const HG *)G, 0, uf);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, uf, ux, ne, true, ux + ne);
    const uint32_t nu = read32(ux + ne);
    UR *ulist = ctx->get<UR>("ch_ulist", std::max<uint32_t>(nu, 1));
    uint32_t *uoff = ctx->get<uint32_t>("ch_uoff", (size_t)nh + 1);
    launch(ctx, "ch_ulist", k_ch_ulist, dim3(grid_for(std::max<uint64_t>(ne, (uint64_t)nh + 1), BLOCK)), dim3(BLOCK), 0, ne, nh, nu,
           (const uint32_t *)uf, (const uint32_t *)ux, (const uint32_t *)eoff, (const uint32_t *)eg, (const HG *)G, ulist, uoff);
    // the same for the uncommitted entries new in this batch
    launch(ctx, "ch_uflag", k_ch_uflag, dim3(grid_for(ne, BLOCK)), dim3(BLOCK), 0, ne, (const uint32_t *)eg, (const HG *)G, 1, uf);
    scan<uint32_t, OpAdd<uint32_t>>(ctx, uf, ux, ne, true, ux + ne);
    const uint32_t nun = read32(ux + ne);
    UR *ulist_n = ctx->get<UR>("ch_ulist_n", std::max<uint32_t>(nun, 1));
    uint32_t *uoff_n = ctx->get<uint32_t>("ch_uoff_n", (size_t)nh + 1);
    launch(ctx, "ch_ulist", k_ch_ulist, dim3(grid_for(std::max<uint64_t>(ne, (uint64_t)nh + 1), BLOCK)), dim3(BLOCK), 0, ne, nh, nun,
           (const uint32_t *)uf, (const uint32_t *)ux, (const uint32_t *)eoff, (const uint32_t *)eg, (const HG *)G, ulist_n, uoff_n);
    const NewList nl{ ulist_n, uoff_n };
    // the groups that crossed to committed in this batch, as a hash set
    XSet xs{ nullptr, 0 };
    {
        uint32_t *xc = ctx->get<uint32_t>("ch_xcnt", 1);
        ACC_HIP(hipMemsetAsync(xc, 0, 4, st));
        launch(ctx, "ch_xcount", k_ch_xcount, dim3(grid_for(ng, BLOCK)), dim3(BLOCK), 0, ng, (const HG *)G, xc);
        const uint32_t nxc = read32(xc);
        if (nxc) {
            uint32_t cap = 1024;
            while (cap < 2 * nxc && cap < (1u << 31)) cap <<= 1;
            xs.slot = ctx->get<ulonglong4>("ch_xset", cap);
            xs.mask = cap - 1;
            ACC_HIP(hipMemsetAsync(xs.slot, 0, (size_t)cap * sizeof(ulonglong4), st));
            launch(ctx, "ch_xbuild", k_ch_xbuild, dim3(grid_for(ng, BLOCK)), dim3(BLOCK), 0, ng, (const HG *)G, xs);
        }
    }
    uint32_t *mcnt = ctx->get<uint32_t>("ch_mcnt", std::max<uint32_t>(ne, 1)), *moff = ctx->get<uint32_t>("ch_moff", (size_t)ne + 1);
    launch(ctx, "ch_mcount", k_ch_miss<false>, dim3(grid_for(ne, BLOCK)), dim3(BLOCK), 0, ne, (const uint32_t *)eg, (const HG *)G,
           (const uint32_t *)eoff, (const UR *)ulist, (const uint32_t *)uoff, urec, u, s, xs, nl, mcnt, (const uint32_t *)nullptr,
           (uint64_t *)nullptr, (uint64_t *)nullptr, (int32_t *)nullptr);
    uint64_t *nm64 = ctx->get<uint64_t>("ch_nm64", 1);
    sum_u32(ctx, mcnt, ne, nm64);   // the u32 offsets below must not wrap
    scan<uint32_t, OpAdd<uint32_t>>(ctx, mcnt, moff, ne, true, moff + ne);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, nm64, 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t nm = ctx->pinned[0];
    if (nm >= 0xFFFFFFFFull) fail(ACC_E_CAP, "CommandsForKey update: more than 2^32-2 missing[] TxnIds over the hot keys");
    uint64_t *mm = ctx->get<uint64_t>("ch_mm", nm), *ml = ctx->get<uint64_t>("ch_ml", nm);
    int32_t *mn = ctx->get<int32_t>("ch_mn", nm);
    if (nm)
        launch(ctx, "ch_memit", k_ch_miss<true>, dim3(grid_for(ne, BLOCK)), dim3(BLOCK), 0, ne, (const uint32_t *)eg, (const HG *)G,
               (const uint32_t *)eoff, (const UR *)ulist, (const uint32_t *)uoff, urec, u, s, xs, nl, (uint32_t *)nullptr,
               (const uint32_t *)moff, mm, ml, mn);
    ctx->stat("cfk.hot_keys", nh);
    ctx->stat("cfk.hot_items", NI);
    ho.nh = nh; ho.ne = ne; ho.nm = nm;
    ho.hk = hk; ho.eg = eg; ho.eoff = eoff; ho.mcnt = mcnt; ho.moff = moff; ho.G = G; ho.mm = mm; ho.ml = ml; ho.mn = mn;
    return true;
}

// ---- the key-major state as the txn-major snapshot of acc_map_reduce_full (acc_cfk_snap_to_batch)
// Entries are sorted by TxnId with the dense-rank dictionary's stable radix sort of the compacted (msb, lsb & IDENTITY_LSB,
// node) bits (the Timestamp order of cmp; only the bits that vary across the entries, so a few passes instead of the 19
// of three full-width sorts); entries of one TxnId keep key order, so each txn's keys come out sorted.
__global__ __launch_bounds__(BLOCK) void k_cb_node(uint64_t NE, const int32_t *__restrict__ en, uint64_t *__restrict__ k)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < NE) k[i] = (uint32_t)en[i] ^ 0x80000000u;
}
struct BatchOut {
    uint64_t *tm, *tl, *xm, *xl, *kc;
    int32_t *tn, *xn;
    uint8_t *st;
    uint32_t *ko, *mcnt;
};
// the sorted position of every entry
__global__ __launch_bounds__(BLOCK) void k_cb_inv(uint64_t NE, const uint32_t *__restrict__ perm, uint32_t *__restrict__ qpos)
{
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < NE) qpos[perm[i]] = (uint32_t)i;
}
// a TxnId's executeAt and InternalStatus in one record, for the per-entry check
struct TxnChk {
    uint64_t xm, xl;
    int32_t xn;
    uint32_t st;
};
// per TxnId (its first entry in sorted order, which is its first key's): the batch's txn columns and its key run start
__global__ __launch_bounds__(BLOCK) void k_cb_first(uint64_t NE, const uint64_t *__restrict__ ntxn, const uint32_t *__restrict__ first,
                                                    const uint32_t *__restrict__ qpos, Snap s, BatchOut b,
                                                    TxnChk *__restrict__ chk)
{
    const uint64_t t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    const uint64_t n = *ntxn;
    if (t >= n) return;
    const uint32_t e = first[t];
    b.tm[t] = s.em[e]; b.tl[t] = s.el[e]; b.tn[t] = s.en[e];
    b.xm[t] = s.xm[e]; b.xl[t] = s.xl[e]; b.xn[t] = s.xn[e];
    b.st[t] = s.st[e];
    chk[t] = TxnChk{ s.xm[e], s.xl[e], s.xn[e], s.st[e] };
    b.ko[t] = qpos[e];
    if (t + 1 == n) b.ko[n] = (uint32_t)NE;
}
// owner key of every entry (the last key whose entries start at or before it)
__global__ __launch_bounds__(BLOCK) void k_cb_owner(uint64_t NE, uint32_t nk, const uint32_t *__restrict__ ent_off,
                                                    uint32_t *__restrict__ owner)
{
    const uint64_t e = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e >= NE) return;
    uint32_t lo = 0, hi = nk;   // first k with ent_off[k + 1] > e
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (ent_off[mid + 1] > e) hi = mid; else lo = mid + 1;
    }
    owner[e] = lo;
}
// per entry, in entry order (its columns read contiguously): its key code and missing count at its sorted position,
// and the check that it carries its TxnId's executeAt and InternalStatus (a TxnId twice on one key is already refused
// by the per-key sort check)
__global__ __launch_bounds__(BLOCK) void k_cb_ent(uint64_t NE, const uint32_t *__restrict__ owner, const uint32_t *__restrict__ rank,
                                                  const uint32_t *__restrict__ qpos, Snap s, const TxnChk *__restrict__ chk,
                                                  BatchOut b, uint64_t *__restrict__ err)
{
    const uint64_t e = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e >= NE) return;
    const uint32_t t = rank[e], i = qpos[e];
    b.kc[i] = s.key[owner[e]];
    b.mcnt[i] = s.miss_off[e + 1] - s.miss_off[e];
    const TxnChk c = chk[t];
    if (s.st[e] != c.st || cmp(Ts{ s.xm[e], s.xl[e], s.xn[e] }, Ts{ c.xm, c.xl, c.xn }) != 0)
        atomicOr((unsigned long long *)err, (unsigned long long)E_STATE);
}
// Each missing TxnId's batch index from an open-addressing hash table of the batch's TxnIds (built once per call: one
// probe of a 32-B slot per lookup, where a binary search over the batch's TxnIds costs ~20 dependent loads of 20 B).
struct TxnHash {
    ulonglong4 *slot;   // (msb, lsb & IDENTITY_LSB, node << 32 | index, used)
    uint32_t mask;
};
constexpr uint64_t TH_EMPTY = 0;
__device__ __forceinline__ uint32_t th_hash(uint64_t m, uint64_t l, int32_t n)
{
    uint64_t x = m * 0x9E3779B97F4A7C15ull ^ (l & IDENTITY_LSB) ^ ((uint64_t)(uint32_t)n << 40);
    x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 29; x *= 0x94D049BB133111EBull; x ^= x >> 32;
    return (uint32_t)x;
}
__global__ __launch_bounds__(BLOCK) void k_cb_hash_build(const uint64_t *__restrict__ ntxn, BatchOut b,
                                                         TxnHash h)
{
    const uint64_t t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (t >= *ntxn) return;
    const uint64_t m = b.tm[t], l = b.tl[t] & IDENTITY_LSB;
    const int32_t n = b.tn[t];
    for (uint32_t i = th_hash(m, l, n) & h.mask;; i = (i + 1) & h.mask)
        if (atomicCAS((unsigned long long *)&h.slot[i].w, (unsigned long long)TH_EMPTY, 1ull) == TH_EMPTY) {
            h.slot[i].x = m; h.slot[i].y = l; h.slot[i].z = ((uint64_t)(uint32_t)n << 32) | (uint32_t)t;
            return;
        }
}
__device__ __forceinline__ uint32_t th_find(const TxnHash &h, const Ts &k, uint64_t &bad)
{
    const uint64_t l = k.l & IDENTITY_LSB;
    for (uint32_t i = th_hash(k.m, l, k.n) & h.mask;; i = (i + 1) & h.mask) {
        const ulonglong4 e = h.slot[i];
        if (e.w == TH_EMPTY) { bad |= E_STATE; return 0; }   // a TxnId that is no entry of the batch
        if (e.x == k.m && e.y == l && (int32_t)(e.z >> 32) == k.n) return (uint32_t)e.z;
    }
}
// missing[] elements in parallel (a thread each, their TxnIds read contiguously): the owning entry of element j from
// a max-scan of the entries' first-element marks; the element's batch index by one hash probe, written at its pair's
// place in the txn-major layout; each element's TxnId must exceed the one before it in its list (sorted unique)
__global__ __launch_bounds__(BLOCK) void k_cb_mhead(uint64_t NE, Snap s, uint32_t *__restrict__ head)
{
    const uint64_t e = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e < NE && s.miss_off[e + 1] > s.miss_off[e]) head[s.miss_off[e]] = (uint32_t)e;
}
__global__ __launch_bounds__(BLOCK) void k_cb_miss_elem(uint64_t NM, const uint32_t *__restrict__ owner,
                                                        const uint32_t *__restrict__ qpos, Snap s, TxnHash h,
                                                        const uint32_t *__restrict__ mo, uint32_t *__restrict__ mt,
                                                        uint64_t *__restrict__ err)
{
    const uint64_t j = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (j >= NM) return;
    uint64_t bad = 0;
    const uint32_t e = owner[j];
    const uint32_t m0 = s.miss_off[e];
    const Ts x{ s.mm[j], s.ml[j], s.mn[j] };
    if (j > m0 && cmp(Ts{ s.mm[j - 1], s.ml[j - 1], s.mn[j - 1] }, x) >= 0) bad |= E_ARG_SORT;
    const uint32_t lo = th_find(h, x, bad);
    mt[mo[qpos[e]] + (j - m0)] = lo;
    if (bad) atomicOr((unsigned long long *)err, (unsigned long long)bad);
}

}  // namespace cd

void cfk_snap_to_batch(acc_ctx *ctx, const acc_cfk_snap *in, acc_cfk_batch_view *view, bool trusted)
{
    using namespace cd;
    if (!in || !view) fail(ACC_E_ARG, "null argument");
    if (in->mem != ACC_MEM_HOST && in->mem != ACC_MEM_DEVICE) fail(ACC_E_ARG, "mem must be ACC_MEM_HOST or ACC_MEM_DEVICE");
    hipStream_t st = ctx->stream;
    const uint32_t nk = in->n_keys;
    const uint64_t NE = in->n_entries, NM = in->n_missing;
    if (nk == 0 && (NE || NM)) fail(ACC_E_ARG, "entries without keys");
    if (NE >= 0xFFFFFFFFull || NM >= 0xFFFFFFFFull) fail(ACC_E_CAP, "more than 2^32-1 entries / missing");
    Snap s{};
    s.key = stage_in(ctx, "cb_skey", in->key, nk, in->mem);
    s.ent_off = stage_in(ctx, "cb_soff", in->ent_off, (size_t)nk + 1, in->mem);
    s.em = stage_in(ctx, "cb_sem", in->txn_id.msb, NE, in->mem);
    s.el = stage_in(ctx, "cb_sel", in->txn_id.lsb, NE, in->mem);
    s.en = stage_in(ctx, "cb_sen", in->txn_id.node, NE, in->mem);
    s.xm = stage_in(ctx, "cb_sxm", in->execute_at.msb, NE, in->mem);
    s.xl = stage_in(ctx, "cb_sxl", in->execute_at.lsb, NE, in->mem);
    s.xn = stage_in(ctx, "cb_sxn", in->execute_at.node, NE, in->mem);
    s.st = stage_in(ctx, "cb_sst", in->status, NE, in->mem);
    s.miss_off = stage_in(ctx, "cb_smoff", in->miss_off, NE + 1, in->mem);
    s.mm = stage_in(ctx, "cb_smm", in->missing.msb, NM, in->mem);
    s.ml = stage_in(ctx, "cb_sml", in->missing.lsb, NM, in->mem);
    s.mn = stage_in(ctx, "cb_smn", in->missing.node, NM, in->mem);
    s.n_keys = nk; s.n_ent = NE; s.n_miss = NM;
    uint64_t *errs = ctx->get<uint64_t>("cb_errs", 1);
    ACC_HIP(hipMemsetAsync(errs, 0, 8, st));
    BatchOut b{};
    b.tm = ctx->get<uint64_t>("cb_tm", NE); b.tl = ctx->get<uint64_t>("cb_tl", NE); b.tn = ctx->get<int32_t>("cb_tn", NE);
    b.xm = ctx->get<uint64_t>("cb_xm", NE); b.xl = ctx->get<uint64_t>("cb_xl", NE); b.xn = ctx->get<int32_t>("cb_xn", NE);
    b.st = ctx->get<uint8_t>("cb_st", NE);
    b.ko = ctx->get<uint32_t>("cb_ko", NE + 1);
    b.kc = ctx->get<uint64_t>("cb_kc", NE);
    b.mcnt = ctx->get<uint32_t>("cb_mcnt", NE);
    uint32_t *mo = ctx->get<uint32_t>("cb_mo", NE + 1), *mt = ctx->get<uint32_t>("cb_mt", NM);
    uint32_t n_txn = 0;
    if (NE == 0) {
        ACC_HIP(hipMemsetAsync(b.ko, 0, 4, st));
        ACC_HIP(hipMemsetAsync(mo, 0, 4, st));
        ctx->sync();
    } else {
        if (!trusted) {   // (acc_cfk_apply_deps hands over acc_cfk_apply's own output: already in this form)
            Upd none{};
            launch(ctx, "cb_check", k_cd_check, dim3(grid_for(std::max<uint64_t>(nk, NE), BLOCK)), dim3(BLOCK), 0, s, none,
                   (uint32_t *)nullptr, errs,
                   (uint64_t *)nullptr);
            ACC_HIP(hipMemcpyAsync(ctx->pinned, errs, 8, hipMemcpyDeviceToHost, st));
            ctx->sync();
            if (ctx->pinned[0] & E_ARG_STATUS) fail(ACC_E_ARG, "invalid InternalStatus ordinal");
            if (ctx->pinned[0] & E_ARG_OFF) fail(ACC_E_ARG, "offsets must be non-decreasing from 0 to their totals");
            if (ctx->pinned[0] & E_ARG_SORT) fail(ACC_E_ARG, "keys / TxnIds must be sorted unique");
        }
        const dim3 g(grid_for(NE, BLOCK));
        uint64_t *k = ctx->get<uint64_t>("cb_key", NE);
        uint32_t *qpos = ctx->get<uint32_t>("cb_qpos", NE);
        TxnChk *chk = ctx->get<TxnChk>("cb_chk", NE);
        // entries in Timestamp order (stable: a TxnId's entries stay in key order) through the dense-rank dictionary's
        // sort of the compacted (msb, lsb & IDENTITY_LSB, node) bits: a few radix passes over the bits that vary
        launch(ctx, "cb_node", k_cb_node, g, dim3(BLOCK), 0, NE, s.en, k);
        const uint64_t *words[3] = { s.em, s.el, k };
        const uint64_t wand[3] = { ~0ull, 0xFFFFFFFFFFFF001EULL, ~0ull };
        DenseRank dr = dense_rank(ctx, "cb_dr", NE, 3, words, wand, nullptr, true);
        const uint32_t *perm = dr.perm;
        if (!perm) {   // every entry carries one TxnId: identity order
            uint32_t *id = ctx->get<uint32_t>("cb_iota", NE);
            launch(ctx, "cb_iota", k_iota, g, dim3(BLOCK), 0, id, (size_t)NE);
            perm = id;
        }
        // the batch's txn columns from each TxnId's first entry, then every entry (entry order) checked against them
        launch(ctx, "cb_inv", k_cb_inv, g, dim3(BLOCK), 0, NE, perm, qpos);
        launch(ctx, "cb_first", k_cb_first, g, dim3(BLOCK), 0, NE, (const uint64_t *)dr.count_dev, (const uint32_t *)dr.first,
               (const uint32_t *)qpos, s, b, chk);
        uint32_t *owner = ctx->get<uint32_t>("cb_owner", NE);
        launch(ctx, "cb_owner", k_cb_owner, g, dim3(BLOCK), 0, NE, nk, s.ent_off, owner);
        launch(ctx, "cb_ent", k_cb_ent, g, dim3(BLOCK), 0, NE, (const uint32_t *)owner, (const uint32_t *)dr.rank, (const uint32_t *)qpos, s, (const TxnChk *)chk, b, errs);
        scan<uint32_t, OpAdd<uint32_t>>(ctx, b.mcnt, mo, NE, true, mo + NE);
        if (NM) {
            // the batch's TxnIds in a hash table of >= 2x their count (one read-back of the count)
            ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, dr.count_dev, 8, hipMemcpyDeviceToHost, st));
            ctx->sync();
            const uint64_t nt = ctx->pinned[1] & 0xFFFFFFFFu;
            uint32_t cap = 1024;
            while (cap < 2 * nt && cap < (1u << 31)) cap <<= 1;
            TxnHash th{ ctx->get<ulonglong4>("cb_hash", cap), cap - 1 };
            ACC_HIP(hipMemsetAsync(th.slot, 0, (size_t)cap * sizeof(ulonglong4), st));
            launch(ctx, "cb_hash", k_cb_hash_build, dim3(grid_for(nt, BLOCK)), dim3(BLOCK), 0, (const uint64_t *)dr.count_dev, b, th);
            uint32_t *head = ctx->get<uint32_t>("cb_mhead", NM), *owner_m = ctx->get<uint32_t>("cb_mowner", NM);
            ACC_HIP(hipMemsetAsync(head, 0, NM * 4, st));
            launch(ctx, "cb_mhead", k_cb_mhead, g, dim3(BLOCK), 0, NE, s, head);
            scan<uint32_t, OpMax<uint32_t>>(ctx, head, owner_m, NM, false, (uint32_t *)nullptr);
            launch(ctx, "cb_miss", k_cb_miss_elem, dim3(grid_for(NM, BLOCK)), dim3(BLOCK), 0, NM, (const uint32_t *)owner_m,
                   (const uint32_t *)qpos, s, th, (const uint32_t *)mo, mt, errs);
        }
        ACC_HIP(hipMemcpyAsync(ctx->pinned, errs, 8, hipMemcpyDeviceToHost, st));
        ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, dr.count_dev, 8, hipMemcpyDeviceToHost, st));
        ctx->sync();
        const uint64_t e = ctx->pinned[0];
        if (e & E_STATE)
            fail(ACC_E_STATE, "a TxnId with different executeAt / InternalStatus on two keys, or a missing[] TxnId "
                              "that is no CommandsForKey entry");
        if (e & E_ARG_SORT) fail(ACC_E_ARG, "a TxnId twice on one key, or a missing[] not sorted unique");
        n_txn = (uint32_t)(ctx->pinned[1] & 0xFFFFFFFFu);
    }
    ctx->stat("cfk_batch.txns", n_txn);
    ctx->stat("cfk_batch.pairs", NE);
    acc_batch_in &o = view->batch;
    o.n_txn = n_txn; o.mem = ACC_MEM_DEVICE; o.n_pairs = NE;
    o.txn_id = acc_ts_cols{ b.tm, b.tl, b.tn };
    o.execute_at = acc_ts_cols{ b.xm, b.xl, b.xn };
    o.status = b.st; o.key_off = b.ko; o.key_code = b.kc;
    view->missing_off = mo; view->missing_txn = mt; view->n_missing = NM;
}

void cfk_apply(acc_ctx *ctx, const acc_cfk_snap *in, const acc_cfk_updates *up, acc_cfk_snap_view *view)
{
    using namespace cd;
    if (!in || !up || !view) fail(ACC_E_ARG, "null argument");
    for (uint32_t m : { in->mem, up->mem })
        if (m != ACC_MEM_HOST && m != ACC_MEM_DEVICE) fail(ACC_E_ARG, "mem must be ACC_MEM_HOST or ACC_MEM_DEVICE");
    hipStream_t st = ctx->stream;
    const uint32_t nk = in->n_keys, nu = up->n_upd;
    const uint64_t NE = in->n_entries, NM = in->n_missing, NP = up->n_pairs, ND = up->n_deps;
    if (nk == 0 && (NE || NM)) fail(ACC_E_ARG, "entries without keys");
    if (nu == 0 && (NP || ND)) fail(ACC_E_ARG, "pairs without updates");
    if (NE >= 0xFFFFFFFFull || NM >= 0xFFFFFFFFull || NP >= 0xFFFFFFFFull || ND >= 0xFFFFFFFFull)
        fail(ACC_E_CAP, "more than 2^32-1 entries / missing / pairs / deps");
    Snap s{};
    s.key = stage_in(ctx, "cd_skey", in->key, nk, in->mem);
    s.ent_off = stage_in(ctx, "cd_soff", in->ent_off, (size_t)nk + 1, in->mem);
    s.em = stage_in(ctx, "cd_sem", in->txn_id.msb, NE, in->mem);
    s.el = stage_in(ctx, "cd_sel", in->txn_id.lsb, NE, in->mem);
    s.en = stage_in(ctx, "cd_sen", in->txn_id.node, NE, in->mem);
    s.xm = stage_in(ctx, "cd_sxm", in->execute_at.msb, NE, in->mem);
    s.xl = stage_in(ctx, "cd_sxl", in->execute_at.lsb, NE, in->mem);
    s.xn = stage_in(ctx, "cd_sxn", in->execute_at.node, NE, in->mem);
    s.st = stage_in(ctx, "cd_sst", in->status, NE, in->mem);
    s.miss_off = stage_in(ctx, "cd_smoff", in->miss_off, NE + 1, in->mem);
    s.mm = stage_in(ctx, "cd_smm", in->missing.msb, NM, in->mem);
    s.ml = stage_in(ctx, "cd_sml", in->missing.lsb, NM, in->mem);
    s.mn = stage_in(ctx, "cd_smn", in->missing.node, NM, in->mem);
    s.n_keys = nk; s.n_ent = NE; s.n_miss = NM;
    Upd u{};
    u.um = stage_in(ctx, "cd_um", up->txn_id.msb, nu, up->mem);
    u.ul = stage_in(ctx, "cd_ul", up->txn_id.lsb, nu, up->mem);
    u.un = stage_in(ctx, "cd_un", up->txn_id.node, nu, up->mem);
    u.uxm = stage_in(ctx, "cd_uxm", up->execute_at.msb, nu, up->mem);
    u.uxl = stage_in(ctx, "cd_uxl", up->execute_at.lsb, nu, up->mem);
    u.uxn = stage_in(ctx, "cd_uxn", up->execute_at.node, nu, up->mem);
    u.st = stage_in(ctx, "cd_ust", up->status, nu, up->mem);
    u.fl = stage_in(ctx, "cd_ufl", up->flags, nu, up->mem);
    u.key_off = stage_in(ctx, "cd_ukoff", up->key_off, (size_t)nu + 1, up->mem);
    u.key = stage_in(ctx, "cd_ukey", up->key, NP, up->mem);
    u.dep_off = stage_in(ctx, "cd_udoff", up->dep_off, NP + 1, up->mem);
    u.dm = stage_in(ctx, "cd_udm", up->deps.msb, ND, up->mem);
    u.dl = stage_in(ctx, "cd_udl", up->deps.lsb, ND, up->mem);
    u.dn = stage_in(ctx, "cd_udn", up->deps.node, ND, up->mem);
    u.n_upd = nu; u.NP = NP; u.ND = ND;
    uint32_t *owner = ctx->get<uint32_t>("cd_owner", NP);
    u.owner = owner;
    uint64_t *errs = ctx->get<uint64_t>("cd_errs", 1);
    ACC_HIP(hipMemsetAsync(errs, 0, 8, st));
    const uint64_t gmax = std::max<uint64_t>({ (uint64_t)nk, (uint64_t)nu, NP, NE, 1 });
    uint64_t *krng = ctx->get<uint64_t>("cd_krng", 2);
    ACC_HIP(hipMemsetAsync(krng, 0xFF, 8, st));
    ACC_HIP(hipMemsetAsync(krng + 1, 0, 8, st));
    launch(ctx, "cd_check", k_cd_check, dim3(grid_for(gmax, BLOCK)), dim3(BLOCK), 0, s, u, owner, errs, krng);
    if (NP) launch(ctx, "cd_depchk", k_cd_depchk, dim3(grid_for(NP, BLOCK)), dim3(BLOCK), 0, u, errs);
    ACC_HIP(hipMemcpyAsync(ctx->pinned, errs, 8, hipMemcpyDeviceToHost, st));
    ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, krng, 16, hipMemcpyDeviceToHost, st));
    ctx->sync();
    const uint64_t kbase = ctx->pinned[1], kspan = ctx->pinned[2] - ctx->pinned[1];
    auto check = [&](uint64_t e) {
        if (e & E_ARG_STATUS) fail(ACC_E_ARG, "invalid InternalStatus ordinal");
        if (e & E_ARG_OFF) fail(ACC_E_ARG, "offsets must be non-decreasing from 0 to their totals");
        if (e & E_ARG_SORT) fail(ACC_E_ARG, "keys / TxnIds / deps must be sorted unique");
        if (e & E_STALE) fail(ACC_E_STATE, "stale status update to CommandsForKey (IllegalStateException)");
        if (e & E_STATE) fail(ACC_E_STATE, "CommandsForKey invariant violated (IllegalStateException)");
        if (e & E_CAP) fail(ACC_E_STATE, "internal: CommandsForKey working space exceeded");
    };
    check(ctx->pinned[0]);

    // ---- 1. keys: the snapshot's and every (update, key) pair's, sorted stably by key code
    const uint64_t T = nk + NP;
    uint64_t *all = ctx->get<uint64_t>("cd_all", T);
    uint32_t nkeys = 0;
    Sorted so{ nullptr, nullptr };
    uint32_t *kflag = ctx->get<uint32_t>("cd_kflag", T), *kinc = ctx->get<uint32_t>("cd_kinc", T);
    if (T) {
        launch(ctx, "cd_keys", k_cd_keys, dim3(grid_for(T, BLOCK)), dim3(BLOCK), 0, nk, NP, s.key, u.key, kbase, all);
        so = radix_sort(ctx, "cd_rs", all, nullptr, T, bits_for(kspan));
        launch(ctx, "cd_kflag", k_cd_kflag, dim3(grid_for(T, BLOCK)), dim3(BLOCK), 0, T, (const uint64_t *)so.keys, kflag);
        scan<uint32_t, OpAdd<uint32_t>>(ctx, kflag, kinc, T, false);
        ACC_HIP(hipMemcpyAsync(ctx->pinned, kinc + T - 1, 4, hipMemcpyDeviceToHost, st));
        ctx->sync();
        nkeys = reinterpret_cast<uint32_t *>(ctx->pinned)[0];
    }
    // ---- 2. working space
    uint32_t *kstart = ctx->get<uint32_t>("cd_kstart", (size_t)nkeys + 1);
    uint64_t *ecap = ctx->get<uint64_t>("cd_ecap", nkeys), *mcap = ctx->get<uint64_t>("cd_mcap", nkeys);
    uint64_t *dcap = ctx->get<uint64_t>("cd_dcap", nkeys), *mmax = ctx->get<uint64_t>("cd_mmax", nkeys);
    uint32_t *ovf = ctx->get<uint32_t>("cd_ovf", nkeys);
    // per wave of 64 keys (their buffers interleaved): the capacities' maxima and the per-lane region offsets
    const uint32_t nwv = (nkeys + (uint32_t)CD_W - 1) / (uint32_t)CD_W;
    uint64_t *ecw = ctx->get<uint64_t>("cd_ecw", nwv), *mcw = ctx->get<uint64_t>("cd_mcw", nwv), *dcw = ctx->get<uint64_t>("cd_dcw", nwv);
    uint64_t *esz = ctx->get<uint64_t>("cd_esz", nwv), *tsz = ctx->get<uint64_t>("cd_tsz", nwv);
    uint64_t *eoffw = ctx->get<uint64_t>("cd_eoffw", (size_t)nwv + 1), *toffw = ctx->get<uint64_t>("cd_toffw", (size_t)nwv + 1);
    uint64_t Ew = 0, Tw = 0;   // per-lane totals (the pools hold CD_W times these)
    const uint32_t *perm = nullptr;   // slot -> key, by entry capacity (set after the bounds)
    uint32_t *kslot = ctx->get<uint32_t>("cd_kslot", nkeys);
    auto wave_layout = [&]() {
        launch(ctx, "cd_wcap", k_cd_wcap, dim3(grid_for(nkeys, BLOCK)), dim3(BLOCK), 0, nkeys, perm, kslot, (const uint64_t *)ecap,
               (const uint64_t *)mcap, (const uint64_t *)dcap, ecw, mcw, dcw, esz, tsz);
        const uint64_t *si[2] = { esz, tsz };
        uint64_t *so[2] = { eoffw, toffw }, *stot[2] = { eoffw + nwv, toffw + nwv };
        const size_t sn[2] = { nwv, nwv };
        scan_multi<uint64_t, OpAdd<uint64_t>>(ctx, 2, si, so, sn, true, stot);
        ACC_HIP(hipMemcpyAsync(ctx->pinned, eoffw + nwv, 8, hipMemcpyDeviceToHost, st));
        ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, toffw + nwv, 8, hipMemcpyDeviceToHost, st));
        ctx->sync();
        Ew = ctx->pinned[0]; Tw = ctx->pinned[1];
    };
    // each (update, key) pair's update record at its sorted position
    UpdRec *urec = ctx->get<UpdRec>("cd_urec", std::max<uint64_t>(T, 1));
    if (NP) {
        uint32_t *qpos = ctx->get<uint32_t>("cd_qpos", NP);
        launch(ctx, "cd_inv", k_cd_inv, dim3(grid_for(T, BLOCK)), dim3(BLOCK), 0, T, (const uint32_t *)so.vals, nk, qpos);
        launch(ctx, "cd_urec", k_cd_urec, dim3(grid_for(NP, BLOCK)), dim3(BLOCK), 0, NP, (const uint32_t *)qpos, u, urec);
    }
    uint8_t *hot = ctx->get<uint8_t>("cd_hot", nkeys);
    const uint32_t hot_thr = ctx->opts.cfk_hot ? ctx->opts.cfk_hot : CH_DEFAULT_HOT;   // acc_opts.cfk_hot
    uint32_t *fin_n = ctx->get<uint32_t>("cd_fin_n", nkeys);
    HotOut ho;
    if (nkeys)
        launch(ctx, "cd_kstart", k_cd_kstart, dim3(grid_for(T, BLOCK)), dim3(BLOCK), 0, T, (const uint32_t *)kflag,
               (const uint32_t *)kinc, nkeys, kstart);
    uint32_t *nhot = ctx->get<uint32_t>("cd_nhot", 1);
    BSum bs{ ctx->get<uint64_t>("cd_bs_e", nkeys), ctx->get<uint64_t>("cd_bs_m", nkeys), ctx->get<uint64_t>("cd_bs_g", nkeys),
             ctx->get<uint32_t>("cd_bs_d", nkeys) };
    if (nkeys) {
        ACC_HIP(hipMemsetAsync(bs.e, 0, (size_t)nkeys * 8, st));
        ACC_HIP(hipMemsetAsync(bs.m, 0, (size_t)nkeys * 8, st));
        ACC_HIP(hipMemsetAsync(bs.g, 0, (size_t)nkeys * 8, st));
        ACC_HIP(hipMemsetAsync(bs.d, 0, (size_t)nkeys * 4, st));
        launch(ctx, "cd_bsum", k_cd_bsum, dim3(grid_for(T, BLOCK)), dim3(BLOCK), 0, T, (const uint32_t *)kinc, (const uint32_t *)so.vals,
               reinterpret_cast<const uint2 *>(urec), nk, s, bs);
    }
    ctx->stat("cfk.hot_keys", 0);
    ctx->stat("cfk.hot_irregular", 0);
    for (int keep_hot = 0; nkeys; keep_hot = 1) {
        ACC_HIP(hipMemsetAsync(nhot, 0, 4, st));
        launch(ctx, "cd_bounds", k_cd_bounds, dim3(grid_for(nkeys, BLOCK)), dim3(BLOCK), 0, nkeys, (const uint32_t *)kstart,
               (const uint32_t *)so.vals, nk, s.ent_off, bs,
               ecap, mcap, mmax, dcap, ovf, hot_thr, keep_hot, hot,
               nhot);
        // keys by entry capacity (bits up to the largest), so interleaved waves hold keys of similar size
        uint64_t *cmax = ctx->get<uint64_t>("cd_cmax", 1);
        ACC_HIP(hipMemsetAsync(cmax, 0, 8, st));
        scan<uint64_t, OpMax<uint64_t>>(ctx, ecap, ctx->get<uint64_t>("cd_cscan", nkeys), nkeys, false, cmax);
        ACC_HIP(hipMemcpyAsync(ctx->pinned, cmax, 8, hipMemcpyDeviceToHost, st));
        ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, nhot, 4, hipMemcpyDeviceToHost, st));
        ctx->sync();
        const uint32_t nh = (uint32_t)ctx->pinned[1];
        {
            const uint32_t *asc = radix_sort(ctx, "cd_rs_cap", ecap, nullptr, nkeys, std::max(1, bits_for(ctx->pinned[0]))).vals;
            uint32_t *desc = ctx->get<uint32_t>("cd_perm_desc", nkeys);
            launch(ctx, "cd_rev", k_cd_rev, dim3(grid_for(nkeys, BLOCK)), dim3(BLOCK), 0, nkeys, asc, desc);
            perm = desc;
        }
        wave_layout();
        // the hot keys' final states; keys found irregular go back to the lane path (layout again)
        if (!nh || hot_keys(ctx, nkeys, hot, kstart, so.vals, nk, s, u, urec, fin_n, errs, ho)) break;
    }
    uint8_t *final_b = ctx->get<uint8_t>("cd_final_b", nkeys);
    uint32_t *fin_m = ctx->get<uint32_t>("cd_fin_m", nkeys);
    // ---- 3. replay, again with grown missing areas while some key outgrows its guess
    Pool p{};
    uint32_t regrow = 0;
    // the kept keys and the output entry offsets, scanned right after each replay (one host sync for both)
    uint32_t *keep = ctx->get<uint32_t>("cd_keep", nkeys), *kpos = ctx->get<uint32_t>("cd_kpos", (size_t)nkeys + 1);
    uint32_t *eall = ctx->get<uint32_t>("cd_eall", (size_t)nkeys + 1);
    uint32_t nko = 0;
    uint64_t NEo = 0, NMo = 0;
    for (;; ++regrow) {
        const uint64_t pool_bytes = (uint64_t)CD_W * (Ew * sizeof(InfoP) + Tw * sizeof(Ts));
        if (pool_bytes > (64ull << 30)) fail(ACC_E_CAP, "CommandsForKey working space beyond 64 GiB for this batch");
        p = Pool{ ctx->get<InfoP>("cd_pool_e", (size_t)CD_W * Ew), ctx->get<Ts>("cd_pool_m", (size_t)CD_W * Tw), ecw, mcw, dcw,
                  eoffw, toffw, perm, kslot };
        if (!nkeys) break;
        unsigned long long *paths = ctx->get<unsigned long long>("cd_paths", 2);
        ACC_HIP(hipMemsetAsync(paths, 0, 16, st));
        launch(ctx, "cd_apply", k_cd_apply, dim3(grid_for(nkeys, BLOCK)), dim3(BLOCK), 0, nkeys, (const uint32_t *)kstart,
               (const uint32_t *)so.vals, (const uint64_t *)ecap, (const uint64_t *)mcap, nk, s, u, p, final_b, fin_n, fin_m,
               ovf, errs, paths, (const UpdRec *)urec, (const uint8_t *)hot);
        launch(ctx, "cd_out1", k_cd_out1, dim3(grid_for(nkeys, BLOCK)), dim3(BLOCK), 0, nkeys, (const uint32_t *)fin_n, keep);
        {
            const uint32_t *si[2] = { keep, fin_n };
            uint32_t *so2[2] = { kpos, eall }, *stot[2] = { kpos + nkeys, eall + nkeys };
            const size_t sn[2] = { nkeys, nkeys };
            scan_multi<uint32_t, OpAdd<uint32_t>>(ctx, 2, si, so2, sn, true, stot);
        }
        ACC_HIP(hipMemcpyAsync(ctx->pinned, errs, 8, hipMemcpyDeviceToHost, st));
        ACC_HIP(hipMemcpyAsync(ctx->pinned + 1, paths, 16, hipMemcpyDeviceToHost, st));
        ACC_HIP(hipMemcpyAsync(ctx->pinned + 3, kpos + nkeys, 4, hipMemcpyDeviceToHost, st));
        ACC_HIP(hipMemcpyAsync(ctx->pinned + 4, eall + nkeys, 4, hipMemcpyDeviceToHost, st));
        ctx->sync();
        ctx->stat("cfk.apply_in_place", ctx->pinned[1]);
        ctx->stat("cfk.apply_rebuilt", ctx->pinned[2]);
        const uint64_t e = ctx->pinned[0];
        check(e & ~E_MCAP);
        nko = (uint32_t)ctx->pinned[3];
        NEo = (uint32_t)ctx->pinned[4];
        if (!(e & E_MCAP)) break;
        ACC_HIP(hipMemsetAsync(errs, 0, 8, st));
        launch(ctx, "cd_grow", k_cd_grow, dim3(grid_for(nkeys, BLOCK)), dim3(BLOCK), 0, nkeys, ovf, mcap,
               (const uint64_t *)mmax, errs, regrow);
        ACC_HIP(hipMemcpyAsync(ctx->pinned, errs, 8, hipMemcpyDeviceToHost, st));
        ctx->sync();
        check(ctx->pinned[0]);
        wave_layout();
    }
    ctx->stat("cfk.apply_regrow", regrow);
    // ---- 4. key-major output
    uint64_t *okey = ctx->get<uint64_t>("cd_okey", nko);
    uint32_t *kkey = ctx->get<uint32_t>("cd_kkey", std::max<uint32_t>(nko, 1));
    Out o{};
    o.ent_off = ctx->get<uint32_t>("cd_oent_off", (size_t)nko + 1);
    if (nko) {
        launch(ctx, "cd_out2", k_cd_out2, dim3(grid_for(nkeys, BLOCK)), dim3(BLOCK), 0, nkeys, (const uint32_t *)keep,
               (const uint32_t *)kpos, (const uint32_t *)kstart, (const uint64_t *)so.keys, kbase, (const uint32_t *)eall, okey,
               o.ent_off, nko, (uint32_t)NEo, kkey);
    } else {
        ACC_HIP(hipMemsetAsync(o.ent_off, 0, 4, st));
    }
    o.em = ctx->get<uint64_t>("cd_oem", NEo); o.el = ctx->get<uint64_t>("cd_oel", NEo); o.en = ctx->get<int32_t>("cd_oen", NEo);
    o.xm = ctx->get<uint64_t>("cd_oxm", NEo); o.xl = ctx->get<uint64_t>("cd_oxl", NEo); o.xn = ctx->get<int32_t>("cd_oxn", NEo);
    o.st = ctx->get<uint8_t>("cd_ost", NEo);
    o.mcnt = ctx->get<uint32_t>("cd_omcnt", NEo);
    o.miss_off = ctx->get<uint32_t>("cd_omoff", NEo + 1);
    if (NEo) {
        launch(ctx, "cd_out3", k_cd_out3e, dim3(grid_for(NEo, BLOCK)), dim3(BLOCK), 0, (uint32_t)NEo, nko, (const uint32_t *)kkey,
               p, (const uint8_t *)final_b, o, (const uint8_t *)hot);
        if (ho.ne)
            launch(ctx, "ch_out3", k_ch_out3, dim3(grid_for(ho.ne, BLOCK)), dim3(BLOCK), 0, ho.ne, ho.eg, ho.G, ho.eoff, ho.hk,
                   (const uint32_t *)kpos, ho.mcnt, o);
        uint64_t *nm64 = ctx->get<uint64_t>("cd_onm64", 1);
        sum_u32(ctx, o.mcnt, NEo, nm64);   // the u32 miss_off of the result must not wrap
        scan<uint32_t, OpAdd<uint32_t>>(ctx, o.mcnt, o.miss_off, NEo, true, o.miss_off + NEo);
        ACC_HIP(hipMemcpyAsync(ctx->pinned, nm64, 8, hipMemcpyDeviceToHost, st));
        ctx->sync();
        if (ctx->pinned[0] >= 0xFFFFFFFFull) fail(ACC_E_CAP, "CommandsForKey update: more than 2^32-2 missing[] TxnIds in the result");
        NMo = (uint32_t)ctx->pinned[0];
    } else {
        ACC_HIP(hipMemsetAsync(o.miss_off, 0, 4, st));
    }
    o.mm = ctx->get<uint64_t>("cd_omm", NMo); o.ml = ctx->get<uint64_t>("cd_oml", NMo); o.mn = ctx->get<int32_t>("cd_omn", NMo);
    if (NMo)
    {
        launch(ctx, "cd_out4", k_cd_out4, dim3(grid_for(nkeys, BLOCK)), dim3(BLOCK), 0, nkeys, (const uint32_t *)keep,
               (const uint32_t *)kpos, (const uint64_t *)ecap, (const uint64_t *)mcap, p, (const uint8_t *)final_b, o,
               (const uint8_t *)hot);
        if (ho.nm)
            launch(ctx, "ch_out4", k_ch_out4, dim3(grid_for(ho.nm, BLOCK)), dim3(BLOCK), 0, ho.nm, ho.ne, ho.eg, ho.G, ho.eoff, ho.hk,
                   (const uint32_t *)kpos, ho.moff, ho.mm, ho.ml, ho.mn, o);
    }
    ctx->sync();
    ctx->stat("cfk.keys", nko);
    ctx->stat("cfk.entries", NEo);
    ctx->stat("cfk.missing", NMo);
    *view = acc_cfk_snap_view{ nko, NEo, NMo, okey, o.ent_off, acc_ts_cols{ o.em, o.el, o.en }, acc_ts_cols{ o.xm, o.xl, o.xn },
                               o.st, o.miss_off, acc_ts_cols{ o.mm, o.ml, o.mn } };
}

}  // namespace acc
