// ranges.hpp — the Ranges algebra of accord-core as host code (see ranges.hip for the C ABI): a Ranges is a sorted,
// deoverlapped list of Range (start, end) u64 key codes of one bound type; every operation restates its reference
// method step by step (file:line in each function).
#pragma once
#include "../../include/accord_amd.h"

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <vector>

namespace acc {
namespace rg {

struct Rg {
    uint64_t s, e;
    bool operator==(const Rg &o) const { return s == o.s && e == o.e; }
};
using V = std::vector<Rg>;

struct ArgError : std::runtime_error { using std::runtime_error::runtime_error; };

inline int cmpu(uint64_t a, uint64_t b) { return a < b ? -1 : a > b ? 1 : 0; }

// Range.compareIntersecting (Range.java:296-305)
inline int cmp_intersecting(const Rg &a, const Rg &b)
{
    if (a.s >= b.e) return 1;
    if (a.e <= b.s) return -1;
    return 0;
}

// Range.compareTo(RoutableKey): EndInclusive (Range.java:48-55), StartInclusive (Range.java:98-105)
inline int cmp_key(const Rg &r, uint64_t k, bool ei)
{
    if (ei) {
        if (k <= r.s) return 1;
        if (k > r.e) return -1;
        return 0;
    }
    if (k < r.s) return 1;
    if (k >= r.e) return -1;
    return 0;
}

enum Search { FAST, CEIL, FLOOR };

// SortedArrays.binarySearch (utils/SortedArrays.java:993-1027); cmp(i) = comparator.compare(find, in[i])
template <class C>
int64_t bsearch(int64_t from, int64_t to, C cmp, Search op)
{
    int64_t found = -1;
    while (from < to) {
        const int64_t i = (from + to) >> 1;
        const int c = cmp(i);
        if (c < 0) to = i;
        else if (c > 0) from = i + 1;
        else {
            if (op == FAST) return i;
            if (op == CEIL) to = found = i;
            else { found = i; from = i + 1; }
        }
    }
    return found >= 0 ? found : -1 - to;
}

// AbstractRanges.indexOf(RoutableKey) (primitives/AbstractRanges.java:51-54): comparator (k, r) -> -r.compareTo(k)
inline int64_t index_of(const V &a, uint64_t k, bool ei)
{
    return bsearch(0, (int64_t)a.size(), [&](int64_t i) { return -cmp_key(a[(size_t)i], k, ei); }, FAST);
}

// AbstractRanges.deoverlapSorted, MERGE_OVERLAPPING (AbstractRanges.java:714-781): neighbours merge only when
// prev.end > next.start (touching ranges stay apart)
inline V deoverlap_sorted(const V &in)
{
    V out;
    out.reserve(in.size());
    size_t i = 0;
    while (i < in.size()) {
        Rg cur = in[i++];
        while (i < in.size() && cur.e > in[i].s) { cur.e = std::max(cur.e, in[i].e); ++i; }
        out.push_back(cur);
    }
    return out;
}

// Ranges.of -> AbstractRanges.sortAndDeoverlap (AbstractRanges.java:689-707): sorted by Range::compare (start, end)
inline V of(V in)
{
    std::stable_sort(in.begin(), in.end(), [](const Rg &x, const Rg &y) { return x.s != y.s ? x.s < y.s : x.e < y.e; });
    return deoverlap_sorted(in);
}

// AbstractRanges.ofSortedAndDeoverlapped (AbstractRanges.java:789-798)
inline const V &check_sorted_deoverlapped(const V &in)
{
    for (size_t i = 1; i < in.size(); ++i)
        if (in[i - 1].e > in[i].s) throw ArgError("ranges are not correctly sorted or deoverlapped");
    return in;
}

// AbstractRanges.supersetLinearMerge (AbstractRanges.java:439-484): (ai, bi) = how far `as` covers a prefix of `bs`
inline void superset_linear_merge(const V &as, const V &bs, size_t &ai_out, size_t &bi_out)
{
    size_t ai = 0, bi = 0;
    while (ai < as.size() && bi < bs.size()) {
        Rg a = as[ai];
        const Rg b = bs[bi];
        int c = cmp_intersecting(a, b);
        if (c < 0) { ai++; continue; }
        if (c > 0) break;
        if (b.s < a.s) break;
        if ((c = cmpu(b.e, a.e)) <= 0) {
            bi++;
            if (c == 0) ai++;
            continue;
        }
        // a run of touching `as` ranges must reach b's end, else stop at the start of the run
        size_t t = ai;
        bool broke = false;
        do {
            if (++t == as.size() || a.e != as[t].s) { broke = true; break; }
            a = as[t];
        } while (a.e < b.e);
        if (broke) break;
        bi++;
        ai = t;
    }
    ai_out = ai;
    bi_out = bi;
}

// AbstractRanges.union(MERGE_OVERLAPPING, left, right) (AbstractRanges.java:496-585) = Ranges.with (Ranges.java:119-127)
inline V with(const V &left, const V &right)
{
    if (&left == &right || right.empty()) return left;
    if (left.empty()) return right;
    const V *pa = &left, *pb = &right;
    {
        const int c = cmpu((*pa)[0].s, (*pb)[0].s);
        if (c > 0 || (c == 0 && pa->back().e < pb->back().e)) std::swap(pa, pb);
    }
    const V &as = *pa, &bs = *pb;
    size_t ai, bi;
    superset_linear_merge(as, bs, ai, bi);
    if (bi == bs.size()) return as;
    V result(as.begin(), as.begin() + (ptrdiff_t)ai);
    while (ai < as.size() && bi < bs.size()) {
        const Rg a = as[ai], b = bs[bi];
        const int c = cmp_intersecting(a, b);
        if (c < 0) { result.push_back(a); ai++; }
        else if (c > 0) { result.push_back(b); bi++; }
        else {
            const uint64_t start = a.s <= b.s ? a.s : b.s;
            uint64_t end = a.e >= b.e ? a.e : b.e;
            ai++; bi++;
            while (ai < as.size() || bi < bs.size()) {
                bool from_a;
                if (ai == as.size()) from_a = false;
                else if (bi == bs.size()) from_a = true;
                else from_a = as[ai].s < bs[bi].s;
                const Rg &mn = from_a ? as[ai] : bs[bi];
                if (mn.s > end) break;
                if (mn.e > end) end = mn.e;
                if (from_a) ai++; else bi++;
            }
            result.push_back({ start, end });
        }
    }
    while (ai < as.size()) result.push_back(as[ai++]);
    while (bi < bs.size()) result.push_back(bs[bi++]);
    return result;
}

// AbstractRanges.subtract(AbstractRanges) (AbstractRanges.java:223-287); findNext = the CEIL search with
// compareIntersecting from a start index (AbstractRanges.java:208-212)
inline V subtract(const V &a, const V &b)
{
    if (b.empty()) return a;
    if (a.empty() || &a == &b) return {};
    auto find_next = [](const V &in, int64_t from, const Rg &find) {
        return bsearch(from, (int64_t)in.size(), [&](int64_t i) { return cmp_intersecting(find, in[(size_t)i]); }, CEIL);
    };
    V result;
    size_t i = 0;
    int64_t j = 0;
    Rg iv = a[0];
    while (true) {
        j = find_next(b, j, iv);
        if (j < 0) {
            j = -1 - j;
            int64_t nexti = j == (int64_t)b.size() ? (int64_t)a.size() : find_next(a, (int64_t)i + 1, b[(size_t)j]);
            if (nexti < 0) nexti = -1 - nexti;
            result.push_back(iv);
            for (int64_t k = (int64_t)i + 1; k < nexti; ++k) result.push_back(a[(size_t)k]);
            if (nexti == (int64_t)a.size()) break;
            iv = a[i = (size_t)nexti];
            continue;
        }
        const Rg jv = b[(size_t)j];
        if (jv.s > iv.s) result.push_back({ iv.s, jv.s });
        if (jv.e >= iv.e) {
            if (++i == a.size()) break;
            iv = a[i];
        } else {
            iv = { jv.e, iv.e };
        }
    }
    return result;
}

// AbstractRanges.mergeTouching / copyAndMergeTouching (AbstractRanges.java:637-675)
inline V merge_touching(const V &a)
{
    if (a.empty()) return a;
    V out;
    Rg prev = a[0];
    uint64_t end = prev.e;
    for (size_t i = 1; i < a.size(); ++i) {
        const Rg &next = a[i];
        if (end != next.s) { out.push_back({ prev.s, end }); prev = next; }
        end = next.e;
    }
    out.push_back({ prev.s, end });
    return out;
}

// AbstractRanges.containsAll(AbstractKeys) (AbstractRanges.java:86-91): the keys the ranges' fold visits == all keys;
// with sorted unique keys and deoverlapped ranges that is "every key lies in some range"
inline bool contains_all_keys(const V &a, const uint64_t *keys, size_t nk, bool ei)
{
    if (a.empty()) return nk == 0;
    for (size_t i = 0; i < nk; ++i)
        if (index_of(a, keys[i], ei) < 0) return false;
    return true;
}

// AbstractRanges.containsAll(AbstractRanges) (AbstractRanges.java:96-101)
inline bool contains_all(const V &a, const V &b)
{
    if (a.empty()) return b.empty();
    if (b.empty()) return true;
    size_t ai, bi;
    superset_linear_merge(a, b, ai, bi);
    return bi == b.size();
}

// RangeDeps.isCoveredBy(Ranges covering) (primitives/RangeDeps.java:595-613): every entry range intersects some
// covering range; `rd` = the RangeDeps' ranges (sorted by Range::compare, may overlap)
inline bool is_covered_by(const V &rd, const V &covering)
{
    auto ceil_start = [&](uint64_t key) {
        int64_t x = bsearch(0, (int64_t)rd.size(), [&](int64_t i) { return cmpu(key, rd[(size_t)i].s); }, CEIL);
        return x < 0 ? -1 - x : x;
    };
    int64_t prev = 0;
    for (const Rg &range : covering) {
        const int64_t start = ceil_start(range.s), end = ceil_start(range.e);
        for (int64_t i = prev; i < start; ++i)
            if (cmp_intersecting(range, rd[(size_t)i]) != 0) return false;
        prev = end;
    }
    return prev == (int64_t)rd.size();
}

inline V load(const acc_rlist *r)
{
    if (!r) throw ArgError("null ranges");
    if (r->n && (!r->start || !r->end)) throw ArgError("null range arrays");
    V v(r->n);
    for (uint32_t i = 0; i < r->n; ++i) v[i] = { r->start[i], r->end[i] };
    return v;
}

inline int store(const V &v, uint64_t *s, uint64_t *e, uint32_t cap, uint32_t *n)
{
    if (!n) return ACC_E_ARG;
    *n = (uint32_t)v.size();
    if (v.size() > cap) return ACC_E_CAP;
    if (!v.empty() && (!s || !e)) return ACC_E_ARG;
    for (size_t i = 0; i < v.size(); ++i) { s[i] = v[i].s; e[i] = v[i].e; }
    return ACC_OK;
}

template <class F>
int guard(F &&f)
{
    try {
        return f();
    } catch (const ArgError &) {
        return ACC_E_ARG;
    } catch (...) {
        return ACC_E_STATE;
    }
}

}  // namespace rg
}  // namespace acc
