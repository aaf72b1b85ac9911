// ranges.hip — the Ranges algebra of accord-core on the host (PartialDeps.covering).
//
// A Ranges is a sorted, deoverlapped list of Range (start, end) u64 key codes of one bound type (Range.EndInclusive
// (s, e] or Range.StartInclusive [s, e), Range.java:40-138). Store slicing, the LatestDeps intervals and
// PartialDeps.covering are a handful of ranges per object, so this is plain host code beside the device kernels;
// every operation restates its reference method step by step (file:line in each function), so results match the
// reference's element for element (e.g. Ranges.with merges touching ranges only inside an overlapping run, as the
// union loop's `min.start() > end` test does).
#include "ranges.hpp"


using namespace acc::rg;

extern "C" {

int acc_ranges_of(const acc_rlist *in, uint64_t *out_start, uint64_t *out_end, uint32_t cap, uint32_t *out_n)
{
    return guard([&] { return store(of(load(in)), out_start, out_end, cap, out_n); });
}

int acc_ranges_with(const acc_rlist *a, const acc_rlist *b, uint64_t *out_start, uint64_t *out_end, uint32_t cap,
                    uint32_t *out_n)
{
    return guard([&] {
        const V x = load(a), y = load(b);
        return store(with(check_sorted_deoverlapped(x), check_sorted_deoverlapped(y)), out_start, out_end, cap, out_n);
    });
}

int acc_ranges_subtract(const acc_rlist *a, const acc_rlist *b, uint64_t *out_start, uint64_t *out_end, uint32_t cap,
                        uint32_t *out_n)
{
    return guard([&] {
        const V x = load(a), y = load(b);
        return store(subtract(check_sorted_deoverlapped(x), check_sorted_deoverlapped(y)), out_start, out_end, cap, out_n);
    });
}

int acc_ranges_merge_touching(const acc_rlist *a, uint64_t *out_start, uint64_t *out_end, uint32_t cap, uint32_t *out_n)
{
    return guard([&] { const V x = load(a); return store(merge_touching(check_sorted_deoverlapped(x)), out_start, out_end, cap, out_n); });
}

int acc_ranges_select(const acc_rlist *a, const uint32_t *idx, uint32_t k, uint64_t *out_start, uint64_t *out_end,
                      uint32_t cap, uint32_t *out_n)
{
    return guard([&] {
        const V x = load(a);
        if (k && !idx) throw ArgError("null indexes");
        V sel(k);
        for (uint32_t i = 0; i < k; ++i) {
            if (idx[i] >= x.size()) throw ArgError("index out of range");
            sel[i] = x[idx[i]];
        }
        return store(check_sorted_deoverlapped(sel), out_start, out_end, cap, out_n);
    });
}

int acc_ranges_index_of(const acc_rlist *a, uint32_t end_inclusive, uint64_t key, int64_t *out_index)
{
    return guard([&] {
        if (!out_index || end_inclusive > 1) throw ArgError("bad argument");
        *out_index = index_of(load(a), key, end_inclusive != 0);
        return ACC_OK;
    });
}

int acc_ranges_contains_all_keys(const acc_rlist *a, uint32_t end_inclusive, const uint64_t *keys, uint32_t n_keys,
                                 int32_t *out)
{
    return guard([&] {
        if (!out || end_inclusive > 1 || (n_keys && !keys)) throw ArgError("bad argument");
        *out = contains_all_keys(load(a), keys, n_keys, end_inclusive != 0) ? 1 : 0;
        return ACC_OK;
    });
}

int acc_ranges_contains_all(const acc_rlist *a, const acc_rlist *b, int32_t *out)
{
    return guard([&] {
        if (!out) throw ArgError("bad argument");
        *out = contains_all(load(a), load(b)) ? 1 : 0;
        return ACC_OK;
    });
}

int acc_rangedeps_is_covered_by(const acc_rlist *range_deps_ranges, const acc_rlist *covering, int32_t *out)
{
    return guard([&] {
        if (!out) throw ArgError("bad argument");
        *out = is_covered_by(load(range_deps_ranges), load(covering)) ? 1 : 0;
        return ACC_OK;
    });
}

}  // extern "C"
