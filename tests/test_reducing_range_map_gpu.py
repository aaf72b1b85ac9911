"""ReducingRangeMapTest's randomized canonical-model check (accord-core/src/test/java/accord/utils/
ReducingRangeMapTest.java:163-474) restated against the store's persistent MaxConflicts map on the device
(acc_maxconflicts_*: a ReducingRangeMap<Timestamp> merged with Timestamp::max, local/MaxConflicts.java:31-96).

The reference's generator (RandomMap.addOneRandom, :263-286): each addition is 1..maxRangeCount ranges of length
2 * random * maxCoverage * MAX_VALUE over the int key space (a chance of ranges pinned to MIN_VALUE + 1 / MAX_VALUE - 1)
with one Timestamp ts(random.nextInt(MAX_VALUE)) = Timestamp.fromValues(1, b, 0, node 1) (:114-117); several maps built
that way are merged (testRandomAdds, :216-241: here each map is one update batch of the persistent map, merged batch by
batch). validate (:380-471) compares get() at every canonical boundary and its neighbours, at random keys, and folds over
random key sets and over the ranges between consecutive keys of such a set (MaxConflicts.get is that fold with
Timestamp::max). The canonical model here is point-wise: the value at a key is the max over the additions whose ranges
contain it, a range query the max over the additions whose ranges intersect it (the reference's TreeMap canonical). Both
Range bound types. Keys: int -> order-preserving u64 code (x - Integer.MIN_VALUE)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

INT_MIN, INT_MAX = -(1 << 31), (1 << 31) - 1


@pytest.fixture(scope="module")
def ctx():
    from accord_amd.deps import Context
    c = Context(0)
    yield c
    c.close()


def code(x):
    return np.asarray(x, np.int64) - INT_MIN


def add_random(rng, count, max_ranges, max_cov, min_chance, hlc_space):
    """RandomMap.addRandom: `count` additions of (ranges, hlc)."""
    out = []
    for _ in range(count):
        n = 1 if max_ranges == 1 else 1 + int(rng.integers(0, max_ranges - 1))
        b = int(rng.integers(0, hlc_space))
        rs = []
        for _ in range(n):
            length = int(2 * rng.random() * max_cov * INT_MAX) or 1
            if rng.random() <= min_chance:
                rs.append((INT_MIN + 1, INT_MIN + 1 + length) if rng.random() < 0.5 else (INT_MAX - length - 1, INT_MAX - 1))
            else:
                s = int(rng.integers(0, INT_MAX - length - 1))
                rs.append((s, s + length))
        # Ranges.of: sorted, overlaps merged (the update's ranges must be sorted and non-overlapping)
        rs.sort()
        merged = []
        for s, e in rs:
            if merged and merged[-1][1] > s:
                merged[-1] = (merged[-1][0], max(merged[-1][1], e))
            else:
                merged.append((s, e))
        out.append((merged, b))
    return out


def as_update(adds, ei):
    import accord_amd.workload as W
    m, l, nd = W.encode_ts(1, np.array([b for _, b in adds], np.uint64), 0, 1)
    ro = np.concatenate([[0], np.cumsum([len(r) for r, _ in adds])]).astype(np.uint32)
    rs = np.array([code(s) for r, _ in adds for s, _ in r], np.uint64)
    re = np.array([code(e) for r, _ in adds for _, e in r], np.uint64)
    return dict(end_inclusive=ei, xmsb=np.asarray(m, np.uint64), xlsb=np.asarray(l, np.uint64),
                xnode=np.asarray(nd, np.int32), key_off=np.zeros(len(adds) + 1, np.uint32), key=np.zeros(0, np.uint64),
                rng_off=ro, rng_start=rs, rng_end=re)


def contains(s, e, k, ei):
    return (s < k) & (k <= e) if ei else (s <= k) & (k < e)


def canonical_key(adds, keys, ei):
    """max hlc (+1; 0 = none) over the additions containing each key"""
    best = np.zeros(len(keys), np.int64)
    k = code(keys)
    for r, b in adds:
        hit = np.zeros(len(keys), bool)
        for s, e in r:
            hit |= contains(code(s), code(e), k, ei)
        best = np.where(hit, np.maximum(best, b + 1), best)
    return best


def canonical_ranges(adds, qs, qe):
    """max hlc (+1) over the additions with a range intersecting any query range (compareIntersecting == 0)"""
    a, z = code(qs), code(qe)
    best = 0
    for r, b in adds:
        if any(((code(s) < z) & (a < code(e))).any() for s, e in r):
            best = max(best, b + 1)
    return best


def got_hlc(res):
    """the hlc (+1) of each query's max, 0 for Timestamp.NONE"""
    msb, lsb = res["msb"].astype(np.uint64), res["lsb"].astype(np.uint64)
    hlc = ((msb & np.uint64((1 << 15) - 1)) << np.uint64(48)) | (lsb >> np.uint64(16))
    none = (msb == 0) & (lsb == 0)
    return np.where(none, 0, hlc.astype(np.int64) + 1)


def key_queries(keys):
    import accord_amd.workload as W
    q0 = W.encode_ts(1, 0, 0, 1)
    n = len(keys)
    return dict(msb=np.full(n, q0[0], np.uint64), lsb=np.full(n, q0[1], np.uint64), node=np.full(n, 1, np.int32),
                is_range=np.zeros(n, np.uint8), part_off=np.arange(n + 1, dtype=np.uint32),
                part_start=np.array([code(k) for k in keys], np.uint64), part_end=np.array([code(k) for k in keys], np.uint64))


def multi_query(parts, is_range):
    """one query per list of parts (keys, or (start, end) ranges)"""
    import accord_amd.workload as W
    q0 = W.encode_ts(1, 0, 0, 1)
    n = len(parts)
    po = np.concatenate([[0], np.cumsum([len(p) for p in parts])]).astype(np.uint32)
    if is_range:
        ps = np.array([code(s) for p in parts for s, _ in p], np.uint64)
        pe = np.array([code(e) for p in parts for _, e in p], np.uint64)
    else:
        ps = np.array([code(k) for p in parts for k in p], np.uint64)
        pe = ps.copy()
    return dict(msb=np.full(n, q0[0], np.uint64), lsb=np.full(n, q0[1], np.uint64), node=np.full(n, 1, np.int32),
                is_range=np.full(n, 1 if is_range else 0, np.uint8), part_off=po, part_start=ps, part_end=pe)


def random_key(rng):
    """ReducingRangeMapTest.rk(Random) (:60-67)"""
    k = int(rng.integers(INT_MIN, INT_MAX, endpoint=True))
    if rng.random() < 0.5:
        k = -k if k != INT_MIN else INT_MAX
    return min(max(k, INT_MIN + 1), INT_MAX - 1)


CASES = [(a, cov, mc) for a in (1, 10, 100) for cov in (0.01, 0.1, 0.5) for mc in (0.01, 0.1)]


@pytest.mark.parametrize("ei", [1, 0])
@pytest.mark.parametrize("adds,cov,min_chance", CASES)
def test_reducing_range_map_random_adds(ctx, ei, adds, cov, min_chance):
    """testRandomAdds(seed, numberOfMerges = 3, numberOfAdditions, 3 ranges per addition, maxCoverage, chance of the
    min / max routing key) (:171-187), a few seeds per shape; the hlc space is small enough for equal timestamps."""
    from accord_amd.deps import MaxConflictsMap
    for seed in range(3):
        rng = np.random.default_rng(hash((seed, adds, cov, min_chance, ei)) & 0xFFFFFFFF)
        m = MaxConflictsMap(ctx, ei)
        try:
            applied = []
            for _merge in range(3):
                batch = add_random(rng, adds, 3, cov, min_chance, hlc_space=4 * adds + 5)
                m.update(as_update(batch, ei))
                applied += batch
                # every boundary of the canonical model and its neighbours, plus random keys (validate, :382-399)
                bounds = sorted({x for r, _ in applied for s, e in r for x in (s, e)} | {INT_MIN + 1, INT_MAX - 1})
                keys = sorted({min(max(x + d, INT_MIN + 1), INT_MAX - 1) for x in bounds for d in (-1, 0, 1)} |
                              {random_key(rng) for _ in range(200)})
                np.testing.assert_array_equal(got_hlc(m.get(key_queries(keys))), canonical_key(applied, keys, ei),
                                              err_msg=f"seed {seed} merge {_merge} point gets")
                # folds over random key sets and the ranges between their consecutive keys (validate, :402-469)
                ksets, rsets = [], []
                for _ in range(40):
                    ks = sorted({random_key(rng) for _ in range(1 + int(rng.integers(0, 20)))})
                    ksets.append(ks)
                    rr, i = [], 0
                    if len(ks) % 2 == 1 and rng.random() < 0.5:
                        rr.append((INT_MIN, ks[0])); i = 1
                    while i + 1 < len(ks):
                        rr.append((ks[i], ks[i + 1])); i += 2
                    if i < len(ks):
                        rr.append((ks[i], INT_MAX))
                    rsets.append([(s, e) for s, e in rr if s < e])
                gk = got_hlc(m.get(multi_query(ksets, False)))
                want_k = [int(canonical_key(applied, ks, ei).max()) for ks in ksets]
                np.testing.assert_array_equal(gk, want_k, err_msg=f"seed {seed} merge {_merge} key folds")
                keep = [i for i, r in enumerate(rsets) if r]
                gr = got_hlc(m.get(multi_query([rsets[i] for i in keep], True)))
                want_r = [canonical_ranges(applied, np.array([s for s, _ in rsets[i]]), np.array([e for _, e in rsets[i]]))
                          for i in keep]
                np.testing.assert_array_equal(gr, want_r, err_msg=f"seed {seed} merge {_merge} range folds")
        finally:
            m.close()


def test_reducing_range_map_one(ctx):
    """ReducingRangeMapTest.testOne's shape (:163-167: 3 merges of 1 addition of up to 3 ranges, coverage 0.1, min-key
    chance 0.1) over 200 seeds, EndInclusive (IntKey.Range)."""
    from accord_amd.deps import MaxConflictsMap
    for seed in range(200):
        rng = np.random.default_rng(8532037884171168001 % (1 << 32) + seed)
        m = MaxConflictsMap(ctx, 1)
        try:
            applied = []
            for _ in range(3):
                batch = add_random(rng, 1, 3, 0.1, 0.1, hlc_space=1 << 20)
                m.update(as_update(batch, 1))
                applied += batch
            bounds = sorted({x for r, _ in applied for s, e in r for x in (s, e)})
            keys = sorted({min(max(x + d, INT_MIN + 1), INT_MAX - 1) for x in bounds for d in (-1, 0, 1)})
            np.testing.assert_array_equal(got_hlc(m.get(key_queries(keys))), canonical_key(applied, keys, 1),
                                          err_msg=f"seed {seed}")
        finally:
            m.close()
