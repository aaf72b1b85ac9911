"""The reference's literal Range vectors (accord-core/src/test/java/accord/utils/RangeTest.java), asserted through the
deps paths that depend on them: the literal values of the Java test are the expectations here, not the oracle's output.

* containsTest :97-110, higherKeyIndexTest :120-140, lowKeyIndexTest :163-188 — a range txn over the CommandsForKey
  of keys(10..16): the keys its KeyDeps covers (`InMemoryCommandStore.mapReduceForKey` :274-289, the `subMap` with the
  range's inclusive flags) are exactly the keys `Range.contains`; the first covered index is `nextCeilKeyIndex` and one
  past the last is `nextHigherKeyIndex`. A range covering none of the keys yields no KeyDeps key; the Java's negative
  (or insertion-point) value for that case is only observable here as "nothing covered".
* compareIntersectingTest :206-226 — a range command r(100,200) against later range txns: a RangeDeps entry iff
  `compareIntersecting == 0` (`InMemoryCommandStore.java:950-959`), both directions, and the stabbing of a built
  RangeDeps (`SearchableRangeList.forEach`, `acc_rangedeps_stab`).
* intersectsTest :244-256 — a range command r(100,200) against later key txns: a RangeDeps entry iff
  `range.intersects(keys)`; and a later range txn over those key txns' CFKs (mixed KeyDeps).
* invalidRangeTest :91-95 — start >= end is an IllegalArgumentException at the ABI.
* intersectionTest :236-242 — `Range.intersection`, as the store slicing (`sharded.slice_ranges`) applies it.

`IntKey.range(start, end)` is `Range.EndInclusive` (tst/impl/IntKey.java:140-150, 206); keys are IntKey codes.
Each case runs on the C oracle (CPU) and through the HIP library (`-m gpu`)."""
import numpy as np
import pytest

import rd_cases
from accord_amd import sharded
from accord_amd import workload as W

BACKENDS = ["oracle", pytest.param("gpu", marks=pytest.mark.gpu)]


def code(v: int) -> int:
    return int(W.int_key_code(np.array([v]))[0])


@pytest.fixture(scope="module")
def gpu_ctx():
    from accord_amd.deps import Context
    c = Context(0)
    yield c
    c.close()


@pytest.fixture
def run(request):
    backend = request.param

    def mixed(rb):
        if backend == "oracle":
            import oracle
            return oracle.keydeps_mixed(rb)
        return request.getfixturevalue("gpu_ctx").calculate_partial_key_deps_mixed(rb)

    def ranges(rb):
        if backend == "oracle":
            import oracle
            return oracle.rangedeps_batch(rb)
        return request.getfixturevalue("gpu_ctx").calculate_partial_range_deps(rb)

    return dict(backend=backend, mixed=mixed, ranges=ranges, request=request)


def covered_keys(res, t):
    """KeyDeps keys (IntKey codes) of txn t."""
    return [int(x) for x in res.kd_key[int(res.kd_off[t]):int(res.kd_off[t + 1])]]


def range_deps(res, t):
    """{(start, end): [dep batch index]} of txn t."""
    r, d, a = res.txn(t)
    out, start = {}, len(r)
    for i, rid in enumerate(r.tolist()):
        end = int(a[i])
        out[(int(res.rng_start[rid]), int(res.rng_end[rid]))] = [int(d[x]) for x in a[start:end]]
        start = end
    return out


KEYS_10_16 = [10, 11, 12, 13, 14, 15, 16]


def key_index_batch(cases, keys=KEYS_10_16):
    """One key txn (Write, PREACCEPTED) per key of `keys`, then one range txn per case: the range txns of one bound
    type go into one batch (one Range type per store). Returns {end_inclusive: (batch, [(case, txn index)])}."""
    out = {}
    for ei in (1, 0):
        mine = [c for c in cases if c[1] == ei]
        if not mine:
            continue
        txns = [dict(kind=W.WRITE, keys=[code(k)]) for k in keys]
        at = []
        for c in mine:
            at.append((c, len(txns)))
            txns.append(dict(kind=W.WRITE, ranges=[(code(c[2]), code(c[3]))]))
        out[ei] = (rd_cases.build(txns, ei), at)
    return out


@pytest.mark.parametrize("run", BACKENDS, indirect=True)
def test_contains(run):
    """RangeTest.containsTest :97-110: EndInclusive(10,20) contains 20 not 10; StartInclusive(10,20) contains 10 not 20.
    Checked both ways: key txns on 10 and 20 against the range command (RangeDeps), and the range txn over their
    CFKs (KeyDeps)."""
    for ei, inside, outside in ((1, 20, 10), (0, 10, 20)):
        rb = rd_cases.build([dict(kind=W.WRITE, ranges=[(code(10), code(20))]),
                             dict(kind=W.WRITE, keys=[code(10)]), dict(kind=W.WRITE, keys=[code(20)]),
                             dict(kind=W.WRITE, ranges=[(code(10), code(20))])], ei)
        rd = run["ranges"](rb)
        got = {k: bool(range_deps(rd, t)) for t, k in ((1, 10), (2, 20))}
        assert got == {inside: True, outside: False}, (ei, got)
        kd = run["mixed"](rb)
        assert covered_keys(kd, 3) == [code(inside)], ei
        # the range txn's KeyDeps entry for the covered key is the key txn on it
        _, d, _ = kd.txn(3)
        assert d.tolist() == [1 if inside == 10 else 2]


# (expected, end_inclusive, start, end) — RangeTest.java:123-139
HIGHER = [(0, 1, 0, 9), (0, 0, 0, 10), (0, 1, 0, 5), (0, 0, 0, 5),
          (1, 1, 9, 10), (0, 0, 9, 10), (5, 1, 11, 14), (4, 0, 11, 14), (6, 1, 11, 15), (5, 0, 11, 15),
          (7, 1, 16, 25), (7, 0, 16, 25), (7, 1, 20, 25), (7, 0, 20, 25)]
# RangeTest.java:166-184
LOWER = [(-1, 1, 0, 5), (-1, 0, 0, 5), (-1, 1, 0, 9), (-1, 0, 0, 9),
         (0, 1, 5, 10), (-1, 0, 5, 10), (2, 1, 11, 15), (1, 0, 11, 15), (3, 1, 12, 14), (2, 0, 12, 14),
         (6, 1, 15, 20), (5, 0, 15, 20),
         (-8, 1, 16, 20), (6, 0, 16, 20), (-8, 1, 20, 25), (-8, 0, 20, 25)]


@pytest.mark.parametrize("run", BACKENDS, indirect=True)
def test_higher_key_index(run):
    """RangeTest.higherKeyIndexTest :120-140 (`Range.nextHigherKeyIndex`, Range.java:361-367): when the range covers a
    key, one past the last covered key's index is the literal; a literal 0 with nothing covered is a range below
    keys(10..16) (or ending where its exclusive end is 10), a literal 7 with nothing covered is a range above."""
    for ei, (rb, at) in key_index_batch(HIGHER).items():
        kd = run["mixed"](rb)
        for (exp, _, s, e), t in at:
            cov = covered_keys(kd, t)
            idx = [KEYS_10_16.index(k - (1 << 31)) for k in cov]
            assert idx == list(range(idx[0], idx[-1] + 1)) if idx else True
            if idx:
                assert idx[-1] + 1 == exp, (ei, s, e, idx)
            else:
                assert exp in (0, 7), (ei, s, e)
                # the range lies wholly below (exp 0) or above (exp 7) every key
                assert (e <= 10) if exp == 0 else (s >= 16), (ei, s, e)


@pytest.mark.parametrize("run", BACKENDS, indirect=True)
def test_low_key_index(run):
    """RangeTest.lowKeyIndexTest :163-188 (`Range.nextCeilKeyIndex`, Range.java:375-378): a non-negative literal is
    the first covered key's index; a negative literal means no key of keys(10..16) is covered (the reference asserts
    `!contains(keys[lowerBound])` and `!contains(keys[last])` there, :150-154)."""
    for ei, (rb, at) in key_index_batch(LOWER).items():
        kd = run["mixed"](rb)
        for (exp, _, s, e), t in at:
            cov = covered_keys(kd, t)
            if exp >= 0:
                assert cov and cov[0] == code(KEYS_10_16[exp]), (ei, s, e, cov)
            else:
                assert cov == [], (ei, s, e, cov)
    # non-intersecting: rangeStartIncl(12, 14) over keys(10, 16) -> -2 (:187)
    (rb, at), = key_index_batch([(-2, 0, 12, 14)], keys=[10, 16]).values()
    assert covered_keys(run["mixed"](rb), at[0][1]) == []


# r(100,200).compareIntersecting(r(s, e)) — RangeTest.java:208-225
COMPARE_INTERSECTING = [(1, 0, 100), (1, 0, 99), (0, 0, 101), (0, 99, 199), (0, 99, 200), (0, 99, 201),
                        (0, 101, 199), (0, 125, 175), (0, 100, 201), (0, 101, 201), (0, 199, 300),
                        (-1, 200, 300), (-1, 201, 300)]


@pytest.mark.parametrize("run", BACKENDS, indirect=True)
def test_compare_intersecting(run):
    """RangeTest.compareIntersectingTest :206-226 through the range-command scan (`mapReduceRangesInternal`,
    InMemoryCommandStore.java:950-959: a stored range becomes a RangeDeps key iff it intersects the query's ranges).
    Forward: the range command r(100,200) then one range txn per case; reverse: every case's range as a command,
    then one r(100,200) txn, whose RangeDeps keys are exactly the intersecting cases."""
    txns = [dict(kind=W.WRITE, ranges=[(code(100), code(200))])]
    txns += [dict(kind=W.WRITE, ranges=[(code(s), code(e))]) for _, s, e in COMPARE_INTERSECTING]
    rb = rd_cases.build(txns, 1)
    rd = run["ranges"](rb)
    for i, (exp, s, e) in enumerate(COMPARE_INTERSECTING):
        deps = range_deps(rd, 1 + i)
        has = (code(100), code(200)) in deps and 0 in deps[(code(100), code(200))]
        assert has == (exp == 0), (s, e, deps)
    # reverse direction: r(100,200) queried last, every case is a command before it
    txns = [dict(kind=W.WRITE, ranges=[(code(s), code(e))]) for _, s, e in COMPARE_INTERSECTING]
    txns.append(dict(kind=W.WRITE, ranges=[(code(100), code(200))]))
    rb = rd_cases.build(txns, 1)
    deps = range_deps(run["ranges"](rb), len(COMPARE_INTERSECTING))
    want = sorted((code(s), code(e)) for exp, s, e in COMPARE_INTERSECTING if exp == 0)
    assert sorted(deps) == want
    # each stored range's TxnIds = the commands that carry it (ranges are distinct here, so one each)
    for i, (exp, s, e) in enumerate(COMPARE_INTERSECTING):
        if exp == 0:
            assert deps[(code(s), code(e))] == [i]


@pytest.mark.gpu
def test_compare_intersecting_stab(gpu_ctx):
    """The same literals through `acc_rangedeps_stab` (SearchableRangeList.forEach over a built RangeDeps): the cases'
    ranges form one RangeDeps (sorted by Range::compare, one TxnId each), queried with the range r(100,200)."""
    from accord_amd.deps import rangedeps_stab
    cases = sorted({(code(s), code(e)) for _, s, e in COMPARE_INTERSECTING})
    n = len(cases)
    m = dict(key_off=np.array([0, n], np.uint64), key_a=np.array([c[0] for c in cases], np.uint64),
             key_b=np.array([c[1] for c in cases], np.uint64), val_off=np.array([0, n], np.uint64),
             k2v_off=np.array([0, 2 * n], np.uint64),
             k2v=np.concatenate([np.arange(n + 1, 2 * n + 1), np.arange(n)]).astype(np.int32))
    got = rangedeps_stab(gpu_ctx, m, np.zeros(1, np.uint32), np.array([code(100)], np.uint64),
                         np.array([code(200)], np.uint64), end_inclusive=True)
    hit = [cases[int(i)] for i in got["range_idx"][int(got["range_off"][0]):int(got["range_off"][1])]]
    want = sorted((code(s), code(e)) for exp, s, e in COMPARE_INTERSECTING if exp == 0)
    assert hit == want


# r(100,200).intersects(keys(...)) — RangeTest.java:247-255
INTERSECTS = [(True, [50, 150, 250]), (True, [150, 250]), (True, [50, 150]),
              (False, []), (False, [50, 75]), (False, [50, 75, 250, 300]), (False, [250, 300])]


@pytest.mark.parametrize("run", BACKENDS, indirect=True)
def test_intersects(run):
    """RangeTest.intersectsTest :244-256: the range command r(100,200) is a RangeDeps entry of a later key txn iff
    `range.intersects(keys)`; and a later range txn r(100,200) over the key txns' CFKs lists exactly the
    intersecting key txns (KeyDeps), under exactly the contained keys."""
    txns = [dict(kind=W.WRITE, ranges=[(code(100), code(200))])]
    txns += [dict(kind=W.WRITE, keys=[code(k) for k in ks]) for _, ks in INTERSECTS]
    txns.append(dict(kind=W.WRITE, ranges=[(code(100), code(200))]))
    rb = rd_cases.build(txns, 1)
    rd = run["ranges"](rb)
    for i, (exp, ks) in enumerate(INTERSECTS):
        assert bool(range_deps(rd, 1 + i)) == exp, ks
    kd = run["mixed"](rb)
    q = len(txns) - 1
    _, d, _ = kd.txn(q)
    assert sorted(d.tolist()) == [1 + i for i, (exp, _) in enumerate(INTERSECTS) if exp]
    assert covered_keys(kd, q) == [code(150)]


@pytest.mark.parametrize("run", BACKENDS, indirect=True)
@pytest.mark.parametrize("end_inclusive", [1, 0])
@pytest.mark.parametrize("s,e", [(1, 1), (2, 1)])
def test_invalid_range(run, end_inclusive, s, e):
    """RangeTest.invalidRangeTest :91-95: start >= end is an IllegalArgumentException (Range.java constructors)."""
    rb = rd_cases.build([dict(kind=W.WRITE, ranges=[(code(s), code(e))]), dict(kind=W.WRITE, keys=[code(1)])],
                        end_inclusive)
    if run["backend"] == "oracle":
        import oracle
        with pytest.raises(oracle.OracleError):
            run["ranges"](rb)
    else:
        from accord_amd.deps import IllegalArgumentException
        with pytest.raises(IllegalArgumentException):
            run["ranges"](rb)
        with pytest.raises(IllegalArgumentException):
            run["mixed"](rb)


def test_intersection_store_slice():
    """RangeTest.intersectionTest :236-242 (`Range.intersection`, both argument orders) as the store slicing applies
    it to range commands (`Ranges.slice`, InMemoryCommandStore.java:756-760)."""
    for (ws, we), (as_, ae), (bs, be) in (((25, 75), (0, 75), (25, 100)), ((0, 75), (0, 75), (0, 100)),
                                          ((25, 100), (0, 100), (25, 100)), ((25, 75), (0, 100), (25, 75)),
                                          ((0, 100), (0, 100), (0, 100))):
        for (x, y), (lo, hi) in (((as_, ae), (bs, be)), ((bs, be), (as_, ae))):
            keep, s, e = sharded.slice_ranges(np.array([x], np.uint64), np.array([y], np.uint64), lo, hi)
            assert bool(keep[0]) and (int(s[0]), int(e[0])) == (ws, we)
