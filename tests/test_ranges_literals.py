"""The reference's literal Ranges expectations, through the library's Ranges algebra (acc_ranges_*, host code of
libaccord_amd.so): accord-core/src/test/java/accord/utils/RangesTest.java:39-116 and
accord-core/src/test/java/accord/primitives/AbstractRangesTest.java:38-64. The algebra is what PartialDeps.covering
(acc_partial_deps_reduce), store slicing and the LatestDeps intervals apply.

RangesTest builds IntKey ranges: IntKey.Range extends Range.EndInclusive (test/.../impl/IntKey.java:140-152), so the
ranges here are (s, e] over integer key codes. Each test runs twice: in the CPU suite and, marked gpu, in the GPU
suite's process (the same host functions of the same library)."""
import numpy as np
import pytest

WHERE = [pytest.param("cpu"), pytest.param("gpu", marks=pytest.mark.gpu)]


def R(*pairs):
    from accord_amd.ranges import Ranges
    return Ranges.of(*pairs)


@pytest.mark.parametrize("where", WHERE)
def test_range_index_for_key(where):
    """RangesTest.rangeIndexForKeyTest (RangesTest.java:39-48)."""
    ranges = R((100, 200), (300, 400))
    assert ranges.index_of(50) == -1
    assert ranges.index_of(150) == 0
    assert ranges.index_of(250) == -2
    assert ranges.index_of(350) == 1
    assert ranges.index_of(450) == -3


@pytest.mark.parametrize("where", WHERE)
def test_difference(where):
    """RangesTest.differenceTest (RangesTest.java:50-76)."""
    assert R((100, 200)).subtract(R((125, 175))) == R((100, 125), (175, 200))
    assert R((100, 200)).subtract(R((100, 125), (175, 200))) == R((125, 175))
    assert R((100, 200)).subtract(R((0, 75), (175, 200))) == R((100, 175))
    assert R((100, 200)).subtract(R((0, 75), (200, 205))) == R((100, 200))
    assert R((100, 200), (250, 350)).subtract(R((0, 125), (175, 300))) == R((125, 175), (300, 350))
    assert R((100, 200), (250, 350)).subtract(R((0, 125), (225, 300))) == R((125, 200), (300, 350))
    assert R((100, 200)).subtract(R((0, 125), (135, 140), (160, 170), (170, 175))) == R((125, 135), (140, 160), (175, 200))


@pytest.mark.parametrize("where", WHERE)
def test_add(where):
    """RangesTest.addTest (RangesTest.java:78-83): touching ranges of different inputs stay apart."""
    assert R((0, 50), (100, 150)).with_(R((50, 100), (150, 200))) == R((0, 50), (50, 100), (100, 150), (150, 200))


@pytest.mark.parametrize("where", WHERE)
def test_merge(where):
    """RangesTest.mergeTest / assertMergeResult (RangesTest.java:85-100): both argument orders."""
    from accord_amd.ranges import Ranges
    cases = [(R((0, 50), (100, 350)), R((100, 250), (300, 350)), R((0, 50), (200, 300), (310, 315))),
             (R((0, 100)), Ranges.EMPTY, R((0, 100)))]
    for expected, a, b in cases:
        assert a.with_(b) == expected
        assert b.with_(a) == expected


@pytest.mark.parametrize("where", WHERE)
def test_merge_touching(where):
    """RangesTest.mergeTouchingTest (RangesTest.java:102-108)."""
    assert R((0, 100), (100, 200), (200, 300), (300, 400)).merge_touching() == R((0, 400))
    assert R((0, 100), (100, 200), (300, 400)).merge_touching() == R((0, 200), (300, 400))
    assert R((0, 100), (200, 300), (300, 400)).merge_touching() == R((0, 100), (200, 400))


@pytest.mark.parametrize("where", WHERE)
def test_select(where):
    """RangesTest.selectTest (RangesTest.java:110-116)."""
    test_ranges = R((0, 100), (100, 200), (200, 300), (300, 400), (400, 500))
    got = test_ranges.select([1, 3])
    assert got == R((100, 200), (300, 400))


@pytest.mark.parametrize("where", WHERE)
def test_select_rejects_unsorted(where):
    """Ranges.select -> ofSortedAndDeoverlapped throws IllegalArgumentException (AbstractRanges.java:789-798)."""
    from accord_amd.deps import IllegalArgumentException
    with pytest.raises(IllegalArgumentException):
        R((0, 100), (100, 200), (200, 300)).select([2, 0])


@pytest.mark.parametrize("where", WHERE)
def test_abstract_ranges_to_string(where):
    """AbstractRangesTest.testToString (AbstractRangesTest.java:38-48): start-inclusive ranges of prefixed keys."""
    from accord_amd.ranges import ranges_to_string
    s = ranges_to_string([0, 10, 20, 30], [10, 20, 30, 40], ["first", "first", "second", "third"],
                         start_inclusive=True, end_inclusive=False)
    assert s == "[first:[[0,10), [10,20)], second:[[20,30)], third:[[30,40)]]"


@pytest.mark.parametrize("where", WHERE)
@pytest.mark.parametrize("seed", range(8))
def test_contains_all_property(where, seed):
    """AbstractRangesTest.testContainsAll (AbstractRangesTest.java:50-64): keys drawn inside the ranges are all
    contained, keys drawn outside are not; both bound types (random ranges over int keys as AccordGens.ranges)."""
    from accord_amd.ranges import Ranges
    rng = np.random.default_rng(seed)
    for ei in (1, 0):
        pts = np.unique(rng.integers(0, 1 << 20, size=2 * int(rng.integers(1, 10))))
        if len(pts) % 2:
            pts = pts[:-1]
        s, e = pts[0::2], pts[1::2]
        ranges = Ranges(s, e, ei)
        lo = s + (1 if ei else 0)                    # first key inside: (s, e] -> s + 1, [s, e) -> s
        width = (e - s).astype(np.int64)
        pick = rng.integers(0, len(s), size=10)
        inside = np.unique(lo[pick] + (rng.random(10) * width[pick]).astype(np.uint64))
        assert ranges.contains_all_keys(inside)
        assert all(ranges.contains(int(k)) for k in inside)
        gaps = [int(x) for x in (s if ei else s - 1)[s > 0]]      # keys just outside each range's start
        gaps += [int(x) + (1 if ei else 0) for x in e]            # and just past its end
        outside = np.unique(np.array([g for g in gaps if not ranges.contains(g)], np.uint64))
        if len(outside):
            assert not ranges.contains_all_keys(np.unique(np.concatenate([inside, outside[:1]])))


@pytest.mark.parametrize("where", WHERE)
def test_contains_all_ranges_and_covered_by(where):
    """AbstractRanges.containsAll(Ranges) (supersetLinearMerge, AbstractRanges.java:96-101, 439-484) and
    RangeDeps.isCoveredBy (primitives/RangeDeps.java:595-613), worked from the reference loops by hand."""
    from accord_amd.ranges import Ranges, range_deps_is_covered_by
    cov = R((0, 100), (100, 200), (300, 400))
    assert cov.contains_all(R((10, 20), (150, 200)))
    assert cov.contains_all(R((50, 150)))            # spans two touching covering ranges
    assert not cov.contains_all(R((150, 250)))
    assert not cov.contains_all(R((250, 260)))
    assert Ranges.EMPTY.contains_all(Ranges.EMPTY) and not Ranges.EMPTY.contains_all(R((1, 2)))
    assert range_deps_is_covered_by([10, 50, 150, 310], [20, 60, 200, 320], cov)
    assert not range_deps_is_covered_by([10, 210], [20, 220], cov)   # (210, 220] meets no covering range
    assert range_deps_is_covered_by([90], [120], cov)                # intersects the first covering range
    assert range_deps_is_covered_by([], [], cov)


@pytest.mark.parametrize("where", WHERE)
@pytest.mark.parametrize("seed", range(6))
def test_with_subtract_against_point_sets(where, seed):
    """with / subtract / mergeTouching as sets of integer points (x in (s, e]) equal the point-set union /
    difference, and every result is sorted and deoverlapped (Ranges' invariant)."""
    from accord_amd.ranges import Ranges
    rng = np.random.default_rng(100 + seed)

    def rand():
        pts = np.unique(rng.integers(0, 400, size=2 * int(rng.integers(0, 8))))
        if len(pts) % 2:
            pts = pts[:-1]
        return Ranges.of(*zip(pts[0::2].tolist(), pts[1::2].tolist())) if len(pts) else Ranges.EMPTY

    def pts(r):
        return {x for s, e in r for x in range(s + 1, e + 1)}

    def ok(r):
        return all(int(r.end[i - 1]) <= int(r.start[i]) for i in range(1, len(r))) and all(s < e for s, e in r)

    for _ in range(30):
        a, b = rand(), rand()
        u, d = a.with_(b), a.subtract(b)
        assert pts(u) == pts(a) | pts(b) and ok(u)
        assert pts(d) == pts(a) - pts(b) and ok(d)
        m = u.merge_touching()
        assert pts(m) == pts(u) and ok(m)
        assert all(int(m.end[i - 1]) < int(m.start[i]) for i in range(1, len(m)))
        assert a.with_(b) == b.with_(a)
