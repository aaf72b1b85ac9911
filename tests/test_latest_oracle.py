"""CPU: the LatestDeps merge restatement (oracle/latest.py) — the interval fold rules and the deps it selects, against
the canonical union of the selected objects' slices."""
import numpy as np
import pytest

import latest
import latest_cases as LC


@pytest.mark.parametrize("seed,commit", [(1, False), (2, False), (3, True), (4, True)])
def test_latest_merge_is_union_of_selected_slices(seed, commit):
    kh, rh = LC.deps_objects(seed, 30)
    gs = LC.groups(seed, 12, 30, [0, 1] if not commit else [0, 1, 2, 4])
    use_local = [bool(g % 2) for g in range(len(gs))]
    r = latest.latest_deps_merge(gs, kh, rh, commit=commit, use_local=use_local)
    for g in range(len(gs)):
        assert LC.result_map(r["key"], g, False) == LC.canonical_union(kh, r["items"][g], False)
        assert LC.result_map(r["range"], g, True) == LC.canonical_union(rh, r["items"][g], True)


def test_latest_reduce_rules():
    D = latest
    b0, b1 = (1, 0, 0), (2, 0, 0)
    a = D.Entry(D.DEPS_UNKNOWN, b0, -1, [1])
    p = D.Entry(D.DEPS_PROPOSED, b1, 5, [2])
    # winner DepsProposed (<= DepsProposed): merged from the ARGUMENTS as passed -> a's phase and coordinatedDeps
    m = D._reduce(a, p)
    assert (m.known, m.coord, m.merge) == (D.DEPS_UNKNOWN, -1, [1, 2])
    k = D.Entry(D.DEPS_KNOWN, b0, 7, [3])
    assert D._reduce(a, k) is k and D._reduce(k, a) is k
    # Accept phase: ballot tie-break
    p2 = D.Entry(D.DEPS_PROPOSED, b0, 6, [])
    assert D._reduce(p2, p).merge == [2]
    # coalescing: contiguous equal neighbours keep the first entry (and its phase)
    x = D.Entry(D.DEPS_KNOWN, b0, 9, [])
    y = D.Entry(D.DEPS_COMMITTED, b1, 9, [])
    starts, values = D.merge_intervals(([0, 10], [x]), ([10, 20], [y]))
    assert starts == [0, 20] and values == [x]


def test_latest_commit_sufficient_for():
    kh, rh = LC.deps_objects(5, 10)
    gs = [[[(0, 10, 4, (1, 0, 0), 1, -1), (10, 20, 0, (1, 0, 0), -1, 2), (30, 40, 2, (1, 0, 0), 3, -1)]]]
    r = latest.latest_deps_merge(gs, kh, rh, commit=True, use_local=[False])
    assert r["sufficient"] == [[(0, 10), (30, 40)]]
    r = latest.latest_deps_merge(gs, kh, rh, commit=True, use_local=[True])
    assert r["sufficient"] == [[(0, 10), (10, 20), (30, 40)]]
    with pytest.raises(latest.InvalidKnownDeps):
        latest.latest_deps_merge([[[(0, 10, 3, (1, 0, 0), 1, -1)]]], kh, rh, commit=True, use_local=[True])
