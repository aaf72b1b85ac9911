"""GPU parity: acc_latest_deps_merge (LatestDeps.mergeProposal / mergeCommit, primitives/LatestDeps.java:306-326, as
Recover calls them, coordinate/Recover.java:295-355) vs the restatement in oracle/latest.py: every merged KeyDeps /
RangeDeps array bit for bit, and sufficientFor."""
import numpy as np
import pytest

import latest
import latest_cases as LC

pytestmark = pytest.mark.gpu

FIELDS = ("key_off", "key_a", "val_off", "msb", "lsb", "node", "k2v_off", "k2v")


@pytest.fixture(scope="module")
def ctx():
    from accord_amd.deps import Context
    c = Context(0)
    yield c
    c.close()


def check(got, ref):
    for half, rng in (("key", False), ("range", True)):
        for f in FIELDS + (("key_b",) if rng else ()):
            np.testing.assert_array_equal(got[half][f], ref[half][f], err_msg=f"{half} {f}")
    assert got["sufficient"] == ref["sufficient"]


@pytest.mark.parametrize("seed,commit", [(1, False), (2, False), (3, True), (4, True), (5, True)])
def test_latest_merge_vs_oracle(ctx, seed, commit):
    from accord_amd.deps import latest_deps_merge
    kh, rh = LC.deps_objects(seed, 40)
    gs = LC.groups(seed, 60, 40, [0, 1] if not commit else [0, 1, 2, 4])
    tids = [(1 << 15, (g + 1) << 16, 1) for g in range(len(gs))]
    exes = [t if g % 2 else (t[0], t[1] + (5 << 16), t[2]) for g, t in enumerate(tids)]
    got = latest_deps_merge(ctx, gs, kh, rh, commit=commit, txn_ids=tids, execute_ats=exes)
    ref = latest.latest_deps_merge(gs, kh, rh, commit=commit, use_local=[bool(g % 2) for g in range(len(gs))])
    check(got, ref)


def test_latest_merge_empty_and_errors(ctx):
    from accord_amd.deps import IllegalArgumentException, IllegalStateException, latest_deps_merge
    kh, rh = LC.deps_objects(9, 8)
    got = latest_deps_merge(ctx, [[], [[]]], kh, rh)
    assert all(int(x) == 0 for x in got["key"]["key_off"]) and got["sufficient"] == [[], []]
    with pytest.raises(IllegalStateException):    # DepsKnown is no proposal phase
        latest_deps_merge(ctx, [[[(0, 10, 4, (1, 0, 0), 1, -1)]]], kh, rh)
    with pytest.raises(IllegalStateException):    # DepsErased is no commit phase
        latest_deps_merge(ctx, [[[(0, 10, 3, (1, 0, 0), 1, -1)]]], kh, rh, commit=True, txn_ids=[(1, 0, 0)],
                          execute_ats=[(1, 0, 0)])
    with pytest.raises(IllegalArgumentException):  # overlapping intervals in one reply
        latest_deps_merge(ctx, [[[(0, 10, 0, (1, 0, 0), -1, 1), (5, 20, 0, (1, 0, 0), -1, 2)]]], kh, rh)
    with pytest.raises(IllegalArgumentException):  # unknown deps object
        latest_deps_merge(ctx, [[[(0, 10, 1, (1, 0, 0), 99, -1)]]], kh, rh)
