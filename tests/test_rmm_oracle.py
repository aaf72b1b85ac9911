"""CPU: the RelationMultiMap restatements (oracle/accord_oracle_rmm.c) against the canonical set model (no GPU)."""
import numpy as np
import pytest

import oracle
import rmm_cases as RC


@pytest.mark.parametrize("is_range", [False, True])
@pytest.mark.parametrize("seed,kw", [
    (1, {}),
    (2, dict(p_flip=0.5)),
    (3, dict(wide=True, p_flip=0.3)),
    (4, dict(nemesis=True)),
    (5, dict(identical=True, p_flip=0.2)),
    (6, dict(p_empty=0.6, p_keyonly=0.4)),
    (7, dict(max_replies=9, n_keys=3, n_txn=6)),
    (8, dict(inthash=True, n_keys=40, p_flip=0.2)),
])
def test_merge_oracle_is_canonical_union(is_range, seed, kw):
    """KeyDeps.merge / RangeDeps.merge == canonical union (KeyDepsTest.testMergedProperty :275-283) over raw TxnIds."""
    if not is_range and (kw.get("nemesis") or kw.get("identical")):
        pytest.skip("range-only generator")
    grp_off, half = RC.gen_groups(seed, 12, 7, is_range=is_range, **kw)
    res = oracle.rmm_merge(grp_off, half, is_range)
    assert RC.as_groups(res, is_range) == RC.canonical_merge(grp_off, half, is_range)
    # every kept instance is an input slot holding an equal TxnId
    src = res["src"].astype(np.int64)
    for f in ("msb", "lsb", "node"):
        assert np.array_equal(res[f], half[f][src])


def test_merge_oracle_instance_rules():
    """SortedArrays.linearUnion (utils/SortedArrays.java:152-281): ties keep LEFT, except in the matched prefix of a
    longer right side (the superset candidate), which is copied from the right."""
    a = (1 << 15, (5 << 16) | 2, 1)           # TxnId A
    b = (1 << 15, (6 << 16) | 2, 1)           # TxnId B > A
    c = (1 << 15, (7 << 16) | 2, 1)
    flip = lambda t: (t[0], t[1] | 0x8000, t[2])   # noqa: E731  equal under Timestamp.equals
    # reply 0: {k1: A}; reply 1 (longer): {k1: A', B, C} -> right is the superset candidate; A' taken from the right
    reps = [([10], [a], {0: [0]}), ([10], [flip(a), b, c], {0: [0, 1, 2]})]
    half = RC.build_half(reps, False)
    res = oracle.rmm_merge(np.array([0, 2], np.uint64), half, False)
    assert int(res["lsb"][0]) == flip(a)[1]
    # reply 1 shorter: left (reply 0) keeps its instance
    reps = [([10], [a, b], {0: [0, 1]}), ([10], [flip(a)], {0: [0]})]
    res = oracle.rmm_merge(np.array([0, 2], np.uint64), RC.build_half(reps, False), False)
    assert int(res["lsb"][0]) == a[1]
