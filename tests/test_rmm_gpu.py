"""GPU parity of the RelationMultiMap helpers against the oracle restatements
(oracle/accord_oracle_rmm.c): invert, KeyDeps/RangeDeps.slice + trimUnusedValues, RangeDeps stabbing queries
(SearchableRangeList.forEach order, RangeDeps.computeTxnIds)."""
import numpy as np
import pytest

import rmm_cases as RC

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from accord_amd.deps import Context
    c = Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("is_range,seed", [(False, 1), (True, 2), (False, 3)])
def test_invert(ctx, is_range, seed):
    import oracle
    from accord_amd.deps import rmm_invert
    _, half = RC.gen_groups(seed, 60, 7, is_range=is_range, p_keyonly=0.3, p_extra=0.5, wide=seed == 3)
    m = RC.as_batch(half)
    off, ints = rmm_invert(ctx, m)
    nk = np.diff(m["key_off"].astype(np.int64)).astype(np.uint64)
    nv = np.diff(m["val_off"].astype(np.int64)).astype(np.uint64)
    roff, rints = oracle.invert(m["k2v_off"], m["k2v"], nk, nv)
    np.testing.assert_array_equal(off, roff)
    np.testing.assert_array_equal(ints, rints)


@pytest.mark.parametrize("is_range,end_inclusive,seed", [(False, True, 4), (False, False, 5), (True, True, 6), (True, False, 7)])
def test_slice(ctx, is_range, end_inclusive, seed):
    import oracle
    from accord_amd.deps import rmm_slice
    _, half = RC.gen_groups(seed, 80, 6, is_range=is_range, p_keyonly=0.2, p_empty=0.2, p_extra=0.4)
    m = RC.as_batch(half)
    n = len(m["key_off"]) - 1
    so, ss, se = RC.gen_select(seed + 50, n)
    got = rmm_slice(ctx, m, so, ss, se, end_inclusive)
    ref = oracle.rmm_slice(m, so, ss, se, is_range, end_inclusive)
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


def _stab_check(ctx, m, grp, qs, qe, end_inclusive):
    import oracle
    from accord_amd.deps import rangedeps_stab
    got = rangedeps_stab(ctx, m, grp, qs, qe, end_inclusive, want_txns=True)
    roff, ridx = oracle.rmm_stab(grp, qs, qe, qe is None, end_inclusive, m["key_off"], m["key_a"], m["key_b"])
    np.testing.assert_array_equal(got["range_off"], roff)
    np.testing.assert_array_equal(got["range_idx"], ridx)
    # computeTxnIds: sorted unique TxnId indices of the hit ranges (primitives/RangeDeps.java:629-643)
    for q in range(0, len(grp), max(1, len(grp) // 200)):
        g = int(grp[q])
        h = m["k2v"][int(m["k2v_off"][g]):int(m["k2v_off"][g + 1])]
        nk = int(m["key_off"][g + 1] - m["key_off"][g])
        ids = set()
        for k in ridx[int(roff[q]):int(roff[q + 1])].tolist():
            ids.update(int(x) for x in h[(nk if k == 0 else int(h[k - 1])):int(h[k])])
        assert got["txn_idx"][int(got["txn_off"][q]):int(got["txn_off"][q + 1])].tolist() == sorted(ids), q


@pytest.mark.parametrize("gen", ["plain", "nemesis", "identical", "wide"])
@pytest.mark.parametrize("end_inclusive", [True, False])
def test_stab_key_and_range_queries(ctx, gen, end_inclusive):
    """RangeDepsTest.Validate (tst/primitives/RangeDepsTest.java:131-148) over the reference's generators: every range
    start, end and random probes, as key and as range queries."""
    kw = {} if gen == "plain" else {gen: True}
    _, half = RC.gen_groups(8, 30, 4, is_range=True, n_keys=25, **kw)
    m = RC.as_batch(half)
    rng = np.random.default_rng(9)
    n = len(m["key_off"]) - 1
    grp, qs, qe = [], [], []
    for g in range(n):
        a0, a1 = int(m["key_off"][g]), int(m["key_off"][g + 1])
        for i in range(a0, a1):
            for x in (int(m["key_a"][i]), int(m["key_b"][i])):
                grp.append(g); qs.append(x)
        hi = (1 << 63) if gen == "wide" else 1500
        for x in rng.integers(0, hi, size=8):
            grp.append(g); qs.append(int(x))
    grp, qs = np.array(grp, np.uint32), np.array(qs, np.uint64)
    _stab_check(ctx, m, grp, qs, None, end_inclusive)
    qe = qs + np.uint64(1) + rng.integers(0, 200, size=len(qs)).astype(np.uint64)
    _stab_check(ctx, m, grp, qs, qe, end_inclusive)


def test_stab_full_world_and_random(ctx):
    """SearchableRangeListTest.fullWorld / random (tst/utils/SearchableRangeListTest.java:36-115): 1000 unit ranges
    against every prefix and suffix query; 10k random ranges against picked / random / spanning queries; ascending
    index order checked against brute force."""
    n = 1000
    m = dict(key_off=np.array([0, n], np.uint64), key_a=np.arange(n, dtype=np.uint64),
             key_b=np.arange(1, n + 1, dtype=np.uint64), val_off=np.array([0, 1], np.uint64),
             k2v_off=np.array([0, 2 * n], np.uint64),
             k2v=np.concatenate([np.arange(n + 1, 2 * n + 1), np.zeros(n)]).astype(np.int32))
    qs = np.concatenate([np.arange(n), np.zeros(n)]).astype(np.uint64)
    qe = np.concatenate([np.full(n, n), n - np.arange(n)]).astype(np.uint64)
    _stab_check(ctx, m, np.zeros(2 * n, np.uint32), qs, qe, True)
    s, e = RC.random_range_list(10, 10_000)
    nr = len(s)
    m = dict(key_off=np.array([0, nr], np.uint64), key_a=s, key_b=e, val_off=np.array([0, 1], np.uint64),
             k2v_off=np.array([0, 2 * nr], np.uint64),
             k2v=np.concatenate([np.arange(nr + 1, 2 * nr + 1), np.zeros(nr)]).astype(np.int32))
    rng = np.random.default_rng(11)
    sel = rng.integers(0, 3, size=1000)
    pick = rng.integers(0, nr, size=1000)
    rs_ = rng.integers(0, (1 << 32) - 1000, size=1000).astype(np.uint64)
    off = rng.integers(1, 1000, size=1000).astype(np.uint64)
    a = rng.integers(0, nr, size=1000)
    b = a + (rng.random(1000) * (nr - a)).astype(np.int64)
    qs = np.where(sel == 0, s[pick], np.where(sel == 1, rs_, s[a]))
    qe = np.where(sel == 0, e[pick], np.where(sel == 1, rs_ + off, e[np.minimum(b, nr - 1)]))
    qe = np.maximum(qe, qs + np.uint64(1))
    _stab_check(ctx, m, np.zeros(1000, np.uint32), qs.astype(np.uint64), qe.astype(np.uint64), True)
