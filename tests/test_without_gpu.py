"""GPU parity of acc_rmm_without (RelationMultiMap.remove = KeyDeps.without / RangeDeps.without,
utils/RelationMultiMap.java:843-905) and acc_recovery_deps_reduce (Deps.merge then .without(committed::contains),
coordinate/Recover.java:320-322, messages/BeginRecovery.java:180-183) against the oracle restatements, with
KeyDepsTest.testWithout's property (tst/primitives/KeyDepsTest.java:116-153) checked on the GPU output."""
import numpy as np
import pytest

import rmm_cases as RC
import without_cases as WC

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from accord_amd.deps import Context
    c = Context(0)
    yield c
    c.close()


FIELDS = ("key_off", "key_idx", "val_off", "val_idx", "k2v_off", "k2v", "kind")


def check(got, ref):
    for k in FIELDS:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


@pytest.mark.parametrize("is_range,seed,kw", [(False, 1, {}), (True, 2, {}), (False, 3, dict(p_empty=0.4, p_keyonly=0.4)),
                                              (True, 4, dict(wide=True, p_extra=0.5)), (False, 5, dict(n_keys=2, n_txn=4)),
                                              (False, 6, dict(p_flip=0.5))])
def test_without_vs_oracle(ctx, is_range, seed, kw):
    import oracle
    from accord_amd.deps import rmm_without
    m = WC.one_per_group(seed, 300, is_range, **kw)
    sa, sb = WC.make_sets(seed + 100, m)
    got = rmm_without(ctx, m, sa, sb)
    check(got, oracle.rmm_without(m, sa, sb))
    assert got["counts"] == tuple(int((got["kind"] == k).sum()) for k in range(3))


def test_without_one_set_or_none(ctx):
    import oracle
    from accord_amd.deps import rmm_without
    m = WC.one_per_group(8, 100, False)
    sa, _ = WC.make_sets(9, m)
    check(rmm_without(ctx, m, sa, None), oracle.rmm_without(m, sa, None))
    check(rmm_without(ctx, m, None, sa), oracle.rmm_without(m, None, sa))
    got = rmm_without(ctx, m, None, None)
    assert (got["kind"] == 0).all()
    check(got, oracle.rmm_without(m, None, None))


def test_without_property_on_gpu(ctx):
    """KeyDepsTest.testWithout on the GPU output: no match -> the same object; all match -> NONE; removing one TxnId
    removes it from txnIds and from every key, other TxnIds keep their keys. All single removals of all groups in one
    batch: group (g, t) of the batch is group g with remove set {t}."""
    from accord_amd.deps import rmm_without
    m = WC.one_per_group(10, 60, False, p_empty=0.0)
    ng = len(m["key_off"]) - 1
    got = rmm_without(ctx, m, WC.pack_sets([[] for _ in range(ng)]), None)
    assert (got["kind"] == 0).all()
    got = rmm_without(ctx, m, None, WC.pack_sets([WC.group_vals(m, g) for g in range(ng)]))
    assert (got["kind"] == 1).all() and int(got["key_off"][-1]) == 0 and int(got["k2v_off"][-1]) == 0
    # replicate every group once per TxnId it holds
    rep, sets = [], []
    for g in range(ng):
        for t in WC.group_vals(m, g):
            rep.append(g)
            sets.append([t])
    mm = replicate(m, rep)
    r = rmm_without(ctx, mm, WC.pack_sets(sets), None)
    base = rmm_without(ctx, mm, None, None)
    for i, g in enumerate(rep):
        tk = RC.ts_key(*sets[i][0])
        bl, bids = WC.group_lists(mm, base, i)
        lists, ids = WC.group_lists(mm, r, i)
        assert ids == [x for x in bids if x != tk]
        for k, lst in bl.items():
            assert lists.get(k, []) == [x for x in lst if x != tk]


def replicate(m, rep):
    """The batch whose group i is m's group rep[i]."""
    out = {k: [] for k in ("key_a", "key_b", "msb", "lsb", "node", "k2v")}
    ko, vo, oo = [0], [0], [0]
    for g in rep:
        k0, k1 = int(m["key_off"][g]), int(m["key_off"][g + 1])
        v0, v1 = int(m["val_off"][g]), int(m["val_off"][g + 1])
        o0, o1 = int(m["k2v_off"][g]), int(m["k2v_off"][g + 1])
        out["key_a"].extend(m["key_a"][k0:k1])
        if "key_b" in m:
            out["key_b"].extend(m["key_b"][k0:k1])
        for f in ("msb", "lsb", "node"):
            out[f].extend(m[f][v0:v1])
        out["k2v"].extend(m["k2v"][o0:o1])
        ko.append(len(out["key_a"])); vo.append(len(out["msb"])); oo.append(len(out["k2v"]))
    r = dict(key_off=np.array(ko, np.uint64), val_off=np.array(vo, np.uint64), k2v_off=np.array(oo, np.uint64),
             key_a=np.array(out["key_a"], np.uint64), msb=np.array(out["msb"], np.uint64),
             lsb=np.array(out["lsb"], np.uint64), node=np.array(out["node"], np.int32), k2v=np.array(out["k2v"], np.int32))
    if "key_b" in m:
        r["key_b"] = np.array(out["key_b"], np.uint64)
    return r


def test_without_large_batch(ctx):
    """Many groups (multi-block scans, every return kind spread over the batch)."""
    import oracle
    from accord_amd.deps import rmm_without
    m = WC.one_per_group(11, 20000, False, n_keys=6, n_txn=20)
    sa, sb = WC.make_sets(12, m)
    check(rmm_without(ctx, m, sa, sb), oracle.rmm_without(m, sa, sb))


def test_without_errors(ctx):
    from accord_amd.deps import IllegalArgumentException, rmm_without
    m = WC.one_per_group(13, 20, False, p_empty=0.0)
    sa, _ = WC.make_sets(14, m, modes=("all",))
    g = int(np.argmax(np.diff(sa["off"].astype(np.int64))))
    q0 = int(sa["off"][g])
    bad = {k: v.copy() for k, v in sa.items()}
    for f in ("msb", "lsb", "node"):   # two TxnIds of one group out of order
        bad[f][q0], bad[f][q0 + 1] = sa[f][q0 + 1], sa[f][q0]
    with pytest.raises(IllegalArgumentException):
        rmm_without(ctx, m, bad, None)
    broken = {k: v.copy() for k, v in m.items()}
    o0 = int(m["k2v_off"][0])
    broken["k2v"][o0] = int(m["k2v"][o0]) + 1000   # the first key's end offset past the int[]
    with pytest.raises(IllegalArgumentException):
        rmm_without(ctx, broken, sa, None)


@pytest.mark.parametrize("seed,groups,replies", [(21, 60, 5), (22, 200, 3), (23, 30, 12), (24, 5000, 4)])
def test_recovery_deps_reduce(ctx, seed, groups, replies):
    """earlierAcceptedNoWitness = Deps.merge(...).without(Deps.merge(earlierCommittedWitness)::contains), per recovered
    txn, against the oracle's merge and without restatements."""
    import oracle
    from accord_amd.deps import recovery_deps_reduce
    grp_off, cw, anw = WC.gen_recovery(seed, groups, replies)
    got = recovery_deps_reduce(ctx, dict(grp_off=grp_off, **cw), dict(grp_off=grp_off, **anw))
    rck, rcr = oracle.rmm_merge(grp_off, cw["key"], False), oracle.rmm_merge(grp_off, cw["range"], True)
    rak, rar = oracle.rmm_merge(grp_off, anw["key"], False), oracle.rmm_merge(grp_off, anw["range"], True)
    for name, g, r, isr in (("ck", got["committed"]["key"], rck, False), ("cr", got["committed"]["range"], rcr, True),
                            ("ak", got["accepted_merged"]["key"], rak, False),
                            ("ar", got["accepted_merged"]["range"], rar, True)):
        for f in ("key_off", "key_a", "val_off", "msb", "lsb", "node", "k2v_off", "k2v") + (("key_b",) if isr else ()):
            np.testing.assert_array_equal(g[f], r[f], err_msg=name + " " + f)
    sets = [dict(off=h["val_off"], msb=h["msb"], lsb=h["lsb"], node=h["node"]) for h in (rck, rcr)]
    ok, orr = oracle.rmm_without(rak, *sets), oracle.rmm_without(rar, *sets)
    check(got["accepted_key"], ok)
    check(got["accepted_range"], orr)
    if groups >= 60:
        assert set(ok["kind"].tolist()) == {0, 1, 2}
