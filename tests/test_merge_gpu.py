"""GPU parity: acc_keydeps_merge (batched KeyDeps.merge) vs the C restatement of LinearMerger/linearUnion
and the canonical union (KeyDepsTest.testMergedProperty, KeyDepsTest.java:275-283)."""
import numpy as np
import pytest

import canonical
from test_oracle import gen_keydeps, pack_groups

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from accord_amd.deps import Context
    c = Context(0)
    yield c
    c.close()


def check_groups(out, groups):
    for gi, g in enumerate(groups):
        keys, vals, k2v = canonical.merge_union(g)
        a, b = int(out["key_off"][gi]), int(out["key_off"][gi + 1])
        assert out["key_code"][a:b].tolist() == keys, gi
        a, b = int(out["val_off"][gi]), int(out["val_off"][gi + 1])
        assert out["txn_rank"][a:b].tolist() == vals, gi
        a, b = int(out["k2v_off"][gi]), int(out["k2v_off"][gi + 1])
        assert out["k2v"][a:b].tolist() == k2v, gi


@pytest.mark.parametrize("seed", range(4))
def test_merge_random_groups(ctx, seed):
    import oracle
    from accord_amd.deps import keydeps_merge
    rng = np.random.RandomState(100 + seed)
    groups = [[gen_keydeps(rng) for _ in range(rng.randint(0, 20))] for _ in range(40)]
    m = pack_groups(groups)
    out = keydeps_merge(ctx, m)
    ref = oracle.keydeps_merge(m)
    for k in ref:
        np.testing.assert_array_equal(out[k], ref[k], err_msg=k)
    check_groups(out, groups)


def test_merge_empty_replies_and_keys_without_values(ctx):
    from accord_amd.deps import keydeps_merge
    # reply A: keys [5, 9], key 5 has no entries, key 9 -> txn 3 (non-empty: its key 5 is kept)
    a = ([5, 9], [3, 7], [2, 3, 0])
    # reply B: empty (keys but no entries) -> skipped entirely, including its txnIds
    b = ([1, 2], [11], [2, 2])
    c = ([9, 12], [3, 8], [3, 4, 0, 1])
    groups = [[a, b, c], [b], [], [b, b], [c, a]]
    out = keydeps_merge(ctx, pack_groups(groups))
    check_groups(out, groups)
    assert out["key_code"][int(out["key_off"][0]):int(out["key_off"][1])].tolist() == [5, 9, 12]


def test_merge_rejects_bad_layout(ctx):
    from accord_amd.deps import IllegalArgumentException, keydeps_merge
    bad = ([5, 9], [3], [2, 2, 0])   # last offset != length
    with pytest.raises(IllegalArgumentException):
        keydeps_merge(ctx, pack_groups([[bad]]))
    good = ([5, 9], [3], [3, 4, 0, 0])
    keydeps_merge(ctx, pack_groups([[good]]))


def test_merge_config5_shape(ctx):
    """Config-5 shaped input at reduced size: every txn's true deps replicated over 16 replies with
    entries dropped (p=0.1) and spurious entries added (5%)."""
    import oracle
    from accord_amd import workload as W
    from accord_amd.deps import keydeps_merge
    m = W.merge_batch(n_txn=1500, replies=16, seed=0xACC00006, n_keys=2000)
    out = keydeps_merge(ctx, m)
    ref = oracle.keydeps_merge(m)
    for k in ref:
        np.testing.assert_array_equal(out[k], ref[k], err_msg=k)


def test_merge_lds_tier_vs_global_path(ctx):
    """The LDS tier (every group fits) and the global sort path (forced) give identical arrays; a group beyond the
    LDS caps sends the batch to the global path."""
    import oracle
    from accord_amd import workload as W
    from accord_amd.deps import Context, keydeps_merge
    m = W.merge_batch(n_txn=3000, replies=64, seed=0xACC00016, n_keys=5000)
    a = keydeps_merge(ctx, m)
    assert ctx.stats()["merge.lds_tier"] == 1
    with Context(0, force_replay=True) as c2:
        b = keydeps_merge(c2, m)
        assert c2.stats()["merge.lds_tier"] == 0
    ref = oracle.keydeps_merge(m)
    for k in ref:
        np.testing.assert_array_equal(a[k], ref[k], err_msg=k)
        np.testing.assert_array_equal(b[k], ref[k], err_msg=k)
    rng = np.random.RandomState(7)
    groups = [[gen_keydeps(rng) for _ in range(300)]] + [[gen_keydeps(rng) for _ in range(5)] for _ in range(10)]
    out = keydeps_merge(ctx, pack_groups(groups))
    assert ctx.stats()["merge.lds_tier"] == 0
    check_groups(out, groups)


@pytest.mark.parametrize("force_global", [False, True])
def test_merge_errors_both_paths(force_global):
    from accord_amd.deps import Context, IllegalArgumentException, IllegalStateException, keydeps_merge
    with Context(0, force_replay=force_global) as c:
        for bad, exc in ((([9, 5], [3], [3, 4, 0, 0]), IllegalArgumentException),     # keys not sorted
                         (([5, 9], [7, 3], [3, 4, 0, 1]), IllegalArgumentException),   # txnIds not sorted
                         (([5, 9], [3], [3, 4, 0, 1]), IllegalArgumentException),      # entry out of range
                         (([5], [3, 7], [3, 1, 1]), IllegalStateException),            # duplicate value per key
                         (([5, 9], [3], [2, 2, 0]), IllegalArgumentException)):        # last offset != length
            with pytest.raises(exc):
                keydeps_merge(c, pack_groups([[gen_keydeps(np.random.RandomState(1))], [bad]]))


def test_merge_wide_key_codes_general_path(ctx):
    """Full-width u64 key codes (hashed keys) on the general radix path (> 256 replies in a group, beyond the LDS tier):
    the composite sort runs on dense ranks of the codes instead of failing with ACC_E_CAP."""
    import oracle
    from accord_amd.deps import keydeps_merge
    rng = np.random.RandomState(77)
    wide = rng.randint(0, 2**63, size=400, dtype=np.int64).astype(np.uint64) * np.uint64(2) + np.uint64(1)
    groups = []
    for g in range(3):
        reps = []
        for _ in range(300 if g == 0 else 5):
            keys, vals, kv = gen_keydeps(rng, n_keys_range=(2, 20), total_range=(1, 60))
            reps.append(([int(wide[k]) for k in keys], vals, kv))
        groups.append(reps)
    # the remapped codes no longer follow the original key order: re-sort each reply's keys
    m = pack_groups([[_sorted_reply(r) for r in g] for g in groups])
    out = keydeps_merge(ctx, m)
    assert ctx.stats().get("merge.lds_tier") == 0
    assert ctx.stats().get("merge.dense_keys") == 1
    ref = oracle.keydeps_merge(m)
    for k in ref:
        np.testing.assert_array_equal(out[k], ref[k], err_msg=k)


def _sorted_reply(r):
    """Re-sort a reply whose key codes were remapped (order changed): keys ascending, the header and the per-key
    index lists moved with their keys."""
    keys, vals, kv = r
    nk = len(keys)
    lists, prev = [], nk
    for i in range(nk):
        lists.append(kv[prev:kv[i]])
        prev = kv[i]
    order = sorted(range(nk), key=lambda i: keys[i])
    hdr, body = [], []
    for i in order:
        body += list(lists[i])
        hdr.append(nk + len(body))
    return [keys[i] for i in order], vals, hdr + body


@pytest.mark.parametrize("scale", [1, 5, 40, 1 << 18])
def test_merge_txnid_bitmap_and_merge_tree_paths(ctx, scale):
    """The LDS tier unions a group's TxnIds through a bitmap when their rank span fits 32768 and through the merge tree
    otherwise: ranks scaled so that groups fall on either side (and, within one launch, on both)."""
    import oracle
    from accord_amd.deps import keydeps_merge
    rng = np.random.RandomState(7000 + scale)
    groups = []
    for gi in range(30):
        g = []
        for _ in range(rng.randint(0, 16)):
            keys, vals, k2v = gen_keydeps(rng)
            s = scale if gi % 2 == 0 else 1
            g.append((keys, [v * s + (gi % 3) for v in vals], k2v))
        groups.append(g)
    m = pack_groups(groups)
    out = keydeps_merge(ctx, m)
    ref = oracle.keydeps_merge(m)
    for k in ref:
        np.testing.assert_array_equal(out[k], ref[k], err_msg=k)
    check_groups(out, groups)
