"""GPU parity: acc_deps_merge (Deps.merge = KeyDeps.merge + RangeDeps.merge over raw TxnIds, primitives/Deps.java:256-260)
vs the C restatement of the LinearMerger / linearUnion fold with instance tracking (oracle/accord_oracle_rmm.c) and the
canonical union (KeyDepsTest.testMergedProperty, tst/primitives/KeyDepsTest.java:275-283)."""
import numpy as np
import pytest

import rmm_cases as RC

pytestmark = pytest.mark.gpu

FIELDS = ("key_off", "key_a", "val_off", "msb", "lsb", "node", "k2v_off", "k2v")


@pytest.fixture(scope="module")
def ctx():
    from accord_amd.deps import Context
    c = Context(0)
    yield c
    c.close()


def check_half(got, grp_off, half, is_range):
    import oracle
    ref = oracle.rmm_merge(grp_off, half, is_range)
    for f in FIELDS + (("key_b",) if is_range else ()):
        np.testing.assert_array_equal(got[f], ref[f], err_msg=f)
    # the reported source slot holds the kept instance's raw bits
    src = got["src"].astype(np.int64)
    for f in ("msb", "lsb", "node"):
        np.testing.assert_array_equal(half[f][src], got[f], err_msg="src " + f)
    assert RC.as_groups(got, is_range) == RC.canonical_merge(grp_off, half, is_range)


CASES = [
    (11, {}),
    (12, dict(p_flip=0.5)),                    # equals-ties with differing raw bits: the exact instance replay
    (13, dict(wide=True, p_flip=0.2)),         # full-width u64 keys / range codes and TxnId words
    (14, dict(p_empty=0.7, p_keyonly=0.5)),    # empty replies, keys without entries
    (15, dict(max_replies=12, n_keys=2, n_txn=5)),
]


@pytest.mark.parametrize("seed,kw", CASES)
def test_deps_merge_both_halves(ctx, seed, kw):
    from accord_amd.deps import deps_merge
    grp_off, kh = RC.gen_groups(seed, 30, 9, is_range=False, **kw)
    # the range half over the same groups and reply counts (one Deps per reply: KeyDeps + RangeDeps)
    _, rh = RC.gen_groups(seed + 1000, 30, 9, is_range=True, counts=np.diff(grp_off.astype(np.int64)), **kw)
    out = deps_merge(ctx, dict(grp_off=grp_off, key=kh, range=rh))
    check_half(out["key"], grp_off, kh, False)
    check_half(out["range"], grp_off, rh, True)


def test_keydeps_merge_inthash_keys(ctx):
    """KeyDepsTest.Deps.generate key space (tst/primitives/KeyDepsTest.java:315-374): IntHashKey.key(nextInt(keyRange))
    ordered by its 16-bit CRC32 hash only (tst/impl/IntHashKey.java:255-279), TxnIds (epoch < 3, hlc < 500, node < 4)."""
    from accord_amd.deps import deps_merge
    for seed in (41, 42, 43):
        grp_off, kh = RC.gen_groups(seed, 25, 12, is_range=False, n_keys=150, n_txn=200, inthash=True, p_flip=0.1)
        out = deps_merge(ctx, dict(grp_off=grp_off, key=kh))
        check_half(out["key"], grp_off, kh, False)


@pytest.mark.parametrize("gen", ["nemesis", "identical"])
def test_rangedeps_merge_reference_generators(ctx, gen):
    """RangeDepsTest.generateNemesisRanges / generateIdenticalTxns shapes (tst/primitives/RangeDepsTest.java:166-192):
    duplicate and overlapping range pieces across replies."""
    from accord_amd.deps import deps_merge
    grp_off, rh = RC.gen_groups(21, 40, 8, is_range=True, n_keys=20, n_txn=60, **{gen: True})
    out = deps_merge(ctx, dict(grp_off=grp_off, range=rh))
    check_half(out["range"], grp_off, rh, True)
    assert int(out["key"]["key_off"][-1]) == 0


def test_deps_merge_global_path(ctx):
    """Groups beyond the LDS tier (> 256 replies, > 1024 keys) with full-width codes: the general radix merge path on
    dense key ranks (no composite-width failure)."""
    from accord_amd.deps import deps_merge
    grp_off, kh = RC.gen_groups(31, 3, 300, is_range=False, n_keys=40, n_txn=80, wide=True, p_flip=0.05)
    _, kh2 = RC.gen_groups(32, 2, 8, is_range=False, n_keys=1500, n_txn=40, wide=True)
    # two groups of 1500-key replies: > ML_KC key slots
    grp = np.concatenate([grp_off, grp_off[-1] + np.array([8, 16], np.uint64)])
    half = {k: (np.concatenate([kh[k], kh2[k]]) if not k.endswith("_off") else
                np.concatenate([kh[k], kh2[k][1:] + kh[k][-1]])) for k in kh}
    out = deps_merge(ctx, dict(grp_off=grp, key=half))
    assert ctx.stats().get("merge.lds_tier") == 0
    check_half(out["key"], grp, half, False)


def test_deps_merge_errors(ctx):
    from accord_amd.deps import IllegalArgumentException, IllegalStateException, deps_merge
    t = RC.txn_pool(np.random.default_rng(5), 3)
    bad_order = RC.build_half([([9, 5], [t[0]], {0: [0], 1: [0]})], False)
    with pytest.raises(IllegalArgumentException):
        deps_merge(ctx, dict(grp_off=np.array([0, 1], np.uint64), key=bad_order))
    bad_range = RC.build_half([([(7, 7)], [t[0]], {0: [0]})], True)
    with pytest.raises(IllegalArgumentException):
        deps_merge(ctx, dict(grp_off=np.array([0, 1], np.uint64), range=bad_range))
    unsorted_txn = RC.build_half([([5], [t[1], t[0]], {0: [0, 1]})], False)
    with pytest.raises(IllegalArgumentException):
        deps_merge(ctx, dict(grp_off=np.array([0, 1], np.uint64), key=unsorted_txn))
    dup = RC.build_half([([5], [t[0], t[1]], {0: [1, 1]})], False)
    with pytest.raises(IllegalStateException):
        deps_merge(ctx, dict(grp_off=np.array([0, 1], np.uint64), key=dup))


def test_deps_merge_config5_full(ctx):
    """BASELINE config 5 at full size (16,384 coordinated txns x 64 replies) through the raw-TxnId boundary: the merged
    TxnIds equal the rank-space acc_keydeps_merge result mapped to TxnIds, and both equal the oracle."""
    import oracle
    from accord_amd import workload as W
    from accord_amd.deps import deps_merge, keydeps_merge
    m = W.merge_batch(n_txn=16_384, replies=64)
    half = W.merge_batch_raw(m)
    out = deps_merge(ctx, dict(grp_off=m["grp_off"], key=half))["key"]
    ref = oracle.keydeps_merge(m)
    rk = keydeps_merge(ctx, m)
    for f in ("key_off", "val_off", "k2v_off", "k2v"):
        np.testing.assert_array_equal(out[f], ref[f], err_msg=f)
        np.testing.assert_array_equal(rk[f], ref[f], err_msg=f)
    np.testing.assert_array_equal(out["key_a"], ref["key_code"])
    msb, lsb, node = W.raw_txn_ids(ref["txn_rank"])
    np.testing.assert_array_equal(out["msb"], msb)
    np.testing.assert_array_equal(out["lsb"], lsb)
    np.testing.assert_array_equal(out["node"], node)
