"""GPU parity: acc_keydeps_mixed (HIP, gfx950) vs the C restatement (oracle/ orc_keydeps_mixed): KeyDeps of every txn
of a mixed key/range batch — key txns as acc_keydeps_batch, range txns over every CommandsForKey inside their ranges
(InMemoryCommandStore.mapReduceForKey :274-289). Bit-exact on every array including the key codes."""
import numpy as np
import pytest

import rd_cases
from accord_amd import workload as W

pytestmark = pytest.mark.gpu
FIELDS = ("arena_off", "arena", "kd_off", "key_idx", "u_off", "dep_txn", "kd_key")


@pytest.fixture(scope="module")
def ctx():
    from accord_amd.deps import Context
    c = Context(0)
    yield c
    c.close()


def assert_same(g, o, label=""):
    for f in FIELDS:
        np.testing.assert_array_equal(getattr(g, f), getattr(o, f), err_msg=f"{label} {f}")


@pytest.mark.parametrize("end_inclusive", [1, 0])
def test_handmade(ctx, end_inclusive):
    import oracle
    rb = rd_cases.handmade(end_inclusive)
    g = ctx.calculate_partial_key_deps_mixed(rb)
    assert_same(g, oracle.keydeps_mixed(rb), "handmade")
    # key txns: identical to acc_keydeps_batch
    k = ctx.calculate_partial_deps(rb.keys)
    for t in range(rb.n_txn):
        if int(rb.rng_off[t + 1]) == int(rb.rng_off[t]):
            for x, y in zip(k.txn(t), g.txn(t)):
                np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("end_inclusive", [1, 0])
def test_dense_random(ctx, seed, end_inclusive):
    import oracle
    rb = rd_cases.dense(300 + seed, n=4000, end_inclusive=end_inclusive, ranges_per_txn=1 + seed)
    g = ctx.calculate_partial_key_deps_mixed(rb)
    o = oracle.keydeps_mixed(rb)
    assert g.total_edges == o.total_edges > 0
    assert_same(g, o, f"dense {seed}")


def test_replay_path(ctx):
    """Forced exact-replay context: the CFK replay columns come from keydeps_core itself."""
    import oracle
    from accord_amd.deps import Context
    rb = rd_cases.dense(41, n=3000)
    with Context(0, force_replay=True) as c2:
        g = c2.calculate_partial_key_deps_mixed(rb)
        assert c2.stats()["keydeps.path_replay"] == 1
    assert_same(g, oracle.keydeps_mixed(rb), "replay")


def test_unsorted_batch_and_wide_codes(ctx):
    import oracle
    rb = rd_cases.dense(51, n=3000)
    perm = np.random.RandomState(9).permutation(rb.n_txn)
    kb = rb.keys.permuted(perm)
    cnt = np.diff(rb.rng_off.astype(np.int64))[perm]
    off = np.zeros(rb.n_txn + 1, np.uint32)
    np.cumsum(cnt, out=off[1:])
    starts = rb.rng_off[:-1].astype(np.int64)[perm]
    idx = np.repeat(starts - off[:-1].astype(np.int64), cnt) + np.arange(int(off[-1]), dtype=np.int64)
    rb2 = W.RangeBatch(kb, off, rb.rng_start[idx], rb.rng_end[idx], rb.end_inclusive)
    assert_same(ctx.calculate_partial_key_deps_mixed(rb2), oracle.keydeps_mixed(rb2), "unsorted")
    rb3 = rd_cases.wide_codes(12, n=3000)
    assert_same(ctx.calculate_partial_key_deps_mixed(rb3), oracle.keydeps_mixed(rb3), "wide codes")


def test_config4_scaled(ctx):
    """BASELINE config 4's mixed batch at 1/50 scale (400k txns, full int32 key space): structural properties of every
    txn plus a strided oracle sample."""
    import oracle
    rb = W.config4(0.02)
    g = ctx.calculate_partial_key_deps_mixed(rb)
    assert ctx.stats()["keydeps.range_key_queries"] > 0
    n = rb.n_txn
    nk = np.diff(g.kd_off.astype(np.int64))
    na = np.diff(g.arena_off.astype(np.int64))
    nu = np.diff(g.u_off.astype(np.int64))
    assert (na >= nk).all() and ((na > nk) == (nk > 0)).all() and ((nu > 0) == (nk > 0)).all()
    isr = (rb.keys.txn_lsb & 1).astype(bool)
    assert nk[isr].sum() > 0
    o = oracle.keydeps_mixed(rb, query_lo=0, query_hi=n, query_stride=499)
    for t in range(0, n, 499):
        for x, y in zip(g.txn(t), o.txn(t)):
            np.testing.assert_array_equal(x, y, err_msg=f"txn {t}")
        np.testing.assert_array_equal(g.kd_key[g.kd_off[t]:g.kd_off[t + 1]], o.kd_key[o.kd_off[t]:o.kd_off[t + 1]])


def test_empty_and_one_sided(ctx):
    import oracle
    only_keys = rd_cases.build([dict(keys=[1, 2]), dict(keys=[3, 2 + 2]), dict(keys=[1], kind=W.READ)])
    assert_same(ctx.calculate_partial_key_deps_mixed(only_keys), oracle.keydeps_mixed(only_keys), "only keys")
    only_ranges = rd_cases.build([dict(ranges=[(0, 10)]), dict(ranges=[(5, 15)], kind=W.READ)])
    g = ctx.calculate_partial_key_deps_mixed(only_ranges)
    assert g.total_edges == 0 and len(g.arena) == 0
    empty = rd_cases.build([])
    assert len(ctx.calculate_partial_key_deps_mixed(empty).arena_off) == 1


def test_errors(ctx):
    from accord_amd.deps import IllegalArgumentException
    for bad in (rd_cases.build([dict(keys=[3]), dict(ranges=[(5, 5)])]),
                rd_cases.build([dict(keys=[3]), dict(ranges=[(5, 10), (8, 12)])])):
        with pytest.raises(IllegalArgumentException):
            ctx.calculate_partial_key_deps_mixed(bad)
    rb = rd_cases.build([dict(keys=[1]), dict(ranges=[(0, 4)])])
    rb.keys.key_off[:] = [0, 0, 1]
    rb.keys.key_code[:] = [1]
    with pytest.raises(IllegalArgumentException):
        ctx.calculate_partial_key_deps_mixed(rb)


def test_union_tiers(ctx):
    """Range txns whose entries exceed the wave tier (block tier) and the block tier (global (txn, rank) sort)."""
    import oracle
    n_keys = 5000
    txns = [dict(kind=W.WRITE, keys=[10 * i + 5]) for i in range(n_keys)]
    txns += [dict(kind=W.WRITE, ranges=[(0, 10 * 300)])]            # ~300 entries: wave-LDS tier
    txns += [dict(kind=W.WRITE, ranges=[(0, 10 * 2000)])]           # ~2000 entries: block tier
    txns += [dict(kind=W.READ, ranges=[(0, 10 * n_keys + 10)])]     # 5000 entries: beyond the block tier
    rb = rd_cases.build(txns)
    g = ctx.calculate_partial_key_deps_mixed(rb)
    assert_same(g, oracle.keydeps_mixed(rb), "union tiers + fallback")
    rb = rd_cases.build(txns[:-1])
    g = ctx.calculate_partial_key_deps_mixed(rb)
    st = ctx.stats()
    assert st["keydeps.range_block_txns"] >= 1 and st["keydeps.range_mid_txns"] >= 1
    assert_same(g, oracle.keydeps_mixed(rb), "union tiers")


def test_union_register_tiers(ctx):
    """Range txns of 65-128 and 129-256 entries (the register-sort union, 2 and 4 entries per lane) and 16-64 (lane
    groups), over key txns of three keys each so a range txn meets most of its TxnIds on several keys (dedupe)."""
    import oracle
    txns = [dict(kind=W.WRITE, keys=[30 * i + 5, 30 * i + 15, 30 * i + 25]) for i in range(400)]
    for w in (20, 40, 100, 170, 250):   # covered keys ~ 3 w / ... : entries from ~20 to ~250
        txns += [dict(kind=W.WRITE, ranges=[(0, 10 * w)]), dict(kind=W.READ, ranges=[(3000, 3000 + 10 * w)])]
    rb = rd_cases.build(txns)
    g = ctx.calculate_partial_key_deps_mixed(rb)
    assert ctx.stats()["keydeps.range_mid_txns"] >= 4
    assert_same(g, oracle.keydeps_mixed(rb), "register unions")


@pytest.mark.parametrize("end_inclusive", [1, 0])
def test_partial_deps_fused(ctx, end_inclusive):
    """acc_partial_deps_batch: both PartialDeps halves in one call over one dictionary pass, identical to the two
    separate calls and to the oracle's KeyDeps and RangeDeps."""
    import oracle
    rb = rd_cases.dense(77, n=5000, end_inclusive=end_inclusive, ranges_per_txn=2)
    k, r = ctx.calculate_partial_deps_mixed(rb)
    assert ctx.stats()["rangedeps.shared_dictionary"] == 1
    assert_same(k, oracle.keydeps_mixed(rb), "fused key half")
    r2 = ctx.calculate_partial_range_deps(rb)
    assert ctx.stats()["rangedeps.shared_dictionary"] == 0
    for f in ("rng_start", "rng_end", "arena_off", "arena", "rd_off", "range_id", "u_off", "dep_txn"):
        np.testing.assert_array_equal(getattr(r, f), getattr(r2, f), err_msg=f)
    o = oracle.rangedeps_batch(rb)
    for f in ("arena_off", "arena", "rd_off", "u_off", "dep_txn"):
        np.testing.assert_array_equal(getattr(r, f), getattr(o, f), err_msg=f)
    # a batch without key pairs: the RangeDeps half builds its own dictionary
    only = rd_cases.dense(78, n=600, end_inclusive=end_inclusive, p_range=1.0)
    k, r = ctx.calculate_partial_deps_mixed(only)
    assert ctx.stats()["rangedeps.shared_dictionary"] == 0
    assert_same(k, oracle.keydeps_mixed(only), "range-only key half")


def test_partial_deps_fused_errors_and_repeat(ctx):
    """acc_partial_deps_batch runs its RangeDeps half on a child context from a second host thread: a rejected batch
    raises (whichever half finds it first) and leaves the context usable; repeated calls reuse the child and give the
    same arrays as the first, equal to the oracle."""
    import oracle
    from accord_amd.deps import IllegalArgumentException
    for bad in (rd_cases.build([dict(keys=[3]), dict(ranges=[(5, 5)])]),
                rd_cases.build([dict(keys=[3]), dict(ranges=[(5, 10), (8, 12)])])):
        with pytest.raises(IllegalArgumentException):
            ctx.calculate_partial_deps_mixed(bad)
    rb = rd_cases.dense(79, n=3000, end_inclusive=1, ranges_per_txn=2)
    k1, r1 = ctx.calculate_partial_deps_mixed(rb)
    k2, r2 = ctx.calculate_partial_deps_mixed(rb)
    for f in ("arena_off", "arena", "kd_off", "key_idx", "u_off", "dep_txn"):
        np.testing.assert_array_equal(getattr(k1, f), getattr(k2, f), err_msg=f)
    for f in ("rng_start", "rng_end", "arena_off", "arena", "rd_off", "range_id", "u_off", "dep_txn"):
        np.testing.assert_array_equal(getattr(r1, f), getattr(r2, f), err_msg=f)
    assert_same(k1, oracle.keydeps_mixed(rb), "fused key half after errors")
    o = oracle.rangedeps_batch(rb)
    for f in ("arena_off", "arena", "rd_off", "u_off", "dep_txn"):
        np.testing.assert_array_equal(getattr(r1, f), getattr(o, f), err_msg=f)
