"""GPU parity: acc_rangedeps_batch (HIP, gfx950) vs the C restatement of mapReduceRangesInternal (oracle/).

Bit-exact on every array: the stored-range dictionary, RangeDeps.ranges (dictionary ids), RangeDeps.txnIds (batch
indices) and the Java rangesToTxnIds int[] of every txn; hand-made boundary cases, dense random batches for both
Range bound types, u64 codes over the whole range (split sorts), every build tier, the config-4 golden fixture
and error behaviour."""
import os

import numpy as np
import pytest

import rd_cases
from accord_amd import workload as W

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
FIELDS = ("rng_start", "rng_end", "arena_off", "arena", "rd_off", "range_id", "u_off", "dep_txn")


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
    assert_same(ctx.calculate_partial_range_deps(rb), oracle.rangedeps_batch(rb), "handmade")


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("end_inclusive", [1, 0])
def test_dense_random(ctx, seed, end_inclusive):
    import oracle
    rb = rd_cases.dense(200 + seed, n=4000, end_inclusive=end_inclusive, ranges_per_txn=1 + seed)
    g = ctx.calculate_partial_range_deps(rb)
    o = oracle.rangedeps_batch(rb)
    assert g.total_edges == o.total_edges > 0
    assert_same(g, o, f"dense {seed}")


def test_block_and_global_tiers(ctx):
    import oracle
    rb = rd_cases.dense(7, n=6000, key_bits=9, max_width_log2=7, ranges_per_txn=3)   # txns of 65..8192 entries
    g = ctx.calculate_partial_range_deps(rb)
    st = ctx.stats()
    assert st["rangedeps.block_txns"] > 0 and st["rangedeps.s16_txns"] > 0 and st["rangedeps.s64_txns"] > 0
    assert st["rangedeps.s32_txns"] > 0
    assert_same(g, oracle.rangedeps_batch(rb), "block tier")
    rb = rd_cases.global_tier(9000)
    g = ctx.calculate_partial_range_deps(rb)
    assert ctx.stats()["rangedeps.global_txns"] > 0
    assert_same(g, oracle.rangedeps_batch(rb), "global tier")


@pytest.mark.parametrize("wide", [False, True])
def test_identical_ranges(ctx, wide):
    """Range commands sharing one stored range (64 keys, widths <= 8: ~500 distinct ranges for ~1,500 range txns), so
    the lane-group tiers see range ids held by several TxnIds: the 32-bit (range id, lane) sort falls back to the 64-bit
    one for those waves (acc_opts ACC_OPT_RD_WIDE_SORT: the 64-bit sorts throughout)."""
    import oracle
    from accord_amd.deps import Context
    rb = rd_cases.dense(11, n=3000, key_bits=6, max_width_log2=3, ranges_per_txn=1)
    c = Context(0, rd_wide_sort=True) if wide else ctx
    try:
        g = c.calculate_partial_range_deps(rb)
        st = c.stats()
    finally:
        if wide:
            c.close()
    assert st["rangedeps.narrow_sorts"] == (0 if wide else 1)
    assert st["rangedeps.s16_txns"] > 0 and st["rangedeps.s32_txns"] + st["rangedeps.s64_txns"] > 0
    assert st["rangedeps.stored_ranges"] < st["rangedeps.entries"] // 2
    assert_same(g, oracle.rangedeps_batch(rb), "identical ranges")


def test_unsorted_batch(ctx):
    """Txns not given in TxnId order: TxnId positions differ from batch indices (txn_of_tpos path)."""
    import oracle
    rb = rd_cases.dense(31, n=3000)
    perm = np.random.RandomState(5).permutation(rb.n_txn)
    kb = rb.keys.permuted(perm)
    cnt = np.diff(rb.rng_off.astype(np.int64))[perm]
    off = np.zeros(rb.n_txn + 1, np.uint32)
    np.cumsum(cnt, out=off[1:])
    starts = rb.rng_off[:-1].astype(np.int64)[perm]
    idx = np.repeat(starts - off[:-1].astype(np.int64), cnt) + np.arange(int(off[-1]), dtype=np.int64)
    rb2 = W.RangeBatch(kb, off, rb.rng_start[idx], rb.rng_end[idx], rb.end_inclusive)
    assert_same(ctx.calculate_partial_range_deps(rb2), oracle.rangedeps_batch(rb2), "unsorted")


def test_wide_codes(ctx):
    import oracle
    rb = rd_cases.wide_codes(11, n=3000)
    assert_same(ctx.calculate_partial_range_deps(rb), oracle.rangedeps_batch(rb), "wide codes")


def test_config4_golden(ctx):
    z = np.load(os.path.join(HERE, "golden", "config4s.npz"))
    rb = W.RangeBatch(W.Batch(z["txn_msb"], z["txn_lsb"], z["txn_node"], z["exe_msb"], z["exe_lsb"], z["exe_node"],
                              z["status"], z["key_off"], z["key_code"]), z["rng_off"], z["rng_start"], z["rng_end"],
                      int(z["end_inclusive"]))
    g = ctx.calculate_partial_range_deps(rb)
    for f in FIELDS:
        np.testing.assert_array_equal(getattr(g, f), z["out_" + f], err_msg=f)


def test_config4_scaled_properties(ctx):
    """BASELINE config 4 at 1/20 scale (1M txns, full key space): structural properties over every txn plus a
    strided oracle sample (the oracle scan is O(range commands) per query)."""
    import oracle
    rb = W.config4(0.05)
    g = ctx.calculate_partial_range_deps(rb)
    n = rb.n_txn
    nr = np.diff(g.rd_off.astype(np.int64))
    na = np.diff(g.arena_off.astype(np.int64))
    nu = np.diff(g.u_off.astype(np.int64))
    assert (na >= nr).all() and ((na > nr) == (nr > 0)).all() and ((nu > 0) == (nr > 0)).all()
    # dictionary strictly sorted by (start, end)
    ds, de = g.rng_start.astype(np.uint64), g.rng_end.astype(np.uint64)
    assert ((ds[1:] > ds[:-1]) | ((ds[1:] == ds[:-1]) & (de[1:] > de[:-1]))).all()
    o = oracle.rangedeps_batch(rb, query_lo=0, query_hi=n, query_stride=997)
    for t in range(0, n, 997):
        for x, y in zip(g.txn(t), o.txn(t)):
            np.testing.assert_array_equal(x, y, err_msg=f"txn {t}")


def test_empty_and_one_sided(ctx):
    import oracle
    only_keys = rd_cases.build([dict(keys=[1, 2]), dict(keys=[3])])
    g = ctx.calculate_partial_range_deps(only_keys)
    assert g.total_edges == 0 and len(g.arena) == 0
    only_ranges = rd_cases.build([dict(ranges=[(0, 10)]), dict(ranges=[(5, 15)], kind=W.READ)])
    assert_same(ctx.calculate_partial_range_deps(only_ranges), oracle.rangedeps_batch(only_ranges), "only ranges")
    empty = rd_cases.build([])
    g = ctx.calculate_partial_range_deps(empty)
    assert len(g.arena_off) == 1


def test_errors(ctx):
    from accord_amd.deps import IllegalArgumentException
    for bad in (rd_cases.build([dict(ranges=[(5, 5)])]),
                rd_cases.build([dict(ranges=[(5, 10), (8, 12)])])):
        with pytest.raises(IllegalArgumentException):
            ctx.calculate_partial_range_deps(bad)
    # a key txn listing ranges (domain mismatch)
    rb = rd_cases.build([dict(keys=[1]), dict(ranges=[(0, 4)])])
    rb.keys.key_off[:] = [0, 0, 1]   # the range txn now lists the key too
    rb.keys.key_code[:] = [1]
    with pytest.raises(IllegalArgumentException):
        ctx.calculate_partial_range_deps(rb)
