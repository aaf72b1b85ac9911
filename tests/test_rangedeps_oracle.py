"""CPU tests: the RangeDeps restatement (oracle/accord_oracle.c orc_rangedeps_batch, InMemoryCommandStore
.mapReduceRangesInternal :883-1016) against the independent set model (oracle/canonical.py) and the committed
config-4 golden fixture; RangeDepsTest-style brute-force overlap sets (RangeDepsTest.java:131-148)."""
import os

import numpy as np
import pytest

import canonical
import oracle
import rd_cases
from accord_amd import workload as W

HERE = os.path.dirname(os.path.abspath(__file__))


def check_same(rb):
    o = oracle.rangedeps_batch(rb)
    ds, de, c = canonical.rangedeps_batch(rb)
    np.testing.assert_array_equal(o.rng_start, ds)
    np.testing.assert_array_equal(o.rng_end, de)
    for t in range(rb.n_txn):
        r, d, a = o.txn(t)
        assert (list(r), list(d), list(a)) == c[t], t
    return o


@pytest.mark.parametrize("end_inclusive", [1, 0])
def test_handmade(end_inclusive):
    rb = rd_cases.handmade(end_inclusive)
    o = check_same(rb)
    # stored ranges: (0,100) is erased, so (5,12) (10,20) (11,13) (15,35) (19,31) (30,40) (0,50)
    assert [(int(s), int(e)) for s, e in zip(o.rng_start, o.rng_end)] == \
        [(0, 50), (5, 12), (10, 20), (11, 13), (15, 35), (19, 31), (30, 40)]
    # txn 4 (write, keys 10 11 20 21 30 40) sees cmds 0, 1 (writes), 2 (read); not 3 (erased)
    r, d, a = o.txn(4)
    ranges = {(int(o.rng_start[x]), int(o.rng_end[x])) for x in r}
    if end_inclusive:   # (s, e]: 11 and 20 in (10,20]; 21 30 in (15,35]; 40 in (30,40]
        assert ranges == {(10, 20), (15, 35), (30, 40)}
    else:               # [s, e): 10 11 in [10,20); 20 21 30 in [15,35); 30 in [30,40)
        assert ranges == {(10, 20), (15, 35), (30, 40)}
    # txn 6 (Accept-style, executeAt beyond txn 8) depends on 7 and 8 but not on itself
    r, d, a = o.txn(6)
    assert 6 not in set(d.tolist()) and 7 in set(d.tolist())
    assert 8 not in set(d.tolist())   # a SyncPoint: Write witnesses only Reads and Writes (Txn.java:221-236)
    # txn 5 (read) only on writes, one entry per (range, cmd) though both keys are in (10,20]
    r, d, a = o.txn(5)
    assert set(d.tolist()) == {0, 1}


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("end_inclusive", [1, 0])
def test_dense_random(seed, end_inclusive):
    rb = rd_cases.dense(100 + seed, n=700, end_inclusive=end_inclusive, ranges_per_txn=1 + seed % 3)
    o = check_same(rb)
    assert o.total_edges > 0


def test_wide_codes():
    check_same(rd_cases.wide_codes(5, n=400))


def test_query_window_and_stride():
    rb = rd_cases.dense(9, n=600)
    full = oracle.rangedeps_batch(rb)
    part = oracle.rangedeps_batch(rb, query_lo=100, query_hi=400, query_stride=3)
    for t in range(100, 400, 3):
        for x, y in zip(full.txn(t), part.txn(t)):
            np.testing.assert_array_equal(x, y)
    assert part.queried == len(range(100, 400, 3))


def test_errors():
    bad = rd_cases.build([dict(ranges=[(5, 5)])])
    with pytest.raises(oracle.OracleError):
        oracle.rangedeps_batch(bad)
    bad = rd_cases.build([dict(ranges=[(5, 10), (8, 12)])])
    with pytest.raises(oracle.OracleError):
        oracle.rangedeps_batch(bad)


def test_config4_golden():
    """tests/golden/config4s.npz: BASELINE config 4's generator at 1/1000 of the txns over a 2^22 key space (the full
    config's stab depth), expected RangeDeps from the C restatement, cross-checked against the canonical model."""
    z = np.load(os.path.join(HERE, "golden", "config4s.npz"))
    rb = W.RangeBatch(W.Batch(z["txn_msb"], z["txn_lsb"], z["txn_node"], z["exe_msb"], z["exe_lsb"], z["exe_node"],
                              z["status"], z["key_off"], z["key_code"]), z["rng_off"], z["rng_start"], z["rng_end"],
                      int(z["end_inclusive"]))
    o = oracle.rangedeps_batch(rb)
    for k in ("rng_start", "rng_end", "arena_off", "arena", "rd_off", "range_id", "u_off", "dep_txn"):
        np.testing.assert_array_equal(getattr(o, k), z["out_" + k], err_msg=k)


# ---- KeyDeps of a mixed batch: range txns scan every CommandsForKey inside their ranges
# (InMemoryCommandStore.mapReduceForKey :274-289)

def check_mixed(rb, n_shards=1):
    o = oracle.keydeps_mixed(rb, n_shards=n_shards)
    c = canonical.keydeps_mixed(rb)
    for t in range(rb.n_txn):
        k, d, a = o.txn(t)
        keys = o.kd_key[o.kd_off[t]:o.kd_off[t + 1]]
        assert (list(keys), list(d), list(a)) == c[t], t
    return o


@pytest.mark.parametrize("end_inclusive", [1, 0])
def test_mixed_keydeps_handmade(end_inclusive):
    rb = rd_cases.handmade(end_inclusive)
    o = check_mixed(rb)
    # txn 2 (read over (15,35]) covers keys 18, 20, 21, 30 (end-inclusive) of writes 4 only (5 is a read, later)
    keys = set(o.kd_key[o.kd_off[2]:o.kd_off[3]].tolist())
    assert keys == set()   # key txns 4, 5 are after txn 2: TxnId >= startedBefore
    # txn 10 (read, APPLIED, over (19,31]) sees write 4 on keys 20/21/30 (end-inclusive) or 20/21/30 (start-incl.)
    k, d, a = o.txn(10)
    keys = o.kd_key[o.kd_off[10]:o.kd_off[11]].tolist()
    assert set(d.tolist()) == {4} and keys == [20, 21, 30]
    # a range txn's key_idx indexes the CFK keys its ranges cover
    cfk = sorted({int(x) for x in rb.keys.key_code})
    lo, hi = 19, 31
    covered = [x for x in cfk if ((lo < x <= hi) if end_inclusive else (lo <= x < hi))]
    assert [covered[i] for i in k.tolist()] == keys
    # key txns agree with the key-only path
    kb = oracle.keydeps_batch(rb.keys)
    for t in range(rb.n_txn):
        if int(rb.rng_off[t + 1]) == int(rb.rng_off[t]):
            for x, y in zip(kb.txn(t), o.txn(t)):
                np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("seed,ei", [(11, 1), (12, 0), (13, 1)])
def test_mixed_keydeps_dense(seed, ei):
    rb = rd_cases.dense(seed, n=600, end_inclusive=ei)
    o = check_mixed(rb)
    assert o.total_edges > 0


def test_mixed_keydeps_shards_invariant():
    """KeyDeps of range txns do not depend on the CommandStore split (keys are disjoint across stores)."""
    rb = rd_cases.dense(21, n=800)
    a = oracle.keydeps_mixed(rb)
    for s in (2, 3, 8):
        b = oracle.keydeps_mixed(rb, n_shards=s)
        for f in ("arena_off", "arena", "kd_off", "key_idx", "u_off", "dep_txn", "kd_key"):
            np.testing.assert_array_equal(getattr(a, f), getattr(b, f))


def test_mixed_keydeps_errors():
    rb = rd_cases.handmade()
    bad = W.RangeBatch(rb.keys, rb.rng_off, rb.rng_start.copy(), rb.rng_end.copy(), rb.end_inclusive)
    bad.rng_start[0] = bad.rng_end[0]
    with pytest.raises(oracle.OracleError):
        oracle.keydeps_mixed(bad)
