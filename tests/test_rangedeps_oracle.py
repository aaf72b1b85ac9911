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
