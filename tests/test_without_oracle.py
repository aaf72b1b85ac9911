"""CPU: the oracle's RelationMultiMap.remove restatement (oracle/accord_oracle_rmm.c orc_rmm_without, following
utils/RelationMultiMap.java:843-905 line by line) against an independent set model, and KeyDepsTest.testWithout's
property (tst/primitives/KeyDepsTest.java:116-153) on the oracle's output."""
import numpy as np
import pytest

import rmm_cases as RC
import without_cases as WC


@pytest.mark.parametrize("is_range,seed,kw", [(False, 1, {}), (True, 2, {}), (False, 3, dict(p_empty=0.4, p_keyonly=0.4)),
                                              (True, 4, dict(wide=True, p_extra=0.5)), (False, 5, dict(n_keys=2, n_txn=4))])
def test_oracle_without_matches_model(is_range, seed, kw):
    import oracle
    m = WC.one_per_group(seed, 200, is_range, **kw)
    sa, sb = WC.make_sets(seed + 100, m)
    ref = oracle.rmm_without(m, sa, sb)
    want = WC.model_batch(m, sa, sb)
    for k in want:
        np.testing.assert_array_equal(ref[k], want[k], err_msg=k)
    # every return of the Java occurs
    assert set(ref["kind"].tolist()) == {0, 1, 2}


def test_oracle_without_property():
    """KeyDepsTest.testWithout: without(_ -> false) is the same object; without(_ -> true) is NONE; removing one TxnId
    drops it from txnIds and from every key, and leaves every other TxnId's keys alone."""
    import oracle
    m = WC.one_per_group(7, 40, False, p_empty=0.0)
    ng = len(m["key_off"]) - 1
    none = WC.pack_sets([[] for _ in range(ng)])
    r = oracle.rmm_without(m, none, None)
    assert (r["kind"] == 0).all()
    alls = WC.pack_sets([WC.group_vals(m, g) for g in range(ng)])
    r = oracle.rmm_without(m, None, alls)
    assert (r["kind"] == 1).all() and r["key_off"][-1] == 0 and r["k2v_off"][-1] == 0
    for g in range(ng):
        vals = WC.group_vals(m, g)
        base_lists, base_ids = WC.group_lists(m, oracle.rmm_without(m, None, None), g)
        for t in vals:
            per = [[] for _ in range(ng)]
            per[g] = [t]
            r = oracle.rmm_without(m, WC.pack_sets(per), None)
            lists, ids = WC.group_lists(m, r, g)
            tk = RC.ts_key(*t)
            assert ids == [x for x in base_ids if x != tk]
            for k, lst in base_lists.items():
                assert lists.get(k, []) == [x for x in lst if x != tk]
