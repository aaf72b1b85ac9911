"""CPU: the C restatement of CommandsForKey.update with deps (oracle/accord_oracle_cfk.c, local/CommandsForKey.java:
657-1149) against a sequence worked out by hand, and its batch properties on generated command lifecycles."""
import numpy as np
import pytest

import cfk_cases as CC
import oracle


def test_handmade_sequence():
    upd, expect = CC.handmade()
    for n, want in expect:
        first, _ = CC.split_updates(upd, n)
        assert CC.describe(oracle.cfk_apply(CC.empty_snapshot(), first)) == want, n


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_batches_compose(seed):
    """Applying a sequence in two batches (the first batch's result as the second's snapshot) equals one batch."""
    upd = CC.cfk_case(seed, n_txn=150)
    whole = oracle.cfk_apply(CC.empty_snapshot(), upd)
    for frac in (0.3, 0.7):
        a, b = CC.split_updates(upd, int(len(upd["msb"]) * frac))
        two = oracle.cfk_apply(oracle.cfk_apply(CC.empty_snapshot(), a), b)
        for k in whole:
            np.testing.assert_array_equal(two[k], whole[k], err_msg=k)


def test_invariants_mid_sequence():
    """missing[] is sorted, holds only TxnIds of the key's uncommitted entries, never the owner; TRANSITIVELY_KNOWN
    entries appear (deps the store had not seen)."""
    upd = CC.cfk_case(3, n_txn=150)
    a, _ = CC.split_updates(upd, len(upd["msb"]) // 3)
    s = oracle.cfk_apply(CC.empty_snapshot(), a)
    assert (s["status"] == CC.TK).any() and len(s["mmsb"]) > 0
    for k in range(len(s["key"])):
        e0, e1 = int(s["ent_off"][k]), int(s["ent_off"][k + 1])
        ids = {(int(s["emsb"][e]), int(s["elsb"][e]) & ~1, int(s["enode"][e])): int(s["status"][e]) for e in range(e0, e1)}
        for e in range(e0, e1):
            m0, m1 = int(s["miss_off"][e]), int(s["miss_off"][e + 1])
            ms = [(int(s["mmsb"][q]), int(s["mlsb"][q]) & ~1, int(s["mnode"][q])) for q in range(m0, m1)]
            assert ms == sorted(ms, key=lambda t: (t[0], t[1] >> 16, t[1] & 0x1E, t[2]))
            for t in ms:
                assert t in ids and ids[t] < CC.COMMITTED
                assert t != (int(s["emsb"][e]), int(s["elsb"][e]) & ~1, int(s["enode"][e]))


def test_stale_status_rejected():
    upd, _ = CC.handmade()
    first, _ = CC.split_updates(upd, 5)
    back = {k: v.copy() for k, v in first.items()}
    back["status"][4] = CC.PRE   # B COMMITTED -> PREACCEPTED after ACCEPTED: goes back
    with pytest.raises(oracle.OracleError):
        oracle.cfk_apply(CC.empty_snapshot(), back)
