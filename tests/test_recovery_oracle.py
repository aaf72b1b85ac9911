"""CPU: the C restatement of CommandsForKey.mapReduceFull (oracle/accord_oracle.c orc_map_reduce_full,
local/CommandsForKey.java:553-612) against the independent set model (oracle/canonical.py map_reduce_full) for every
TestStartedAt x TestDep x TestStatus combination, explicit Kinds masks and the executeAt > testTxnId map filter; and the
range-command half (orc_map_reduce_full_ranges, impl/InMemoryCommandStore.java:883-1016) against answers worked out by
hand plus its invariants on random tables."""
import pytest

import canonical
import oracle
import recovery_cases as RC


@pytest.mark.parametrize("seed,permute", [(1, False), (2, True), (3, False)])
def test_oracle_matches_canonical_all_tests(seed, permute):
    b, mo, mt, q = RC.recovery_case(seed, n=250, n_keys=20, n_query=60, permute=permute)
    nq = len(q["msb"])
    for sa, td, ts in RC.ALL_TESTS:
        o = oracle.map_reduce_full(b, mo, mt, q, sa, td, ts)
        c = canonical.map_reduce_full(b, mo, mt, q, sa, td, ts)
        assert RC.canonical_rows(o, nq) == c, (sa, td, ts)


@pytest.mark.parametrize("kinds,exec_after", [(0x1B, False), (0x02, True), (0x00, False), (0x10, True)])
def test_oracle_kinds_and_filter(kinds, exec_after):
    b, mo, mt, q = RC.recovery_case(11, n=200, n_keys=15, n_query=40)
    nq = len(q["msb"])
    for sa, td, ts in [(0, 1, 1), (2, 2, 0), (1, 0, 2)]:
        o = oracle.map_reduce_full(b, mo, mt, q, sa, td, ts, test_kinds=kinds, exec_after=exec_after)
        c = canonical.map_reduce_full(b, mo, mt, q, sa, td, ts, test_kinds=kinds, exec_after=exec_after)
        assert RC.canonical_rows(o, nq) == c


def test_oracle_recovery_edge_rules():
    """STARTED_AFTER includes X itself when X is on the key; WITH skips keys where X is no member."""
    b, mo, mt, q = RC.recovery_case(5, n=120, n_keys=8, n_query=30)
    nq = len(q["msb"])
    any_self = False
    o = oracle.map_reduce_full(b, mo, mt, q, 1, 2, 0)   # STARTED_AFTER, ANY_DEPS, ANY_STATUS
    tids = {(int(b.txn_msb[t]), int(b.txn_lsb[t]), int(b.txn_node[t])): t for t in range(b.n_txn)}
    for i in range(nq):
        t = tids.get((int(q["msb"][i]), int(q["lsb"][i]), int(q["node"][i])))
        deps = set(int(x) for x in o.dep_txn[int(o.u_off[i]):int(o.u_off[i + 1])])
        witnessed = canonical.WITNESSED_BY[(int(q["lsb"][i]) >> 1) & 7]
        if t is not None and int(b.status[t]) != 0 and ((int(b.txn_lsb[t]) >> 1) & 7) in witnessed:
            assert t in deps
            any_self = True
    assert any_self


def test_oracle_errors():
    b, mo, mt, q = RC.recovery_case(7, n=60, n_keys=6, n_query=5)
    bad = mt.copy()
    if len(bad) >= 2:
        j = int(next(i for i in range(len(mo) - 1) if mo[i + 1] - mo[i] >= 2))
        bad[mo[j]], bad[mo[j] + 1] = bad[mo[j] + 1], bad[mo[j]]
        with pytest.raises(oracle.OracleError):
            oracle.map_reduce_full(b, mo, bad, q, 0, 1, 1)
    q2 = dict(q)
    q2["lsb"] = q["lsb"].copy()
    q2["lsb"][0] = (int(q2["lsb"][0]) & ~0xE & (2**64 - 1)) | (5 << 1)   # LocalOnly testTxnId: witnessedBy() throws
    with pytest.raises(oracle.OracleError):
        oracle.map_reduce_full(b, mo, mt, q2, 0, 1, 1)


# ---- the range-command half (orc_map_reduce_full_ranges, impl/InMemoryCommandStore.java:883-1016)
def test_handmade_answers():
    cmds, q, expected = RC.range_recovery_handmade()
    for (sa, td, ts, ea), want in expected.items():
        got = RC.rangedeps_as_dict(oracle.map_reduce_full_ranges(cmds, q, sa, td, ts, exec_after=ea), 0)
        assert got == want, ((sa, td, ts, ea), got, want)


def test_random_tables_invariants():
    """Per query: ranges ascending, TxnIds ascending and unique, every entry indexes them; the executeAt filter only
    removes entries; WITH and WITHOUT partition the entries ANY_DEPS leaves (for non-historical, deps-known commands)."""
    cmds, q = RC.range_recovery_case(4, n_cmd=200, n_query=60)
    for sa, td, ts in RC.ALL_TESTS:
        full = oracle.map_reduce_full_ranges(cmds, q, sa, td, ts)
        filt = oracle.map_reduce_full_ranges(cmds, q, sa, td, ts, exec_after=True)
        for i in range(len(q["msb"])):
            a, b = RC.rangedeps_as_dict(full, i), RC.rangedeps_as_dict(filt, i)
            keys = list(a)
            assert keys == sorted(keys)
            for r, ds in a.items():
                assert ds == sorted(set(ds))
            for r, ds in b.items():
                assert set(ds) <= set(a.get(r, []))
