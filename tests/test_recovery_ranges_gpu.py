"""GPU parity: acc_map_reduce_full_ranges (the range-command half of SafeCommandStore.mapReduceFull,
InMemorySafeStore.mapReduceRangesInternal, impl/InMemoryCommandStore.java:883-1016, as the BeginRecovery scans call it,
messages/BeginRecovery.java:334-378) vs the C restatement (oracle/accord_oracle.c orc_map_reduce_full_ranges), bit for
bit: every TestStartedAt x TestDep x TestStatus combination with and without the executeAt > testTxnId map filter, key
and range participants, both Range bound types, historical entries (visited for ANY_STATUS + ANY_DEPS only), Erased
entries, repeated ranges, TxnIds present both as a range command and historically, explicit Kinds masks, empty inputs
and the error cases."""
import numpy as np
import pytest

import oracle
import recovery_cases as RC

pytestmark = pytest.mark.gpu

FIELDS = ("rng_start", "rng_end", "arena_off", "arena", "rd_off", "range_id", "u_off", "dep_txn")


@pytest.fixture(scope="module")
def ctx():
    from accord_amd.deps import Context
    c = Context(0)
    yield c
    c.close()


def check(ctx, cmds, q, sa, td, ts, test_kinds=-1, exec_after=False):
    g = ctx.map_reduce_full_ranges(cmds, q, sa, td, ts, test_kinds=test_kinds, executes_after=exec_after)
    o = oracle.map_reduce_full_ranges(cmds, q, sa, td, ts, test_kinds=test_kinds, exec_after=exec_after)
    for f in FIELDS:
        np.testing.assert_array_equal(np.asarray(getattr(g, f)).astype(np.int64), np.asarray(getattr(o, f)).astype(np.int64),
                                      err_msg=f"{f} {(sa, td, ts, exec_after)}")
    return g


@pytest.mark.parametrize("seed,end_inclusive", [(1, 1), (2, 0), (3, 1)])
def test_range_recovery_all_tests(ctx, seed, end_inclusive):
    cmds, q = RC.range_recovery_case(seed, n_cmd=400, n_query=300, end_inclusive=end_inclusive)
    nonempty = 0
    for sa, td, ts in RC.ALL_TESTS:
        for ea in (False, True):
            g = check(ctx, cmds, q, sa, td, ts, exec_after=ea)
            nonempty += int(g.u_off[-1] > 0)
    assert nonempty > 40


def test_range_recovery_begin_recovery_scans(ctx):
    """The four BeginRecovery scans (_lib.RECOVERY_SCANS) over a larger table: many 64-entry chunks per query."""
    from accord_amd import _lib as L
    cmds, q = RC.range_recovery_case(7, n_cmd=5000, n_query=400, span=4000)
    for name, (sa, td, ts, ea) in L.RECOVERY_SCANS.items():
        check(ctx, cmds, q, sa, td, ts, exec_after=ea)
    assert ctx.stats()["recovery.range_chunks"] > 1000


@pytest.mark.parametrize("kinds", [0x1B, 0x02, 0x00, 0x3F])
def test_range_recovery_kinds(ctx, kinds):
    cmds, q = RC.range_recovery_case(11, n_cmd=300, n_query=100)
    for sa, td, ts, ea in [(0, 1, 1, True), (2, 2, 0, False), (1, 0, 2, False), (0, 2, 0, True)]:
        check(ctx, cmds, q, sa, td, ts, test_kinds=kinds, exec_after=ea)


def test_range_recovery_historical_only_any_any(ctx):
    """historicalRangeCommands entries count only when the call is ANY_STATUS + ANY_DEPS (:962-963)."""
    cmds, q = RC.range_recovery_case(5, n_cmd=200, n_query=80, p_hist=0.5, p_hist_only=0.5)
    hist = (cmds["flags"] & RC.ACC_RCMD_HISTORICAL) != 0
    assert hist.any()
    live = drop_rows(cmds, ~hist)
    a, a_live = check(ctx, cmds, q, 2, 2, 0), check(ctx, live, q, 2, 2, 0)
    assert int(a.u_off[-1]) > int(a_live.u_off[-1])          # the historical entries were visited
    for sa, td, ts in [(2, 2, 2), (0, 1, 0), (1, 2, 1)]:     # ... and only for ANY_STATUS + ANY_DEPS
        x, y = check(ctx, cmds, q, sa, td, ts), check(ctx, live, q, sa, td, ts)
        np.testing.assert_array_equal(np.diff(x.u_off), np.diff(y.u_off))


def drop_rows(cmds, keep):
    """the table restricted to the rows where keep is true"""
    idx = np.nonzero(keep)[0]
    out = {k: cmds[k][idx] for k in ("txn_msb", "txn_lsb", "txn_node", "exe_msb", "exe_lsb", "exe_node", "status", "flags")}
    out["end_inclusive"] = cmds["end_inclusive"]
    for off, cols in (("rng_off", ("rng_start", "rng_end")),
                      ("dep_off", ("dep_msb", "dep_lsb", "dep_node", "dep_start", "dep_end", "dep_is_key"))):
        o = cmds[off].astype(np.int64)
        sel = np.concatenate([np.arange(o[i], o[i + 1]) for i in idx] + [np.zeros(0, np.int64)])
        out[off] = np.concatenate([[0], np.cumsum(o[idx + 1] - o[idx])]).astype(np.uint32)
        for c in cols:
            out[c] = cmds[c][sel]
    return out


def test_range_recovery_empty_and_errors(ctx):
    from accord_amd.deps import IllegalArgumentException, IllegalStateException
    cmds, q = RC.range_recovery_case(9, n_cmd=50, n_query=20)
    # no queries; an empty table
    empty_q = {k: v[:0] for k, v in q.items()}
    empty_q["part_off"] = np.zeros(1, np.uint32)
    g = ctx.map_reduce_full_ranges(cmds, empty_q, 0, 1, 1)
    assert len(g.u_off) == 1
    empty_c = {k: (v[:0] if isinstance(v, np.ndarray) else v) for k, v in cmds.items()}
    empty_c["rng_off"] = np.zeros(1, np.uint32)
    empty_c["dep_off"] = np.zeros(1, np.uint32)
    g = check(ctx, empty_c, q, 2, 2, 0)
    assert int(g.u_off[-1]) == 0
    # unsorted table
    bad = dict(cmds)
    bad["txn_lsb"] = cmds["txn_lsb"][::-1].copy()
    bad["txn_msb"] = cmds["txn_msb"][::-1].copy()
    with pytest.raises(IllegalArgumentException):
        ctx.map_reduce_full_ranges(bad, q, 0, 1, 1)
    # a LocalOnly testTxnId: Kind.witnessedBy() throws (AssertionError -> ACC_E_STATE)
    lq = dict(q)
    lq["lsb"] = (q["lsb"] & ~np.uint64(0xE)) | np.uint64(5 << 1)
    with pytest.raises(IllegalStateException):
        ctx.map_reduce_full_ranges(cmds, lq, 0, 1, 1)
    # overlapping query ranges
    oq = dict(q)
    oq["is_range"] = np.ones_like(q["is_range"])
    oq["part_end"] = q["part_start"] + np.uint64(100000)
    with pytest.raises(IllegalArgumentException):
        ctx.map_reduce_full_ranges(cmds, oq, 0, 1, 1)
    # the context stays usable
    check(ctx, cmds, q, 1, 1, 1)


def test_range_recovery_handmade(ctx):
    cmds, q, expected = RC.range_recovery_handmade()
    for (sa, td, ts, ea), want in expected.items():
        g = check(ctx, cmds, q, sa, td, ts, exec_after=ea)
        assert RC.rangedeps_as_dict(g, 0) == want
