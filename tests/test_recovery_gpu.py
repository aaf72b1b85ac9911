"""GPU parity: acc_map_reduce_full (batched CommandsForKey.mapReduceFull, local/CommandsForKey.java:553-612, as the
BeginRecovery scans call it, messages/BeginRecovery.java:334-378) vs the C restatement, bit for bit, for every
TestStartedAt x TestDep x TestStatus combination, permuted batches, hot keys (windows over many 256-entry chunks),
explicit Kinds masks, the executeAt > testTxnId filter, empty inputs and the error cases."""
import numpy as np
import pytest

import oracle
import recovery_cases as RC

pytestmark = pytest.mark.gpu

FIELDS = ("arena_off", "arena", "kd_off", "key_idx", "u_off", "dep_txn")


@pytest.fixture(scope="module")
def ctx():
    from accord_amd.deps import Context
    c = Context(0)
    yield c
    c.close()


def check(ctx, b, mo, mt, q, sa, td, ts, **kw):
    g = ctx.map_reduce_full(b, mo, mt, q, sa, td, ts, test_kinds=kw.get("test_kinds", -1),
                            executes_after=kw.get("exec_after", False))
    o = oracle.map_reduce_full(b, mo, mt, q, sa, td, ts, **kw)
    for f in FIELDS:
        np.testing.assert_array_equal(getattr(g, f), getattr(o, f), err_msg=f"{f} {(sa, td, ts)}")
    return g


@pytest.mark.parametrize("seed,permute", [(1, False), (2, True)])
def test_recovery_all_tests(ctx, seed, permute):
    b, mo, mt, q = RC.recovery_case(seed, n=600, n_keys=25, n_query=120, permute=permute)
    for sa, td, ts in RC.ALL_TESTS:
        check(ctx, b, mo, mt, q, sa, td, ts)


def test_recovery_begin_recovery_scans(ctx):
    from accord_amd import _lib as L
    b, mo, mt, q = RC.recovery_case(3, n=2000, n_keys=60, n_query=400)
    for name, (sa, td, ts, ea) in L.RECOVERY_SCANS.items():
        g = check(ctx, b, mo, mt, q, sa, td, ts, exec_after=ea)
        if name.startswith("has"):
            assert ((np.diff(g.u_off) > 0).any())


def test_recovery_hot_keys_multi_chunk(ctx):
    """Five keys over 6000 txns: every window spans many 256-entry chunks."""
    b, mo, mt, q = RC.recovery_case(4, n=6000, keys_per=2, n_keys=5, n_query=200, p_missing=0.02)
    for sa, td, ts in [(0, 1, 1), (0, 0, 2), (1, 1, 1), (2, 1, 2), (2, 2, 0), (1, 2, 0)]:
        check(ctx, b, mo, mt, q, sa, td, ts)
    assert ctx.stats()["recovery.chunks"] > 1000


@pytest.mark.parametrize("kinds,exec_after", [(0x1B, False), (0x02, True), (0x00, False), (0x3F, True)])
def test_recovery_kinds_and_filter(ctx, kinds, exec_after):
    b, mo, mt, q = RC.recovery_case(11, n=500, n_keys=15, n_query=80)
    for sa, td, ts in [(0, 1, 1), (2, 2, 0), (1, 0, 2)]:
        check(ctx, b, mo, mt, q, sa, td, ts, test_kinds=kinds, exec_after=exec_after)


def test_recovery_empty_inputs(ctx):
    b, mo, mt, q = RC.recovery_case(12, n=50, n_keys=5, n_query=10)
    # no queries
    q0 = dict(msb=q["msb"][:0], lsb=q["lsb"][:0], node=q["node"][:0], key_off=np.zeros(1, np.uint32),
              key_code=q["key_code"][:0])
    g = ctx.map_reduce_full(b, mo, mt, q0, 2, 2, 0)
    assert len(g.u_off) == 1 and g.u_off[0] == 0
    # queries without keys
    qe = dict(q, key_off=np.zeros(len(q["msb"]) + 1, np.uint32), key_code=q["key_code"][:0])
    g = ctx.map_reduce_full(b, mo, mt, qe, 2, 2, 0)
    assert int(g.arena_off[-1]) == 0
    # empty snapshot: every query empty
    from accord_amd import workload as W
    e = W.Batch(*(a[:0] for a in (b.txn_msb, b.txn_lsb, b.txn_node, b.exe_msb, b.exe_lsb, b.exe_node, b.status)),
                np.zeros(1, np.uint32), b.key_code[:0])
    g = ctx.map_reduce_full(e, np.zeros(1, np.uint32), np.zeros(0, np.uint32), q, 2, 2, 0)
    assert int(g.arena_off[-1]) == 0 and len(g.u_off) == len(q["msb"]) + 1


def test_recovery_errors(ctx):
    from accord_amd.deps import IllegalArgumentException, IllegalStateException
    b, mo, mt, q = RC.recovery_case(7, n=60, n_keys=6, n_query=5)
    j = int(next(i for i in range(len(mo) - 1) if mo[i + 1] - mo[i] >= 2))
    bad = mt.copy()
    bad[mo[j]], bad[mo[j] + 1] = bad[mo[j] + 1], bad[mo[j]]
    with pytest.raises(IllegalArgumentException):
        ctx.map_reduce_full(b, mo, bad, q, 0, 1, 1)
    oob = mt.copy()
    oob[0] = b.n_txn
    with pytest.raises(IllegalArgumentException):
        ctx.map_reduce_full(b, mo, oob, q, 0, 1, 1)
    q2 = dict(q, lsb=q["lsb"].copy())
    q2["lsb"][0] = (int(q2["lsb"][0]) & ~0xE & (2**64 - 1)) | (5 << 1)
    with pytest.raises(IllegalStateException):
        ctx.map_reduce_full(b, mo, mt, q2, 0, 1, 1)
    q3 = dict(q, key_code=q["key_code"].copy())
    k0, k1 = int(q["key_off"][0]), int(q["key_off"][1])
    if k1 - k0 >= 2:
        q3["key_code"][k0], q3["key_code"][k0 + 1] = q3["key_code"][k0 + 1], q3["key_code"][k0]
        with pytest.raises(IllegalArgumentException):
            ctx.map_reduce_full(b, mo, mt, q3, 0, 1, 1)
    with pytest.raises(IllegalArgumentException):
        ctx.map_reduce_full(b, mo, mt, q, 3, 1, 1)
    # the context stays usable
    check(ctx, b, mo, mt, q, 0, 1, 1)
