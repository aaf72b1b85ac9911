"""GPU parity: acc_cfk_apply (CommandsForKey.update with each command's deps: missing[] maintenance, TRANSITIVELY_KNOWN
additions, removeMissing on commit; local/CommandsForKey.java:657-1149) vs the C restatement (oracle/accord_oracle_cfk.c),
every output array bit for bit: a hand-worked sequence, generated command lifecycles (interleaved, re-accepted ballots,
bumped executeAts, invalidations, no-op save statuses), batches chained through the device result, many keys, empty
inputs and the error cases."""
import numpy as np
import pytest

import cfk_cases as CC
import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from accord_amd.deps import Context
    c = Context(0)
    yield c
    c.close()


def same(g, o, label):
    for k in o:
        np.testing.assert_array_equal(np.asarray(g[k]), np.asarray(o[k]), err_msg=f"{label}: {k}")


def test_cfk_deps_handmade(ctx):
    from accord_amd.deps import cfk_apply
    upd, expect = CC.handmade()
    for n, want in expect:
        first, _ = CC.split_updates(upd, n)
        g = cfk_apply(ctx, CC.empty_snapshot(), first)
        assert CC.describe(g) == want, n
        same(g, oracle.cfk_apply(CC.empty_snapshot(), first), f"handmade {n}")


@pytest.mark.parametrize("seed,n_txn,n_keys", [(0, 200, 12), (1, 400, 30), (2, 120, 3), (3, 1500, 200)])
def test_cfk_deps_random(ctx, seed, n_txn, n_keys):
    from accord_amd.deps import cfk_apply
    upd = CC.cfk_case(seed, n_txn=n_txn, n_keys=n_keys)
    seen_missing = seen_tk = False
    for frac in (0.1, 0.2, 0.5, 1.0):
        part, _ = CC.split_updates(upd, int(len(upd["msb"]) * frac))
        g = cfk_apply(ctx, CC.empty_snapshot(), part)
        o = oracle.cfk_apply(CC.empty_snapshot(), part)
        same(g, o, f"seed {seed} frac {frac}")
        seen_missing |= len(o["mmsb"]) > 0
        seen_tk |= bool((o["status"] == CC.TK).any())
    assert seen_missing and seen_tk


def test_cfk_deps_chained_batches(ctx):
    """Four batches, each applied to the previous device result: equals the oracle over the whole sequence."""
    from accord_amd.deps import cfk_apply
    upd = CC.cfk_case(7, n_txn=600, n_keys=40)
    n = len(upd["msb"])
    cuts = [0, n // 5, n // 2, 3 * n // 4, n]
    snap = CC.empty_snapshot()
    rest = upd
    done = 0
    for c in cuts[1:]:
        part, rest = CC.split_updates(rest, c - done)
        done = c
        snap = cfk_apply(ctx, snap, part)
        head, _ = CC.split_updates(upd, c)
        same(snap, oracle.cfk_apply(CC.empty_snapshot(), head), f"after {c} updates")


def test_cfk_deps_empty_and_errors(ctx):
    from accord_amd.deps import IllegalStateException, cfk_apply
    e = CC.empty_snapshot()
    u0, _ = CC.split_updates(CC.handmade()[0], 0)
    g = cfk_apply(ctx, e, u0)
    assert len(g["key"]) == 0 and list(g["ent_off"]) == [0]
    upd, _ = CC.handmade()
    back = {k: v.copy() for k, v in upd.items()}
    back["status"][4] = CC.PRE   # B goes back from ACCEPTED to PREACCEPTED
    with pytest.raises(IllegalStateException):
        cfk_apply(ctx, e, back)
    g = cfk_apply(ctx, e, upd)   # the context stays usable
    assert CC.describe(g) == CC.handmade()[1][-1][1]


@pytest.mark.parametrize("seed,end_inclusive,n_upd,n_query,span", [(1, 1, 500, 300, 4000), (2, 0, 800, 400, 300),
                                                                   (3, 1, 20000, 5000, 1 << 20)])
def test_max_conflicts(ctx, seed, end_inclusive, n_upd, n_query, span):
    """acc_max_conflicts (MaxConflicts.get + the PreAccept fast-path test) vs the C restatement: key and range updates,
    key and range queries, both bound types, dense (span 300: every key hot) and sparse key spaces."""
    from accord_amd.deps import max_conflicts
    upd, q = CC.conflicts_case(seed, n_upd=n_upd, n_query=n_query, span=span, end_inclusive=end_inclusive)
    g = max_conflicts(ctx, upd, q)
    o = oracle.max_conflicts(upd, q)
    for k in ("msb", "lsb", "node", "fast"):
        np.testing.assert_array_equal(g[k], o[k], err_msg=k)
    assert 0 < int(o["fast"].sum()) < n_query


def test_max_conflicts_empty(ctx):
    from accord_amd.deps import IllegalArgumentException, max_conflicts
    upd, q = CC.conflicts_case(4, n_upd=10, n_query=5)
    none = dict(end_inclusive=1, xmsb=np.zeros(0, np.uint64), xlsb=np.zeros(0, np.uint64), xnode=np.zeros(0, np.int32),
                key_off=np.zeros(1, np.uint32), key=np.zeros(0, np.uint64), rng_off=np.zeros(1, np.uint32),
                rng_start=np.zeros(0, np.uint64), rng_end=np.zeros(0, np.uint64))
    g = max_conflicts(ctx, none, q)
    assert not g["msb"].any() and g["fast"].all()   # Timestamp.NONE: every TxnId is a fast path
    bad = dict(upd)
    bad["key"] = upd["key"][::-1].copy()
    with pytest.raises(IllegalArgumentException):
        max_conflicts(ctx, bad, q)
