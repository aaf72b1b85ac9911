"""GPU: the device-resident CommandsForKey store (acc_cfk_*, CommandsForKey.update local/CommandsForKey.java:652-706 for
batches of commands) against the dict model of the same rules after every batch, and acc_keydeps_batch read straight
from the store against the oracle over the model's snapshot."""
import numpy as np
import pytest

import cfk_model as CM

pytestmark = pytest.mark.gpu

COLS = ("txn_msb", "txn_lsb", "txn_node", "exe_msb", "exe_lsb", "exe_node", "status", "key_off", "key_code")


@pytest.fixture(scope="module")
def ctx():
    from accord_amd.deps import Context
    c = Context(0)
    yield c
    c.close()


def same(a, b):
    for f in COLS:
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)


def test_cfk_store_updates_match_model(ctx):
    import oracle
    from accord_amd.deps import CfkStore
    rng = np.random.default_rng(3)
    store, model = CfkStore(ctx), CM.Model()
    for rnd in range(12):
        d = CM.delta(rng, model, n_new=int(rng.integers(0, 400)), n_upd=int(rng.integers(0, 150)))
        model.apply(d)
        store.update(d)
        same(store.snapshot(), model.batch())
    assert store.snapshot().n_txn > 1000
    g = store.calculate_partial_deps()
    o = oracle.keydeps_batch(model.batch())
    for f in ("arena_off", "arena", "kd_off", "key_idx", "u_off", "dep_txn"):
        np.testing.assert_array_equal(getattr(g, f), getattr(o, f), err_msg=f)
    store.close()


def test_cfk_store_errors_and_empty(ctx):
    from accord_amd.deps import CfkStore, IllegalArgumentException, IllegalStateException
    rng = np.random.default_rng(4)
    store, model = CfkStore(ctx), CM.Model()
    assert store.snapshot().n_txn == 0
    d = CM.delta(rng, model, n_new=50, n_upd=0)
    model.apply(d)
    store.update(d)
    before = store.snapshot()
    # a stored txn whose status goes back: IllegalStateException, store unchanged
    k = next(iter(model.t.values()))
    if k[6] > 0:
        bad = CM.W.Batch(np.array([k[0]], np.uint64), np.array([k[1]], np.uint64), np.array([k[2]], np.int32),
                         np.array([k[0]], np.uint64), np.array([k[1]], np.uint64), np.array([k[2]], np.int32),
                         np.array([k[6] - 1], np.uint8), np.zeros(2, np.uint32), np.zeros(0, np.uint64))
        with pytest.raises(IllegalStateException):
            store.update(bad)
        same(store.snapshot(), before)
    dup = CM.W.Batch(*(np.concatenate([getattr(d, f)[:1]] * 2) for f in COLS[:7]), np.zeros(3, np.uint32), np.zeros(0, np.uint64))
    with pytest.raises(IllegalArgumentException):
        store.update(dup)
    same(store.snapshot(), before)
    store.close()
