"""BASELINE.json configs at their full size on one MI355X, checked against the oracle on bounded samples plus
size-independent layout properties over every txn (the O(prefix) / O(range commands) restatements are
too slow for every query at these sizes).

  config 3: 100M txn-key pairs (12.5M txns x 8 keys over 2^24 keys), zipf(0.99) and uniform;
  config 4: 10M range txns + 10M key txns x 4 keys (RangeDeps);
  config 5: 16,384 coordinated txns x 64 replies: KeyDeps.merge + levelisation, every array compared.

The config-3 oracle samples are committed fixtures (tests/golden/make_golden.py), computed on a sub-batch that keeps
every txn (TxnIds, statuses, executeAts) but only the keys of the sampled txns: a txn's KeyDeps depend only on the
CommandsForKey of its own keys, so the sampled txns' results are unchanged."""
import os
import sys

import numpy as np
import pytest

from accord_amd import workload as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from accord_amd.deps import Context
    c = Context(0)
    yield c
    c.close()


def check_properties(g, b):
    """Layout properties over every txn (KeyDeps.java:150-172): the header's last end offset is the arena length, TxnIds
    ascend strictly (batch in TxnId order: index order), a non-bumped txn depends only on earlier txns, key indices
    ascend inside the txn's keys, entries index the txn's TxnIds."""
    n = b.n_txn
    kd = np.diff(g.kd_off.astype(np.int64))
    al = np.diff(g.arena_off.astype(np.int64))
    nu = np.diff(g.u_off.astype(np.int64))
    nz = kd > 0
    assert ((nu > 0) == nz).all()
    last_hdr = g.arena[(g.arena_off[:-1].astype(np.int64) + kd - 1)[nz]]
    np.testing.assert_array_equal(last_hdr, al[nz])
    assert int(g.total_edges) == int(al.sum() - kd.sum())
    owner = np.repeat(np.arange(n, dtype=np.int64), nu)
    d = g.dep_txn.astype(np.int64)
    same = owner[1:] == owner[:-1]
    assert (d[1:][same] > d[:-1][same]).all()
    unbumped = (b.exe_msb == b.txn_msb) & (b.exe_lsb == b.txn_lsb) & (b.exe_node == b.txn_node)
    assert (d[unbumped[owner]] < owner[unbumped[owner]]).all()
    kown = np.repeat(np.arange(n, dtype=np.int64), kd)
    ki = g.key_idx.astype(np.int64)
    ks = kown[1:] == kown[:-1]
    assert (ki[1:][ks] > ki[:-1][ks]).all()
    assert (ki < np.diff(b.key_off.astype(np.int64))[kown]).all()


@pytest.mark.parametrize("dist", ["zipf", "uniform"])
def test_config3_full(ctx, dist):
    """BASELINE config 3 on one GPU: 100M txn-key pairs. Oracle sample (committed fixture, tests/golden/make_golden.py
    config3): the 1,000 latest txns (uncommitted window, the hottest outputs) and 1,000 txns strided over the batch,
    each compared by size and digest of its three arrays."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_golden import batch_digest, config3_batch, txn_digest
    b = config3_batch(dist)
    assert b.n_pairs == 100_000_000
    fx = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"config3{dist[0]}_sample.npz")))
    assert batch_digest(b) == bytes(fx["input_sha256"]).hex(), "config-3 generator changed"
    g = ctx.calculate_partial_deps(b)
    assert ctx.stats().get("keydeps.path_replay", 0) == 0
    check_properties(g, b)
    for t, sz, dg in zip(fx["txn"].tolist(), fx["sizes"], fx["digest"]):
        gk, gd, ga = g.txn(t)
        assert (len(gk), len(gd), len(ga)) == tuple(int(x) for x in sz), f"txn {t} sizes"
        assert txn_digest(gk, gd, ga) == bytes(dg), f"txn {t} digest"


def test_config4_full(ctx):
    """BASELINE config 4: RangeDeps of 10M range txns + 10M key txns at full size; every txn's structure, and the oracle
    (a walk of all 10M range commands per query) on 100 strided txns."""
    import oracle
    rb = W.config4(1.0)
    g = ctx.calculate_partial_range_deps(rb)
    n = rb.n_txn
    nr = np.diff(g.rd_off.astype(np.int64))
    na = np.diff(g.arena_off.astype(np.int64))
    nu = np.diff(g.u_off.astype(np.int64))
    assert (na >= nr).all() and ((na > nr) == (nr > 0)).all() and ((nu > 0) == (nr > 0)).all()
    ds, de = g.rng_start.astype(np.uint64), g.rng_end.astype(np.uint64)
    assert ((ds[1:] > ds[:-1]) | ((ds[1:] == ds[:-1]) & (de[1:] > de[:-1]))).all()
    stride = n // 100 + 1
    o = oracle.rangedeps_batch(rb, query_lo=3, query_hi=n, query_stride=stride)
    for t in range(3, n, stride):
        for x, y in zip(g.txn(t), o.txn(t)):
            np.testing.assert_array_equal(x, y, err_msg=f"txn {t}")


def test_config4_fixture_full(ctx):
    """BASELINE config 4 at full size against the committed oracle fixture (tests/golden/make_golden.py config4):
    the RangeDeps of 2,000 txns and the mixed KeyDeps (range txns over the CommandsForKey inside their ranges,
    InMemoryCommandStore.java:274-289) of 1,500 txns, by size and digest; and the fused acc_partial_deps_batch is the
    two separate calls, every array of every txn (PartialDeps.Builder routes both halves, Deps.java:46-96)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_golden import range_batch_digest, range_digest, txn_digest
    rb = W.config4(1.0)
    fx = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "config4_sample.npz")))
    assert range_batch_digest(rb) == bytes(fx["input_sha256"]).hex(), "config-4 generator changed"
    rd = ctx.calculate_partial_range_deps(rb)
    for t, sz, dg in zip(fx["rd_txn"].tolist(), fx["rd_sizes"], fx["rd_digest"]):
        r, d, a = rd.txn(t)
        rr = np.stack([rd.rng_start[r], rd.rng_end[r]], 1) if len(r) else np.zeros((0, 2), np.uint64)
        assert (len(r), len(d), len(a)) == tuple(int(x) for x in sz), f"rangedeps txn {t} sizes"
        assert range_digest(rr, d, a) == bytes(dg), f"rangedeps txn {t} digest"
    kd = ctx.calculate_partial_key_deps_mixed(rb)
    for t, sz, dg in zip(fx["mx_txn"].tolist(), fx["mx_sizes"], fx["mx_digest"]):
        k, d, a = kd.txn(t)
        kk = kd.kd_key[int(kd.kd_off[t]):int(kd.kd_off[t + 1])]
        assert (len(k), len(d), len(a)) == tuple(int(x) for x in sz), f"mixed keydeps txn {t} sizes"
        assert txn_digest(kk, d, a) == bytes(dg), f"mixed keydeps txn {t} digest"
    pk, pr = ctx.calculate_partial_deps_mixed(rb)
    for f in ("arena_off", "arena", "kd_off", "key_idx", "u_off", "dep_txn", "kd_key"):
        np.testing.assert_array_equal(getattr(pk, f), getattr(kd, f), err_msg=f"fused KeyDeps {f}")
    for f in ("rng_start", "rng_end", "arena_off", "arena", "rd_off", "range_id", "u_off", "dep_txn"):
        np.testing.assert_array_equal(getattr(pr, f), getattr(rd, f), err_msg=f"fused RangeDeps {f}")


def test_config5_full(ctx):
    """BASELINE config 5 at full size through the bench's device chain: every array of the merged view (keys, TxnIds,
    keysToTxnIds of all 16,384 coordinated txns) and the level / order of the levelised graph, against the oracle."""
    import torch
    import oracle
    from accord_amd import _lib as L
    from accord_amd.deps import merge_copy_out, merge_levelise_device
    n = 16_384
    m = W.merge_batch(n_txn=n, replies=64)
    er = W.merge_exec_rank(n)
    dev = torch.device("cuda", 0)
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in m.items()}
    er_d = torch.from_numpy(er).to(dev)
    level = torch.empty(n, dtype=torch.int32, device=dev)
    order = torch.empty(n, dtype=torch.int32, device=dev)
    mi = L.MergeIn(L.ACC_MEM_DEVICE, n, len(m["key_off"]) - 1,
                   *(t[k].data_ptr() for k in ("grp_off", "key_off", "key_code", "val_off", "txn_rank", "k2v_off", "k2v")))
    view, nl = merge_levelise_device(ctx, mi, er_d.data_ptr(), level.data_ptr(), order.data_ptr())
    ctx.sync()
    got = merge_copy_out(ctx, view)
    ref = oracle.keydeps_merge(m)
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    l2, o2, nl2 = oracle.levelise(ref["val_off"], ref["txn_rank"], er)
    np.testing.assert_array_equal(level.cpu().numpy().view(np.uint32), l2)
    np.testing.assert_array_equal(order.cpu().numpy().view(np.uint32), o2)
    assert nl == nl2
