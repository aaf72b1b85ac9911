"""CPU tests (no GPU): the C restatement against the independent canonical model, the reference's own
property tests restated (KeyDepsTest merge/with/builder, SortedArrays union), the committed golden
fixtures, and the host-side workload generator."""
import os

import numpy as np
import pytest

import canonical
import oracle
from accord_amd import workload as W

HERE = os.path.dirname(os.path.abspath(__file__))


def same_txn(o, c, t):
    k, d, a = o.txn(t)
    ck, cd, ca = c[t]
    return list(k) == ck and list(d) == cd and list(a) == ca


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("status_model", ["preaccepted", "model"])
def test_oracle_matches_canonical(seed, status_model):
    rng = np.random.RandomState(seed)
    b = W.keydeps_batch(int(rng.randint(50, 800)), int(rng.randint(1, 6)), int(rng.randint(5, 120)),
                        1000 + seed, "uniform" if seed % 2 else "zipf", status_model=status_model,
                        window=int(rng.randint(10, 400)), p_syncpoint=0.05 * (seed % 3))
    if seed % 3 == 0:
        b = b.permuted(rng.permutation(b.n_txn))
    o = oracle.keydeps_batch(b)
    c = canonical.keydeps_batch(b)
    for t in range(b.n_txn):
        assert same_txn(o, c, t), t


@pytest.mark.parametrize("shards", [2, 3, 8])
def test_shard_invariance(shards):
    """KeyDeps of a txn is the same whether its keys live in one CommandStore or are split over many
    and reduced with PartialDeps.with (PreAccept.reduce, PreAccept.java:141-156)."""
    b = W.keydeps_batch(1500, 5, 300, 77 + shards, "zipf", status_model="model", window=300)
    o1 = oracle.keydeps_batch(b)
    os_ = oracle.keydeps_batch(b, n_shards=shards)
    for f in ("arena_off", "arena", "kd_off", "key_idx", "u_off", "dep_txn"):
        np.testing.assert_array_equal(getattr(o1, f), getattr(os_, f), err_msg=f)


def test_accept_style_p1_exclusion():
    """executeAt > txnId: the txn itself sits below insertPos and must be excluded by p1."""
    b = W.keydeps_batch(300, 2, 10, 5, "uniform", status_model="preaccepted")
    b.exe_lsb[:] = b.txn_lsb + (np.uint64(50) << np.uint64(16))
    b.exe_node[:] = 9999
    o = oracle.keydeps_batch(b)
    c = canonical.keydeps_batch(b)
    for t in range(b.n_txn):
        assert same_txn(o, c, t)
        _, d, _ = o.txn(t)
        assert t not in set(d.tolist())


def test_golden_fixtures_reproduce():
    """The committed fixtures are exactly what the oracle computes for BASELINE config 1."""
    for name in ("1a", "1b"):
        z = np.load(os.path.join(HERE, "golden", f"config{name}.npz"))
        b = W.config(name)
        for k, v in b.arrays().items():
            np.testing.assert_array_equal(z[k], v, err_msg=f"generator drift in {k}")
        o = oracle.keydeps_batch(b)
        for f in ("arena_off", "arena", "kd_off", "key_idx", "u_off", "dep_txn"):
            np.testing.assert_array_equal(z["out_" + f], getattr(o, f), err_msg=f)


def test_timestamp_compare_matches_java_semantics():
    # unsigned msb, lowHlc, identity flags 0x1E (domain bit 0 and REJECTED 0x8000 ignored), signed node
    a = (1 << 63, 5 << 16, 1)
    b = (1, 5 << 16, 1)
    assert oracle.ts_compare(a, b) > 0
    assert oracle.ts_compare((1, (5 << 16) | 1, 1), (1, 5 << 16, 1)) == 0          # domain bit
    assert oracle.ts_compare((1, (5 << 16) | 0x8000, 1), (1, 5 << 16, 1)) == 0     # REJECTED flag
    assert oracle.ts_compare((1, (5 << 16) | 2, 1), (1, 5 << 16, 1)) > 0           # kind bits
    assert oracle.ts_compare((1, 5 << 16, -1), (1, 5 << 16, 1)) < 0                # signed node


# ---------------------------------------------------------------- KeyDepsTest properties, restated

def gen_keydeps(rng, n_keys_range=(2, 200), total_range=(1, 1000)):
    """KeyDepsTest.Deps.generate (KeyDepsTest.java:315-374): canonical map over IntHashKey-like keys and
    (epoch<3, hlc<500, node<4) TxnIds, here as u32 order ranks."""
    unique = rng.randint(2, 200)
    vals = rng.choice(3 * 500 * 4, size=unique, replace=False)
    keys = rng.choice(400, size=rng.randint(*n_keys_range), replace=False)
    m = {}
    for _ in range(rng.randint(*total_range)):
        m.setdefault(int(rng.choice(keys)), set()).add(int(rng.choice(vals)))
    return canonical.from_canonical_map(m)


def pack_groups(groups):
    """list of list of (keys, vals, k2v) -> acc_merge_in dict"""
    grp_off, key_off, val_off, k2v_off = [0], [0], [0], [0]
    key_code, txn_rank, k2v = [], [], []
    for g in groups:
        for keys, vals, kv in g:
            key_code += keys
            txn_rank += vals
            k2v += kv
            key_off.append(len(key_code))
            val_off.append(len(txn_rank))
            k2v_off.append(len(k2v))
        grp_off.append(len(key_off) - 1)
    return dict(grp_off=np.array(grp_off, np.uint64), key_off=np.array(key_off, np.uint64),
                key_code=np.array(key_code, np.uint64), val_off=np.array(val_off, np.uint64),
                txn_rank=np.array(txn_rank, np.uint32), k2v_off=np.array(k2v_off, np.uint64),
                k2v=np.array(k2v, np.int32))


@pytest.mark.parametrize("seed", range(5))
def test_merge_is_canonical_union(seed):
    """KeyDepsTest.testMergedProperty (:275-283): merge(list) == fold(with) == canonical union."""
    rng = np.random.RandomState(seed)
    groups = [[gen_keydeps(rng) for _ in range(rng.randint(0, 12))] for _ in range(20)]
    m = oracle.keydeps_merge(pack_groups(groups))
    for gi, g in enumerate(groups):
        keys, vals, k2v = canonical.merge_union(g)
        a, b = m["key_off"][gi], m["key_off"][gi + 1]
        assert m["key_code"][a:b].tolist() == keys
        a, b = m["val_off"][gi], m["val_off"][gi + 1]
        assert m["txn_rank"][a:b].tolist() == vals
        a, b = m["k2v_off"][gi], m["k2v_off"][gi + 1]
        assert m["k2v"][a:b].tolist() == k2v


def test_levelise_oracle_matches_canonical():
    rng = np.random.RandomState(1)
    n = 400
    exec_rank = rng.permutation(n).astype(np.uint32)
    deps = [sorted(rng.choice(n, size=rng.randint(0, 6), replace=False).tolist()) for _ in range(n)]
    off = np.concatenate([[0], np.cumsum([len(d) for d in deps])]).astype(np.uint64)
    dep = np.array([x for d in deps for x in d], dtype=np.uint32)
    l1, o1, nl = oracle.levelise(off, dep, exec_rank)
    l2, o2 = canonical.levelise(off, dep, exec_rank)
    np.testing.assert_array_equal(l1, l2)
    np.testing.assert_array_equal(o1, o2)
    assert nl == int(l1.max()) + 1


def test_workload_is_deterministic():
    a = W.keydeps_batch(2000, 8, 10000, 42, "zipf", 0.99)
    b = W.keydeps_batch(2000, 8, 10000, 42, "zipf", 0.99)
    for k, v in a.arrays().items():
        np.testing.assert_array_equal(v, b.arrays()[k])
    kc = a.key_code.reshape(-1, 8)
    assert (np.diff(kc.astype(np.int64), axis=1) > 0).all()


def test_oracle_matches_canonical_inthash_keys():
    """IntHashKey codes (KeyDepsTest's key type, ordered by a 16-bit CRC32 hash, tst/impl/IntHashKey.java:255-279) with
    colliding int keys sharing one CommandsForKey."""
    import rmm_cases as RC
    from test_keydeps_gpu import inthash_batch
    rng = np.random.default_rng(3)
    b = W.keydeps_batch(600, 4, 200, 0x4A6, "uniform", status_model="model", window=300)
    pairs = RC.int_hash_collisions(1 << 17)[:40]
    pool = np.array([k for p in pairs for k in p] + list(rng.integers(0, 1 << 20, size=60)), np.int64)
    hb = inthash_batch(b, pool[rng.integers(0, len(pool), size=b.n_pairs)])
    o = oracle.keydeps_batch(hb)
    c = canonical.keydeps_batch(hb)
    for t in range(hb.n_txn):
        assert same_txn(o, c, t), t


def test_config2_fixture_reproduces():
    """The committed config-2 sample (tests/golden/config2_sample.npz): the generator still yields the same 1M-txn batch,
    and the oracle reproduces a spread window of it (the whole fixture takes ~2 min to regenerate)."""
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_golden import batch_digest, txn_digest
    fx = dict(np.load(os.path.join(HERE, "golden", "config2_sample.npz")))   # decompress each array once
    b = W.config("2")
    assert batch_digest(b) == bytes(fx["input_sha256"]).hex(), "generator drift"
    assert len(fx["txn"]) >= 20_000
    lo = 444_444
    o = oracle.keydeps_batch(b, query_lo=lo, query_hi=lo + 200)
    pos = {t: i for i, t in enumerate(fx["txn"].tolist())}
    for t in range(lo, lo + 200):
        k, d, a = o.txn(t)
        assert txn_digest(k, d, a) == bytes(fx["digest"][pos[t]]), t


def test_config2_all_fixture_reproduces():
    """tests/golden/config2_all.npz (every config-2 txn's 32-bit KeyDeps hash, made by make_golden.py config2_all on 8
    processes) matches the C restatement re-run here on the first 3,000 txns and on 300 of the hot uncommitted window."""
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_golden import batch_digest, txn_hashes
    b = W.config("2")
    fa = np.load(os.path.join(HERE, "golden", "config2_all.npz"))
    assert batch_digest(b) == bytes(fa["input_sha256"]).hex()
    assert fa["hash32"].shape == (b.n_txn,) and fa["sizes"].shape == (b.n_txn, 3)
    for lo, hi in ((0, 3000), (998_000, 998_300)):
        o = oracle.keydeps_batch(b, query_lo=lo, query_hi=hi)
        np.testing.assert_array_equal(txn_hashes(o, lo, hi), fa["hash32"][lo:hi])
        np.testing.assert_array_equal(np.diff(o.u_off[lo:hi + 1].astype(np.int64)), fa["sizes"][lo:hi, 1].astype(np.int64))
