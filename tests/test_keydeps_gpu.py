"""GPU parity: acc_keydeps_batch (HIP, gfx950) vs the C restatement of the reference (oracle/).

Bit-exact on every array of every txn: KeyDeps.keys (as indices into the txn's keys), KeyDeps.txnIds
(as batch indices) and the Java keysToTxnIds int[]. Mirrors the reference's KeyDepsTest style: random
seeded batches, shuffled inputs, canonical comparisons.
"""
import os
import sys

import numpy as np
import pytest

from accord_amd import workload as W

HERE = os.path.dirname(os.path.abspath(__file__))

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["runs", "replay"])
def ctx(request):
    """Both device paths: the run-based scan (default) and the exact FAST-bisection replay that batches
    with executeAt ties take (forced here with ACC_OPT_FORCE_REPLAY)."""
    from accord_amd.deps import Context
    c = Context(0, force_replay=request.param == "replay")
    yield c
    c.close()


def assert_same(gpu, orc, n, label=""):
    np.testing.assert_array_equal(gpu.arena_off, orc.arena_off, err_msg=f"{label} arena_off")
    np.testing.assert_array_equal(gpu.kd_off, orc.kd_off, err_msg=f"{label} kd_off")
    np.testing.assert_array_equal(gpu.u_off, orc.u_off, err_msg=f"{label} u_off")
    np.testing.assert_array_equal(gpu.arena, orc.arena, err_msg=f"{label} arena")
    np.testing.assert_array_equal(gpu.key_idx, orc.key_idx, err_msg=f"{label} key_idx")
    np.testing.assert_array_equal(gpu.dep_txn, orc.dep_txn, err_msg=f"{label} dep_txn")


@pytest.mark.parametrize("status_model", ["preaccepted", "model"])
@pytest.mark.parametrize("permute", [False, True])
def test_small_uniform(ctx, status_model, permute):
    import oracle
    b = W.keydeps_batch(3000, 4, 300, 0x1234, "uniform", status_model=status_model, window=800)
    if permute:
        b = b.permuted(np.random.RandomState(7).permutation(b.n_txn))
    g = ctx.calculate_partial_deps(b)
    o = oracle.keydeps_batch(b)
    assert g.total_edges == o.total_edges
    assert_same(g, o, b.n_txn, f"{status_model} permute={permute}")


@pytest.mark.parametrize("name", ["1a", "1b"])
def test_config1_vs_oracle(ctx, name):
    import oracle
    b = W.config(name)
    g = ctx.calculate_partial_deps(b)
    o = oracle.keydeps_batch(b)
    assert_same(g, o, b.n_txn, name)


def test_config1_golden(ctx):
    """Committed golden fixtures (tests/golden/make_golden.py) for BASELINE config 1."""
    import os
    here = os.path.join(os.path.dirname(__file__), "golden")
    for name in ("config1a", "config1b"):
        z = np.load(os.path.join(here, f"{name}.npz"))
        b = W.Batch(z["txn_msb"], z["txn_lsb"], z["txn_node"], z["exe_msb"], z["exe_lsb"], z["exe_node"],
                    z["status"], z["key_off"], z["key_code"])
        g = ctx.calculate_partial_deps(b)
        for k in ("arena_off", "arena", "kd_off", "key_idx", "u_off", "dep_txn"):
            np.testing.assert_array_equal(getattr(g, k), z["out_" + k], err_msg=f"{name} {k}")


def inthash_batch(b, key_ints):
    """The batch with IntHashKey keys: each pair's int key -> its 16-bit hash code (IntHashKey.compareTo orders by the
    hash alone, tst/impl/IntHashKey.java:275-279); a txn's Keys are sorted unique by that order, so keys of one txn
    whose hashes collide collapse to one (Keys.of dedups by compareTo)."""
    import rmm_cases as RC
    codes = np.array([RC.int_hash_key(int(k)) for k in key_ints], np.uint64)
    off, kc = [0], []
    for t in range(b.n_txn):
        ks = sorted(set(int(x) for x in codes[int(b.key_off[t]):int(b.key_off[t + 1])]))
        kc.extend(ks)
        off.append(len(kc))
    return W.Batch(b.txn_msb, b.txn_lsb, b.txn_node, b.exe_msb, b.exe_lsb, b.exe_node, b.status,
                   np.array(off, np.uint32), np.array(kc, np.uint64))


def test_inthash_keys(ctx):
    """IntHashKey key space (KeyDepsTest's key type): codes are 16-bit hashes, so distinct int keys with colliding
    hashes share one CommandsForKey, and key order is hash order, not int order."""
    import oracle
    import rmm_cases as RC
    rng = np.random.default_rng(9)
    b = W.keydeps_batch(4000, 4, 1000, 0x4A5, "uniform", status_model="model", window=900)
    pairs = RC.int_hash_collisions(1 << 17)[:200]
    pool = np.array([k for p in pairs for k in p] + list(rng.integers(0, 1 << 20, size=600)), np.int64)
    key_ints = pool[rng.integers(0, len(pool), size=b.n_pairs)]
    hb = inthash_batch(b, key_ints)
    g = ctx.calculate_partial_deps(hb)
    o = oracle.keydeps_batch(hb)
    assert_same(g, o, hb.n_txn, "inthash")
    assert g.total_edges > 0


def test_zipf_hot_keys(ctx):
    """Skewed keys (hot CFK segments) with the status model; multi-pass rank and pair sorts."""
    import oracle
    b = W.keydeps_batch(20000, 8, 5000, 0x77, "zipf", 0.99, status_model="model", window=1500)
    g = ctx.calculate_partial_deps(b)
    o = oracle.keydeps_batch(b)
    assert_same(g, o, b.n_txn, "zipf")


@pytest.mark.parametrize("n,k,nkeys,window", [(4000, 16, 3000, 2000), (6000, 16, 4000, 3000)])
def test_inline_txns_beyond_stream_cap(ctx, n, k, nkeys, window):
    """16-key txns whose every pair keeps its entries inline (<= 15 each) yet sum past the stream pass's 128-entry
    buffer (E up to ~265; 161 / 192 such txns here): the mark pass routes them to the block tiers, every txn equals the
    oracle."""
    import oracle
    b = W.keydeps_batch(n, k, nkeys, 0x5EED, "uniform", status_model="model", window=window)
    g = ctx.calculate_partial_deps(b)
    o = oracle.keydeps_batch(b)
    E = np.diff(o.arena_off.astype(np.int64)) - np.diff(o.kd_off.astype(np.int64))
    assert E.max() > 200
    assert_same(g, o, b.n_txn, f"{k}-key inline txns past the stream cap")


def test_mixed_kinds_and_accept_style(ctx):
    """SyncPoint kinds, random executeAt bumps on uncommitted txns (Accept-style queries with p1)."""
    import oracle
    b = W.keydeps_batch(4000, 3, 200, 0x99, "uniform", status_model="model", window=2000, p_syncpoint=0.05)
    rng = np.random.RandomState(3)
    # bump executeAt of some ACCEPTED txns (executeAt > txnId, p1 != null)
    acc = np.where(b.status == W.ACCEPTED)[0]
    pick = acc[rng.rand(len(acc)) < 0.3]
    hlc = (b.txn_lsb[pick] >> np.uint64(16)) + np.uint64(5)
    b.exe_lsb[pick] = hlc << np.uint64(16)
    b.exe_node[pick] = 2000
    g = ctx.calculate_partial_deps(b)
    o = oracle.keydeps_batch(b)
    assert_same(g, o, b.n_txn, "mixed")


def test_exec_ties_fast_bisection(ctx):
    """Equal executeAts on committed entries exercise the FAST-bisection '--i' quirk
    (CommandsForKey.java:619-621); the GPU replays the same bisection on ranks."""
    import oracle
    b = W.keydeps_batch(2000, 2, 20, 0x5151, "uniform", status_model="model", window=300)
    rng = np.random.RandomState(11)
    com = np.where((b.status >= W.COMMITTED) & (b.status <= W.APPLIED))[0]
    # give groups of committed txns an identical executeAt (a later timestamp)
    for grp in np.array_split(rng.permutation(com)[:600], 150):
        top = int(max(b.txn_lsb[grp] >> np.uint64(16))) + 3
        b.exe_msb[grp] = b.txn_msb[grp[0]]
        b.exe_lsb[grp] = np.uint64(top) << np.uint64(16)
        b.exe_node[grp] = 4242
    g = ctx.calculate_partial_deps(b)
    o = oracle.keydeps_batch(b)
    assert_same(g, o, b.n_txn, "ties")


def test_wide_timestamps_multiword_sort(ctx):
    """Timestamps whose varying bits exceed 64 force the 3-word LSD dictionary sort."""
    import oracle
    b = W.keydeps_batch(1500, 3, 100, 0x4242, "uniform", status_model="model", window=500)
    rng = np.random.RandomState(5)
    n = b.n_txn
    epochs = rng.randint(1, 1 << 20, size=n).astype(np.uint64)
    order = np.argsort(epochs, kind="stable")
    b = b.permuted(order)  # keep txn order consistent with the new epochs below
    epochs = np.sort(epochs)
    b.txn_msb[:] = epochs << np.uint64(15)
    b.exe_msb[:] = epochs << np.uint64(15)
    b.txn_node[:] = rng.randint(-2**31, 2**31 - 1, size=n).astype(np.int32)
    b.exe_node[:] = b.txn_node
    g = ctx.calculate_partial_deps(b)
    o = oracle.keydeps_batch(b)
    assert_same(g, o, b.n_txn, "wide")


def set_kind(b, idx, kind):
    b.txn_lsb[idx] = (b.txn_lsb[idx] & ~np.uint64(0xE)) | np.uint64(kind << 1)
    b.exe_msb[idx], b.exe_lsb[idx], b.exe_node[idx] = b.txn_msb[idx], b.txn_lsb[idx], b.txn_node[idx]


@pytest.mark.parametrize("hot_every,tail", [(10, 5), (40, 3), (2, 3)])
def test_tiers_medium_big_fallback(ctx, hot_every, tail):
    """One hot key of committed Reads closed by a few PREACCEPTED Writes: those Writes depend on every
    earlier entry (E up to ~9000), exercising the block tier (E <= 8192) and the global-sort tier."""
    import oracle
    b = W.keydeps_batch(90_000, 1, 1_000_000, 0x5EED + hot_every, "uniform", status_model="model", window=0)
    hot = np.arange(0, b.n_txn, hot_every)
    b.key_code[hot] = W.int_key_code(np.array([1 << 30]))[0]
    set_kind(b, hot, W.READ)
    b.status[hot] = W.APPLIED
    last = hot[-tail:]
    set_kind(b, last, W.WRITE)
    b.status[last] = W.PREACCEPTED
    g = ctx.calculate_partial_deps(b)
    o = oracle.keydeps_batch(b)
    assert_same(g, o, b.n_txn, "tiers")
    st = ctx.stats()
    if st.get("keydeps.path_replay") == 0 and hot_every == 10:
        assert st["keydeps.huge_txns"] > 0         # E ~9000: the 32768-record block tier
    if st.get("keydeps.path_replay") == 0 and hot_every == 2:
        assert st["keydeps.fallback_txns"] > 0     # E ~45000: the global-sort tier


@pytest.mark.parametrize("nk", [8, 12, 24])
def test_window_tier(nk):
    """The uncommitted window's txns on hot keys (E up to thousands) through the per-key bitmap tier (<= 8 and
    <= 16 keys: k_v2_write_win) or, beyond 16 keys, the sorting tiers run after the host sync: bit-exact with the
    oracle on the window's txns and, on every txn, with the sorting tiers alone (acc_opts ACC_OPT_NO_WINDOW_TIER)."""
    import oracle
    from accord_amd.deps import Context
    b = W.keydeps_batch(40_000, nk, 12_000, 0xB17 + nk, "zipf", 0.99, status_model="model", window=2500)
    with Context(0) as c:
        g = c.calculate_partial_deps(b)
        st = c.stats()
    if nk <= 16:
        assert st["keydeps.window_txns"] > 0
    else:
        assert st["keydeps.window_txns"] == 0 and st["keydeps.medium_txns"] + st["keydeps.big_txns"] > 0
    with Context(0, no_window_tier=True) as c:
        s = c.calculate_partial_deps(b)
    assert_same(g, s, b.n_txn, f"window vs sorting tiers, {nk} keys")
    n = b.n_txn
    o = oracle.keydeps_batch(b, query_lo=n - 400, query_hi=n)
    for t in range(n - 400, n):
        for x, y, what in zip(g.txn(t), o.txn(t), ("keys", "txnIds", "keysToTxnIds")):
            np.testing.assert_array_equal(x, y, err_msg=f"txn {t} {what}")


def test_path_selection():
    """Tie-free batches take the run-based path; executeAt ties switch to the exact replay."""
    from accord_amd.deps import Context
    b = W.keydeps_batch(3000, 4, 300, 0x31, "zipf", status_model="model", window=500)
    with Context(0, timing=True) as c:
        c.calculate_partial_deps(b)
        names = set(c.timing())
    assert "v3_stream" in names and "query_emit" not in names
    com = np.where((b.status >= W.COMMITTED) & (b.status <= W.APPLIED))[0][:2]
    b.exe_msb[com] = b.exe_msb[com[0]]
    b.exe_lsb[com] = b.txn_lsb[com].max() + (np.uint64(7) << np.uint64(16))
    b.exe_node[com] = 77
    with Context(0, timing=True) as c:
        c.calculate_partial_deps(b)
        names = set(c.timing())
    assert "query_emit" in names


def test_edge_cases(ctx):
    import oracle
    # single txn, no deps
    b = W.keydeps_batch(1, 3, 10, 1, "uniform", status_model="preaccepted")
    g = ctx.calculate_partial_deps(b)
    assert g.arena_off.tolist() == [0, 0] and len(g.dep_txn) == 0
    # ragged key counts including txns with zero keys
    b = W.keydeps_batch(500, 4, 40, 2, "uniform", status_model="model", window=200)
    counts = np.random.RandomState(2).randint(0, 5, size=b.n_txn)
    keep = np.concatenate([np.arange(int(b.key_off[t]), int(b.key_off[t]) + c) for t, c in enumerate(counts)])
    b.key_code = b.key_code[keep]
    b.key_off = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint32)
    g = ctx.calculate_partial_deps(b)
    o = oracle.keydeps_batch(b)
    assert_same(g, o, b.n_txn, "ragged")


def test_errors(ctx):
    from accord_amd.deps import IllegalArgumentException, IllegalStateException
    b = W.keydeps_batch(100, 3, 50, 3, "uniform", status_model="model", window=50)
    bad = W.Batch(**{k: v.copy() for k, v in b.arrays().items()})
    bad.key_code[1], bad.key_code[2] = bad.key_code[2], bad.key_code[1]
    with pytest.raises(IllegalArgumentException):
        ctx.calculate_partial_deps(bad)
    dup = W.Batch(**{k: v.copy() for k, v in b.arrays().items()})
    dup.txn_lsb[5] = dup.txn_lsb[4]
    dup.txn_node[5] = dup.txn_node[4]
    dup.txn_msb[5] = dup.txn_msb[4]
    with pytest.raises(IllegalArgumentException):
        ctx.calculate_partial_deps(dup)
    local = W.Batch(**{k: v.copy() for k, v in b.arrays().items()})
    local.txn_lsb[3] = (local.txn_lsb[3] & ~np.uint64(0xE)) | np.uint64(5 << 1)
    with pytest.raises(IllegalStateException):
        ctx.calculate_partial_deps(local)
    # key_off[n_txn] != n_pairs (checked on the device by the prep pass, ACC_E_ARG)
    from accord_amd import _lib as L
    a = {k: np.ascontiguousarray(v) for k, v in b.arrays().items()}
    kc = np.concatenate([a["key_code"], a["key_code"][-1:]])   # n_pairs + 1 codes (kept alive for the call)
    bi = L.BatchIn(b.n_txn, L.ACC_MEM_HOST, b.n_pairs + 1,
                   L.TsCols(a["txn_msb"].ctypes.data, a["txn_lsb"].ctypes.data, a["txn_node"].ctypes.data),
                   L.TsCols(a["exe_msb"].ctypes.data, a["exe_lsb"].ctypes.data, a["exe_node"].ctypes.data),
                   a["status"].ctypes.data, a["key_off"].ctypes.data, kc.ctypes.data)
    with pytest.raises(IllegalArgumentException, match="n_pairs"):
        ctx.keydeps_batch_raw(bi)
    # the context stays usable after errors
    g = ctx.calculate_partial_deps(b)
    assert g.arena_off[-1] == len(g.arena)


def test_config2_sample_and_properties(ctx):
    """BASELINE config 2 (1M txns x 8 keys, zipf 0.99 over 1M keys) on the GPU, bit-exact against the oracle on EVERY
    txn: the committed per-txn sizes and 32-bit hashes of all 1M txns' KeyDeps arrays (tests/golden/config2_all.npz,
    the C restatement run over the whole batch on 8 cores by make_golden.py config2_all), the 20,000-txn fixture's
    16-byte digests and full arrays, and size-independent layout properties over every txn."""
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_golden import batch_digest, txn_digest, txn_hashes
    b = W.config("2")
    fx = dict(np.load(os.path.join(HERE, "golden", "config2_sample.npz")))   # decompress each array once
    assert batch_digest(b).encode() == bytes(fx["input_sha256"]).hex().encode(), "config-2 generator changed"
    g = ctx.calculate_partial_deps(b)
    n = b.n_txn
    fa = dict(np.load(os.path.join(HERE, "golden", "config2_all.npz")))
    assert bytes(fa["input_sha256"]) == bytes(fx["input_sha256"])
    sz = np.stack([np.diff(g.kd_off.astype(np.int64)), np.diff(g.u_off.astype(np.int64)),
                   np.diff(g.arena_off.astype(np.int64))], axis=1)
    bad = np.flatnonzero((sz != fa["sizes"].astype(np.int64)).any(axis=1))
    assert len(bad) == 0, f"{len(bad)} txns differ in size from the oracle, first {bad[:5].tolist()}"
    bad = np.flatnonzero(txn_hashes(g, 0, n) != fa["hash32"])
    assert len(bad) == 0, f"{len(bad)} txns differ from the oracle, first {bad[:5].tolist()}"
    # the committed oracle sample (tests/golden/make_golden.py config2): 20,000 query txns, the hottest 2,000 among
    # them; per-txn sizes + digests for all, full arrays for the spread windows
    for t, sz, dg in zip(fx["txn"].tolist(), fx["sizes"], fx["digest"]):
        gk, gd, ga = g.txn(t)
        assert (len(gk), len(gd), len(ga)) == tuple(int(x) for x in sz), f"txn {t} sizes"
        assert txn_digest(gk, gd, ga) == bytes(dg), f"txn {t} digest"
    ko, do, ao = (fx[f].astype(np.int64) for f in ("full_key_off", "full_dep_off", "full_k2v_off"))
    for i, t in enumerate(fx["full_txn"].tolist()):
        gk, gd, ga = g.txn(t)
        np.testing.assert_array_equal(gk, fx["full_keys"][ko[i]:ko[i + 1]], err_msg=f"txn {t} keys")
        np.testing.assert_array_equal(gd, fx["full_deps"][do[i]:do[i + 1]], err_msg=f"txn {t} txnIds")
        np.testing.assert_array_equal(ga, fx["full_k2v"][ao[i]:ao[i + 1]], err_msg=f"txn {t} keysToTxnIds")
    # properties for every txn: header ends at array end, indices strictly increasing per key,
    # every txnId referenced, deps strictly increasing in TxnId order and earlier than the txn
    kd = np.diff(g.kd_off.astype(np.int64))
    al = np.diff(g.arena_off.astype(np.int64))
    nz = kd > 0
    last_hdr = g.arena[(g.arena_off[:-1].astype(np.int64) + kd - 1)[nz]]
    np.testing.assert_array_equal(last_hdr, al[nz])
    assert int(g.total_edges) == int(al.sum() - kd.sum())


def test_runs_vs_replay_beyond_one_scan_chunk():
    """9.6M pairs (> 8192 tiles of 1024 positions): the per-tile column scans carry across chunks. The run-based
    path is compared bit-for-bit with the independent FAST-bisection replay path on every txn, and with the oracle on
    a sample of the hottest (latest) txns."""
    import oracle
    from accord_amd.deps import Context
    b = W.keydeps_batch(1_200_000, 8, 1_200_000, 0xC4A1, "zipf", 0.99, status_model="model")
    assert b.n_pairs > 8192 * 1024
    with Context(0) as c:
        g = c.calculate_partial_deps(b)
        assert c.stats().get("keydeps.path_replay", 0) == 0
    with Context(0, force_replay=True) as c:
        r = c.calculate_partial_deps(b)
    assert_same(g, r, b.n_txn, "runs vs replay")
    n = b.n_txn
    o = oracle.keydeps_batch(b, query_lo=n - 200, query_hi=n)
    for t in range(n - 200, n):
        for x, y, what in zip(g.txn(t), o.txn(t), ("keys", "txnIds", "keysToTxnIds")):
            np.testing.assert_array_equal(x, y, err_msg=f"txn {t} {what}")


def test_txn_with_more_than_65536_keys(ctx):
    """A txn listing 70,000 keys (Keys has no cap) with deps on many of them: the global write tier's key-index field is
    sized from the batch (17 bits here), not fixed at 16 bits."""
    import oracle
    rng = np.random.RandomState(65)
    n, big, nk_big = 300, 200, 70_000
    kinds = rng.choice([W.READ, W.WRITE], size=n)
    msb, lsb, node = W.encode_ts(np.ones(n), np.arange(1, n + 1), kinds.astype(np.uint64) << np.uint64(1),
                                 1 + np.arange(n) % 8)
    lsb[big] = (lsb[big] & ~np.uint64(0xE)) | np.uint64(W.WRITE << 1)
    keys = []
    for t in range(n):
        keys.append(np.arange(nk_big) if t == big else np.sort(rng.choice(nk_big, size=6, replace=False)))
    off = np.zeros(n + 1, np.uint32)
    np.cumsum([len(k) for k in keys], out=off[1:])
    b = W.Batch(msb, lsb, node.astype(np.int32), msb.copy(), lsb.copy(), node.astype(np.int32).copy(),
                np.full(n, W.PREACCEPTED, np.uint8), off, W.int_key_code(np.concatenate(keys)))
    g = ctx.calculate_partial_deps(b)
    o = oracle.keydeps_batch(b)
    k, d, a = o.txn(big)
    assert len(d) > 100 and int(np.max(k)) > 65536
    assert_same(g, o, b.n_txn, ">65536 keys")
