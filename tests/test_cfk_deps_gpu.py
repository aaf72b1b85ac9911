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


@pytest.fixture(scope="module")
def lane_ctx():
    """Every key through the one-lane replay (acc_opts.cfk_hot above any key's size)."""
    from accord_amd.deps import Context
    c = Context(0, cfk_hot=1_000_000)
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


@pytest.fixture(scope="module", params=[0.0, 0.5], ids=["no_deps", "half_deps"])
def hot_key_case(request):
    """One hot key, 600 txns / ~2,700 updates with events spread over the whole batch (everything in flight at once):
    with p_dep 0.5 the deps total ~120K and the quadratic working-space bound of round 3 was ~1e10-1e11 Ts (0.4-2 TB,
    the call failed); with p_dep 0 the missing[] arrays (12K-23K TxnIds) outgrow the linear first guess, so the replay
    regrows them. (A key's updates replay serially in one lane, so a hot key costs its whole history per update: the
    size here keeps that to seconds.)"""
    upd = CC.cfk_case(11, n_txn=600, n_keys=1, keys_per=1, window=600, p_dep=request.param)
    return request.param, upd


@pytest.mark.parametrize("path", ["hot", "lane"])
@pytest.mark.parametrize("frac", [0.3, 0.6, 1.0])
def test_cfk_deps_hot_key(ctx, lane_ctx, hot_key_case, frac, path):
    """The hot key through the hot-key closed form (its ~2,700 updates are above acc_opts.cfk_hot's default) and
    through the one-lane replay (threshold raised)."""
    from accord_amd.deps import cfk_apply
    if path == "lane":
        ctx = lane_ctx
    p_dep, upd = hot_key_case
    part, _ = CC.split_updates(upd, int(len(upd["msb"]) * frac))
    g = cfk_apply(ctx, CC.empty_snapshot(), part)
    st = ctx.stats()
    o = oracle.cfk_apply(CC.empty_snapshot(), part)
    same(g, o, f"hot key p_dep {p_dep} frac {frac} {path}")
    if path == "hot" and frac > 0.5:
        assert st["cfk.hot_keys"] == 1 and st["cfk.hot_irregular"] == 0
    if p_dep == 0.0 and frac < 1.0:
        assert len(o["mmsb"]) > 10_000
        if path == "lane":
            assert st["cfk.apply_regrow"] > 0


@pytest.fixture(scope="module", params=[1, 3], ids=["hot_gt1", "hot_gt3"])
def hot_all(request):
    """A context whose acc_opts.cfk_hot sends every key with more than 1 (3) sorted elements (its snapshot + its
    updates) through the hot-key closed form."""
    from accord_amd.deps import Context
    c = Context(0, cfk_hot=request.param)
    yield c
    c.close()


def test_cfk_hot_path_handmade(hot_all):
    ctx = hot_all
    from accord_amd.deps import cfk_apply
    upd, expect = CC.handmade()
    for n, want in expect:
        first, _ = CC.split_updates(upd, n)
        g = cfk_apply(ctx, CC.empty_snapshot(), first)
        assert CC.describe(g) == want, n
        same(g, oracle.cfk_apply(CC.empty_snapshot(), first), f"handmade {n}")


@pytest.mark.parametrize("seed,n_txn,n_keys", [(0, 200, 12), (1, 400, 30), (2, 120, 3), (3, 1500, 200)])
def test_cfk_hot_path_random(hot_all, seed, n_txn, n_keys):
    """Generated lifecycles (TRANSITIVELY_KNOWN additions, re-accepted ballots, bumped executeAts, invalidations):
    the closed form equals the serial restatement bit for bit."""
    ctx = hot_all
    from accord_amd.deps import cfk_apply
    upd = CC.cfk_case(seed, n_txn=n_txn, n_keys=n_keys)
    hot = 0
    for frac in (0.1, 0.5, 1.0):
        part, _ = CC.split_updates(upd, int(len(upd["msb"]) * frac))
        g = cfk_apply(ctx, CC.empty_snapshot(), part)
        hot += ctx.stats()["cfk.hot_keys"]
        same(g, oracle.cfk_apply(CC.empty_snapshot(), part), f"seed {seed} frac {frac}")
    assert hot > 0


def test_cfk_hot_path_chained(hot_all):
    """Batches applied to the previous result: the snapshot's missing[] carried (less the TxnIds committed since), new
    uncommitted TxnIds added."""
    ctx = hot_all
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


def test_cfk_hot_path_stream_and_errors(hot_all):
    ctx = hot_all
    from accord_amd import workload as W
    from accord_amd.deps import IllegalStateException, cfk_apply
    upd = W.cfk_update_stream(5_000, 4, 800)
    o = oracle.cfk_apply(CC.empty_snapshot(), upd)
    same(cfk_apply(ctx, CC.empty_snapshot(), upd), o, "update stream")
    a, b = CC.split_updates(upd, len(upd["msb"]) // 3)
    same(cfk_apply(ctx, cfk_apply(ctx, CC.empty_snapshot(), a), b), o, "update stream, chained")
    h, _ = CC.handmade()
    back = {k: v.copy() for k, v in h.items()}
    back["status"][4] = CC.PRE   # B goes back from ACCEPTED to PREACCEPTED
    with pytest.raises(IllegalStateException):
        cfk_apply(ctx, CC.empty_snapshot(), back)


def test_cfk_zipf_update_stream(ctx):
    """A zipf(0.99) update stream (workload.cfk_update_stream, 20,000 txns x 4 keys over 3,000 keys: the hottest key
    holds ~9K pairs): the hot keys take the closed form, the rest the lanes; equal to the serial restatement."""
    from accord_amd import workload as W
    from accord_amd.deps import cfk_apply
    upd = W.cfk_update_stream(20_000, 4, 3_000, dist="zipf")
    o = oracle.cfk_apply(CC.empty_snapshot(), upd)
    g = cfk_apply(ctx, CC.empty_snapshot(), upd)
    st = ctx.stats()
    same(g, o, "zipf update stream")
    assert st["cfk.hot_keys"] > 0 and st["cfk.hot_irregular"] == 0


def test_cfk_zipf_bench_stream_key_sample(ctx):
    """N4 at bench size: the bench's zipf(0.99) update stream (1M txns x 8 keys over 1M keys: 2M updates, 15.9M
    (update, key) pairs, 190M deps; the hottest key holds 835K pairs) applied to an empty store on the GPU, and the final
    CommandsForKey state of 3,047 sampled keys -- hot keys up to ~54K updates among them -- compared with the C
    restatement run on the stream restricted to those keys (tests/golden/cfk_zipf_sample.npz; keys are independent)."""
    import hashlib
    import os
    from accord_amd import workload as W
    from accord_amd.deps import cfk_apply
    here = os.path.dirname(os.path.abspath(__file__))
    fx = np.load(os.path.join(here, "golden", "cfk_zipf_sample.npz"))
    upd = W.cfk_update_stream(1_000_000, 8, 1_000_000, dist="zipf")
    h = hashlib.sha256()
    for k in sorted(set(upd) - {"time"}):   # (the event times are not part of the CFK_UPD layout)
        h.update(k.encode())
        h.update(np.ascontiguousarray(upd[k]).tobytes())
    assert h.digest() == bytes(fx["stream_sha256"]), "update-stream generator changed"
    g = cfk_apply(ctx, CC.empty_snapshot(), upd)
    st = ctx.stats()
    assert st["cfk.hot_keys"] > 10_000 and st["cfk.hot_irregular"] == 0
    kh, ne, nm = CC.key_hashes(g, fx["keys"])
    np.testing.assert_array_equal(ne, fx["entries"].astype(np.int64))
    np.testing.assert_array_equal(nm, fx["missing"].astype(np.int64))
    bad = np.flatnonzero(kh != fx["hash64"])
    assert len(bad) == 0, f"{len(bad)} keys differ, first {fx['keys'][bad[:5]].tolist()}"


def test_cfk_update_stream(ctx):
    """The bench leg's update stream (workload.cfk_update_stream: Accept with deps, then commit / stable / apply /
    invalidate with deps, interleaved) at 20,000 txns x 4 keys, applied in one call and in two chained halves."""
    from accord_amd import workload as W
    from accord_amd.deps import cfk_apply
    upd = W.cfk_update_stream(20_000, 4, 3_000)
    o = oracle.cfk_apply(CC.empty_snapshot(), upd)
    assert len(o["mmsb"]) > 0 and (o["status"] >= CC.COMMITTED).any()
    same(cfk_apply(ctx, CC.empty_snapshot(), upd), o, "update stream")
    a, b = CC.split_updates(upd, len(upd["msb"]) // 2)
    same(cfk_apply(ctx, cfk_apply(ctx, CC.empty_snapshot(), a), b), o, "update stream, chained halves")


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


@pytest.mark.parametrize("seed,end_inclusive,span,batches", [(5, 1, 4000, 4), (6, 0, 300, 7), (7, 1, 1 << 40, 3)])
def test_max_conflicts_persistent(ctx, seed, end_inclusive, span, batches):
    """acc_maxconflicts_*: the store's MaxConflicts kept on the device and merged batch by batch
    (CommandStore.updateMaxConflicts, local/CommandStore.java:280-290); after each batch every query equals the C
    restatement over all updates so far (MaxConflicts.merge is a pointwise Timestamp::max, MaxConflicts.java:62-65)."""
    from accord_amd.deps import MaxConflictsMap
    upd, q = CC.conflicts_case(seed, n_upd=3000, n_query=800, span=span, end_inclusive=end_inclusive)
    n = len(upd["xmsb"])
    cuts = [n * b // batches for b in range(batches + 1)]
    m = MaxConflictsMap(ctx, end_inclusive)
    try:
        for b in range(batches):
            m.update(CC.conflicts_slice(upd, cuts[b], cuts[b + 1]))
            g = m.get(q)
            o = oracle.max_conflicts(CC.conflicts_slice(upd, 0, cuts[b + 1]), q)
            for k in ("msb", "lsb", "node", "fast"):
                np.testing.assert_array_equal(g[k], o[k], err_msg=f"batch {b} {k}")
            assert 0 < m.size() <= 2 * (int(upd["key_off"][cuts[b + 1]]) + int(upd["rng_off"][cuts[b + 1]]))
        # the map is the store's state: an empty batch and a bad batch leave it as it is
        with pytest.raises(Exception):
            bad = CC.conflicts_slice(upd, 0, 5)
            bad["key"] = bad["key"][::-1].copy()
            m.update(bad)
        np.testing.assert_array_equal(m.get(q)["msb"], oracle.max_conflicts(upd, q)["msb"])
    finally:
        m.close()


def test_max_conflicts_code_space_ends(ctx):
    """Keys and ranges at both ends of the u64 code space (0, 2^64 - 1) through the persistent map."""
    from accord_amd.deps import MaxConflictsMap
    import accord_amd.workload as W
    top = (1 << 64) - 1
    for ei in (1, 0):
        ts = [tuple(int(x) for x in W.encode_ts(1, h, 0, 1)) for h in (10, 20, 30, 40)]
        upd = dict(end_inclusive=ei, xmsb=np.array([t[0] for t in ts], np.uint64), xlsb=np.array([t[1] for t in ts], np.uint64),
                   xnode=np.array([t[2] for t in ts], np.int32), key_off=np.array([0, 1, 2, 2, 2], np.uint32),
                   key=np.array([0, top], np.uint64), rng_off=np.array([0, 0, 0, 1, 2], np.uint32),
                   rng_start=np.array([0, top - 5], np.uint64), rng_end=np.array([3, top], np.uint64))
        qk = [0, 1, 2, 3, 4, top - 5, top - 4, top - 1, top]
        q = dict(msb=np.full(len(qk) + 1, ts[0][0], np.uint64), lsb=np.full(len(qk) + 1, ts[0][1], np.uint64),
                 node=np.full(len(qk) + 1, 1, np.int32), is_range=np.array([0] * len(qk) + [1], np.uint8),
                 part_off=np.arange(len(qk) + 2, dtype=np.uint32),
                 part_start=np.array(qk + [0], np.uint64), part_end=np.array(qk + [top], np.uint64))
        m = MaxConflictsMap(ctx, ei)
        try:
            m.update(upd)
            g = m.get(q)
        finally:
            m.close()
        o = oracle.max_conflicts(upd, q)
        for k in ("msb", "lsb", "node", "fast"):
            np.testing.assert_array_equal(g[k], o[k], err_msg=f"ei {ei} {k}")


def test_max_conflicts_keeps_existing_instance(ctx):
    """Equal executeAts under compareTo that differ in non-identity flag bits (lsb bit 5 / 6): the merged map keeps the
    existing instance, then the earliest update of a batch, as MaxConflicts.merge(existing, update) does with
    Timestamp.max (a.compareTo(b) >= 0 ? a : b; Timestamp.java:265-268, MaxConflicts.java:77-79)."""
    from accord_amd.deps import MaxConflictsMap
    import accord_amd.workload as W

    def upd(flags_keys):
        ts = [tuple(int(x) for x in W.encode_ts(1, 100, f, 1)) for f, _ in flags_keys]
        ko = np.concatenate([[0], np.cumsum([len(k) for _, k in flags_keys])]).astype(np.uint32)
        return dict(end_inclusive=1, xmsb=np.array([t[0] for t in ts], np.uint64),
                    xlsb=np.array([t[1] for t in ts], np.uint64), xnode=np.array([t[2] for t in ts], np.int32),
                    key_off=ko, key=np.array([k for _, ks in flags_keys for k in ks], np.uint64),
                    rng_off=np.zeros(len(flags_keys) + 1, np.uint32), rng_start=np.zeros(0, np.uint64),
                    rng_end=np.zeros(0, np.uint64))

    def get(m, keys):
        q0 = W.encode_ts(1, 50, 0, 1)
        n = len(keys)
        q = dict(msb=np.full(n, q0[0], np.uint64), lsb=np.full(n, q0[1], np.uint64), node=np.full(n, 1, np.int32),
                 is_range=np.zeros(n, np.uint8), part_off=np.arange(n + 1, dtype=np.uint32),
                 part_start=np.array(keys, np.uint64), part_end=np.array(keys, np.uint64))
        return m.get(q)["lsb"] & np.uint64(0xFFFF)

    m = MaxConflictsMap(ctx, 1)
    try:
        # isolated keys (no two adjacent: equal neighbours would coalesce into one instance, as the builder does)
        m.update(upd([(0x20, [5]), (0x40, [20]), (0x80, [20])]))     # within a batch: the earlier update on key 20
        np.testing.assert_array_equal(get(m, [5, 20]), [0x20, 0x40])
        m.update(upd([(0x100, [5, 30]), (0x200, [20, 40])]))         # across batches: the stored instance
        np.testing.assert_array_equal(get(m, [5, 30, 20, 40]), [0x20, 0x100, 0x40, 0x200])
    finally:
        m.close()


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


FIELDS = ("arena_off", "arena", "kd_off", "key_idx", "u_off", "dep_txn")


@pytest.mark.parametrize("seed,n_txn,n_keys", [(4, 160, 10), (6, 1500, 40)])
def test_cfk_recovery_in_place(ctx, seed, n_txn, n_keys):
    """acc_cfk_apply -> acc_cfk_snap_to_batch -> acc_map_reduce_full with nothing leaving HBM, against the C
    restatements on the host restatement of the same conversion: the txn-major snapshot and missing[] indices bit for
    bit, then every TestStartedAt x TestDep x TestStatus scan."""
    import recovery_cases as RC
    from accord_amd.deps import cfk_apply, cfk_batch_host, cfk_map_reduce_full, cfk_snap_to_batch
    upd = CC.cfk_case(seed, n_txn=n_txn, n_keys=n_keys)
    seen = 0
    for frac in (0.4, 1.0):
        head, _ = CC.split_updates(upd, int(len(upd["msb"]) * frac))
        v = cfk_apply(ctx, CC.empty_snapshot(), head, keep_device=True)
        bv = cfk_snap_to_batch(ctx, v)
        b, mo, mt = CC.snap_as_batch(oracle.cfk_apply(CC.empty_snapshot(), head))
        gb, gmo, gmt = cfk_batch_host(ctx, bv)
        for f in ("txn_msb", "txn_lsb", "txn_node", "exe_msb", "exe_lsb", "exe_node", "status", "key_off", "key_code"):
            np.testing.assert_array_equal(getattr(gb, f), getattr(b, f), err_msg=f)
        np.testing.assert_array_equal(gmo, mo)
        np.testing.assert_array_equal(gmt, mt)
        seen += len(mt)
        q = CC.recovery_queries(b, seed, 120)
        for sa, td, ts in RC.ALL_TESTS:
            g = cfk_map_reduce_full(ctx, bv, q, sa, td, ts)
            o = oracle.map_reduce_full(b, mo, mt, q, sa, td, ts)
            for f in FIELDS:
                np.testing.assert_array_equal(getattr(g, f), getattr(o, f), err_msg=f"{frac} {f} {(sa, td, ts)}")
    assert seen


def test_cfk_snap_to_batch_errors(ctx):
    from accord_amd.deps import IllegalArgumentException, IllegalStateException, cfk_snap_to_batch
    upd = CC.cfk_case(7, n_txn=80, n_keys=6)
    snap = oracle.cfk_apply(CC.empty_snapshot(), upd)
    e = cfk_snap_to_batch(ctx, CC.empty_snapshot())
    assert e.batch.n_txn == 0 and e.batch.n_pairs == 0
    ok = cfk_snap_to_batch(ctx, snap)
    assert ok.batch.n_pairs == len(snap["status"])
    # one TxnId with two statuses on two keys
    b, _, _ = CC.snap_as_batch(snap)
    t = int(np.nonzero(np.diff(b.key_off.astype(np.int64)) > 1)[0][0])
    tid = (b.txn_msb[t], b.txn_lsb[t], b.txn_node[t])
    e0 = [i for i in range(len(snap["status"])) if (snap["emsb"][i], snap["elsb"][i], snap["enode"][i]) == tid][0]
    bad = {k: v.copy() for k, v in snap.items()}
    bad["status"][e0] = CC.INVALID if bad["status"][e0] != CC.INVALID else CC.APPLIED
    with pytest.raises(IllegalStateException):
        cfk_snap_to_batch(ctx, bad)
    # a missing[] TxnId that is no entry of the store
    if len(snap["mmsb"]):
        bad = {k: v.copy() for k, v in snap.items()}
        bad["mlsb"][0] = np.uint64(int(bad["mlsb"][0]) ^ (1 << 17))
        with pytest.raises(IllegalStateException):
            cfk_snap_to_batch(ctx, bad)
    bad = {k: v.copy() for k, v in snap.items()}
    bad["ent_off"][1] = bad["ent_off"][-1] + 1
    with pytest.raises(IllegalArgumentException):
        cfk_snap_to_batch(ctx, bad)
    assert cfk_snap_to_batch(ctx, snap).batch.n_txn == ok.batch.n_txn   # the context stays usable


def test_cfk_store_one_state(ctx):
    """One device CommandsForKey store for the update with deps and every scan (acc_cfk_apply_deps; the reference's
    one CommandsForKey per key, local/CommandsForKey.java:614-706, 1085-1149): three chained batches applied to the
    store; after each, its key-major state equals the C restatement over all updates so far, its txn-major view and
    missing[] indices equal the host restatement of that state, and calculatePartialDeps / mapReduceFull read the store
    in place with the same results as the host batch."""
    import recovery_cases as RC
    from accord_amd.deps import CfkStore, IllegalStateException, cfk_batch_host, cfk_map_reduce_full
    upd = CC.cfk_case(9, n_txn=700, n_keys=30)
    n = len(upd["msb"])
    cuts = [0, n // 3, 2 * n // 3, n]
    st = CfkStore(ctx)
    try:
        rest, done = upd, 0
        for c in cuts[1:]:
            part, rest = CC.split_updates(rest, c - done)
            done = c
            st.apply_deps(part)
            head, _ = CC.split_updates(upd, c)
            o = oracle.cfk_apply(CC.empty_snapshot(), head)
            same(st.state(), o, f"state after {c}")
            b, mo, mt = CC.snap_as_batch(o)
            gb, gmo, gmt = cfk_batch_host(ctx, st.missing_view())
            for f in ("txn_msb", "txn_lsb", "txn_node", "exe_msb", "exe_lsb", "exe_node", "status", "key_off", "key_code"):
                np.testing.assert_array_equal(getattr(gb, f), getattr(b, f), err_msg=f"{c} {f}")
            np.testing.assert_array_equal(gmo, mo)
            np.testing.assert_array_equal(gmt, mt)
            g = st.calculate_partial_deps()
            r = ctx.calculate_partial_deps(b)
            for f in FIELDS:
                np.testing.assert_array_equal(getattr(g, f), getattr(r, f), err_msg=f"keydeps {c} {f}")
            q = CC.recovery_queries(b, c, 60)
            for sa, td, ts in RC.ALL_TESTS[::3]:
                g = cfk_map_reduce_full(ctx, st.missing_view(), q, sa, td, ts)
                o2 = oracle.map_reduce_full(b, mo, mt, q, sa, td, ts)
                for f in FIELDS:
                    np.testing.assert_array_equal(getattr(g, f), getattr(o2, f), err_msg=f"recovery {c} {f} {(sa, td, ts)}")
        # a rejected batch leaves the store as it was; status-only updates are refused on a store holding missing[]
        before = st.state()
        back = {k: v.copy() for k, v in CC.split_updates(upd, 40)[0].items()}
        back["status"][:] = CC.PRE
        back["flags"][:] = 0
        with pytest.raises(IllegalStateException):
            st.apply_deps(back)
        same(st.state(), before, "after a rejected batch")
        with pytest.raises(IllegalStateException):
            st.update(b)
    finally:
        st.close()


def test_cfk_store_modes(ctx):
    """A store keeps missing[] from its first acc_cfk_apply_deps on: deps updates on a store holding status-only state
    (acc_cfk_update) and the key-major / missing views of such a store are ACC_E_STATE; an empty store takes either."""
    from accord_amd.deps import CfkStore, IllegalStateException
    upd = CC.cfk_case(3, n_txn=60, n_keys=5)
    b, _, _ = CC.snap_as_batch(oracle.cfk_apply(CC.empty_snapshot(), upd))
    st = CfkStore(ctx)
    try:
        st.update(b)                       # status-only state
        with pytest.raises(IllegalStateException):
            st.apply_deps(upd)
        with pytest.raises(IllegalStateException):
            st.state()
        with pytest.raises(IllegalStateException):
            st.missing_view()
    finally:
        st.close()
    st = CfkStore(ctx)
    try:
        st.apply_deps(upd)                 # from empty: the deps state
        same(st.state(), oracle.cfk_apply(CC.empty_snapshot(), upd), "store from empty")
    finally:
        st.close()


def test_cfk_deps_order_checked(ctx):
    """Each (update, key) pair's deps must be strictly ascending (KeyDeps.txnIds(key) is a SortedList): a swapped or
    repeated dep inside one pair's range is IllegalArgumentException; a larger dep ending one pair before a smaller
    dep starting the next is legal (the check sees range boundaries)."""
    from accord_amd import workload as W
    from accord_amd.deps import IllegalArgumentException, cfk_apply
    upd = W.cfk_update_stream(3_000, 4, 400)
    off = upd["dep_off"].astype(np.int64)
    cnt = np.diff(off)
    p = int(np.nonzero(cnt >= 3)[0][5])
    a = int(off[p])
    for mode in ("swap", "repeat"):
        bad = {k: v.copy() for k, v in upd.items()}
        for col in ("dmsb", "dlsb", "dnode"):
            if mode == "swap":
                bad[col][a], bad[col][a + 1] = upd[col][a + 1], upd[col][a]
            else:
                bad[col][a + 1] = upd[col][a]
        with pytest.raises(IllegalArgumentException):
            cfk_apply(ctx, CC.empty_snapshot(), bad)
    # pair boundaries: consecutive pairs' ranges abut, the next range may start below the previous one's end
    q = int(np.nonzero((cnt[:-1] >= 2) & (cnt[1:] >= 2))[0][3])
    b = int(off[q + 1])
    assert (upd["dmsb"][b - 1], upd["dlsb"][b - 1]) != (upd["dmsb"][b], upd["dlsb"][b])
    g = cfk_apply(ctx, CC.empty_snapshot(), upd)
    same(g, oracle.cfk_apply(CC.empty_snapshot(), upd), "ordered deps")
