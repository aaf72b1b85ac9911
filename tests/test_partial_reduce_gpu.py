"""acc_partial_deps_reduce: PreAccept.reduce of a store's whole PartialDeps behind the C ABI (messages/PreAccept.java:
141-156; PartialDeps.with = KeyDeps.with + RangeDeps.with, primitives/PartialDeps.java:80-86). Each rank is one
CommandStore over an EvenSplit key range holding its store-sliced mixed batch (range commands sliced to the store,
impl/InMemoryCommandStore.java:739-761); acc_partial_deps_batch, then one size exchange and one grouped all-to-all(v)
of both halves' fragments. On the home rank: the KeyDeps half equals the single-store KeyDeps of the whole batch
(KeyDeps is shard-invariant) and the RangeDeps half equals the oracle's RangeDeps.with fold over the same store split
(the reference's result depends on the split)."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu
RANGE_FIELDS = ("key_off", "key_a", "key_b", "val_off", "msb", "lsb", "node", "k2v_off", "k2v")
KEY_FIELDS = ("key_off", "key_code", "val_off", "txn_rank", "k2v_off", "k2v")


def _batch(seed, n, end_inclusive=1):
    from accord_amd import workload as W
    return W.rangedeps_batch(n, seed, p_range=0.5, keys_per_txn=3, ranges_per_txn=2, key_bits=18, max_width_log2=13,
                             window=min(n, 2000), end_inclusive=end_inclusive)


def _expected(rb, world, rank):
    """(key half, range half) expected on `rank`: KeyDeps of the whole batch on one store (GPU, checked against the
    oracle by test_keydeps_mixed_gpu) restricted to the home txns; the oracle's RangeDeps fold over the store split."""
    import oracle
    from accord_amd import sharded as S
    from accord_amd.deps import Context
    with Context(0) as ctx:
        kd = ctx.calculate_partial_key_deps_mixed(rb)
    key_off, val_off, k2v_off, keys, vals, k2v = [0], [0], [0], [], [], []
    for t in S.home_txns(rb.n_txn, rank, world).tolist():
        k, d, a = kd.txn(t)
        kc = kd.kd_key[int(kd.kd_off[t]):int(kd.kd_off[t + 1])]
        keys.append(kc); vals.append(d); k2v.append(a)
        key_off.append(key_off[-1] + len(kc)); val_off.append(val_off[-1] + len(d)); k2v_off.append(k2v_off[-1] + len(a))
    cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)  # noqa: E731
    key = dict(key_off=np.array(key_off, np.uint64), key_code=cat(keys, np.uint64), val_off=np.array(val_off, np.uint64),
               txn_rank=cat(vals, np.uint32), k2v_off=np.array(k2v_off, np.uint64), k2v=cat(k2v, np.int32))
    m = S.range_reduce_local(rb, world, lambda sub: oracle.rangedeps_batch(sub))[rank]
    return key, oracle.rmm_merge(m["grp_off"], m["half"], True)


def _bounds(rb, world):
    from accord_amd import sharded as S
    return S.even_split(np.concatenate([rb.keys.key_code, rb.rng_start, rb.rng_end]).astype(np.uint64), world)


def _store_covering(rb, world, rank):
    """Store `rank`'s Ranges in the batch's bound type (its EvenSplit key range; sharded.store_ranges_bound)"""
    from accord_amd import sharded as S
    lo, hi = S.store_ranges_bound(_bounds(rb, world), rank, rb.end_inclusive)
    return np.array([lo], np.uint64), np.array([hi], np.uint64)


def _expected_covering(rb, world, rank):
    """Per home txn of `rank`: the stores whose batch holds it, and its covering = the fold that.covering.with(
    this.covering) over them (PartialDeps.java:80-86) -- for disjoint store ranges, a set union that leaves touching
    ranges of different stores apart (RangesTest.addTest): the stores' ranges in store order."""
    from accord_amd import sharded as S
    b = _bounds(rb, world)
    member = np.zeros((world, rb.n_txn), bool)
    for s in range(world):
        member[s, S.store_range_batch(rb, b, s)[1].astype(np.int64)] = True
    home = S.home_txns(rb.n_txn, rank, world)
    out = []
    for t in home.tolist():
        stores = [s for s in range(world) if member[s, t]]
        cov = [_store_covering(rb, world, s) for s in stores]
        mask = sum(1 << s for s in stores)
        out.append((mask, np.array([c[0][0] for c in cov], np.uint64), np.array([c[1][0] for c in cov], np.uint64)))
    return out


def _run_store(ctx, comm, rb, world, rank):
    """This rank's store: its sliced batch through acc_partial_deps_batch (+ the store covering's invariant checks),
    then acc_partial_deps_reduce with the store's covering; host copies."""
    from accord_amd import sharded as S
    from accord_amd.deps import rmm_copy_out
    sub, gidx = S.store_range_batch(rb, _bounds(rb, world), rank)
    keep = []
    rbi = ctx.range_batch_in(sub, keep)
    ctx.partial_deps_batch_raw(rbi)
    cov = _store_covering(rb, world, rank)
    S.partial_deps_covering(ctx, rbi, cov)
    kv, rv, cv = S.partial_deps_reduce(ctx, comm, rbi, rb.n_txn, gidx.astype(np.uint32), covering=cov)
    ng = int(kv.n_groups)
    key = S.merged_to_host(ctx, kv)
    rng = rmm_copy_out(ctx, ng, rv.range_deps, True)
    return key, rng, S.covering_to_host(ctx, cv)


def _check_covering(got, want, label):
    cid, mask, table = got
    assert len(cid) == len(want), label
    for i, (m, ws, we) in enumerate(want):
        assert int(mask[i]) == m, (label, i, int(mask[i]), m)
        gs, ge = table[int(cid[i])]
        assert np.array_equal(gs, ws) and np.array_equal(ge, we), (label, i, gs, ge, ws, we)


def _check(key, rng, want_key, want_rng, label):
    for f in KEY_FIELDS:
        np.testing.assert_array_equal(np.asarray(key[f]), np.asarray(want_key[f]), err_msg=f"{label} key {f}")
    for f in RANGE_FIELDS:
        g, w = np.asarray(rng[f]).astype(np.int64), np.asarray(want_rng[f]).astype(np.int64)
        assert g.shape == w.shape and np.array_equal(g, w), (label, "range", f)


def test_partial_deps_reduce_rccl_world_one():
    from accord_amd import sharded as S
    from accord_amd.deps import Context
    rb = _batch(0x7A71, 12_000)
    want_key, want_rng = _expected(rb, 1, 0)
    with Context(0) as ctx:
        comm = S.Comm.rccl(ctx, 1, 0)
        key, rng, cov = _run_store(ctx, comm, rb, 1, 0)
        comm.close()
    _check(key, rng, want_key, want_rng, "rccl world 1")
    _check_covering(cov, _expected_covering(rb, 1, 0), "rccl world 1")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, end_inclusive, errq):
    sys.path[:0] = [os.path.join(ROOT, "cassandra-accord_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    from accord_amd import sharded as S
    from accord_amd.deps import Context
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rb = _batch(0x7B72 + world, 10_000, end_inclusive)
        with Context(0) as ctx:
            comm = S.Comm.host(ctx, world, rank)
            key, rng, cov = _run_store(ctx, comm, rb, world, rank)
            comm.close()
        want_key, want_rng = _expected(rb, world, rank)
        _check(key, rng, want_key, want_rng, f"rank {rank}/{world}")
        _check_covering(cov, _expected_covering(rb, world, rank), f"rank {rank}/{world}")
        dist.barrier()
    except Exception as e:
        errq.put(f"rank {rank}: {e!r}")
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,end_inclusive", [(2, 1), (3, 0), (8, 1)])
def test_partial_deps_reduce_host_transport(world, end_inclusive):
    """World 2, 3 and 8 (the node's 8 CommandStores, CommandStores.java:575-592) over the host transport, every rank on
    GPU 0: each home rank's reduced PartialDeps against the oracle's fold over the same store split."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, end_inclusive, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_partial_deps_covering_invariants():
    """The PartialDeps constructor's checks (PartialDeps.java:52-58): a covering that misses a store key, or a range of
    a RangeDeps, is IllegalStateException; the store's own covering passes."""
    from accord_amd import sharded as S
    from accord_amd.deps import Context, IllegalStateException
    rb = _batch(0x7C73, 4_000)
    with Context(0) as ctx:
        keep = []
        rbi = ctx.range_batch_in(rb, keep)
        ctx.partial_deps_batch_raw(rbi)
        lo, hi = _store_covering(rb, 1, 0)
        S.partial_deps_covering(ctx, rbi, (lo, hi))
        kd = ctx.calculate_partial_key_deps_mixed(rb)
        ctx.partial_deps_batch_raw(rbi)
        keys = np.unique(kd.kd_key)
        mid = int(keys[len(keys) // 2])
        with pytest.raises(IllegalStateException):   # the upper half of the key space uncovered
            S.partial_deps_covering(ctx, rbi, (lo, np.array([mid - 1], np.uint64)))
        with pytest.raises(IllegalStateException):   # no covering at all, deps present
            S.partial_deps_covering(ctx, rbi, (np.zeros(0, np.uint64), np.zeros(0, np.uint64)))
        S.partial_deps_covering(ctx, rbi, (lo, hi))  # the context stays usable
