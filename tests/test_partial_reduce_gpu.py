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


def _run_store(ctx, comm, rb, world, rank):
    """This rank's store: its sliced batch through acc_partial_deps_batch, then acc_partial_deps_reduce; host copies."""
    from accord_amd import sharded as S
    from accord_amd.deps import rmm_copy_out
    bounds = S.even_split(np.concatenate([rb.keys.key_code, rb.rng_start, rb.rng_end]).astype(np.uint64), world)
    sub, gidx = S.store_range_batch(rb, bounds, rank)
    keep = []
    rbi = ctx.range_batch_in(sub, keep)
    ctx.partial_deps_batch_raw(rbi)
    kv, rv = S.partial_deps_reduce(ctx, comm, rbi, rb.n_txn, gidx.astype(np.uint32))
    ng = int(kv.n_groups)
    key = S.merged_to_host(ctx, kv)
    rng = rmm_copy_out(ctx, ng, rv.range_deps, True)
    return key, rng


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
        key, rng = _run_store(ctx, comm, rb, 1, 0)
        comm.close()
    _check(key, rng, want_key, want_rng, "rccl world 1")


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
            key, rng = _run_store(ctx, comm, rb, world, rank)
            comm.close()
        want_key, want_rng = _expected(rb, world, rank)
        _check(key, rng, want_key, want_rng, f"rank {rank}/{world}")
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
