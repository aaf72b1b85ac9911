"""Range-sharded RangeDeps on the GPU: per store acc_rangedeps_batch over the store-sliced batch,
fragments to the home rank, RangeDeps.with fold in store order by acc_deps_merge; parity with the oracle given the
same store split (tests/test_range_shard_cpu.py covers the split's semantics)."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu
FIELDS = ("key_off", "key_a", "key_b", "val_off", "msb", "lsb", "node", "k2v_off", "k2v")


def _batch(seed, n, end_inclusive=1, ranges_per_txn=2):
    from accord_amd import workload as W
    return W.rangedeps_batch(n, seed, p_range=0.5, keys_per_txn=3, ranges_per_txn=ranges_per_txn, key_bits=18,
                             max_width_log2=13, window=min(n, 2000), end_inclusive=end_inclusive)


def _oracle_merged(rb, world):
    import oracle
    from accord_amd import sharded as S
    per = S.range_reduce_local(rb, world, lambda sub: oracle.rangedeps_batch(sub))
    return {d: oracle.rmm_merge(m["grp_off"], m["half"], True) for d, m in per.items()}


def _check(got, want, label):
    for k in FIELDS:
        g, w = np.asarray(got[k]), np.asarray(want[k])
        assert g.shape == w.shape and np.array_equal(g.astype(np.int64), w.astype(np.int64)), (label, k)


@pytest.mark.parametrize("world,end_inclusive", [(1, 1), (2, 1), (3, 0), (4, 1)])
def test_range_shard_single_process(world, end_inclusive):
    from accord_amd import sharded as S
    from accord_amd.deps import Context, deps_merge
    rb = _batch(0x5151 + world, 20_000, end_inclusive)
    want = _oracle_merged(rb, world)
    with Context(0) as ctx:
        per = S.range_reduce_local(rb, world, lambda sub: ctx.calculate_partial_range_deps(sub))
        for d, m in per.items():
            got = deps_merge(ctx, dict(grp_off=m["grp_off"], key=None, range=m["half"]))["range"]
            _check(got, want[d], (world, d))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, errq):
    sys.path[:0] = [os.path.join(ROOT, "cassandra-accord_amd"), os.path.join(ROOT, "oracle")]
    import torch.distributed as dist
    from accord_amd import sharded as S
    from accord_amd.deps import Context, deps_merge
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rb = _batch(0x6262, 12_000)
        bounds = S.even_split(np.concatenate([rb.keys.key_code, rb.rng_start, rb.rng_end]).astype(np.uint64), world)
        sub, gidx = S.store_range_batch(rb, bounds, rank)
        with Context(0) as ctx:
            frags = S.pack_range_fragments(ctx.calculate_partial_range_deps(sub), gidx, world)
            recv, counts = S.exchange(frags)
            m = S.unpack_range_merge(recv, counts, S.home_txns(rb.n_txn, rank, world), rb)
            got = deps_merge(ctx, dict(grp_off=m["grp_off"], key=None, range=m["half"]))["range"]
        _check(got, _oracle_merged(rb, world)[rank], rank)
        dist.barrier()
    except Exception as e:
        errq.put(f"rank {rank}: {e!r}")
        raise
    finally:
        dist.destroy_process_group()


def test_range_shard_two_processes_gloo():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, errq)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
