"""acc_comm + acc_shard_reduce: the CommandStore exchange behind the C ABI (PreAccept.reduce,
messages/PreAccept.java:141-156). World 1 over RCCL (a one-rank communicator: the self send/recv path), and two
processes on the one GPU over the host transport (the library stages the fragment streams and calls back for the
all-to-all(v); here gloo): the home-txn merge equals the single-store KeyDeps."""
import os
import socket
import sys

import numpy as np
import pytest

from accord_amd import workload as W

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MERGE_FIELDS = ("key_off", "key_code", "val_off", "txn_rank", "k2v_off", "k2v")


def _check_home(merged, expect, label):
    for f in MERGE_FIELDS:
        np.testing.assert_array_equal(merged[f], expect[f], err_msg=f"{label} {f}")


def test_rccl_world_one():
    import torch
    from accord_amd import sharded as S
    from accord_amd.deps import Context
    dev = torch.device("cuda", 0)
    b = W.keydeps_batch(20000, 8, 20000, 0xC0AA, "zipf", 0.99, status_model="model", window=2000)
    with Context(0) as ctx:
        full = ctx.calculate_partial_deps(b)
        comm = S.Comm.rccl(ctx, 1, 0)
        bi, keep = S.batch_in_device(b, dev)
        ctx.keydeps_batch_raw(bi)
        view = S.shard_reduce(ctx, comm, bi, b.n_txn)
        merged = S.merged_to_host(ctx, view)
        comm.close()
    _check_home(merged, S.home_result_from_full(full, b, 0, 1), "rccl world 1")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, store_local, errq):
    sys.path[:0] = [os.path.join(ROOT, "cassandra-accord_amd"), os.path.join(ROOT, "oracle")]
    import torch
    import torch.distributed as dist
    import oracle
    from accord_amd import sharded as S
    from accord_amd.deps import Context
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        b = W.keydeps_batch(6000, 6, 3000, 0xC033 + world, "zipf", 0.99, status_model="model", window=800)
        bounds = S.even_split(b.key_code, world)
        gidx = None
        if store_local:
            local, g = S.store_batch(b, bounds, rank)
            gidx = g.astype(np.uint32)
        else:
            local = S.shard_batch(b, bounds, rank)
        with Context(0) as ctx:
            comm = S.Comm.host(ctx, world, rank)
            bi, keep = S.batch_in_device(local, dev)
            ctx.keydeps_batch_raw(bi)
            gdev = torch.from_numpy(gidx.astype(np.int32)).to(dev) if gidx is not None else None
            view = S.shard_reduce(ctx, comm, bi, b.n_txn, gdev)
            merged = S.merged_to_host(ctx, view)
            comm.close()
        _check_home(merged, S.home_result_from_full(oracle.keydeps_batch(b), b, rank, world), f"rank {rank}")
        dist.barrier()
    except Exception as e:
        errq.put(f"rank {rank}: {e!r}")
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,store_local", [(2, False), (3, True)])
def test_host_transport_processes(world, store_local):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, store_local, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
