"""World-size-2 (and 3) gloo tests of the key-range sharded path on CPU: per-shard calculatePartialDeps,
all-to-allv of per-txn fragments to the home rank, PartialDeps.with-equivalent merge there. The per-shard
compute and the merge use the oracle here (no GPU); on GPUs the same plumbing runs acc_keydeps_batch and
acc_keydeps_merge over RCCL."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, seed, errq):
    sys.path[:0] = [os.path.join(ROOT, "cassandra-accord_amd"), os.path.join(ROOT, "oracle")]
    import torch.distributed as dist
    import oracle
    from accord_amd import sharded as S
    from accord_amd import workload as W
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = W.keydeps_batch(3000, 4, 500, seed, "zipf", 0.99, status_model="model", window=600)
        bounds = S.even_split(b.key_code, world)
        local = S.shard_batch(b, bounds, rank)
        res = oracle.keydeps_batch(local)
        recv, counts = S.exchange(S.pack_fragments(res, local, world))
        homes = S.home_txns(b.n_txn, rank, world)
        merged = oracle.keydeps_merge(S.unpack_to_merge(recv, counts, homes))
        full = oracle.keydeps_batch(b)
        for gi, t in enumerate(homes.tolist()):
            k, d, a = full.txn(t)
            keys = b.key_code[int(b.key_off[t]) + k.astype(np.int64)]
            ka, kb = int(merged["key_off"][gi]), int(merged["key_off"][gi + 1])
            va, vb = int(merged["val_off"][gi]), int(merged["val_off"][gi + 1])
            oa, ob = int(merged["k2v_off"][gi]), int(merged["k2v_off"][gi + 1])
            assert merged["key_code"][ka:kb].tolist() == keys.tolist(), (rank, t)
            assert merged["txn_rank"][va:vb].tolist() == d.tolist(), (rank, t)
            assert merged["k2v"][oa:ob].tolist() == a.tolist(), (rank, t)
        dist.barrier()
    except Exception as e:  # surface the failure to the parent
        errq.put(f"rank {rank}: {e!r}")
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_reduce_equals_single_store(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 0xABC + world, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_even_split_covers_domain():
    from accord_amd import sharded as S
    kc = np.array([5, 9, 100, 1000], dtype=np.uint64)
    b = S.even_split(kc, 4)
    assert b[0] == 5 and b[-1] == 1001 and (np.diff(b.astype(np.int64)) > 0).all()


def _store_slice_worker(rank, world, port, dist_name, errq):
    sys.path[:0] = [os.path.join(ROOT, "cassandra-accord_amd"), os.path.join(ROOT, "oracle")]
    import torch.distributed as dist
    from accord_amd import sharded as S
    from accord_amd import workload as W
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, k, nk, seed = 6000, 8, 700, 0xACC0_0002
        sub, g, bounds = S.keydeps_store_batch(n, k, nk, seed, dist_name, world, rank, window=900)
        full = W.keydeps_batch(n, k, nk, seed, dist_name, 0.99, status_model="model", window=900)
        b2 = S.even_split(full.key_code, world)
        assert np.array_equal(bounds, b2), (bounds, b2)
        ref, g2 = S.store_batch(full, b2, rank)
        assert np.array_equal(g, g2)
        for f, v in ref.arrays().items():
            assert np.array_equal(getattr(sub, f), v), f
        dist.barrier()
    except Exception as e:  # surface the failure to the parent
        errq.put(f"rank {rank}: {e!r}")
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,dist_name", [(3, "zipf"), (8, "zipf"), (2, "uniform")])
def test_store_slice_generation_equals_full_batch(world, dist_name):
    """bench.py --gpus N at N > 1: each rank draws 1/N of the txns' keys (duplicate redraws coordinated by an
    all-gather) and receives its key range's pairs by one all-to-all(v); the store batch equals
    store_batch(keydeps_batch(...)) of the single-host generator, array for array."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_store_slice_worker, args=(r, world, port, dist_name, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
