"""GPU parity of the device-side CommandStore-shard reduce (acc_shard_pack -> all-to-all(v) -> acc_shard_merge):
the per-home-txn merge of per-shard KeyDeps equals the single-store KeyDeps (KeyDeps does not depend on the shard
split; PreAccept.reduce, PreAccept.java:141-156). Single process with the exchange simulated by
concatenation, and two processes on one GPU exchanging through gloo (the RCCL path differs only in the backend)."""
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


@pytest.mark.parametrize("store_local,reverse", [(False, False), (True, False), (True, True)])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_reduce_single_process(world, store_local, reverse):
    """reverse: sources concatenated in descending shard order, so a txn's replies are not in ascending key order
    and the fused reduce must hand over to the general KeyDeps.merge (same canonical result)."""
    b = W.keydeps_batch(20000, 8, 20000, 0x5EED + world, "zipf", 0.99, status_model="model", window=2000)
    _run_single(b, world, store_local, reverse)


def test_shard_reduce_big_groups():
    """Home txns whose replies carry 8192..32768 TxnIds (the 1024-thread fused-reduce tier): a hot key of committed
    Reads closed by PREACCEPTED Writes that depend on all of them."""
    def set_kind(idx, kind):
        b.txn_lsb[idx] = (b.txn_lsb[idx] & ~np.uint64(0xE)) | np.uint64(kind << 1)
        b.exe_msb[idx], b.exe_lsb[idx], b.exe_node[idx] = b.txn_msb[idx], b.txn_lsb[idx], b.txn_node[idx]
    b = W.keydeps_batch(60000, 1, 1_000_000, 0xB16, "uniform", status_model="model", window=0)
    hot = np.arange(0, b.n_txn, 4)
    b.key_code[hot] = W.int_key_code(np.array([1 << 30]))[0]
    set_kind(hot, W.READ)
    b.status[hot] = W.APPLIED
    last = hot[-3:]
    set_kind(last, W.WRITE)
    b.status[last] = W.PREACCEPTED
    stats = _run_single(b, 2, True, False)
    assert stats["shard.big_groups"] > 0


def _run_single(b, world, store_local, reverse):
    import torch
    from accord_amd import sharded as S
    from accord_amd.deps import Context
    dev = torch.device("cuda", 0)
    stats = {}
    with Context(0) as ctx:
        full = ctx.calculate_partial_deps(b)
        bounds = S.even_split(b.key_code, world)
        sent, counts, keep = [], [], []
        for s in range(world):
            gidx = None
            if store_local:   # the store's batch holds only the txns touching its keys
                local, g = S.store_batch(b, bounds, s)
                gidx = torch.from_numpy(g.astype(np.int32)).to(dev)
                keep.append(gidx)
            else:
                local = S.shard_batch(b, bounds, s)
            bi, t = S.batch_in_device(local, dev)
            keep.append(t)
            ctx.keydeps_batch_raw(bi)
            bufs, c = S.shard_pack(ctx, bi, world, dev, gidx)
            sent.append(bufs)
            counts.append(c)
        for h in range(world):
            recv, rc = {}, np.zeros((4, world), np.int64)
            order = list(range(world))[::-1] if reverse else list(range(world))
            for q, (name, mult, _) in enumerate(S.STREAMS):
                parts = []
                for i, s in enumerate(order):
                    off = np.concatenate([[0], np.cumsum(counts[s][q])]) * mult
                    parts.append(sent[s][name][int(off[h]):int(off[h + 1])])
                    rc[q, i] = counts[s][q][h]
                recv[name] = torch.cat(parts)
            view = S.shard_merge(ctx, recv, rc, world, h, b.n_txn)
            merged = S.merged_to_host(ctx, view)
            _check_home(merged, S.home_result_from_full(full, b, h, world), f"world {world} home {h}")
            assert ctx.stats()["shard.general_merge"] == (1 if reverse and world > 1 else 0)
            for k, v in ctx.stats().items():
                stats[k] = max(stats.get(k, 0), v)
    return stats


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, errq):
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
        b = W.keydeps_batch(6000, 6, 3000, 0xD15C, "zipf", 0.99, status_model="model", window=800)
        local = S.shard_batch(b, S.even_split(b.key_code, world), rank)
        with Context(0) as ctx:
            bi, keep = S.batch_in_device(local, dev)
            ctx.keydeps_batch_raw(bi)
            bufs, counts = S.shard_pack(ctx, bi, world, dev)
            recv, rc = S.exchange_streams(bufs, counts)
            view = S.shard_merge(ctx, recv, rc, world, rank, b.n_txn)
            merged = S.merged_to_host(ctx, view)
        _check_home(merged, S.home_result_from_full(oracle.keydeps_batch(b), b, rank, world), f"rank {rank}")
        dist.barrier()
    except Exception as e:
        errq.put(f"rank {rank}: {e!r}")
        raise
    finally:
        dist.destroy_process_group()


def test_shard_reduce_two_processes_gloo():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, errq)) for r in range(2)]
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
