#!/usr/bin/env python3
"""Bench: batched Accord dependency calculation (PreAccept.calculatePartialDeps for every txn of a
CommandsForKey snapshot) on MI355X through the C ABI.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload = BASELINE.json configs[1]: 1M txns x 8 keys, zipf(0.99) over 1M keys, read/write mix,
status model of SURVEY.md §8(d). A step = one acc_keydeps_batch over the whole batch with inputs
already resident in HBM (device pointers) and results left device-resident (acc_keydeps_view).
Multi-GPU: each rank is one CommandStore shard holding its own 1M-txn snapshot (independent seed), no
data-path collective: weak scaling. Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "cassandra-accord_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip-level parameters)


def algorithmic_bytes(n_txn, n_pairs, sum_kd, sum_e, sum_u):
    """compulsory traffic, each input read once and each output written once."""
    b_in = 8 * n_pairs + 4 * (n_txn + 1) + 41 * n_txn
    b_out = 4 * (sum_kd + sum_e) + 4 * sum_kd + 4 * sum_u + 8 * (n_txn + 1)
    return b_in, b_out


def cpu_baseline(batch, seconds_target):
    """The C restatement (oracle, kind "port") on a strided sample of query txns, single thread."""
    import oracle
    n = batch.n_txn
    stride = max(1, int(os.environ.get("ACC_CPU_STRIDE", "100")))
    o = oracle.keydeps_batch(batch, query_lo=0, query_hi=n, query_stride=stride)
    return {
        "value": round(o.queried_pairs / o.query_s, 1),
        "unit": "txn-key pairs/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"every {stride}th txn of the same config-2 batch ({o.queried_pairs} (txn,key) queries, "
                   f"{o.query_s:.1f} s of CommandsForKey.mapReduceActive O(prefix) scans + KeyDeps.Builder; "
                   f"CFK snapshot build {o.build_s:.1f} s excluded)"),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of config 2 (testing only)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)

    from accord_amd import _lib as L
    from accord_amd import workload as W
    from accord_amd.deps import Context

    # each rank: an independent CommandStore snapshot of config 2 (rank 0 = the canonical seed)
    seed = W.CONFIG_SEEDS["2"] + 0x1000 * rank
    n_txn = int(1_000_000 * args.scale)
    batch = W.keydeps_batch(n_txn, 8, max(1000, n_txn), seed, "zipf", 0.99, status_model="model")

    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in batch.arrays().items()}
    torch.cuda.synchronize()
    bi = L.BatchIn(batch.n_txn, L.ACC_MEM_DEVICE, batch.n_pairs,
                   L.TsCols(t["txn_msb"].data_ptr(), t["txn_lsb"].data_ptr(), t["txn_node"].data_ptr()),
                   L.TsCols(t["exe_msb"].data_ptr(), t["exe_lsb"].data_ptr(), t["exe_node"].data_ptr()),
                   t["status"].data_ptr(), t["key_off"].data_ptr(), t["key_code"].data_ptr())

    ctx = Context(local, timing=True)
    view = None
    for _ in range(args.warmup):
        view = ctx.keydeps_batch_raw(bi)
    ctx.timing_reset()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        view = ctx.keydeps_batch_raw(bi)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())

    timing = ctx.timing()  # per kernel name: (total ms over the timed steps, launches)
    ms_per_step = elapsed * 1000.0 / args.steps
    kernel_ms = sum(v[0] for v in timing.values()) / args.steps
    dom_name, (dom_total, dom_launches) = max(timing.items(), key=lambda kv: kv[1][0])

    b_in, b_out = algorithmic_bytes(batch.n_txn, batch.n_pairs, view.total_keys, view.total_edges,
                                    view.total_deps)
    step_bytes = b_in + b_out
    achieved = step_bytes / (kernel_ms / 1000.0) / 1e9

    pairs_total = batch.n_pairs * world
    value = pairs_total * args.steps / elapsed

    result = {
        "metric": "txn-key conflict pairs resolved/sec (node)",
        "value": round(value, 1),
        "unit": "txn-key pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32/u64 (integer)",
        "data": "synthetic (seeded SplitMix64, SURVEY.md §8(d) status model)",
        "config": {
            "workload": "config2: KeyDeps batch, 1M txns x 8 keys, zipf(0.99) over 1M keys, p_write 0.5, "
                        "uncommitted window 10k, per-GPU CommandStore snapshot",
            "n_txn_per_gpu": batch.n_txn,
            "pairs_per_gpu": batch.n_pairs,
            "dep_edges_per_gpu": int(view.total_edges),
            "parallelism": f"keyspace shards x{world} (independent CommandStores)",
        },
        "dep_edges_per_s": round(int(view.total_edges) * world * args.steps / elapsed, 1),
        "roofline": {
            "bound": "hbm",
            "scope": "step: SURVEY §8(d) algorithmic bytes of one batch / device time of all kernels of the step",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "algorithmic_bytes_per_step": int(step_bytes),
            "kernel_ms_per_step": round(kernel_ms, 4),
            "dominant_kernel": {"name": dom_name, "avg_ms": round(dom_total / max(dom_launches, 1), 4),
                                "launches_per_step": dom_launches / args.steps,
                                "share_of_step": round(dom_total / args.steps / kernel_ms, 3)},
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(batch, args.cpu_seconds)
    result["path_stats"] = ctx.stats()
    if os.environ.get("ACC_BENCH_KERNELS"):
        result["kernels_ms_per_step"] = {k: round(v[0] / args.steps, 4) for k, v in
                                         sorted(timing.items(), key=lambda kv: -kv[1][0])}
    ctx.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
