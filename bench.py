#!/usr/bin/env python3
"""Bench: batched Accord dependency calculation on MI355X through the C ABI.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

--config 2 (default; BASELINE.json configs[1], the metric's workload): KeyDeps of 1M txns x 8 keys, zipf(0.99) over
1M keys, read/write mix, status model of SURVEY.md §8(d). A step = one acc_keydeps_batch over the whole batch
(PreAccept.calculatePartialDeps for every txn of a CommandsForKey snapshot) with inputs already resident in HBM
(device pointers) and results left device-resident (acc_keydeps_view).
--config 3 (configs[2]): 100M txn-key pairs (12.5M txns x 8 keys, zipf(0.99) over 2^24 keys, status model): on one GPU
one acc_keydeps_batch over the whole batch; at N > 1 the same global batch range-sharded over the N GPUs (strong
scaling) through the multi-GPU path below.
--config 4 (configs[3]): RangeDeps of 10M range txns (1 EndInclusive range each, log-uniform widths <= 2^16)
interleaved with 10M key txns x 4 keys over the int32 key space; a step = one acc_rangedeps_batch.
--config 5 (configs[4]): KeyDeps.merge of 16,384 coordinated txns x 64 replica replies, then acc_levelise of the
merged graph by executeAt; a step = one acc_keydeps_merge + one acc_levelise on device-resident inputs.

Multi-GPU (--config 2, N > 1): one global batch of N x 1M txns x 8 keys, zipf(0.99) over N x 1M keys (seeded
permutation), key range-sharded over the N GPUs the way CommandStores shard a node (EvenSplit); each rank is one
CommandStore holding the txns that touch its keys. A step = the store's acc_keydeps_batch + acc_shard_pack + the
all-to-all(v) of per-txn fragments to the txn's home GPU (RCCL over xGMI) + acc_shard_merge (PartialDeps.with fold =
batched KeyDeps.merge): PreAccept.reduce on device. Weak scaling (~8M pairs per GPU); value = global pairs / the
slowest rank's time. --config 4 at N > 1 runs independent snapshots per rank. Prints ONE JSON line on rank 0.
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


def keydeps_bytes(n_txn, n_pairs, sum_kd, sum_e, sum_u):
    """SURVEY.md §8(d) KeyDeps batch: compulsory traffic, each input read once and each output written once."""
    b_in = 8 * n_pairs + 4 * (n_txn + 1) + 41 * n_txn
    b_out = 4 * (sum_kd + sum_e) + 4 * sum_kd + 4 * sum_u + 8 * (n_txn + 1)
    return b_in, b_out


def rangedeps_bytes(n_txn, n_pairs, n_ranges, sum_rd, sum_e, sum_u, n_dict):
    """SURVEY.md §8(d) RangeDeps batch: range bounds + owners + txn columns + keys in; Java arena, range ids, TxnId
    indices, three offset arrays and the stored-range dictionary out."""
    b_in = 16 * n_ranges + 8 * (n_txn + 1) + 41 * n_txn + 8 * n_pairs
    b_out = 4 * (sum_rd + sum_e) + 4 * sum_rd + 4 * sum_u + 24 * (n_txn + 1) + 16 * n_dict
    return b_in, b_out


def profile_traffic(kernel, config=None):
    """HBM bytes per launch of `kernel` from the newest committed rocprof summary (profiles/*_summary.json: FETCH_SIZE
    x 2 per the gfx950 correction + WRITE_SIZE, MI355X_MICROARCH.md §HBM), or None."""
    import glob
    best = None
    pattern = f"*_config{config}_summary.json" if config else "*_summary.json"
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", pattern))):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        k = d.get("kernels", {}).get("k_" + kernel) or d.get("kernels", {}).get(kernel)
        if k and "hbm_read_bytes_per_launch" in k:
            best = (k["hbm_read_bytes_per_launch"] + k["hbm_write_bytes_per_launch"], os.path.relpath(p, ROOT))
    return best


def roofline(step_bytes, timing, steps, config=None):
    """Contract roofline for the dominant kernel: achieved = algorithmic bytes of the batch one launch processes /
    that kernel's average launch (HIP events on the context stream). step_* = the same bytes over the device time of
    every kernel of the step (the whole pipeline as one launch: the stricter figure)."""
    kernel_ms = sum(v[0] for v in timing.values()) / steps
    dom_name, (dom_total, dom_launches) = max(timing.items(), key=lambda kv: kv[1][0])
    dom_avg_ms = dom_total / max(dom_launches, 1)
    achieved = step_bytes / (dom_avg_ms / 1000.0) / 1e9
    step_achieved = step_bytes / (kernel_ms / 1000.0) / 1e9
    tr = profile_traffic(dom_name, config)
    return {
        "bound": "hbm",
        "kernel": dom_name,
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": int(tr[0]) if tr else None,
        "traffic_source": tr[1] if tr else None,
        "algorithmic_bytes_per_launch": int(step_bytes),
        "kernel_avg_ms": round(dom_avg_ms, 4),
        "launches_per_step": dom_launches / steps,
        "share_of_step": round(dom_total / steps / kernel_ms, 3),
        "step_kernel_ms": round(kernel_ms, 4),
        "step_achieved": round(step_achieved, 1),
        "step_frac": round(step_achieved / HBM_PEAK_GBS, 4),
    }


def keydeps_cpu_baseline(batch):
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


def rangedeps_cpu_baseline(rb):
    """The C restatement of mapReduceRangesInternal (a linear walk of every range command per query, as the
    reference's TreeMap forEach) on a strided sample of query txns, single thread."""
    import oracle
    n = rb.n_txn
    stride = max(1, int(os.environ.get("ACC_CPU_STRIDE_RD", str(max(1, n // 120)))))
    o = oracle.rangedeps_batch(rb, query_lo=0, query_hi=n, query_stride=stride)
    kp = np.diff(rb.keys.key_off.astype(np.int64)) + np.diff(rb.rng_off.astype(np.int64))
    probes = int(kp[::stride].sum())
    return {
        "value": round(probes / o.query_s, 1),
        "unit": "key probes/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"every {stride}th txn of the same config-4 batch ({o.queried} txns, {probes} key/range probes, "
                   f"{o.query_s:.1f} s of range-command scans + RangeDeps.Builder)"),
    }


def dist_setup(args):
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal hook (tests only): every rank on GPU 0 with gloo, to exercise the N > 1 path on a one-GPU box
    if os.environ.get("ACC_BENCH_REHEARSE") == "1":
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("gloo" if os.environ.get("ACC_BENCH_REHEARSE") == "1" else "nccl")
    return world, rank, local, torch.device("cuda", local)


def timed_steps(args, world, dev, step):
    import torch
    import torch.distributed as dist
    for _ in range(args.warmup):
        step()
    step.ctx.timing_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    return elapsed


class Step:
    def __init__(self, ctx, fn):
        self.ctx, self.fn, self.view = ctx, fn, None

    def __call__(self):
        self.view = self.fn()


def run_config2(args, world, rank, local, dev):
    import torch
    from accord_amd import _lib as L
    from accord_amd import workload as W
    from accord_amd.deps import Context

    c3 = args.config == "3"
    seed = W.CONFIG_SEEDS["3z" if c3 else "2"] + 0x1000 * rank
    n_txn = int((12_500_000 if c3 else 1_000_000) * args.scale)
    n_keys = int((1 << 24) * args.scale) if c3 else n_txn
    batch = W.keydeps_batch(n_txn, 8, max(1000, n_keys), seed, "zipf", 0.99, status_model="model")
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in batch.arrays().items()}
    torch.cuda.synchronize()
    bi = L.BatchIn(batch.n_txn, L.ACC_MEM_DEVICE, batch.n_pairs,
                   L.TsCols(t["txn_msb"].data_ptr(), t["txn_lsb"].data_ptr(), t["txn_node"].data_ptr()),
                   L.TsCols(t["exe_msb"].data_ptr(), t["exe_lsb"].data_ptr(), t["exe_node"].data_ptr()),
                   t["status"].data_ptr(), t["key_off"].data_ptr(), t["key_code"].data_ptr())
    ctx = Context(local, timing=True)
    step = Step(ctx, lambda: ctx.keydeps_batch_raw(bi))
    elapsed = timed_steps(args, world, dev, step)
    view = step.view
    timing = ctx.timing()
    b_in, b_out = keydeps_bytes(batch.n_txn, batch.n_pairs, view.total_keys, view.total_edges, view.total_deps)
    result = {
        "metric": "txn-key conflict pairs resolved/sec (node)",
        "value": round(batch.n_pairs * world * args.steps / elapsed, 1),
        "unit": "txn-key pairs/s",
        "dtype": "u32/u64 (integer)",
        "data": "synthetic (seeded SplitMix64, SURVEY.md §8(d) status model)",
        "config": {
            "workload": ("config3 on one GPU: KeyDeps batch of 100M txn-key pairs (12.5M txns x 8 keys), zipf(0.99) "
                         "over 2^24 keys, p_write 0.5, uncommitted window 10k, one CommandStore snapshot") if c3 else
                        ("config2: KeyDeps batch, 1M txns x 8 keys, zipf(0.99) over 1M keys, p_write 0.5, "
                         "uncommitted window 10k, per-GPU CommandStore snapshot"),
            "n_txn_per_gpu": batch.n_txn,
            "pairs_per_gpu": batch.n_pairs,
            "dep_edges_per_gpu": int(view.total_edges),
            "parallelism": f"keyspace shards x{world} (independent CommandStores)",
        },
        "dep_edges_per_s": round(int(view.total_edges) * world * args.steps / elapsed, 1),
        "roofline": roofline(b_in + b_out, timing, args.steps, args.config),
    }
    if rank == 0 and world == 1 and not args.no_cpu and not c3:   # config 3: the O(prefix) CPU scan takes hours
        result["cpu_baseline"] = keydeps_cpu_baseline(batch)
    return ctx, timing, elapsed, result


def run_config2_sharded(args, world, rank, local, dev):
    import torch
    from accord_amd import sharded as S
    from accord_amd import workload as W
    from accord_amd.deps import Context

    c3 = args.config == "3"   # config 3: 100M pairs in total over the N GPUs (strong scaling); else N x config 2
    n_global = int(12_500_000 * args.scale) if c3 else int(1_000_000 * args.scale) * world
    n_keys = int((1 << 24) * args.scale) if c3 else n_global
    batch = W.keydeps_batch(n_global, 8, max(1000, n_keys), W.CONFIG_SEEDS["3z" if c3 else "2"], "zipf", 0.99,
                            status_model="model")
    bounds = S.even_split(batch.key_code, world)
    sub, g = S.store_batch(batch, bounds, rank)
    bi, keep = S.batch_in_device(sub, dev)
    gidx = torch.from_numpy(g.astype(np.int32)).to(dev)
    del batch
    ctx = Context(local, timing=True)
    info = {}

    def fn():
        v = ctx.keydeps_batch_raw(bi)
        bufs, counts = S.shard_pack(ctx, bi, world, dev, gidx)
        torch.cuda.synchronize(dev)
        recv, rc = S.exchange_streams(bufs, counts)
        mv = S.shard_merge(ctx, recv, rc, world, rank, n_global)
        info["kd"], info["counts"], info["merge"] = v, counts, mv
        return v

    step = Step(ctx, fn)
    elapsed = timed_steps(args, world, dev, step)
    view = info["kd"]
    timing = ctx.timing()
    b_in, b_out = keydeps_bytes(sub.n_txn, sub.n_pairs, view.total_keys, view.total_edges, view.total_deps)
    sent = info["counts"]
    sent_bytes = int(16 * sent[0].sum() + 8 * sent[1].sum() + 4 * sent[2].sum() + 4 * sent[3].sum())
    import torch.distributed as dist
    loc = torch.tensor([sub.n_pairs, sent_bytes], dtype=torch.float64,
                       device=dev if dist.get_backend() == "nccl" else "cpu")
    tot = loc.clone()
    dist.all_reduce(tot)
    mx = loc.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    result = {
        "metric": "txn-key conflict pairs resolved/sec (node)",
        "value": round(n_global * 8 * args.steps / elapsed, 1),
        "unit": "txn-key pairs/s",
        "dtype": "u32/u64 (integer)",
        "data": "synthetic (seeded SplitMix64, SURVEY.md §8(d) status model)",
        "config": {
            "workload": f"{'config3' if c3 else f'config2 x{world}'} range-sharded: KeyDeps of {n_global} txns x 8 keys, "
                        f"zipf(0.99) over {n_keys} keys, key ranges EvenSplit over {world} GPUs (one CommandStore each), "
                        "PreAccept.reduce of per-store PartialDeps by RCCL all-to-all(v) + on-device KeyDeps.merge",
            "n_txn_global": n_global,
            "pairs_global": n_global * 8,
            "pairs_per_gpu_max": int(mx[0].item()),
            "parallelism": f"key-range shards x{world} (CommandStores) + all-to-all(v) reduce",
        },
        "exchange": {"bytes_sent_total": int(tot[1].item()), "bytes_sent_max_rank": int(mx[1].item()),
                     "backend": dist.get_backend() + (" (RCCL over xGMI)" if dist.get_backend() == "nccl" else "")},
        "roofline": roofline(b_in + b_out, timing, args.steps, args.config),
    }
    return ctx, timing, elapsed, result


def run_config4(args, world, rank, local, dev):
    import torch
    from accord_amd import _lib as L
    from accord_amd import workload as W
    from accord_amd.deps import Context

    rb = W.rangedeps_batch(int(20_000_000 * args.scale), W.CONFIG_SEEDS["4"] + 0x1000 * rank)
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in rb.arrays().items()}
    torch.cuda.synchronize()
    P, R = rb.keys.n_pairs, rb.n_ranges
    bi = L.RangeBatchIn(rb.n_txn, L.ACC_MEM_DEVICE, P, R,
                        L.TsCols(t["txn_msb"].data_ptr(), t["txn_lsb"].data_ptr(), t["txn_node"].data_ptr()),
                        L.TsCols(t["exe_msb"].data_ptr(), t["exe_lsb"].data_ptr(), t["exe_node"].data_ptr()),
                        t["status"].data_ptr(), t["key_off"].data_ptr(), t["key_code"].data_ptr(),
                        t["rng_off"].data_ptr(), t["rng_start"].data_ptr(), t["rng_end"].data_ptr(),
                        int(rb.end_inclusive), 0)
    ctx = Context(local, timing=True)
    step = Step(ctx, lambda: ctx.rangedeps_batch_raw(bi))
    elapsed = timed_steps(args, world, dev, step)
    view = step.view
    timing = ctx.timing()
    b_in, b_out = rangedeps_bytes(rb.n_txn, P, R, view.total_ranges, view.total_edges, view.total_deps, view.n_ranges)
    probes = P + R
    result = {
        "metric": "RangeDeps key probes resolved/sec (node)",
        "value": round(probes * world * args.steps / elapsed, 1),
        "unit": "key probes/s",
        "dtype": "u32/u64 (integer)",
        "data": "synthetic (seeded SplitMix64, SURVEY.md §8(d) config 4)",
        "config": {
            "workload": "config4: RangeDeps of a mixed batch, 10M range txns (1 EndInclusive range, width log-uniform "
                        "in [1, 2^16], start uniform over int32) + 10M key txns x 4 uniform keys, interleaved 50/50",
            "n_txn_per_gpu": rb.n_txn,
            "key_probes_per_gpu": probes,
            "range_commands_per_gpu": R,
            "dep_entries_per_gpu": int(view.total_edges),
            "parallelism": f"keyspace shards x{world} (independent CommandStores)",
        },
        "dep_entries_per_s": round(int(view.total_edges) * world * args.steps / elapsed, 1),
        "roofline": roofline(b_in + b_out, timing, args.steps, args.config),
    }
    if os.environ.get("ACC_BENCH_MIXED", "1") != "0":
        result["keydeps_mixed"] = mixed_keydeps_leg(bi, local)
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = rangedeps_cpu_baseline(rb)
    return ctx, timing, elapsed, result


def mixed_keydeps_leg(bi, local, calls=3):
    """The key half of the same mixed batch's PartialDeps (acc_keydeps_mixed: key txns' CommandsForKey scans plus every
    range txn over the CFKs inside its range), timed separately on its own context: 1 warmup + `calls` timed calls."""
    import torch
    from accord_amd.deps import Context
    with Context(local, timing=True) as c:
        c.keydeps_mixed_raw(bi)
        c.timing_reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(calls):
            v = c.keydeps_mixed_raw(bi)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1000.0 / calls
        tm = c.timing()
        top = sorted(tm.items(), key=lambda kv: -kv[1][0])[:6]
        return {"ms_per_call": round(ms, 3), "range_key_queries": int(c.stats().get("keydeps.range_key_queries", 0)),
                "dep_entries": int(v.total_edges), "kd_keys": int(v.total_keys),
                "top_kernels_ms": {k: round(x[0] / calls, 3) for k, x in top}}


def merge_bytes(m, view, n_txn, n_edges):
    """SURVEY.md §8(d) merge + levelise: every reply's keys / TxnIds / keysToTxnIds and offsets in, the merged
    per-txn CSR out; levelise reads the merged graph (val_off, TxnIds, executeAt ranks) and writes level + order."""
    nr = len(m["key_off"]) - 1
    b_in = 8 * len(m["key_code"]) + 4 * len(m["txn_rank"]) + 4 * len(m["k2v"]) + 24 * (nr + 1) + 8 * (n_txn + 1)
    b_out = 8 * view.total_keys + 4 * view.total_vals + 4 * view.total_k2v + 24 * (n_txn + 1)
    b_lv = 8 * (n_txn + 1) + 4 * n_edges + 4 * n_txn + 8 * n_txn
    return b_in + b_out + b_lv


def merge_prefix(m, g):
    """The first g groups of an acc_merge_in dict (groups and their replies are contiguous)."""
    r = int(m["grp_off"][g])
    ko, vo, oo = (int(m[k][r]) for k in ("key_off", "val_off", "k2v_off"))
    return dict(grp_off=m["grp_off"][:g + 1], key_off=m["key_off"][:r + 1], key_code=m["key_code"][:ko],
                val_off=m["val_off"][:r + 1], txn_rank=m["txn_rank"][:vo], k2v_off=m["k2v_off"][:r + 1],
                k2v=m["k2v"][:oo])


def merge_cpu_baseline(m, exec_rank, n_in):
    """The C restatement (LinearMerger fold of linearUnion per txn, then the levelisation walk) on a prefix of the
    same config-5 batch, single thread; unit = input entries merged/s."""
    import oracle
    n = len(m["grp_off"]) - 1
    g = min(n, max(1, int(os.environ.get("ACC_CPU_GROUPS_MERGE", str(n)))))
    sub = merge_prefix(m, g)
    entries = int(len(sub["k2v"]) - (len(sub["key_code"])))
    t0 = time.perf_counter()
    ref = oracle.keydeps_merge(sub)
    t1 = time.perf_counter()
    er = np.argsort(np.argsort(exec_rank[:g], kind="stable"), kind="stable").astype(np.uint32)
    dep = ref["txn_rank"]
    oracle.levelise(ref["val_off"], dep, er)
    t2 = time.perf_counter()
    return {
        "value": round(entries / (t2 - t0), 1),
        "unit": "input entries/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"first {g} of {n} coordinated txns ({entries} reply entries of {n_in}): KeyDeps.merge "
                   f"{t1 - t0:.2f} s + levelise of their merged graph {t2 - t1:.3f} s"),
    }


def run_config5(args, world, rank, local, dev):
    import torch
    from accord_amd import _lib as L
    from accord_amd import workload as W
    from accord_amd.deps import Context, merge_levelise_device

    seed = W.CONFIG_SEEDS["5"] + 0x1000 * rank
    n_txn = int(16_384 * args.scale)
    m = W.merge_batch(n_txn=n_txn, replies=64, seed=seed)
    exec_rank = W.merge_exec_rank(n_txn, seed)
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in m.items()}
    er = torch.from_numpy(exec_rank).to(dev)
    level = torch.empty(n_txn, dtype=torch.int32, device=dev)
    order = torch.empty(n_txn, dtype=torch.int32, device=dev)
    nl = np.zeros(1, np.uint32)
    torch.cuda.synchronize()
    mi = L.MergeIn(L.ACC_MEM_DEVICE, n_txn, len(m["key_off"]) - 1,
                   *(t[k].data_ptr() for k in ("grp_off", "key_off", "key_code", "val_off", "txn_rank", "k2v_off",
                                               "k2v")))
    ctx = Context(local, timing=True)

    def fn():
        view, nl[0] = merge_levelise_device(ctx, mi, er.data_ptr(), level.data_ptr(), order.data_ptr())
        return view

    step = Step(ctx, fn)
    elapsed = timed_steps(args, world, dev, step)
    view = step.view
    timing = ctx.timing()
    n_in = int(view.total_in_entries)
    result = {
        "metric": "Deps.merge input entries merged/sec + executeAt levelisation (node)",
        "value": round(n_in * world * args.steps / elapsed, 1),
        "unit": "input entries/s",
        "dtype": "u32/u64 (integer)",
        "data": "synthetic (seeded SplitMix64, SURVEY.md §8(d) config 5)",
        "config": {
            "workload": f"config5: KeyDeps.merge of {n_txn} coordinated txns x 64 replica replies (zipf keys, each "
                        "reply drops 10% of the true entries and adds 5% spurious ones), then levelisation of the "
                        "merged graph by executeAt",
            "n_txn_per_gpu": n_txn,
            "replies_per_gpu": n_txn * 64,
            "input_entries_per_gpu": n_in,
            "merged_entries_per_gpu": int(view.total_k2v - view.total_keys),
            "levels": int(nl[0]),
            "parallelism": f"independent coordinators x{world}",
        },
        "roofline": roofline(merge_bytes(m, view, n_txn, int(view.total_vals)), timing, args.steps, args.config),
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = merge_cpu_baseline(m, exec_rank, n_in)
    return ctx, timing, elapsed, result


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="2", choices=["2", "3", "4", "5"])
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of the config (testing only)")
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world, rank, local, dev = dist_setup(args)
    keyed = run_config2 if world == 1 else run_config2_sharded
    run = {"2": keyed, "3": keyed, "4": run_config4, "5": run_config5}[args.config]
    ctx, timing, elapsed, result = run(args, world, rank, local, dev)
    out = {
        "metric": result.pop("metric"),
        "value": result.pop("value"),
        "unit": result.pop("unit"),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1000.0 / args.steps, 3),
        "higher_is_better": True,
        "scaling": "strong" if args.config == "3" and world > 1 else "weak",
        "vs_baseline": None,
    }
    out.update(result)
    out["path_stats"] = ctx.stats()
    if os.environ.get("ACC_BENCH_KERNELS"):
        out["kernels_ms_per_step"] = {k: round(v[0] / args.steps, 4) for k, v in
                                      sorted(timing.items(), key=lambda kv: -kv[1][0])}
    ctx.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
