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
slowest rank's time. --config 4 at N > 1: the config-4 batch EvenSplit over N stores, each step a store's whole
PartialDeps + acc_partial_deps_reduce (strong scaling). Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "cassandra-accord_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip-level parameters)

# KeyDeps tiers launched on a side stream, concurrently with the stream pass (csrc/keydeps.hip keydeps_core)
SIDE_STREAM_TAGS = {"v2_write_med", "v2_write_big", "v2_write_huge", "v2_write_medium", "v2_write_win", "v2_write_win16",
                    "v3_stream_runs",
                    # RangeDeps build tiers on side streams beside the wave tier (csrc/rangedeps.hip rangedeps_batch)
                    "rd_build_s16", "rd_build_s32", "rd_build_block"}

# launch tags whose kernel is one instance of a template launched under several tags (csrc/keydeps.hip tiers)
TAG_KERNEL = {
    "v2_write_med": "k_v2_write_big<1024,256>",
    "v2_write_big": "k_v2_write_big<8192,512>",
    "v2_write_huge": "k_v2_write_big<16384,1024>",
    "v2_write_win": "k_v2_write_win<8>",
    "v2_write_win16": "k_v2_write_win<16>",
    # the stream pass: k_v3_stream<EntT, NT, G, N2, LIST, RUNS> (lean pass / RUNS pass on a side stream; either EntT)
    "v3_stream": ("k_v3_stream<", "false,false>"),
    "v3_stream_runs": ("k_v3_stream<", "true,true>"),
    # the RangeDeps lane-group tiers: k_rd_build_seg<S, NARROW> (prefix: either sort width)
    "rd_build_s16": "k_rd_build_seg<16,",
    "rd_build_s32": "k_rd_build_seg<32,",
    "rd_build_s64": "k_rd_build_seg<64,",
    # the levelise walk tiers (levelise.hip: one tag per tier)
    "lv_walk_lds": "k_lv_lds",
    "lv_walk_win": "k_lw_step<",
    "lv_walk_waves": "k_lv_waves",
}


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


def profile_summary(config, variant=""):
    """The newest committed rocprof summary for this bench config (profiles/r??_config<cfg><variant>_summary.json):
    (summary dict, relative path) or (None, None)."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_config{config}{variant}_summary.json")))
    for p in reversed(paths):
        try:
            return json.load(open(p)), os.path.relpath(p, ROOT)
        except Exception:
            continue
    return None, None


def roofline(step_bytes, step, steps, ms_per_step, config, variant="", profiled=True):
    """HBM roofline of the whole step (the pipeline is one launch chain per step): achieved = the step's algorithmic
    bytes (each input read once, each output written once) / the timed ms_per_step; `traffic` = the
    HBM bytes per step of the committed rocprof PMC summary of the same config (FETCH_SIZE x2 + WRITE_SIZE, the upper
    bound; traffic_raw = FETCH_SIZE x1 + WRITE_SIZE, the lower bound: tools/calib_fetch.hip calibration). The dominant
    kernel is reported beside it with its HIP-event average and the committed rocprof average for the same kernel.
    profiled=False (a scaled or store-sharded workload, not the one the committed profile measured): no traffic."""
    timing, dsteps = step.diag, DIAG_STEPS
    if not timing:   # ACC_BENCH_NOTIME probe: no per-kernel events were recorded
        timing, dsteps = {"unrecorded": (ms_per_step * steps, steps)}, steps
    kernel_ms = sum(v[0] for v in timing.values()) / dsteps
    # the dominant kernel for the rocprof cross-check is taken among the context-stream kernels (the side-stream tiers
    # overlap the stream pass, so their durations include waiting for CUs); its average is the one measured live over
    # the timed region (the only kernel bracketed by events there)
    main = {k: v for k, v in timing.items() if k not in SIDE_STREAM_TAGS} or timing
    dom_name = max(main.items(), key=lambda kv: kv[1][0])[0]
    dom_total, dom_launches = (step.live or {}).get(dom_name, (timing[dom_name][0] * steps / dsteps,
                                                                timing[dom_name][1] * steps // dsteps))
    achieved = step_bytes / (ms_per_step / 1000.0) / 1e9
    prof, prof_path = profile_summary(config, variant) if profiled else (None, None)
    traffic = traffic_raw = dom_prof_ms = None
    if prof:
        traffic = int(prof.get("hbm_bytes_per_step", 0)) or None
        if "hbm_read_bytes_per_step_raw" in prof:
            traffic_raw = int(prof["hbm_read_bytes_per_step_raw"] + prof["hbm_write_bytes_per_step"])
        # rocprof names carry template arguments (k_v3_stream<unsignedint,512>): launch tags of one kernel's template
        # variants map to their instance, the others match on the base name
        kernels = prof.get("kernels", {})
        exact = TAG_KERNEL.get(dom_name)
        if isinstance(exact, tuple):   # (prefix, suffix): one template instance whatever its leading arguments
            ks = [v for name, v in kernels.items() if name.startswith(exact[0]) and name.endswith(exact[1])]
        elif exact and exact in kernels:
            ks = [kernels[exact]]
        elif exact and exact.endswith((",", "<")):
            ks = [v for name, v in kernels.items() if name.startswith(exact)]
        else:
            ks = [v for name, v in kernels.items() if name.split("<")[0] in ("k_" + dom_name, dom_name)]
        if ks:
            calls = sum(v["calls"] for v in ks)
            dom_prof_ms = round(sum(v["total_ns"] for v in ks) / max(calls, 1) / 1e6, 4)
    return {
        "bound": "hbm",
        "kernel": "pipeline: every kernel of one step (algorithmic bytes of the step / timed ms_per_step)",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 5),
        "traffic": traffic,
        "traffic_raw": traffic_raw,
        "traffic_source": prof_path,
        "traffic_over_algorithmic": round(traffic / step_bytes, 2) if traffic else None,
        "algorithmic_bytes_per_step": int(step_bytes),
        "device_kernel_ms_per_step": round(kernel_ms, 4),
        "device_frac": round(step_bytes / (kernel_ms / 1000.0) / 1e9 / HBM_PEAK_GBS, 5),
        "side_stream_kernels_ms_per_step": {k: round(v[0] / dsteps, 4) for k, v in timing.items() if k in SIDE_STREAM_TAGS},
        "dominant_kernel": {"name": dom_name, "avg_ms": round(dom_total / max(dom_launches, 1), 4),
                            "avg_ms_rocprof": dom_prof_ms, "launches_per_step": dom_launches / steps,
                            "share_of_device_time": round(dom_total / steps / kernel_ms, 3),
                            "measured": "HIP events on the launch stream around this kernel's launches only, over the "
                                        "timed steps"},
        "breakdown": f"device_kernel_ms_per_step and kernels_ms_per_step: {DIAG_STEPS} untimed steps after the warmup "
                     "with every launch bracketed by HIP events",
    }


def cpu_info():
    """(lscpu model name, CPUs this process may use). The GPU box grants 16 CPUs per GPU (nproc shows the machine)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 1
    return model, avail


def cpu_threads():
    return max(1, min(int(os.environ.get("ACC_CPU_THREADS", "16")), cpu_info()[1]))


def run_threads(fn, parts):
    """fn(part) on one thread per part (the oracle's C code releases the GIL inside ctypes): results, wall seconds."""
    from concurrent.futures import ThreadPoolExecutor
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=len(parts)) as ex:
        res = list(ex.map(fn, parts))
    return res, time.perf_counter() - t0


def keydeps_cpu_baseline(batch, label, stride_env="ACC_CPU_STRIDE", default_stride=100):
    """The C restatement (oracle, kind "port") of the reference's concurrency model: S CommandStores
    (EvenSplit of the key domain, one thread each) running calculatePartialDeps for a strided sample of their txns,
    plus the same sample on one thread. The per-txn PartialDeps.with fold across stores is not timed."""
    import oracle
    from accord_amd import sharded as S
    stride = max(1, int(os.environ.get(stride_env, str(default_stride))))
    o1 = oracle.keydeps_batch(batch, query_lo=0, query_hi=batch.n_txn, query_stride=stride)
    nth = cpu_threads()
    bounds = S.even_split(batch.key_code, nth)
    stores = [S.store_batch(batch, bounds, s)[0] for s in range(nth)]
    res, wall = run_threads(lambda b: oracle.keydeps_batch(b, query_lo=0, query_hi=b.n_txn, query_stride=stride), stores)
    pairs = sum(r.queried_pairs for r in res)
    qmax = max(r.query_s for r in res)
    model, avail = cpu_info()
    return {
        "value": round(pairs / qmax, 1),
        "unit": "txn-key pairs/s",
        "cores": nth,
        "kind": "port",
        "cpu_model": model,
        "cpus_available": avail,
        "single_thread_value": round(o1.queried_pairs / o1.query_s, 1),
        "sample": (f"{label}: {nth} CommandStores (EvenSplit key ranges, one thread each) evaluate every {stride}th txn "
                   f"of their store ({pairs} (txn,key) queries, slowest store {qmax:.1f} s of CommandsForKey."
                   f"mapReduceActive O(prefix) scans + KeyDeps.Builder; snapshot builds and the cross-store "
                   f"PartialDeps.with fold excluded); single thread: every {stride}th txn of the whole batch "
                   f"({o1.queried_pairs} queries, {o1.query_s:.1f} s)"),
    }


def rangedeps_cpu_baseline(rb):
    """The C restatement of mapReduceRangesInternal (a linear walk of every range command per query, as the
    reference's TreeMap forEach): S threads over disjoint query ranges of a strided sample, plus one thread."""
    import oracle
    n = rb.n_txn
    stride = max(1, int(os.environ.get("ACC_CPU_STRIDE_RD", str(max(1, n // 120)))))
    kp = np.diff(rb.keys.key_off.astype(np.int64)) + np.diff(rb.rng_off.astype(np.int64))
    o1 = oracle.rangedeps_batch(rb, query_lo=0, query_hi=n, query_stride=stride)
    probes1 = int(kp[::stride].sum())
    nth = cpu_threads()
    # thread s evaluates the sampled txns s, s + nth, ... of the stride-spaced sample
    parts = [(s * stride, nth * stride) for s in range(nth)]
    res, wall = run_threads(lambda p: oracle.rangedeps_batch(rb, query_lo=p[0], query_hi=n, query_stride=p[1]), parts)
    probes = sum(int(kp[p0::st].sum()) for p0, st in parts)
    qmax = max(r.query_s for r in res)
    model, avail = cpu_info()
    return {
        "value": round(probes / qmax, 1),
        "unit": "key probes/s",
        "cores": nth,
        "kind": "port",
        "cpu_model": model,
        "cpus_available": avail,
        "single_thread_value": round(probes1 / o1.query_s, 1),
        "sample": (f"every {stride}th txn of the same config-4 batch split over {nth} threads ({probes} key/range probes, "
                   f"slowest thread {qmax:.1f} s of range-command scans + RangeDeps.Builder); single thread: "
                   f"{probes1} probes in {o1.query_s:.1f} s"),
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


DIAG_STEPS = 2


def timed_steps(args, world, dev, step):
    """W warmup steps; then (timing contexts) DIAG_STEPS untimed steps with every kernel bracketed by HIP events, for
    the per-kernel breakdown and the dominant kernel; then the K timed steps with events around the dominant kernel's
    launches only (each timed launch adds two event records to the stream, ~8 us a launch when every kernel is timed).
    step.diag = the breakdown's timing dict (None without a timing context)."""
    import torch
    import torch.distributed as dist
    for _ in range(args.warmup):
        step()
    step.diag = None
    if step.ctx.timing_enabled:
        step.ctx.timing_reset()
        for _ in range(DIAG_STEPS):
            step()
        torch.cuda.synchronize()
        step.diag = step.ctx.timing()
        main = {k: v for k, v in step.diag.items() if k not in SIDE_STREAM_TAGS} or step.diag
        step.ctx.timing_filter([max(main.items(), key=lambda kv: kv[1][0])[0]])
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
    if step.ctx.timing_enabled:
        step.live = step.ctx.timing()   # the dominant kernel's events over the timed region
        step.ctx.timing_filter(None)
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    return elapsed


class Step:
    def __init__(self, ctx, fn):
        self.ctx, self.fn, self.view = ctx, fn, None
        self.diag = self.live = None

    def __call__(self):
        self.view = self.fn()


def run_config2(args, world, rank, local, dev):
    import torch
    from accord_amd import _lib as L
    from accord_amd import workload as W
    from accord_amd.deps import Context

    c3 = args.config == "3"
    dist, permute = args.dist, not args.unpermuted
    seed = W.CONFIG_SEEDS[("3z" if dist == "zipf" else "3u") if c3 else "2"] + 0x1000 * rank
    n_txn = int((12_500_000 if c3 else 1_000_000) * args.scale)
    n_keys = int((1 << 24) * args.scale) if c3 else n_txn
    batch = W.keydeps_batch(n_txn, 8, max(1000, n_keys), seed, dist, 0.99, status_model="model", permute_keys=permute)
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in batch.arrays().items()}
    torch.cuda.synchronize()
    bi = L.BatchIn(batch.n_txn, L.ACC_MEM_DEVICE, batch.n_pairs,
                   L.TsCols(t["txn_msb"].data_ptr(), t["txn_lsb"].data_ptr(), t["txn_node"].data_ptr()),
                   L.TsCols(t["exe_msb"].data_ptr(), t["exe_lsb"].data_ptr(), t["exe_node"].data_ptr()),
                   t["status"].data_ptr(), t["key_off"].data_ptr(), t["key_code"].data_ptr())
    ctx = Context(local, timing=os.environ.get("ACC_BENCH_NOTIME") != "1")   # NOTIME: overhead probe only
    step = Step(ctx, lambda: ctx.keydeps_batch_raw(bi))
    elapsed = timed_steps(args, world, dev, step)
    view = step.view
    timing = step.diag
    kdesc = "zipf(0.99)" + ("" if permute else " unpermuted") if dist == "zipf" else "uniform"
    variant = ("" if dist == "zipf" else "u") + ("" if permute or dist != "zipf" else "np")
    b_in, b_out = keydeps_bytes(batch.n_txn, batch.n_pairs, view.total_keys, view.total_edges, view.total_deps)
    result = {
        "metric": "txn-key conflict pairs resolved/sec (node)",
        "value": round(batch.n_pairs * world * args.steps / elapsed, 1),
        "unit": "txn-key pairs/s",
        "dtype": "u32/u64 (integer)",
        "data": "synthetic (seeded SplitMix64, SURVEY.md §8(d) status model)",
        "config": {
            "workload": (f"config3 on one GPU: KeyDeps batch of 100M txn-key pairs (12.5M txns x 8 keys), {kdesc} "
                         "over 2^24 keys, p_write 0.5, uncommitted window 10k, one CommandStore snapshot") if c3 else
                        (f"config2: KeyDeps batch, 1M txns x 8 keys, {kdesc} over 1M keys, p_write 0.5, "
                         "uncommitted window 10k, per-GPU CommandStore snapshot"),
            "key_distribution": dist,
            "keys_permuted": permute if dist == "zipf" else None,
            "n_txn_per_gpu": batch.n_txn,
            "pairs_per_gpu": batch.n_pairs,
            "dep_edges_per_gpu": int(view.total_edges),
            "parallelism": f"keyspace shards x{world} (independent CommandStores)",
        },
        "dep_edges_per_s": round(int(view.total_edges) * world * args.steps / elapsed, 1),
        "roofline": roofline(b_in + b_out, step, args.steps, elapsed * 1000.0 / args.steps, args.config, variant,
                             profiled=args.scale == 1.0),
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        # config 3: the O(prefix) scans of the 5M-txn hot key make each sampled query cost ~10 ms: sparser sample
        result["cpu_baseline"] = (keydeps_cpu_baseline(batch, "config 3", "ACC_CPU_STRIDE3", 20_000) if c3 else
                                  keydeps_cpu_baseline(batch, "config 2"))
    if rank == 0 and world == 1 and not c3 and args.scale == 1.0 and os.environ.get("ACC_BENCH_CFK", "1") != "0":
        result["cfk_apply"] = cfk_apply_leg(local)
        # the same stream shape over zipf(0.99) keys (the hottest key ~835K pairs): the hot keys take acc_cfk_apply's
        # closed form (csrc/cfkdeps.hip, hot keys)
        result["cfk_apply_zipf"] = cfk_apply_leg(local, calls=2, dist="zipf")
        # a replica in steady state: 100K-txn PreAccept batches against a resident 1M-txn store
        result["cfk_steady"] = cfk_steady_leg(local)
        result["cfk_steady_zipf"] = cfk_steady_leg(local, dist="zipf")
    return ctx, timing, elapsed, result


def cfk_steady_leg(local, dist="uniform", n_init=1_000_000, batch=100_000, n_batches=5, top_n=10):
    """N4 in steady state (messages/PreAccept.java:107-138, local/CommandStore.java:280-345,
    local/CommandsForKey.java:652-706): a device store built from the first n_init txns of workload.cfk_update_stream
    (8 keys per txn over 1M keys), then n_batches batches of `batch` new txns (plus the final statuses that fall due,
    workload.cfk_stream_cuts). Each batch: MaxConflicts proposes every new txn's executeAt (acc_maxconflicts_get), the
    batch's executeAts merge into it (acc_maxconflicts_update), CommandsForKey.update with deps on the resident store
    (acc_cfk_apply_deps: key-major update + the txn-major view / missing[] indices), and the KeyDeps scan of the whole
    store in place (acc_cfk_view -> acc_keydeps_batch). Inputs resident in HBM. Pass 1 times each phase (wall clock,
    synchronised); pass 2 replays it on a fresh store with every kernel timed for the breakdown."""
    import torch
    from accord_amd import _lib as L
    from accord_amd import workload as W
    from accord_amd.deps import Context
    t0 = time.perf_counter()
    u = W.cfk_update_stream(n_init + batch * n_batches, 8, 1_000_000, dist=dist)
    cuts = W.cfk_stream_cuts(u, n_init, batch, n_batches)
    parts = [W.cfk_slice(u, 0, cuts[0])] + [W.cfk_slice(u, cuts[b], cuts[b + 1]) for b in range(n_batches)]
    qs = [W.preaccept_queries(p) for p in parts]
    t_gen = time.perf_counter() - t0
    dev = torch.device("cuda", local)
    keep = []

    def up(a):
        t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        keep.append(t)
        return t.data_ptr()

    ins = []
    for p, q in zip(parts, qs):
        P = {k: up(v) for k, v in p.items()}
        U = len(p["msb"])
        ui = L.CfkUpdates(L.ACC_MEM_DEVICE, U, len(p["key"]), len(p["dmsb"]), L.TsCols(P["msb"], P["lsb"], P["node"]),
                          L.TsCols(P["xmsb"], P["xlsb"], P["xnode"]), P["status"], P["flags"], P["key_off"], P["key"],
                          P["dep_off"], L.TsCols(P["dmsb"], P["dlsb"], P["dnode"]))
        z = up(np.zeros(U + 1, np.uint32))
        ci = L.ConflictsIn(L.ACC_MEM_DEVICE, U, 1, len(p["key"]), 0, L.TsCols(P["xmsb"], P["xlsb"], P["xnode"]),
                           P["key_off"], P["key"], z, z, z)
        Q = {k: up(v) for k, v in q.items()}
        nq = len(q["msb"])
        qi = L.PreacceptIn(L.ACC_MEM_DEVICE, nq, len(q["part_start"]), L.TsCols(Q["msb"], Q["lsb"], Q["node"]),
                           Q["is_range"], Q["part_off"], Q["part_start"], Q["part_end"])
        qo = L.PreacceptOut(L.ACC_MEM_DEVICE, up(np.zeros(nq, np.uint64)), up(np.zeros(nq, np.uint64)),
                            up(np.zeros(nq, np.int32)), up(np.zeros(nq, np.uint8)))
        ins.append((ui, ci, qi, qo))
    torch.cuda.synchronize()

    scan_stats = {}

    def run(timing):
        nonlocal scan_stats
        rows, tm = [], {}
        with Context(local, timing=timing) as c:
            lib = c._lib
            h, m = C.c_void_p(), C.c_void_p()
            c.check(lib.acc_cfk_create(c.handle, C.byref(h)))
            c.check(lib.acc_maxconflicts_create(c.handle, 1, C.byref(m)))
            try:
                ui, ci, _, _ = ins[0]
                c.check(lib.acc_maxconflicts_update(c.handle, m, C.byref(ci)))
                c.check(lib.acc_cfk_apply_deps(c.handle, h, C.byref(ui)))
                v, kv = L.BatchIn(), L.KeydepsView()
                c.check(lib.acc_cfk_view(c.handle, h, C.byref(v)))
                c.check(lib.acc_keydeps_batch(c.handle, C.byref(v), C.byref(kv)))   # warm the scan's buffers
                torch.cuda.synchronize()
                c.timing_reset()
                for ui, ci, qi, qo in ins[1:]:
                    t = [time.perf_counter()]
                    c.check(lib.acc_maxconflicts_get(c.handle, m, C.byref(qi), C.byref(qo)))
                    torch.cuda.synchronize(); t.append(time.perf_counter())
                    c.check(lib.acc_maxconflicts_update(c.handle, m, C.byref(ci)))
                    torch.cuda.synchronize(); t.append(time.perf_counter())
                    c.check(lib.acc_cfk_apply_deps(c.handle, h, C.byref(ui)))
                    torch.cuda.synchronize(); t.append(time.perf_counter())
                    st = c.stats()
                    c.check(lib.acc_cfk_view(c.handle, h, C.byref(v)))
                    c.check(lib.acc_keydeps_batch(c.handle, C.byref(v), C.byref(kv)))
                    torch.cuda.synchronize(); t.append(time.perf_counter())
                    d = [(t[i + 1] - t[i]) * 1e3 for i in range(4)]
                    scan_stats = {k: v for k, v in c.stats().items() if k.startswith("keydeps.")}
                    rows.append(dict(propose_ms=d[0], maxconflicts_update_ms=d[1], cfk_update_ms=d[2],
                                     cfk_apply_ms=st.get("cfk.apply_us", 0) / 1e3, view_ms=st.get("cfk.view_us", 0) / 1e3,
                                     keydeps_scan_ms=d[3], total_ms=sum(d), store_txns=int(v.n_txn),
                                     store_pairs=int(v.n_pairs), dep_edges=int(kv.total_edges)))
                if timing:
                    tm = c.timing()
            finally:
                lib.acc_maxconflicts_destroy(m)
                lib.acc_cfk_destroy(h)
        return rows, tm

    rows, _ = run(False)
    _, tm = run(True)
    nb = len(rows)
    mean = {k: round(sum(r[k] for r in rows) / nb, 3) for k in rows[0] if k.endswith("_ms")}
    top = sorted(tm.items(), key=lambda kv: -kv[1][0])[:top_n]
    return {"workload": f"workload.cfk_update_stream({(n_init + batch * n_batches) // 1000}K txns x 8 {dist} keys over "
                        f"1M keys): a {n_init // 1000}K-txn device store, then {n_batches} PreAccept batches of "
                        f"{batch // 1000}K new txns (MaxConflicts propose + merge, CommandsForKey.update with deps, "
                        "KeyDeps scan of the whole store in place)",
            "ms_per_batch": mean["total_ms"], **{k: v for k, v in mean.items() if k != "total_ms"},
            "batch_updates": [int(cuts[b + 1] - cuts[b]) for b in range(n_batches)],
            "final_store_txns": rows[-1]["store_txns"], "final_store_pairs": rows[-1]["store_pairs"],
            "final_dep_edges": rows[-1]["dep_edges"],
            "per_batch_total_ms": [round(r["total_ms"], 3) for r in rows],
            "per_batch_view_ms": [round(r["view_ms"], 3) for r in rows],
            "setup_gen_s": round(t_gen, 2), "last_scan_stats": scan_stats,
            "top_kernels_ms_per_batch": {k: round(x[0] / nb, 3) for k, x in top}}


def cfk_apply_leg(local, calls=3, dist="uniform"):
    """N4: a config-2-sized CommandsForKey update stream (workload.cfk_update_stream: 1M txns x 8
    uniform keys, ~2M updates / 16M (update, key) pairs / 63M deps, Accept then commit / stable / apply / invalidate,
    interleaved) applied by ONE acc_cfk_apply call to an empty key-major store, inputs resident in HBM; then
    acc_cfk_snap_to_batch of the result (the txn-major view acc_map_reduce_full reads). 1 warmup + `calls` timed calls
    on its own context."""
    import torch
    from accord_amd import _lib as L
    from accord_amd import workload as W
    from accord_amd.deps import Context, _view_as_snap
    t0 = time.perf_counter()
    u = W.cfk_update_stream(1_000_000, dist=dist)
    t_gen = time.perf_counter() - t0
    dev = torch.device("cuda", local)
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in u.items()}
    z64 = torch.zeros(1, dtype=torch.int64, device=dev)
    z32 = torch.zeros(1, dtype=torch.int32, device=dev)
    zp = z64.data_ptr()
    snap = L.CfkSnap(L.ACC_MEM_DEVICE, 0, 0, 0, zp, z32.data_ptr(), L.TsCols(zp, zp, zp), L.TsCols(zp, zp, zp), zp,
                     z32.data_ptr(), L.TsCols(zp, zp, zp))
    ptr = lambda k: d[k].data_ptr()  # noqa: E731
    ui = L.CfkUpdates(L.ACC_MEM_DEVICE, len(u["msb"]), len(u["key"]), len(u["dmsb"]),
                      L.TsCols(ptr("msb"), ptr("lsb"), ptr("node")), L.TsCols(ptr("xmsb"), ptr("xlsb"), ptr("xnode")),
                      ptr("status"), ptr("flags"), ptr("key_off"), ptr("key"), ptr("dep_off"),
                      L.TsCols(ptr("dmsb"), ptr("dlsb"), ptr("dnode")))
    torch.cuda.synchronize()
    with Context(local, timing=True) as c:
        v = L.CfkSnapView()
        c.check(c._lib.acc_cfk_apply(c.handle, C.byref(snap), C.byref(ui), C.byref(v)))
        c.timing_reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(calls):
            c.check(c._lib.acc_cfk_apply(c.handle, C.byref(snap), C.byref(ui), C.byref(v)))
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1000.0 / calls
        tm = c.timing()
        top = sorted(tm.items(), key=lambda kv: -kv[1][0])[:5]
        cst = c.stats()
        regrow = int(cst.get("cfk.apply_regrow", 0))
        out = L.CfkBatchView()
        si = _view_as_snap(v)
        c.check(c._lib.acc_cfk_snap_to_batch(c.handle, C.byref(si), C.byref(out)))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(calls):
            c.check(c._lib.acc_cfk_snap_to_batch(c.handle, C.byref(si), C.byref(out)))
        torch.cuda.synchronize()
        ms_b = (time.perf_counter() - t0) * 1000.0 / calls
        # the unified store's update (acc_cfk_apply_deps: the update, the txn-major view rebuilt, both kept in the
        # store), each call on a fresh empty store
        ms_s = []
        for _ in range(calls + 1):
            h = C.c_void_p()
            c.check(c._lib.acc_cfk_create(c.handle, C.byref(h)))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            c.check(c._lib.acc_cfk_apply_deps(c.handle, h, C.byref(ui)))
            torch.cuda.synchronize()
            ms_s.append((time.perf_counter() - t0) * 1000.0)
            c._lib.acc_cfk_destroy(h)
        n_upd, n_pairs, n_deps = len(u["msb"]), len(u["key"]), len(u["dmsb"])
        return {"workload": f"workload.cfk_update_stream(1M txns x 8 {dist} keys over 1M keys, deps = latest 16 txns "
                            "below on the key, final status at lag 64): one acc_cfk_apply to an empty store",
                "store_update_ms": round(sum(ms_s[1:]) / calls, 3),
                "hot_keys": int(cst.get("cfk.hot_keys", 0)), "hot_items": int(cst.get("cfk.hot_items", 0)),
                "updates": n_upd, "update_key_pairs": n_pairs, "deps": n_deps,
                "ms_per_call": round(ms, 3), "update_key_pairs_per_s": round(n_pairs / ms * 1e3, 1),
                "deps_per_s": round(n_deps / ms * 1e3, 1), "apply_regrow_rounds": regrow,
                "out_keys": int(v.n_keys), "out_entries": int(v.n_entries), "out_missing": int(v.n_missing),
                "snap_to_batch_ms": round(ms_b, 3), "setup_gen_s": round(t_gen, 2),
                "top_kernels_ms": {k: round(x[0] / calls, 3) for k, x in top}}


def run_config2_sharded(args, world, rank, local, dev):
    import torch
    from accord_amd import sharded as S
    from accord_amd import workload as W
    from accord_amd.deps import Context

    c3 = args.config == "3"   # config 3: 100M pairs in total over the N GPUs (strong scaling); else N x config 2
    n_global = int(12_500_000 * args.scale) if c3 else int(1_000_000 * args.scale) * world
    n_keys = int((1 << 24) * args.scale) if c3 else n_global
    # setup (untimed): each rank draws 1/N of the global batch's keys and receives its key range's (txn, key) pairs by
    # one all-to-all(v) (sharded.keydeps_store_batch: the same store batch as slicing the single-host generator's)
    import torch.distributed as dist
    t_gen = time.perf_counter()
    sub, g, bounds = S.keydeps_store_batch(n_global, 8, max(1000, n_keys), W.CONFIG_SEEDS["3z" if c3 else "2"], "zipf",
                                           world, rank, device=dev if dist.get_backend() == "nccl" else None)
    t_gen = time.perf_counter() - t_gen
    bi, keep = S.batch_in_device(sub, dev)
    gidx = torch.from_numpy(g.astype(np.int32)).to(dev)
    ctx = Context(local, timing=True)
    info = {}
    # the exchange behind the C ABI (what a JVM host calls): an acc_comm over RCCL (its 128-byte id broadcast once at
    # setup) and acc_shard_reduce = pack + one size exchange + one grouped all-to-all(v) + KeyDeps.with fold
    comm, exchange = None, "acc_comm (RCCL over xGMI) + acc_shard_reduce"
    try:
        if dist.get_backend() == "gloo":   # the one-GPU rehearsal: every rank on GPU 0, the host transport over gloo
            comm, exchange = S.Comm.host(ctx, world, rank), "acc_comm (host transport over gloo) + acc_shard_reduce"
        else:
            comm = S.Comm.rccl(ctx, world, rank)
    except Exception as e:  # noqa: BLE001 - recorded in the result line
        exchange = f"torch all_to_all_single + acc_shard_pack/merge (acc_comm unavailable: {e})"
    ctx.comm = comm   # closed before the context (main)

    def fn():
        v = ctx.keydeps_batch_raw(bi)
        if comm is not None:
            mv = S.shard_reduce(ctx, comm, bi, n_global, gidx)
            counts = None
        else:
            bufs, counts = S.shard_pack(ctx, bi, world, dev, gidx)
            torch.cuda.synchronize(dev)
            recv, rc = S.exchange_streams(bufs, counts)
            mv = S.shard_merge(ctx, recv, rc, world, rank, n_global)
        info["kd"], info["counts"], info["merge"] = v, counts, mv
        return v

    step = Step(ctx, fn)
    elapsed = timed_steps(args, world, dev, step)
    view = info["kd"]
    timing = step.diag
    b_in, b_out = keydeps_bytes(sub.n_txn, sub.n_pairs, view.total_keys, view.total_edges, view.total_deps)
    sent = info["counts"]
    sent_bytes = (int(ctx.stats().get("exchange.bytes_sent", 0)) if sent is None else
                  int(16 * sent[0].sum() + 8 * sent[1].sum() + 4 * sent[2].sum() + 4 * sent[3].sum()))
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
            "pairs_per_gpu_mean": round(float(tot[0].item()) / world, 1),
            "imbalance_max_over_mean": round(float(mx[0].item()) * world / float(tot[0].item()), 4) if tot[0].item() else None,
            "setup_store_batch_s": round(t_gen, 2),
            "parallelism": f"key-range shards x{world} (CommandStores) + all-to-all(v) reduce",
        },
        "exchange": {"bytes_sent_total": int(tot[1].item()), "bytes_sent_max_rank": int(mx[1].item()),
                     "path": exchange,
                     "setup_backend": dist.get_backend() + (" (RCCL over xGMI)" if dist.get_backend() == "nccl" else "")},
        "roofline": roofline(b_in + b_out, step, args.steps, elapsed * 1000.0 / args.steps, args.config, profiled=False),
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
    timing = step.diag
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
        "roofline": roofline(b_in + b_out, step, args.steps, elapsed * 1000.0 / args.steps, args.config,
                             profiled=args.scale == 1.0),
    }
    if os.environ.get("ACC_BENCH_MIXED", "1") != "0":
        result["keydeps_mixed"] = mixed_keydeps_leg(bi, local)
        result["partial_deps"] = partial_deps_leg(bi, local)
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = rangedeps_cpu_baseline(rb)
    return ctx, timing, elapsed, result


def run_config4_sharded(args, world, rank, local, dev):
    """Config 4 over N CommandStores (N > 1): the one config-4 mixed batch, EvenSplit over N key ranges; each rank
    holds its store's slice (range commands sliced to the store, impl/InMemoryCommandStore.java:739-761), and a step is
    the store's whole PartialDeps (acc_partial_deps_batch: KeyDeps of key and range txns + RangeDeps) and PreAccept.reduce
    across the stores (acc_partial_deps_reduce: one size exchange + one grouped all-to-all(v) over acc_comm, KeyDeps.with
    / RangeDeps.with / covering folds on the home rank; PreAccept.java:141-156, CommandStores.java:575-592). Strong
    scaling: value = the global batch's key probes / the slowest rank's step."""
    import torch
    import torch.distributed as dist
    from accord_amd import _lib as L
    from accord_amd import sharded as S
    from accord_amd import workload as W
    from accord_amd.deps import Context

    t_gen = time.perf_counter()
    rb = W.rangedeps_batch(int(20_000_000 * args.scale), W.CONFIG_SEEDS["4"])
    bounds = S.even_split(np.concatenate([rb.keys.key_code, rb.rng_start, rb.rng_end]).astype(np.uint64), world)
    sub, g = S.store_range_batch(rb, bounds, rank)
    lo, hi = S.store_ranges_bound(bounds, rank, rb.end_inclusive)
    cov = (np.array([lo], np.uint64), np.array([hi], np.uint64))
    n_global, probes_global = rb.n_txn, rb.keys.n_pairs + rb.n_ranges
    del rb
    t_gen = time.perf_counter() - t_gen
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in sub.arrays().items()}
    gidx = torch.from_numpy(g.astype(np.int32)).to(dev)
    torch.cuda.synchronize()
    P, R = sub.keys.n_pairs, sub.n_ranges
    bi = L.RangeBatchIn(sub.n_txn, L.ACC_MEM_DEVICE, P, R,
                        L.TsCols(t["txn_msb"].data_ptr(), t["txn_lsb"].data_ptr(), t["txn_node"].data_ptr()),
                        L.TsCols(t["exe_msb"].data_ptr(), t["exe_lsb"].data_ptr(), t["exe_node"].data_ptr()),
                        t["status"].data_ptr(), t["key_off"].data_ptr(), t["key_code"].data_ptr(),
                        t["rng_off"].data_ptr(), t["rng_start"].data_ptr(), t["rng_end"].data_ptr(),
                        int(sub.end_inclusive), 0)
    ctx = Context(local, timing=True)
    if dist.get_backend() == "gloo":   # the one-GPU rehearsal: every rank on GPU 0, the host transport over gloo
        comm, exchange = S.Comm.host(ctx, world, rank), "acc_comm (host transport over gloo) + acc_partial_deps_reduce"
    else:
        comm, exchange = S.Comm.rccl(ctx, world, rank), "acc_comm (RCCL over xGMI) + acc_partial_deps_reduce"
    ctx.comm = comm
    info = {}

    def fn():
        kv, rv = ctx.partial_deps_batch_raw(bi)
        info["kv"], info["rv"] = kv, rv
        info["red"] = S.partial_deps_reduce(ctx, comm, bi, n_global, gidx, covering=cov)
        return kv

    step = Step(ctx, fn)
    elapsed = timed_steps(args, world, dev, step)
    kv, rv = info["kv"], info["rv"]
    b_in, b_out = rangedeps_bytes(sub.n_txn, P, R, rv.total_ranges, rv.total_edges, rv.total_deps, rv.n_ranges)
    sent = int(ctx.stats().get("exchange.bytes_sent", 0))
    loc = torch.tensor([P + R, sent, int(kv.total_edges) + int(rv.total_edges)], dtype=torch.float64,
                       device=dev if dist.get_backend() == "nccl" else "cpu")
    tot, mx = loc.clone(), loc.clone()
    dist.all_reduce(tot)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    mean = float(tot[0].item()) / world
    result = {
        "metric": "PartialDeps key probes resolved/sec (node)",
        "value": round(probes_global * args.steps / elapsed, 1),
        "unit": "key probes/s",
        "dtype": "u32/u64 (integer)",
        "data": "synthetic (seeded SplitMix64, SURVEY.md §8(d) config 4)",
        "config": {
            "workload": f"config4 range-sharded: the mixed batch of {n_global} txns (10M range txns, 1 EndInclusive range "
                        f"each + 10M key txns x 4 keys) EvenSplit over {world} stores; per step each store's "
                        "acc_partial_deps_batch (KeyDeps + RangeDeps) and acc_partial_deps_reduce (KeyDeps.with, "
                        "RangeDeps.with and covering folds on the home rank)",
            "n_txn_global": n_global,
            "key_probes_global": probes_global,
            "key_probes_per_gpu_max": int(mx[0].item()),
            "key_probes_per_gpu_mean": round(mean, 1),
            "imbalance_max_over_mean": round(float(mx[0].item()) / mean, 4) if mean else None,
            "dep_entries_total": int(tot[2].item()),
            "setup_store_batch_s": round(t_gen, 2),
            "parallelism": f"key-range shards x{world} (CommandStores) + all-to-all(v) PartialDeps reduce",
        },
        "exchange": {"bytes_sent_total": int(tot[1].item()), "bytes_sent_max_rank": int(mx[1].item()), "path": exchange,
                     "setup_backend": dist.get_backend() + (" (RCCL over xGMI)" if dist.get_backend() == "nccl" else "")},
        "roofline": roofline(b_in + b_out, step, args.steps, elapsed * 1000.0 / args.steps, args.config, profiled=False),
    }
    return ctx, step.diag, elapsed, result


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
        top = sorted(tm.items(), key=lambda kv: -kv[1][0])[:16]
        return {"ms_per_call": round(ms, 3), "range_key_queries": int(c.stats().get("keydeps.range_key_queries", 0)),
                "dep_entries": int(v.total_edges), "kd_keys": int(v.total_keys),
                "top_kernels_ms": {k: round(x[0] / calls, 3) for k, x in top}}


def partial_deps_leg(bi, local, calls=3):
    """The whole PartialDeps of the same mixed batch as ONE timed step (acc_partial_deps_batch: the KeyDeps half of
    acc_keydeps_mixed and the RangeDeps half of acc_rangedeps_batch over one shared dictionary pass): 1 warmup +
    `calls` timed calls on its own context."""
    import torch
    from accord_amd.deps import Context
    with Context(local, timing=True) as c:
        c.partial_deps_batch_raw(bi)
        c.timing_reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(calls):
            kv, rv = c.partial_deps_batch_raw(bi)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1000.0 / calls
        tm = c.timing()
        top = sorted(tm.items(), key=lambda kv_: -kv_[1][0])[:8]
        return {"ms_per_step": round(ms, 3), "key_dep_entries": int(kv.total_edges), "range_dep_entries": int(rv.total_edges),
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


def merge_slice(m, g0, g1):
    """Groups [g0, g1) of an acc_merge_in dict as a standalone acc_merge_in dict (offsets rebased)."""
    r0, r1 = int(m["grp_off"][g0]), int(m["grp_off"][g1])
    ko0, ko1 = int(m["key_off"][r0]), int(m["key_off"][r1])
    vo0, vo1 = int(m["val_off"][r0]), int(m["val_off"][r1])
    oo0, oo1 = int(m["k2v_off"][r0]), int(m["k2v_off"][r1])
    return dict(grp_off=m["grp_off"][g0:g1 + 1] - np.uint64(r0), key_off=m["key_off"][r0:r1 + 1] - np.uint64(ko0),
                key_code=m["key_code"][ko0:ko1], val_off=m["val_off"][r0:r1 + 1] - np.uint64(vo0),
                txn_rank=m["txn_rank"][vo0:vo1], k2v_off=m["k2v_off"][r0:r1 + 1] - np.uint64(oo0), k2v=m["k2v"][oo0:oo1])


def merge_cpu_baseline(m, exec_rank, n_in):
    """The C restatement (LinearMerger fold of linearUnion per txn) over every coordinated txn of the same config-5
    batch, split over S threads (coordinators merge independently), then the levelisation walk on one thread (the
    reference's execution order is event-driven per store); unit = input entries merged/s. Plus the single-thread
    merge rate."""
    import oracle
    n = len(m["grp_off"]) - 1
    nth = cpu_threads()
    cuts = [n * s // nth for s in range(nth + 1)]
    parts = [merge_slice(m, cuts[s], cuts[s + 1]) for s in range(nth)]
    t_single0 = time.perf_counter()
    one = oracle.keydeps_merge(parts[0])
    t_single = time.perf_counter() - t_single0
    e_one = int(len(parts[0]["k2v"]) - len(parts[0]["key_code"]))
    res, wall = run_threads(oracle.keydeps_merge, parts)
    # the merged graph (deps of txn t = its merged TxnIds) for the levelisation walk
    vo = [np.diff(r["val_off"].astype(np.int64)) for r in res]
    val_off = np.zeros(n + 1, np.uint64)
    np.cumsum(np.concatenate(vo), out=val_off[1:])
    dep = np.concatenate([r["txn_rank"] for r in res])
    er = np.argsort(np.argsort(exec_rank, kind="stable"), kind="stable").astype(np.uint32)
    t2 = time.perf_counter()
    oracle.levelise(val_off, dep, er)
    t_lv = time.perf_counter() - t2
    entries = int(len(m["k2v"]) - len(m["key_code"]))
    model, avail = cpu_info()
    del one
    return {
        "value": round(entries / (wall + t_lv), 1),
        "unit": "input entries/s",
        "cores": nth,
        "kind": "port",
        "cpu_model": model,
        "cpus_available": avail,
        "single_thread_value": round(e_one / t_single, 1),
        "sample": (f"all {n} coordinated txns ({entries} reply entries): KeyDeps.merge split over {nth} threads "
                   f"{wall:.2f} s + levelise of the merged graph {t_lv:.3f} s (one thread); single thread: "
                   f"{cuts[1]} txns ({e_one} entries) in {t_single:.2f} s"),
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
    timing = step.diag
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
        "roofline": roofline(merge_bytes(m, view, n_txn, int(view.total_vals)), step, args.steps,
                             elapsed * 1000.0 / args.steps, args.config, profiled=args.scale == 1.0),
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
    ap.add_argument("--dist", default="zipf", choices=["zipf", "uniform"], help="key distribution (configs 2, 3)")
    ap.add_argument("--unpermuted", action="store_true", help="zipf hot keys at the low end of the key space")
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world, rank, local, dev = dist_setup(args)
    keyed = run_config2 if world == 1 else run_config2_sharded
    run = {"2": keyed, "3": keyed, "4": run_config4 if world == 1 else run_config4_sharded, "5": run_config5}[args.config]
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
        "scaling": "strong" if args.config in ("3", "4") and world > 1 else "weak",
        "vs_baseline": None,
    }
    out.update(result)
    out["path_stats"] = ctx.stats()
    if os.environ.get("ACC_BENCH_KERNELS") and timing:
        out["kernels_ms_per_step"] = {k: round(v[0] / DIAG_STEPS, 4) for k, v in
                                      sorted(timing.items(), key=lambda kv: -kv[1][0])}
    if getattr(ctx, "comm", None) is not None:
        ctx.comm.close()
    ctx.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
