"""Key-range sharding of the deps path across GPUs (one CommandStore per GPU), and the per-node reduce.

Accord splits a node's keyspace into CommandStores (local/ShardDistributor.java:106-156, EvenSplit); each
store computes `calculatePartialDeps` over its own keys and the per-store results are folded with
`PartialDeps.with` (PreAccept.reduce, messages/PreAccept.java:141-156). Here:

  1. every rank holds the whole batch's txn table (TxnIds are global) and keeps only the keys of its shard;
  2. the rank computes its shard's KeyDeps for every txn (acc_keydeps_batch on its GPU);
  3. per-txn fragments go to the txn's home rank (t mod world) with one all-to-allv (RCCL on GPUs,
     gloo on CPU) — the only data-path collective;
  4. the home rank unions its txns' fragments in shard order (acc_keydeps_merge): keys are disjoint across
     shards, so the union is the concatenation of keys with a union of TxnIds, exactly PartialDeps.with.

Dependency values travel as global batch indices; the batch must be in TxnId order (what a CommandStore
hands over) so that index order is TxnId order.
"""
from __future__ import annotations

import numpy as np

from .workload import Batch


def even_split(key_code: np.ndarray, world: int) -> np.ndarray:
    """EvenSplit of the observed key-code domain [min, max] into `world` contiguous shards: world+1 bounds
    (ShardDistributor.EvenSplit.split, local/ShardDistributor.java:106-156, with equal-width pieces)."""
    lo = int(key_code.min()) if len(key_code) else 0
    hi = int(key_code.max()) if len(key_code) else 0
    span = hi - lo + 1
    b = [lo + (span * s) // world for s in range(world)] + [hi + 1]
    return np.array(b, dtype=np.uint64)


def shard_batch(batch: Batch, bounds: np.ndarray, rank: int) -> Batch:
    """Same txns (global indices), key lists restricted to [bounds[rank], bounds[rank+1])."""
    lo, hi = np.uint64(bounds[rank]), np.uint64(bounds[rank + 1])
    kc = batch.key_code
    keep = (kc >= lo) & (kc < hi)
    counts = np.add.reduceat(keep.astype(np.int64), batch.key_off[:-1].astype(np.int64)) if len(kc) else \
        np.zeros(batch.n_txn, np.int64)
    # reduceat misbehaves on empty segments: fix them
    empty = np.diff(batch.key_off.astype(np.int64)) == 0
    counts[empty] = 0
    off = np.zeros(batch.n_txn + 1, dtype=np.uint32)
    np.cumsum(counts, out=off[1:])
    return Batch(batch.txn_msb, batch.txn_lsb, batch.txn_node, batch.exe_msb, batch.exe_lsb, batch.exe_node,
                 batch.status, off, kc[keep], dict(batch.meta, shard=rank))


def pack_fragments(res, local: Batch, world: int):
    """Per destination rank, one int64 stream of fragments [t, nk, nv, no, keys..., txnIds..., k2v...] for every
    txn with a non-empty shard result (KeyDeps.isEmpty fragments carry nothing: PartialDeps.with skips them)."""
    n = local.n_txn
    nk = np.diff(res.kd_off.astype(np.int64))
    na = np.diff(res.arena_off.astype(np.int64))
    nv = np.diff(res.u_off.astype(np.int64))
    ts = np.nonzero(na > nk)[0]
    streams = [[] for _ in range(world)]
    for t in ts:
        k0, k1 = int(res.kd_off[t]), int(res.kd_off[t + 1])
        keys = local.key_code[int(local.key_off[t]) + res.key_idx[k0:k1].astype(np.int64)].astype(np.int64)
        vals = res.dep_txn[int(res.u_off[t]):int(res.u_off[t + 1])].astype(np.int64)
        k2v = res.arena[int(res.arena_off[t]):int(res.arena_off[t + 1])].astype(np.int64)
        streams[int(t) % world].append(np.concatenate([[t, k1 - k0, len(vals), len(k2v)], keys, vals, k2v]))
    out = [np.concatenate(s) if s else np.zeros(0, np.int64) for s in streams]
    return out


def exchange(send: list, group=None, device=None):
    """all-to-allv of int64 streams (torch.distributed; nccl = RCCL over xGMI on MI355X, gloo on CPU)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = device or torch.device("cpu")
    counts = torch.tensor([len(s) for s in send], dtype=torch.int64, device=dev)
    recv_counts = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv_counts, counts, group=group)
    send_t = torch.from_numpy(np.concatenate(send) if send else np.zeros(0, np.int64)).to(dev)
    recv_t = torch.empty(int(recv_counts.sum().item()), dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv_t, send_t, output_split_sizes=recv_counts.tolist(),
                           input_split_sizes=counts.tolist(), group=group)
    return recv_t.cpu().numpy(), recv_counts.cpu().numpy()


def unpack_to_merge(recv: np.ndarray, recv_counts: np.ndarray, home_txns: np.ndarray) -> dict:
    """Fragments received from every source rank -> acc_merge_in with one group per home txn (ascending),
    its replies in source-rank (= shard) order, the order of PreAccept.reduce's fold."""
    frags = {}
    pos = 0
    for src, c in enumerate(recv_counts.tolist()):
        end = pos + c
        while pos < end:
            t, nk, nv, no = (int(x) for x in recv[pos:pos + 4])
            body = recv[pos + 4:pos + 4 + nk + nv + no]
            frags.setdefault(t, []).append((src, body[:nk], body[nk:nk + nv], body[nk + nv:]))
            pos += 4 + nk + nv + no
    grp_off, key_off, val_off, k2v_off = [0], [0], [0], [0]
    key_code, txn_rank, k2v = [], [], []
    for t in home_txns.tolist():
        for _, keys, vals, kv in sorted(frags.get(t, []), key=lambda f: f[0]):
            key_code.append(keys)
            txn_rank.append(vals)
            k2v.append(kv)
            key_off.append(key_off[-1] + len(keys))
            val_off.append(val_off[-1] + len(vals))
            k2v_off.append(k2v_off[-1] + len(kv))
        grp_off.append(len(key_off) - 1)
    cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)  # noqa: E731
    return dict(grp_off=np.array(grp_off, np.uint64), key_off=np.array(key_off, np.uint64),
                key_code=cat(key_code, np.uint64), val_off=np.array(val_off, np.uint64),
                txn_rank=cat(txn_rank, np.uint32), k2v_off=np.array(k2v_off, np.uint64), k2v=cat(k2v, np.int32))


def home_txns(n_txn: int, rank: int, world: int) -> np.ndarray:
    return np.arange(rank, n_txn, world, dtype=np.int64)


# ---------------------------------------------------------------- device path (acc_shard_pack / acc_shard_merge)
#
# The same reduce with every data-path step on the GPU: acc_shard_pack writes the fragment streams (destination-
# major) straight into torch device buffers, four all_to_all_single calls move them (RCCL over xGMI with the nccl
# backend; host copies with gloo), acc_shard_merge orders them by txn and runs the batched KeyDeps.merge.

STREAMS = (("hdr", 4, "int32"), ("keys", 1, "int64"), ("vals", 1, "int32"), ("k2v", 1, "int32"))


def batch_in_device(batch: Batch, dev):
    """acc_batch_in over torch device copies of a batch's columns (kept alive in the returned dict)."""
    import torch
    from . import _lib as L
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in batch.arrays().items()}
    bi = L.BatchIn(batch.n_txn, L.ACC_MEM_DEVICE, batch.n_pairs,
                   L.TsCols(t["txn_msb"].data_ptr(), t["txn_lsb"].data_ptr(), t["txn_node"].data_ptr()),
                   L.TsCols(t["exe_msb"].data_ptr(), t["exe_lsb"].data_ptr(), t["exe_node"].data_ptr()),
                   t["status"].data_ptr(), t["key_off"].data_ptr(), t["key_code"].data_ptr())
    return bi, t


def store_batch(batch: Batch, bounds: np.ndarray, rank: int):
    """The CommandStore's own batch: only the txns with at least one key in [bounds[rank], bounds[rank+1]), keys
    restricted to the shard, in TxnId order; plus each kept txn's global index (u32)."""
    local = shard_batch(batch, bounds, rank)
    cnt = np.diff(local.key_off.astype(np.int64))
    keep = np.nonzero(cnt > 0)[0]
    off = np.zeros(len(keep) + 1, dtype=np.uint32)
    np.cumsum(cnt[keep], out=off[1:])
    sub = Batch(batch.txn_msb[keep], batch.txn_lsb[keep], batch.txn_node[keep], batch.exe_msb[keep],
                batch.exe_lsb[keep], batch.exe_node[keep], batch.status[keep], off, local.key_code,
                dict(batch.meta, shard=rank, store_local=True))
    return sub, keep.astype(np.uint32)


def run_key_rows(gens):
    """Drive distinct_key_rows generators of consecutive slices in one process (the exchange is a prefix sum)."""
    nds = [next(g) for g in gens]
    out = [None] * len(gens)
    while True:
        total = sum(nds)
        before = np.concatenate([[0], np.cumsum(nds)[:-1]]).astype(np.int64).tolist()
        nxt = []
        for q, g in enumerate(gens):
            try:
                nxt.append(g.send((before[q], total)))
            except StopIteration as e:
                out[q] = e.value
                nxt.append(None)
        if total == 0:
            return out
        nds = nxt


def keydeps_store_batch(n_txn: int, keys_per_txn: int, n_keys: int, seed: int, key_dist: str, world: int, rank: int,
                        group=None, device=None, **kw):
    """This rank's CommandStore batch of W.keydeps_batch(n_txn, ...) split by EvenSplit over `world` stores, without
    any rank building the whole batch: rank r draws the keys of txns [r n / world, (r+1) n / world) (the duplicate
    redraws coordinated by an all-gather of per-rank counts, so the keys are bit-identical to the single-host
    generator's), the key-code bounds come from an all-reduce, each (txn, key) pair goes to its key's store in one
    all-to-all(v), and the store regenerates the TxnId / executeAt / status columns of its txns from their global
    indices. Returns (store batch, global txn indices u32, bounds) = store_batch(keydeps_batch(...), bounds, rank)."""
    import torch
    import torch.distributed as dist
    from . import workload as W
    dev = device or torch.device("cpu")
    lo, hi = n_txn * rank // world, n_txn * (rank + 1) // world
    sampler = W.key_sampler(seed, key_dist, n_keys, kw.get("zipf_s", 0.99), kw.get("permute_keys", True))
    gen = W.distinct_key_rows(n_txn, keys_per_txn, sampler, lo, hi)
    nd = next(gen)
    while True:
        t = torch.tensor([nd], dtype=torch.int64, device=dev)
        allc = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
        dist.all_gather(allc, t, group=group)
        c = [int(x.item()) for x in allc]
        try:
            nd = gen.send((sum(c[:rank]), sum(c)))
        except StopIteration as e:
            keys = e.value
            break
    kc = W.int_key_code(keys.reshape(-1))
    mm = torch.tensor([int(kc.min()) if len(kc) else (1 << 62), -(int(kc.max()) if len(kc) else 0)], dtype=torch.int64,
                      device=dev)
    dist.all_reduce(mm, op=dist.ReduceOp.MIN, group=group)
    kmin, kmax = int(mm[0].item()), -int(mm[1].item())
    span = kmax - kmin + 1
    bounds = np.array([kmin + (span * s) // world for s in range(world)] + [kmax + 1], dtype=np.uint64)
    txn = np.repeat(np.arange(lo, hi, dtype=np.int64), keys_per_txn)
    owner = np.searchsorted(bounds[1:-1], kc, side="right")
    order = np.argsort(owner, kind="stable")
    send_cnt = np.bincount(owner, minlength=world).astype(np.int64)
    payload = np.stack([txn[order], kc[order].astype(np.int64)], 1).reshape(-1)
    sc = torch.from_numpy(send_cnt * 2).to(dev)
    rc = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(rc, sc, group=group)
    recv = torch.empty(int(rc.sum().item()), dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv, torch.from_numpy(payload).to(dev), output_split_sizes=rc.tolist(),
                           input_split_sizes=sc.tolist(), group=group)
    r = recv.cpu().numpy().reshape(-1, 2)
    rt, rk = r[:, 0], r[:, 1].astype(np.uint64)   # source slices in rank order: txn order, keys sorted per txn
    g, cnt = np.unique(rt, return_counts=True)
    off = np.zeros(len(g) + 1, dtype=np.uint32)
    np.cumsum(cnt, out=off[1:])
    cols = W.keydeps_txn_columns(n_txn, g, seed, kw.get("status_model", "model"), kw.get("window", 10_000),
                                 kw.get("p_write", 0.5), kw.get("p_syncpoint", 0.0))
    sub = W.Batch(*cols, off, rk, dict(n_txn=n_txn, shard=rank, store_local=True))
    return sub, g.astype(np.uint32), bounds


def shard_pack(ctx, bi, world: int, dev, txn_global=None):
    """Fragments of the last acc_keydeps_batch on ctx for every home rank: (streams dict of torch tensors on dev,
    per-destination element counts [4, world] int64 numpy). txn_global: optional device u32/int32 tensor mapping
    the batch's txns to global indices (store-local batches)."""
    import ctypes as C
    import torch
    from . import _lib as L
    offs = [np.zeros(world + 1, np.uint64) for _ in range(4)]
    fs = L.FragStreams()
    fs.world, fs.mem = world, L.ACC_MEM_DEVICE
    fs.frag_off, fs.key_off, fs.val_off, fs.k2v_off = (o.ctypes.data for o in offs)
    fs.txn_global = txn_global.data_ptr() if txn_global is not None else None
    rc = ctx._lib.acc_shard_pack(ctx.handle, C.byref(bi), C.byref(fs))
    if rc != L.ACC_E_CAP:
        ctx.check(rc)
    need = [int(o[-1]) for o in offs]
    bufs = {}
    for (name, mult, dt), cnt in zip(STREAMS, need):
        bufs[name] = torch.empty(max(cnt * mult, 1), dtype=getattr(torch, dt), device=dev)
    fs.cap_frag, fs.cap_keys, fs.cap_vals, fs.cap_k2v = need
    fs.hdr, fs.keys, fs.vals, fs.k2v = (bufs[n].data_ptr() for n, _, _ in STREAMS)
    ctx.check(ctx._lib.acc_shard_pack(ctx.handle, C.byref(bi), C.byref(fs)))
    counts = np.stack([np.diff(o.astype(np.int64)) for o in offs])   # [stream, dest]
    for (name, mult, _), cnt in zip(STREAMS, need):
        bufs[name] = bufs[name][:cnt * mult]
    return bufs, counts


def exchange_streams(bufs: dict, counts: np.ndarray, group=None):
    """all-to-all(v) of the four fragment streams: returns (received streams in source order, received counts
    [4, world]). nccl (RCCL) moves device tensors directly; gloo goes through host copies."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    backend = dist.get_backend(group)
    dev = bufs["hdr"].device
    cdev = dev if backend == "nccl" else torch.device("cpu")
    send_c = torch.from_numpy(np.ascontiguousarray(counts.T.reshape(-1))).to(cdev)   # [dest, stream]
    recv_c = torch.empty_like(send_c)
    dist.all_to_all_single(recv_c, send_c, group=group)
    rc = recv_c.cpu().numpy().reshape(world, 4).T                                    # [stream, source]
    out = {}
    for q, (name, mult, dt) in enumerate(STREAMS):
        src = bufs[name] if backend == "nccl" else bufs[name].cpu()
        recv = torch.empty(int(rc[q].sum()) * mult, dtype=src.dtype, device=src.device)
        dist.all_to_all_single(recv, src, output_split_sizes=(rc[q] * mult).tolist(),
                               input_split_sizes=(counts[q] * mult).tolist(), group=group)
        out[name] = recv.to(dev)
    return out, rc


def shard_merge(ctx, recv: dict, rcounts: np.ndarray, world: int, rank: int, n_txn: int):
    """acc_shard_merge on received device streams; returns the merge view (device result on ctx)."""
    import ctypes as C
    import torch
    from . import _lib as L
    # all_to_all_single only orders torch's current stream after the collective; the library reads `recv` on its own
    # (non-blocking) stream, so wait for the collective to land before handing the buffers over
    dev = recv["hdr"].device
    if dev.type == "cuda":
        torch.cuda.current_stream(dev).synchronize()
    cnt = [np.ascontiguousarray(rcounts[q], dtype=np.uint64) for q in range(4)]
    fr = L.FragRecv(L.ACC_MEM_DEVICE, world, rank, n_txn, *(c.ctypes.data for c in cnt),
                    *(recv[n].data_ptr() if recv[n].numel() else 0 for n, _, _ in STREAMS))
    view = L.MergeView()
    ctx.check(ctx._lib.acc_shard_merge(ctx.handle, C.byref(fr), C.byref(view)))
    return view


def merged_to_host(ctx, view) -> dict:
    """Copy the last merge result on ctx (acc_merge_copy_out) to host arrays."""
    from .deps import merge_copy_out
    return merge_copy_out(ctx, view)


def home_result_from_full(res, batch: Batch, rank: int, world: int) -> dict:
    """The single-store KeyDeps of every home txn of `rank` in the acc_merge_view layout (for parity checks)."""
    ts = home_txns(batch.n_txn, rank, world)
    key_off, val_off, k2v_off = [0], [0], [0]
    keys, vals, k2v = [], [], []
    for t in ts.tolist():
        k, d, a = res.txn(t)
        kc = batch.key_code[int(batch.key_off[t]) + k.astype(np.int64)]
        keys.append(kc); vals.append(d); k2v.append(a)
        key_off.append(key_off[-1] + len(kc)); val_off.append(val_off[-1] + len(d)); k2v_off.append(k2v_off[-1] + len(a))
    cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)  # noqa: E731
    return dict(key_off=np.array(key_off, np.uint64), key_code=cat(keys, np.uint64), val_off=np.array(val_off, np.uint64),
                txn_rank=cat(vals, np.uint32), k2v_off=np.array(k2v_off, np.uint64), k2v=cat(k2v, np.int32))


# ---------------------------------------------------------------- range-sharded RangeDeps (range commands per store)
#
# A CommandStore keeps each range command's ranges sliced to its own ranges (InMemoryCommandStore's update hook:
# keysOrRanges.slice(ranges().allBetween(...), Minimal), impl/InMemoryCommandStore.java:739-761), so a range spanning
# two stores is two stored ranges; a query txn's RangeDeps from each store lists those pieces, and PreAccept.reduce
# folds the stores' PartialDeps with RangeDeps.with (= RelationMultiMap.linearUnion over Range::compare,
# primitives/RangeDeps.java:567-582) in store order. The same split is given to the oracle for parity.

def store_ranges_bound(bounds: np.ndarray, rank: int, end_inclusive: int):
    """The store's range over integer key codes, in the batch's Range bound type: keys [lo, hi) are
    (lo - 1, hi - 1] for Range.EndInclusive, [lo, hi) for Range.StartInclusive (Range.java:40-138)."""
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    return (lo - 1, hi - 1) if end_inclusive else (lo, hi)


def slice_ranges(start: np.ndarray, end: np.ndarray, slo: int, shi: int):
    """Ranges.slice(store, Minimal) of ranges against one store range of the same bound type: the intersections
    (max(start, slo), min(end, shi)) that are non-empty, in order. Returns (keep mask, new start, new end)."""
    s = np.maximum(start.astype(np.int64), slo)   # codes < 2^63
    e = np.minimum(end.astype(np.int64), shi)
    return s < e, s, e


def store_range_batch(rb, bounds: np.ndarray, rank: int):
    """The store's mixed batch: key txns with keys in the store (restricted to them), range txns whose ranges
    intersect the store (sliced to it), every other txn dropped; TxnId order kept. Returns (RangeBatch, global index
    u32 of each kept txn)."""
    from .workload import RangeBatch
    b = rb.keys
    n = b.n_txn
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    kc = b.key_code.astype(np.int64)
    kin = (kc >= lo) & (kc < hi)
    kown = np.repeat(np.arange(n), np.diff(b.key_off.astype(np.int64)))
    kcnt = np.bincount(kown[kin], minlength=n)
    slo, shi = store_ranges_bound(bounds, rank, rb.end_inclusive)
    rown = np.repeat(np.arange(n), np.diff(rb.rng_off.astype(np.int64)))
    rkeep, rs, re = slice_ranges(rb.rng_start, rb.rng_end, slo, shi)
    rcnt = np.bincount(rown[rkeep], minlength=n)
    keep = np.nonzero((kcnt > 0) | (rcnt > 0))[0]
    key_off = np.zeros(len(keep) + 1, np.uint32)
    np.cumsum(kcnt[keep], out=key_off[1:])
    rng_off = np.zeros(len(keep) + 1, np.uint32)
    np.cumsum(rcnt[keep], out=rng_off[1:])
    sel_k = kin & np.isin(kown, keep)
    sel_r = rkeep & np.isin(rown, keep)
    kb = Batch(b.txn_msb[keep], b.txn_lsb[keep], b.txn_node[keep], b.exe_msb[keep], b.exe_lsb[keep], b.exe_node[keep],
               b.status[keep], key_off, b.key_code[sel_k], dict(b.meta, store=rank))
    sub = RangeBatch(kb, rng_off, rs[sel_r].astype(np.uint64), re[sel_r].astype(np.uint64), rb.end_inclusive,
                     dict(rb.meta, store=rank))
    return sub, keep.astype(np.uint32)


def pack_range_fragments(res, gidx: np.ndarray, world: int):
    """Per destination rank one int64 stream of RangeDeps fragments [t, nr, nv, no, (start, end) x nr, txnIds...,
    rangesToTxnIds...] for every store txn with a non-empty RangeDeps (t and txnIds as global indices; empty
    fragments skipped as RangeDeps.with skips empties). `res` = per-store result in the acc_rangedeps_view layout."""
    n = len(gidx)
    nr = np.diff(res.rd_off.astype(np.int64))
    streams = [[] for _ in range(world)]
    for t in np.nonzero(nr > 0)[0].tolist():
        r, d, a = res.txn(t)
        g = int(gidx[t])
        se = np.stack([res.rng_start[r].astype(np.int64), res.rng_end[r].astype(np.int64)], 1).reshape(-1)
        streams[g % world].append(np.concatenate([[g, len(r), len(d), len(a)], se, gidx[d].astype(np.int64),
                                                  a.astype(np.int64)]))
    return [np.concatenate(s) if s else np.zeros(0, np.int64) for s in streams]


def unpack_range_merge(recv: np.ndarray, recv_counts: np.ndarray, home: np.ndarray, batch) -> dict:
    """Received RangeDeps fragments -> Deps.merge input (acc_rmm_in layout, raw TxnIds) with one group per home txn,
    its replies in source-rank (= store) order: the order of PreAccept.reduce's RangeDeps.with fold."""
    frags = {}
    pos = 0
    for src, c in enumerate(recv_counts.tolist()):
        end = pos + c
        while pos < end:
            t, nr, nv, no = (int(x) for x in recv[pos:pos + 4])
            body = recv[pos + 4:pos + 4 + 2 * nr + nv + no]
            frags.setdefault(t, []).append((src, body[:2 * nr], body[2 * nr:2 * nr + nv], body[2 * nr + nv:]))
            pos += 4 + 2 * nr + nv + no
    grp_off, key_off, val_off, k2v_off = [0], [0], [0], [0]
    ka, kb_, vals, k2v = [], [], [], []
    for t in home.tolist():
        for _, se, v, kv in sorted(frags.get(t, []), key=lambda f: f[0]):
            ka.append(se[0::2]); kb_.append(se[1::2]); vals.append(v); k2v.append(kv)
            key_off.append(key_off[-1] + len(se) // 2)
            val_off.append(val_off[-1] + len(v))
            k2v_off.append(k2v_off[-1] + len(kv))
        grp_off.append(len(key_off) - 1)
    cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)  # noqa: E731
    v = cat(vals, np.int64)
    kbk = batch.keys if hasattr(batch, "keys") else batch
    return dict(grp_off=np.array(grp_off, np.uint64),
                half=dict(key_off=np.array(key_off, np.uint64), key_a=cat(ka, np.uint64), key_b=cat(kb_, np.uint64),
                          val_off=np.array(val_off, np.uint64), msb=kbk.txn_msb[v].astype(np.uint64),
                          lsb=kbk.txn_lsb[v].astype(np.uint64), node=kbk.txn_node[v].astype(np.int32),
                          k2v_off=np.array(k2v_off, np.uint64), k2v=cat(k2v, np.int32)))


def range_reduce_local(rb, world: int, compute) -> dict:
    """All `world` stores in one process (oracle-side reference and single-GPU parity): per store `compute(store
    batch)` -> per-txn RangeDeps, fragments to every home rank, and per home rank the Deps.merge input. Returns
    {rank: merge input}."""
    bounds = even_split(np.concatenate([rb.keys.key_code, rb.rng_start, rb.rng_end]).astype(np.uint64), world)
    streams = [[] for _ in range(world)]
    for s in range(world):
        sub, gidx = store_range_batch(rb, bounds, s)
        out = pack_range_fragments(compute(sub), gidx, world)
        for d in range(world):
            streams[d].append(out[d])
    res = {}
    for d in range(world):
        recv = np.concatenate(streams[d]) if streams[d] else np.zeros(0, np.int64)
        counts = np.array([len(x) for x in streams[d]], np.int64)
        res[d] = unpack_range_merge(recv, counts, home_txns(rb.n_txn, d, world), rb)
    return res


# ---------------------------------------------------------------- acc_comm / acc_shard_reduce (exchange behind the ABI)

class Comm:
    """An acc_comm: RCCL (Comm.rccl: rank 0's acc_comm_unique_id shared through torch.distributed) or the host
    transport over a torch.distributed group (Comm.host: the library stages the streams in host memory and calls back
    for an all-to-all(v) of bytes; a JVM host would plug in its own messaging here)."""

    def __init__(self, ctx, handle, keep=None):
        self.ctx, self.handle, self._keep = ctx, handle, keep

    @classmethod
    def rccl(cls, ctx, world: int, rank: int, group=None):
        import ctypes as C
        import torch
        import torch.distributed as dist
        from . import _lib as L
        uid = np.zeros(L.ACC_COMM_ID_BYTES, np.uint8)
        if rank == 0:
            ctx.check(ctx._lib.acc_comm_unique_id(uid.ctypes.data))
        if world > 1:
            t = torch.from_numpy(uid.astype(np.int64))
            if dist.get_backend(group) == "nccl":   # the nccl (RCCL) backend moves device tensors only
                t = t.to(torch.device("cuda", torch.cuda.current_device()))
            dist.broadcast(t, 0, group=group)
            uid = t.cpu().numpy().astype(np.uint8)
        h = C.c_void_p()
        ctx.check(ctx._lib.acc_comm_init_rccl(ctx.handle, world, rank, uid.ctypes.data, C.byref(h)))
        return cls(ctx, h)

    @classmethod
    def host(cls, ctx, world: int, rank: int, group=None):
        import ctypes as C
        import torch
        import torch.distributed as dist
        from . import _lib as L

        def a2av(user, send, send_bytes, recv, recv_bytes):
            try:
                sb = [int(send_bytes[i]) for i in range(world)]
                rbytes = [int(recv_bytes[i]) for i in range(world)]
                src = np.ctypeslib.as_array((C.c_uint8 * max(sum(sb), 1)).from_address(send)) if sum(sb) else \
                    np.zeros(0, np.uint8)
                out = torch.empty(sum(rbytes), dtype=torch.uint8)
                dist.all_to_all_single(out, torch.from_numpy(src[:sum(sb)].copy()), output_split_sizes=rbytes,
                                       input_split_sizes=sb, group=group)
                if sum(rbytes):
                    C.memmove(recv, out.numpy().ctypes.data, sum(rbytes))
                return 0
            except Exception:  # noqa: BLE001 - reported to the library as a transport failure
                return 1

        fn = L.AllToAllvFn(a2av)
        h = C.c_void_p()
        ctx.check(ctx._lib.acc_comm_init_host(ctx.handle, world, rank, fn, None, C.byref(h)))
        return cls(ctx, h, keep=fn)

    def close(self):
        if self.handle:
            self.ctx._lib.acc_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def shard_reduce(ctx, comm: Comm, bi, n_global: int, txn_global=None):
    """acc_shard_reduce: PreAccept.reduce of the last acc_keydeps_batch on ctx (batch `bi`) over `comm`; returns the
    merge view of this rank's home txns. txn_global: u32 array (host or device, same placement as bi) or None."""
    import ctypes as C
    from . import _lib as L
    ptr = None
    if txn_global is not None:
        ptr = txn_global.data_ptr() if hasattr(txn_global, "data_ptr") else np.ascontiguousarray(txn_global).ctypes.data
    view = L.MergeView()
    ctx.check(ctx._lib.acc_shard_reduce(ctx.handle, comm.handle, C.byref(bi), ptr, n_global, C.byref(view)))
    return view


def _rlist(covering):
    """(start[], end[]) -> (acc_rlist, the arrays it points into)"""
    from . import _lib as L
    s = np.ascontiguousarray(covering[0], dtype=np.uint64)
    e = np.ascontiguousarray(covering[1], dtype=np.uint64)
    return L.RList(s.ctypes.data if len(s) else None, e.ctypes.data if len(e) else None, len(s), 0), (s, e)


def partial_deps_reduce(ctx, comm: Comm, rbi, n_global: int, txn_global=None, covering=None):
    """acc_partial_deps_reduce: PreAccept.reduce of both PartialDeps halves of the last acc_partial_deps_batch on ctx
    (mixed batch `rbi`, an acc_range_batch_in) over `comm`, one exchange; returns (KeyDeps merge view, Deps.merge view
    whose range half is the RangeDeps.with fold in store order), plus the PartialDeps.covering view when this store's
    `covering` ((start[], end[]): its Ranges) is given."""
    import ctypes as C
    from . import _lib as L
    ptr = None
    if txn_global is not None:
        ptr = txn_global.data_ptr() if hasattr(txn_global, "data_ptr") else np.ascontiguousarray(txn_global).ctypes.data
    kv, rv, cv = L.MergeView(), L.DepsMergeView(), L.CoveringView()
    rl, keep = _rlist(covering) if covering is not None else (None, None)
    ctx.check(ctx._lib.acc_partial_deps_reduce(ctx.handle, comm.handle, C.byref(rbi), ptr, n_global,
                                               C.byref(rl) if rl is not None else None, C.byref(kv), C.byref(rv),
                                               C.byref(cv) if rl is not None else None))
    return (kv, rv, cv) if covering is not None else (kv, rv)


def partial_deps_covering(ctx, rbi, covering):
    """acc_partial_deps_covering: the store's Ranges as every txn's PartialDeps.covering for the last
    acc_partial_deps_batch on ctx, with the PartialDeps constructor's invariant checks (PartialDeps.java:52-58)."""
    import ctypes as C
    rl, keep = _rlist(covering)
    ctx.check(ctx._lib.acc_partial_deps_covering(ctx.handle, C.byref(rbi), C.byref(rl)))


def covering_to_host(ctx, cv):
    """The covering view on the host: (cov_id[n_groups], store_mask[n_groups], list of (start[], end[]) per distinct
    covering)."""
    from . import _lib as L
    ng, nd = int(cv.n_groups), int(cv.n_coverings)
    cid = np.zeros(max(ng, 1), np.uint32)
    msk = np.zeros(max(ng, 1), np.uint64)
    off = np.zeros(nd + 1, np.uint64)
    for dst, src, nb in ((cid, cv.cov_id, 4 * ng), (msk, cv.store_mask, 8 * ng), (off, cv.cov_off, 8 * (nd + 1))):
        if nb:
            ctx.check(ctx._lib.acc_copy_out(ctx.handle, dst.ctypes.data, src, nb, L.ACC_MEM_HOST))
    tot = int(off[-1]) if nd else 0
    cs, ce = np.zeros(max(tot, 1), np.uint64), np.zeros(max(tot, 1), np.uint64)
    if tot:
        ctx.check(ctx._lib.acc_copy_out(ctx.handle, cs.ctypes.data, cv.cov_start, 8 * tot, L.ACC_MEM_HOST))
        ctx.check(ctx._lib.acc_copy_out(ctx.handle, ce.ctypes.data, cv.cov_end, 8 * tot, L.ACC_MEM_HOST))
    table = [(cs[int(off[i]):int(off[i + 1])].copy(), ce[int(off[i]):int(off[i + 1])].copy()) for i in range(nd)]
    return cid[:ng], msk[:ng], table
