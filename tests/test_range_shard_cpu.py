"""Range-sharded RangeDeps: every CommandStore keeps its range commands sliced to its own ranges
(impl/InMemoryCommandStore.java:739-761), computes its PartialDeps.rangeDeps, and the home rank folds the stores'
fragments with RangeDeps.with in store order (primitives/RangeDeps.java:567-582, PreAccept.reduce). CPU: the oracle
computes each store and the fold; the exchange runs over gloo with world size 2."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _batch(seed=0x77, n=3000, end_inclusive=1):
    from accord_amd import workload as W
    return W.rangedeps_batch(n, seed, p_range=0.5, keys_per_txn=3, ranges_per_txn=2, key_bits=16, max_width_log2=12,
                             window=400, end_inclusive=end_inclusive)


def _union(intervals):
    out = []
    for s, e in sorted(intervals):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return [tuple(x) for x in out]


def _per_dep_cover(key_a, key_b, lsb, k2v):
    """{dep TxnId lsb: union of its ranges} of one RangeDeps (rangesToTxnIds layout)."""
    nr = len(key_a)
    cov, start = {}, nr
    for i in range(nr):
        end = int(k2v[i])
        for x in k2v[start:end]:
            cov.setdefault(int(lsb[x]), []).append((int(key_a[i]), int(key_b[i])))
        start = end
    return {d: _union(v) for d, v in cov.items()}


def _merged(world, rb):
    import oracle
    from accord_amd import sharded as S
    per = S.range_reduce_local(rb, world, lambda sub: oracle.rangedeps_batch(sub))
    return {d: oracle.rmm_merge(m["grp_off"], m["half"], True) for d, m in per.items()}


@pytest.mark.parametrize("end_inclusive", [1, 0])
def test_one_store_equals_unsharded(end_inclusive):
    import oracle
    from accord_amd import sharded as S
    rb = _batch(end_inclusive=end_inclusive)
    full = oracle.rangedeps_batch(rb)
    merged = _merged(1, rb)[0]
    for t in S.home_txns(rb.n_txn, 0, 1).tolist():
        r, d, a = full.txn(t)
        ka, kb = int(merged["key_off"][t]), int(merged["key_off"][t + 1])
        va, vb = int(merged["val_off"][t]), int(merged["val_off"][t + 1])
        oa, ob = int(merged["k2v_off"][t]), int(merged["k2v_off"][t + 1])
        assert merged["key_a"][ka:kb].tolist() == full.rng_start[r].tolist(), t
        assert merged["key_b"][ka:kb].tolist() == full.rng_end[r].tolist(), t
        assert merged["lsb"][va:vb].tolist() == rb.keys.txn_lsb[d].tolist(), t
        assert merged["k2v"][oa:ob].tolist() == a.tolist(), t


def _pts(intervals, end_inclusive):
    """Key points of Range intervals as sorted disjoint half-open [a, b)."""
    d = 1 if end_inclusive else 0
    return _union([(s + d, e + d) for s, e in intervals])


def _inter(x, y):
    out, i, j = [], 0, 0
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if a < b:
            out.append((a, b))
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return out


@pytest.mark.parametrize("world", [2, 3])
def test_split_stores_cover_the_same_points(world):
    """Split stores list range pieces: every piece lies inside one store, each dep's pieces are inside its unsplit
    ranges, and they still cover every point of those ranges that the query txn itself touches."""
    import oracle
    from accord_amd import sharded as S
    rb = _batch()
    ei = rb.end_inclusive
    full = oracle.rangedeps_batch(rb)
    merged = _merged(world, rb)
    bounds = S.even_split(np.concatenate([rb.keys.key_code, rb.rng_start, rb.rng_end]).astype(np.uint64), world)
    stores = [S.store_ranges_bound(bounds, s, ei) for s in range(world)]
    b = rb.keys
    pieces = 0
    for dst, m in merged.items():
        for gi, t in enumerate(S.home_txns(rb.n_txn, dst, world).tolist()):
            if rb.rng_off[t + 1] > rb.rng_off[t]:
                q = _pts(zip(rb.rng_start[rb.rng_off[t]:rb.rng_off[t + 1]].tolist(),
                             rb.rng_end[rb.rng_off[t]:rb.rng_off[t + 1]].tolist()), ei)
            else:
                q = _union([(k, k + 1) for k in b.key_code[b.key_off[t]:b.key_off[t + 1]].tolist()])
            r, d, a = full.txn(t)
            want = _per_dep_cover(full.rng_start[r], full.rng_end[r], b.txn_lsb[d], a)
            ka, kb = int(m["key_off"][gi]), int(m["key_off"][gi + 1])
            va = int(m["val_off"][gi])
            oa, ob = int(m["k2v_off"][gi]), int(m["k2v_off"][gi + 1])
            got = _per_dep_cover(m["key_a"][ka:kb], m["key_b"][ka:kb], m["lsb"][va:], m["k2v"][oa:ob])
            assert set(got) <= set(want), (world, t)
            for dep, w in want.items():
                wp, gp = _pts(w, ei), _pts(got.get(dep, []), ei)
                assert _inter(gp, wp) == gp, (world, t, dep)           # pieces inside the unsplit ranges
                assert _inter(_inter(wp, q), gp) == _inter(wp, q), (world, t, dep)   # query points still covered
            for s_, e_ in zip(m["key_a"][ka:kb].tolist(), m["key_b"][ka:kb].tolist()):
                assert any(lo <= s_ and e_ <= hi for lo, hi in stores), (t, s_, e_)
            pieces += kb - ka
    assert pieces > 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, errq):
    sys.path[:0] = [os.path.join(ROOT, "cassandra-accord_amd"), os.path.join(ROOT, "oracle")]
    import torch.distributed as dist
    import oracle
    from accord_amd import sharded as S
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rb = _batch(seed=0x91)
        bounds = S.even_split(np.concatenate([rb.keys.key_code, rb.rng_start, rb.rng_end]).astype(np.uint64), world)
        sub, gidx = S.store_range_batch(rb, bounds, rank)
        recv, counts = S.exchange(S.pack_range_fragments(oracle.rangedeps_batch(sub), gidx, world))
        m = S.unpack_range_merge(recv, counts, S.home_txns(rb.n_txn, rank, world), rb)
        got = oracle.rmm_merge(m["grp_off"], m["half"], True)
        want = _merged(world, rb)[rank]
        for k in ("key_off", "key_a", "key_b", "val_off", "lsb", "msb", "node", "k2v_off", "k2v"):
            assert np.array_equal(got[k], want[k]), (rank, k)
        dist.barrier()
    except Exception as e:
        errq.put(f"rank {rank}: {e!r}")
        raise
    finally:
        dist.destroy_process_group()


def test_range_reduce_two_processes_gloo():
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
