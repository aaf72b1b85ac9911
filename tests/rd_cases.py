"""Shared RangeDeps test batches (CPU oracle tests and GPU parity tests)."""
import numpy as np

from accord_amd import workload as W


def build(txns, end_inclusive=1):
    """txns: list of dicts {kind, status, keys | ranges, bump (executeAt hlc offset, 0 = executeAt == txnId)}
    in TxnId order (hlc = index + 1). Returns a RangeBatch."""
    n = len(txns)
    i = np.arange(n, dtype=np.int64)
    isr = np.array([1 if "ranges" in t else 0 for t in txns], np.int64)
    kind = np.array([t.get("kind", W.WRITE) for t in txns], np.int64)
    t_msb, t_lsb, t_node = W.encode_ts(np.ones(n), i + 1, (kind << 1) | isr, 1 + (i % 8))
    bump = np.array([t.get("bump", 0) for t in txns], np.int64)
    e_msb, e_lsb, e_node = W.encode_ts(np.ones(n), i + 1 + bump, np.zeros(n), 1000 + (i % 1024))
    exe_msb = np.where(bump > 0, e_msb, t_msb).astype(np.uint64)
    exe_lsb = np.where(bump > 0, e_lsb, t_lsb).astype(np.uint64)
    exe_node = np.where(bump > 0, e_node, t_node).astype(np.int32)
    status = np.array([t.get("status", W.PREACCEPTED) for t in txns], np.uint8)
    keys = [np.array(sorted(t.get("keys", [])), np.uint64) for t in txns]
    ranges = [t.get("ranges", []) for t in txns]
    key_off = np.zeros(n + 1, np.uint32)
    np.cumsum([len(k) for k in keys], out=key_off[1:])
    rng_off = np.zeros(n + 1, np.uint32)
    np.cumsum([len(r) for r in ranges], out=rng_off[1:])
    kc = np.concatenate(keys) if n else np.zeros(0, np.uint64)
    rs = np.array([s for r in ranges for s, _ in r], np.uint64)
    re = np.array([e for r in ranges for _, e in r], np.uint64)
    kb = W.Batch(t_msb, t_lsb, t_node, exe_msb, exe_lsb, exe_node, status, key_off, kc.astype(np.uint64))
    return W.RangeBatch(kb, rng_off, rs, re, end_inclusive)


def handmade(end_inclusive=1):
    """Boundary keys, duplicate stored ranges, a range covering two keys of one txn, Accept-style range txn (p1),
    an erased range command, kind filters, multi-range txns."""
    R, K = W.READ, W.WRITE
    return build([
        dict(kind=K, ranges=[(10, 20)]),                                  # 0
        dict(kind=K, ranges=[(10, 20), (30, 40)]),                        # 1 same (10,20) as 0: one stored range
        dict(kind=R, ranges=[(15, 35)]),                                  # 2 a read: only writes witness it
        dict(kind=K, ranges=[(0, 100)], status=W.INVALID_OR_TRUNCATED),   # 3 erased range command
        dict(kind=K, keys=[10, 11, 20, 21, 30, 40]),                      # 4 boundary keys of 0/1/2
        dict(kind=R, keys=[12, 18]),                                      # 5 both keys in (10,20]: one entry per cmd
        dict(kind=K, ranges=[(5, 12)], bump=3),                           # 6 Accept-style: executeAt past txn 8
        dict(kind=K, ranges=[(11, 13)]),                                  # 7
        dict(kind=W.SYNC_POINT, ranges=[(0, 50)]),                        # 8
        dict(kind=W.EXCLUSIVE_SYNC_POINT, keys=[12]),                     # 9 ESP witnesses SyncPoints
        dict(kind=R, ranges=[(19, 31)], status=W.APPLIED),                # 10 range query over ranges
        dict(kind=K, keys=[15], status=W.INVALID_OR_TRUNCATED),           # 11 invalid key txn still queries
    ], end_inclusive)


def dense(seed, n=3000, end_inclusive=1, ranges_per_txn=2, key_bits=12, max_width_log2=8, p_range=0.5):
    return W.rangedeps_batch(n, seed, p_range=p_range, keys_per_txn=4, ranges_per_txn=ranges_per_txn, key_bits=key_bits,
                             max_width_log2=max_width_log2, window=n // 3, p_syncpoint=0.05,
                             end_inclusive=end_inclusive)


def global_tier(n_cmds=9000):
    """One key txn after n_cmds range commands that all cover it: a txn beyond the LDS tiers."""
    txns = [dict(kind=W.WRITE, ranges=[(i % 7, 1000 + (i % 13))]) for i in range(n_cmds)]
    txns += [dict(kind=W.WRITE, keys=[500, 501])]
    txns += [dict(kind=W.WRITE, ranges=[(400, 600)])]
    return build(txns)


def wide_codes(seed, n=2000):
    """u64 codes spanning the full range (split dictionary and class sorts), widths up to 2^62."""
    rng = np.random.RandomState(seed)
    txns = []
    for t in range(n):
        if rng.rand() < 0.5:
            s = int(rng.randint(0, 2**62, dtype=np.int64)) * 3
            w = 1 << int(rng.randint(0, 62))
            txns.append(dict(kind=int(rng.randint(0, 2)), ranges=[(s, min(s + w, 2**64 - 1))]))
        else:
            ks = sorted({int(rng.randint(0, 2**62, dtype=np.int64)) * 3 + int(rng.randint(0, 3)) for _ in range(3)})
            txns.append(dict(kind=int(rng.randint(0, 2)), keys=ks))
    return build(txns)
