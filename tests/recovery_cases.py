"""Seeded recovery-scan cases (CommandsForKey.mapReduceFull, local/CommandsForKey.java:553-612) — TEST INFRASTRUCTURE.

A CommandsForKey snapshot (acc_batch_in) with every InternalStatus and the durable kinds, executeAts bumped for the
statuses that carry info, a missing[] list per (txn, key) entry (TxnInfoWithMissing, :385-410: other members of that
key's CFK the txn's deps lack, sorted by TxnId), and BeginRecovery-style queries (messages/BeginRecovery.java:334-378):
the recovered txn X is a batch member (its own keys, plus keys it is not on), a foreign TxnId between batch TxnIds, or
a timestamp equal to some bumped executeAt (the "executeAt > X" boundary).
"""
from __future__ import annotations

import numpy as np

from accord_amd import workload as W

KINDS = np.array([0, 1, 3, 4])   # Read, Write, SyncPoint, ExclusiveSyncPoint


def recovery_case(seed, n=400, keys_per=3, n_keys=30, n_query=80, p_missing=0.3, permute=False, p_bump=0.4,
                  max_bump=40):
    rng = np.random.default_rng(seed)
    kind = rng.choice(KINDS, size=n, p=[0.4, 0.4, 0.1, 0.1]).astype(np.int64)
    hlc = 2 * np.arange(n, dtype=np.int64) + 2                     # batch TxnIds on even hlcs
    node = 1 + rng.integers(0, 4, size=n)
    t_msb, t_lsb, t_node = W.encode_ts(np.ones(n), hlc, kind << 1, node)
    status = rng.integers(0, 8, size=n).astype(np.uint8)
    has_info = (status >= 3) & (status <= 6)
    bump = has_info & (rng.random(n) < p_bump)
    e_hlc = hlc + rng.integers(1, max_bump, size=n)
    e_msb, e_lsb, e_node = W.encode_ts(np.ones(n), e_hlc, np.zeros(n, np.int64), 1 + rng.integers(0, 4, size=n))
    exe_msb = np.where(bump, e_msb, t_msb).astype(np.uint64)
    exe_lsb = np.where(bump, e_lsb, t_lsb).astype(np.uint64)
    exe_node = np.where(bump, e_node, t_node).astype(np.int32)
    keys = np.stack([np.sort(rng.choice(n_keys, size=keys_per, replace=False)) for _ in range(n)])
    key_off = (np.arange(n + 1) * keys_per).astype(np.uint32)
    key_code = (keys.reshape(-1) * 7 + 1000).astype(np.uint64)
    b = W.Batch(t_msb, t_lsb, t_node, exe_msb, exe_lsb, exe_node, status, key_off, key_code)
    if permute:
        b = b.permuted(rng.permutation(n))

    # missing[] per pair: other members of the key's CFK, sorted by TxnId
    order_key = [(int(b.txn_msb[t]), int(b.txn_lsb[t]) >> 16, int(b.txn_lsb[t]) & 0x1E, int(b.txn_node[t])) for t in range(n)]
    members: dict[int, list[int]] = {}
    for t in range(n):
        for j in range(int(b.key_off[t]), int(b.key_off[t + 1])):
            members.setdefault(int(b.key_code[j]), []).append(t)
    miss_off, miss = [0], []
    for t in range(n):
        for j in range(int(b.key_off[t]), int(b.key_off[t + 1])):
            cand = [d for d in members[int(b.key_code[j])] if d != t and rng.random() < p_missing]
            miss.extend(sorted(cand, key=lambda d: order_key[d]))
            miss_off.append(len(miss))

    # queries
    qm, ql, qn, qo, qk = [], [], [], [0], []
    all_codes = np.unique(b.key_code)
    for _ in range(n_query):
        r = rng.random()
        if r < 0.55:       # a batch member, its own keys plus maybe a key it is not on / one with no CFK
            t = int(rng.integers(0, n))
            m, l, nd = int(b.txn_msb[t]), int(b.txn_lsb[t]), int(b.txn_node[t])
            ks = set(int(x) for x in b.key_code[int(b.key_off[t]):int(b.key_off[t + 1])])
            if rng.random() < 0.4:
                ks.add(int(rng.choice(all_codes)))
            if rng.random() < 0.2:
                ks.add(999)
        elif r < 0.85:     # a foreign TxnId on an odd hlc
            k = int(rng.choice(KINDS))
            m, l, nd = (int(x) for x in W.encode_ts(1, 2 * int(rng.integers(0, n + 2)) + 1, k << 1, 1 + int(rng.integers(0, 4))))
            ks = set(int(x) for x in rng.choice(all_codes, size=int(rng.integers(1, 5)), replace=False))
        else:              # equal to some bumped executeAt (kind Read: flags 0)
            cand = np.nonzero((b.exe_msb != b.txn_msb) | (b.exe_lsb != b.txn_lsb) | (b.exe_node != b.txn_node))[0]
            t = int(rng.choice(cand)) if len(cand) else 0
            m, l, nd = int(b.exe_msb[t]), int(b.exe_lsb[t]), int(b.exe_node[t])
            ks = set(int(x) for x in rng.choice(all_codes, size=int(rng.integers(1, 5)), replace=False))
        qm.append(m); ql.append(l); qn.append(nd)
        qk.extend(sorted(ks))
        qo.append(len(qk))
    queries = dict(msb=np.array(qm, np.uint64), lsb=np.array(ql, np.uint64), node=np.array(qn, np.int32),
                   key_off=np.array(qo, np.uint32), key_code=np.array(qk, np.uint64))
    return b, np.array(miss_off, np.uint32), np.array(miss, np.uint32), queries


def canonical_rows(res, nq):
    """oracle / GPU result -> [(key_idx list, dep list, keysToTxnIds list)] per query"""
    out = []
    for q in range(nq):
        k = [int(x) for x in res.key_idx[int(res.kd_off[q]):int(res.kd_off[q + 1])]]
        d = [int(x) for x in res.dep_txn[int(res.u_off[q]):int(res.u_off[q + 1])]]
        a = [int(x) for x in res.arena[int(res.arena_off[q]):int(res.arena_off[q + 1])]]
        out.append((k, d, a))
    return out


# every combination the reference's enums allow, the four BeginRecovery scans among them
ALL_TESTS = [(sa, td, ts) for sa in (0, 1, 2) for td in (0, 1, 2) for ts in (0, 1, 2)]
