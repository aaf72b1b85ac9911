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


def _ranges(rng, n_ranges, span, pool, p_pool=0.3):
    """n sorted, non-overlapping [s, e) ranges in [0, span); some drawn from a shared pool (repeated ranges)"""
    out = []
    for _ in range(n_ranges):
        if pool and rng.random() < p_pool:
            out.append(pool[int(rng.integers(0, len(pool)))])
        else:
            s = int(rng.integers(0, span - 2))
            out.append((s, s + int(rng.integers(1, 60))))
    out.sort()
    res = []
    for s, e in out:                  # deoverlap (Ranges.ofSortedAndDeoverlapped keeps them disjoint)
        if res and s < res[-1][1]:
            continue
        res.append((s, min(e, span)))
    return res


def range_recovery_case(seed, n_cmd=300, n_query=120, span=1000, p_hist=0.15, p_hist_only=0.08, end_inclusive=1,
                        p_deps=0.7, max_deps=8):
    """A store's range-command table (rangeCommands + historicalRangeCommands, InMemoryCommandStore.java:100-101) sorted
    by TxnId, each entry with a Status ordinal, flags (Erased, hasProposedOrDecidedDeps), executeAt (bumped for some),
    1-3 ranges and a PartialDeps as (TxnId, key | range) pairs; recovery queries over keys or ranges whose testTxnId is
    a table TxnId, a foreign TxnId that deps may name, or an executeAt (the executeAt boundary)."""
    rng = np.random.default_rng(seed)
    foreign_hlc = 2 * rng.integers(0, n_cmd + 2, size=40) + 1              # odd hlcs: not table TxnIds
    foreign = [tuple(int(x) for x in W.encode_ts(1, int(h), (int(rng.choice(KINDS)) << 1) | int(rng.integers(0, 2)),
                                                  1 + int(rng.integers(0, 4)))) for h in foreign_hlc]
    pool = [(int(s), int(s) + int(w)) for s, w in zip(rng.integers(0, span - 80, size=12), rng.integers(1, 70, size=12))]
    rows = []   # (msb, lsb, node, emsb, elsb, enode, status, flags, ranges, deps)
    ids = []
    for i in range(n_cmd):
        kind = int(rng.choice(KINDS, p=[0.4, 0.4, 0.1, 0.1]))
        m, l, nd = (int(x) for x in W.encode_ts(1, 2 * i + 2, (kind << 1) | 1, 1 + int(rng.integers(0, 4))))
        ids.append((m, l, nd))
    for i in range(n_cmd):
        m, l, nd = ids[i]
        status = int(rng.integers(0, 11))
        if rng.random() < 0.45:
            em, el, en = (int(x) for x in W.encode_ts(1, 2 * i + 2 + int(rng.integers(1, 40)), 0, 1 + int(rng.integers(0, 4))))
        else:
            em, el, en = m, l, nd
        flags = 0
        if rng.random() < 0.05:
            flags |= ACC_RCMD_ERASED
        if rng.random() < p_deps:
            flags |= ACC_RCMD_HAS_DEPS
        rs = _ranges(rng, int(rng.integers(1, 4)), span, pool, p_pool=0.6)
        deps = []
        for _ in range(int(rng.integers(0, max_deps + 1))):
            u = rng.random()
            if u < 0.5:                     # a neighbour (the txns a recovery may find witnessed or not)
                t = ids[min(n_cmd - 1, max(0, i + int(rng.integers(-5, 25))))]
            elif u < 0.8:
                t = ids[int(rng.integers(0, n_cmd))]
            else:
                t = foreign[int(rng.integers(0, len(foreign)))]
            if rng.random() < 0.5:          # a KeyDeps entry: a key inside one of the ranges, or anywhere
                if rng.random() < 0.7:
                    s, e = rs[int(rng.integers(0, len(rs)))]
                    k = int(rng.integers(s, e + 1))
                else:
                    k = int(rng.integers(0, span))
                deps.append((t, k, 0, 1))
            else:
                s = int(rng.integers(0, span - 2))
                deps.append((t, s, s + int(rng.integers(1, 50)), 0))
        deps.sort(key=lambda d: (d[0][0], d[0][1] >> 16, d[0][1] & 0x1E, d[0][2]))
        only_hist = rng.random() < p_hist_only
        rows.append((m, l, nd, em, el, en, status, flags | (ACC_RCMD_HISTORICAL if only_hist else 0), rs, deps))
        if not only_hist and rng.random() < p_hist:   # also in historicalRangeCommands
            rows.append((m, l, nd, m, l, nd, 0, ACC_RCMD_HISTORICAL, _ranges(rng, int(rng.integers(1, 3)), span, pool), []))
    cmds = dict(end_inclusive=end_inclusive)
    cols = list(zip(*[r[:8] for r in rows]))
    for k, dt, col in zip(("txn_msb", "txn_lsb", "txn_node", "exe_msb", "exe_lsb", "exe_node", "status", "flags"),
                          (np.uint64, np.uint64, np.int32, np.uint64, np.uint64, np.int32, np.uint8, np.uint8), cols):
        cmds[k] = np.array(col, dt)
    cmds["rng_off"] = np.concatenate([[0], np.cumsum([len(r[8]) for r in rows])]).astype(np.uint32)
    cmds["rng_start"] = np.array([s for r in rows for s, _ in r[8]], np.uint64)
    cmds["rng_end"] = np.array([e for r in rows for _, e in r[8]], np.uint64)
    cmds["dep_off"] = np.concatenate([[0], np.cumsum([len(r[9]) for r in rows])]).astype(np.uint32)
    dl = [d for r in rows for d in r[9]]
    cmds["dep_msb"] = np.array([d[0][0] for d in dl], np.uint64)
    cmds["dep_lsb"] = np.array([d[0][1] for d in dl], np.uint64)
    cmds["dep_node"] = np.array([d[0][2] for d in dl], np.int32)
    cmds["dep_start"] = np.array([d[1] for d in dl], np.uint64)
    cmds["dep_end"] = np.array([d[2] for d in dl], np.uint64)
    cmds["dep_is_key"] = np.array([d[3] for d in dl], np.uint8)

    qm, ql, qn, qr, qo, ps, pe = [], [], [], [], [0], [], []
    for _ in range(n_query):
        r = rng.random()
        own = None
        pairs = [(row, d) for row in rows if row[9] for d in row[9]] if r < 0.2 else []
        if pairs:                           # X named in some command's deps, over that command's ranges
            row, d = pairs[int(rng.integers(0, len(pairs)))]
            x, own = d[0], row[8]
        elif r < 0.5:                       # recovering a table txn, often over its own ranges
            i = int(rng.integers(0, n_cmd))
            x = ids[i]
            own = next(row[8] for row in rows if row[:3] == x) if rng.random() < 0.6 else None
        elif r < 0.85:
            x = foreign[int(rng.integers(0, len(foreign)))]
        else:
            j = int(rng.integers(0, len(rows)))
            x = (rows[j][3], rows[j][4], rows[j][5])   # an executeAt (a bumped one has kind Read)
        qm.append(x[0]); ql.append(x[1]); qn.append(x[2])
        if own is not None:
            qr.append(1); ps.extend(s_ for s_, _ in own); pe.extend(e_ for _, e_ in own)
        elif rng.random() < 0.5:
            ks = sorted(set(int(k) for k in rng.integers(0, span, size=int(rng.integers(1, 12)))))
            qr.append(0); ps.extend(ks); pe.extend([0] * len(ks))
        else:
            rr = _ranges(rng, int(rng.integers(1, 5)), span, pool, p_pool=0.5)
            qr.append(1); ps.extend(s for s, _ in rr); pe.extend(e for _, e in rr)
        qo.append(len(ps))
    queries = dict(msb=np.array(qm, np.uint64), lsb=np.array(ql, np.uint64), node=np.array(qn, np.int32),
                   is_range=np.array(qr, np.uint8), part_off=np.array(qo, np.uint32), part_start=np.array(ps, np.uint64),
                   part_end=np.array(pe, np.uint64))
    return cmds, queries


ACC_RCMD_ERASED, ACC_RCMD_HAS_DEPS, ACC_RCMD_HISTORICAL = 1, 2, 4


def range_recovery_handmade():
    """A four-entry table and one query whose four BeginRecovery-scan answers are worked out by hand from
    impl/InMemoryCommandStore.java:883-1016 (see tests/test_recovery_oracle.py). TxnIds on hlc 2, 4, 3 (historical),
    6; X = hlc 5, a Write over [0, 100); StartInclusive ranges."""
    def tid(h, kind=1, domain=1):
        return tuple(int(x) for x in W.encode_ts(1, h, (kind << 1) | domain, 1))
    t2, t3, t4, t6, x = tid(2), tid(3), tid(4), tid(6), tid(5, domain=0)
    e4 = tid(9, kind=0, domain=0)
    rows = [  # (txn, exe, status, flags, ranges, deps[(txn, start, end, is_key)])
        (t2, t2, 3, ACC_RCMD_HAS_DEPS, [(10, 20)], [(x, 15, 0, 1)]),
        (t3, t3, 0, ACC_RCMD_HISTORICAL, [(10, 20)], []),
        (t4, e4, 5, ACC_RCMD_HAS_DEPS, [(30, 40)], []),
        (t6, t6, 6, ACC_RCMD_HAS_DEPS, [(10, 20)], [(x, 0, 12, 0)]),
    ]
    cmds = dict(end_inclusive=0)
    for k, dt, f in (("txn_msb", np.uint64, lambda r: r[0][0]), ("txn_lsb", np.uint64, lambda r: r[0][1]),
                     ("txn_node", np.int32, lambda r: r[0][2]), ("exe_msb", np.uint64, lambda r: r[1][0]),
                     ("exe_lsb", np.uint64, lambda r: r[1][1]), ("exe_node", np.int32, lambda r: r[1][2]),
                     ("status", np.uint8, lambda r: r[2]), ("flags", np.uint8, lambda r: r[3])):
        cmds[k] = np.array([f(r) for r in rows], dt)
    cmds["rng_off"] = np.array([0, 1, 2, 3, 4], np.uint32)
    cmds["rng_start"] = np.array([r[4][0][0] for r in rows], np.uint64)
    cmds["rng_end"] = np.array([r[4][0][1] for r in rows], np.uint64)
    deps = [d for r in rows for d in r[5]]
    cmds["dep_off"] = np.concatenate([[0], np.cumsum([len(r[5]) for r in rows])]).astype(np.uint32)
    cmds["dep_msb"] = np.array([d[0][0] for d in deps], np.uint64)
    cmds["dep_lsb"] = np.array([d[0][1] for d in deps], np.uint64)
    cmds["dep_node"] = np.array([d[0][2] for d in deps], np.int32)
    cmds["dep_start"] = np.array([d[1] for d in deps], np.uint64)
    cmds["dep_end"] = np.array([d[2] for d in deps], np.uint64)
    cmds["dep_is_key"] = np.array([d[3] for d in deps], np.uint8)
    q = dict(msb=np.array([x[0]], np.uint64), lsb=np.array([x[1]], np.uint64), node=np.array([x[2]], np.int32),
             is_range=np.array([1], np.uint8), part_off=np.array([0, 1], np.uint32), part_start=np.array([0], np.uint64),
             part_end=np.array([100], np.uint64))
    # expected: {(start, end): [table index, ...]} per (started_at, test_dep, test_status, exec_after)
    expected = {
        (0, 1, 1, True): {(30, 40): [2]},                      # acceptedOrCommittedStartedBeforeWithoutWitnessing
        (1, 1, 1, False): {},                                  # hasAcceptedOrCommittedStartedAfterWithoutWitnessing
        (2, 0, 2, False): {(10, 20): [3]},                     # WITH over ranges: [0, 12) intersects [10, 20)
        (0, 0, 2, False): {},                                  # stableStartedBeforeAndWitnessed: none Stable before X
        (2, 1, 2, False): {},                                  # hasStableExecutesAfterWithoutWitnessing
        (2, 2, 0, False): {(10, 20): [0, 1, 3], (30, 40): [2]},   # ANY/ANY/ANY_STATUS: historical entry included
        (0, 2, 0, False): {(10, 20): [0, 1], (30, 40): [2]},   # STARTED_BEFORE, ANY_DEPS: txnId < X only
        (1, 2, 0, False): {(10, 20): [3]},
        (0, 0, 1, False): {},                                  # T2 witnessed X but executes before X: skipped
    }
    return cmds, q, expected


def rangedeps_as_dict(res, q):
    """one query of a rangedeps-layout result -> {(start, end): [dep table indices]}"""
    out = {}
    r0, r1 = int(res.rd_off[q]), int(res.rd_off[q + 1])
    a0 = int(res.arena_off[q])
    deps = res.dep_txn[int(res.u_off[q]):int(res.u_off[q + 1])]
    nr = r1 - r0
    prev = nr
    for i in range(nr):
        rid = int(res.range_id[r0 + i])
        end = int(res.arena[a0 + i])
        out[(int(res.rng_start[rid]), int(res.rng_end[rid]))] = [int(deps[int(res.arena[a0 + j])]) for j in range(prev, end)]
        prev = end
    return out
