"""Independent canonical model of the batch deps semantics — TEST INFRASTRUCTURE ONLY.

Written from the reference semantics as set definitions (dict of sorted sets), NOT as a port of the
loops, so it cross-checks the line-by-line C restatement in accord_oracle.c:

  * Timestamp order/identity: tuple (msb, lsb>>>16, lsb & 0x1E, node) (Timestamp.java:208-249).
  * deps of T on key k (CommandsForKey.mapReduceActive, CommandsForKey.java:614-650):
        { D on k : D.txnId < S, T.kind.witnesses(D.kind), D.status not in {TRANSITIVELY_KNOWN,
          INVALID_OR_TRUNCATED}, and (D not committed or M is None or D.executeAt >= M) } minus p1
    with S = T.executeAt, M = max executeAt of committed Writes on k with executeAt < S.
    (This set form is exact when committed executeAts on a key are distinct; the FAST-bisection tie
    quirk is exercised against the C restatement only.)
  * KeyDeps layout (KeyDeps.java:150-172): keys with >=1 dep, txnIds = sorted union, keysToTxnIds.
  * KeyDeps.merge == canonical union (KeyDepsTest.java:275-283).
Pure-Python loops: small inputs only.
"""
from __future__ import annotations

import numpy as np

WS = {1}
RS_OR_WS = {0, 1}
ANY_VISIBLE = {0, 1, 3, 4}
WITNESSES = {0: WS, 2: WS, 1: RS_OR_WS, 3: RS_OR_WS, 4: ANY_VISIBLE}  # Txn.java:221-236


def ts_key(msb, lsb, node):
    msb, lsb = int(msb), int(lsb)
    return (msb, lsb >> 16, lsb & 0x1E, int(node))


def kind_of(lsb) -> int:
    return (int(lsb) >> 1) & 7


def keydeps_batch(b, query_lo=0, query_hi=None):
    """Returns list per txn of (key_idx list, dep_txn list, keysToTxnIds list)."""
    n = b.n_txn
    tid = [ts_key(b.txn_msb[i], b.txn_lsb[i], b.txn_node[i]) for i in range(n)]
    tex = [ts_key(b.exe_msb[i], b.exe_lsb[i], b.exe_node[i]) for i in range(n)]
    kinds = [kind_of(b.txn_lsb[i]) for i in range(n)]
    status = [int(s) for s in b.status]
    by_key: dict[int, list[int]] = {}
    for t in range(n):
        for j in range(int(b.key_off[t]), int(b.key_off[t + 1])):
            by_key.setdefault(int(b.key_code[j]), []).append(t)
    committed = {4, 5, 6}
    out = []
    hi = n if query_hi is None else query_hi
    for t in range(n):
        if not (query_lo <= t < hi):
            out.append(([], [], []))
            continue
        S = tex[t]
        wk = WITNESSES[kinds[t]]
        p1 = None if tex[t] == tid[t] else t
        per_key = []
        keys = [int(x) for x in b.key_code[int(b.key_off[t]):int(b.key_off[t + 1])]]
        for ki, k in enumerate(keys):
            entries = by_key[k]
            cw = [tex[d] for d in entries if status[d] in committed and kinds[d] == 1 and tex[d] < S]
            M = max(cw) if cw else None
            deps = sorted((d for d in entries
                           if tid[d] < S and kinds[d] in wk and status[d] not in (0, 7)
                           and (status[d] not in committed or M is None or tex[d] >= M)
                           and d != p1), key=lambda d: tid[d])
            if deps:
                per_key.append((ki, deps))
        union = sorted({d for _, ds in per_key for d in ds}, key=lambda d: tid[d])
        pos = {d: i for i, d in enumerate(union)}
        k2v = []
        end = len(per_key)
        for _, ds in per_key:
            end += len(ds)
            k2v.append(end)
        for _, ds in per_key:
            k2v.extend(pos[d] for d in ds)
        out.append(([ki for ki, _ in per_key], union, k2v))
    return out


def to_canonical_map(keys, txnids, k2v):
    """KeyDeps arrays -> {key: [txnId...]} (the KeyDepsTest canonical TreeMap form)."""
    m = {}
    nk = len(keys)
    start = nk
    for i, k in enumerate(keys):
        end = k2v[i]
        m[k] = [txnids[x] for x in k2v[start:end]]
        start = end
    return m


def from_canonical_map(m):
    """{key: set(txn ranks)} -> (keys, txnIds, keysToTxnIds) in Java layout."""
    keys = sorted(m)
    vals = sorted({v for vs in m.values() for v in vs})
    pos = {v: i for i, v in enumerate(vals)}
    k2v = []
    end = len(keys)
    for k in keys:
        end += len(m[k])
        k2v.append(end)
    for k in keys:
        k2v.extend(pos[v] for v in sorted(m[k]))
    return keys, vals, k2v


def merge_union(replies):
    """KeyDeps.merge == canonical union of {key: set(txnIds)} (KeyDepsTest.java:275-283); values of the
    result are the union of every reply's txnIds array (RelationMultiMap.linearUnion :575-576)."""
    m: dict = {}
    allvals = set()
    for keys, vals, k2v in replies:
        if len(k2v) == len(keys):  # KeyDeps.isEmpty (KeyDeps.java:292-295)
            continue
        allvals.update(vals)
        for k, ts in to_canonical_map(keys, vals, k2v).items():
            m.setdefault(k, set()).update(ts)
    keys = sorted(m)
    vals = sorted(allvals)
    pos = {v: i for i, v in enumerate(vals)}
    k2v = []
    end = len(keys)
    for k in keys:
        end += len(m[k])
        k2v.append(end)
    for k in keys:
        k2v.extend(pos[v] for v in sorted(m[k]))
    return keys, vals, k2v


def levelise(off, dep, exec_rank):
    n = len(exec_rank)
    order_by_exec = sorted(range(n), key=lambda t: (exec_rank[t], t))
    level = [0] * n
    for t in order_by_exec:
        preds = [int(d) for d in dep[int(off[t]):int(off[t + 1])] if exec_rank[int(d)] < exec_rank[t]]
        level[t] = 1 + max(level[d] for d in preds) if preds else 0
    order = sorted(range(n), key=lambda t: (level[t], exec_rank[t], t))
    return np.array(level, dtype=np.uint32), np.array(order, dtype=np.uint32)


def rangedeps_batch(rb, query_lo=0, query_hi=None):
    """RangeDeps of a mixed key/range batch as set definitions (InMemoryCommandStore.mapReduceRangesInternal,
    InMemoryCommandStore.java:883-1016, under PreAccept.calculatePartialDeps, PreAccept.java:245-265):

        deps(T) = { (r, C) : C a range command (range-domain txn, status != INVALID_OR_TRUNCATED),
                    C.txnId < T.executeAt, T.kind.witnesses(C.kind), r in C.ranges, r intersects T's keys
                    (Range.contains) or T's ranges (start < that.end && end > that.start) } minus C == p1

    grouped as a RangeDeps map {Range: {TxnId}} in Java layout. Returns (dict_start, dict_end, per txn
    (range ids, dep txn list, rangesToTxnIds)), range ids indexing the sorted distinct stored ranges."""
    b = rb.keys
    n = b.n_txn
    tid = [ts_key(b.txn_msb[i], b.txn_lsb[i], b.txn_node[i]) for i in range(n)]
    tex = [ts_key(b.exe_msb[i], b.exe_lsb[i], b.exe_node[i]) for i in range(n)]
    kinds = [kind_of(b.txn_lsb[i]) for i in range(n)]
    is_range = [int(b.txn_lsb[i]) & 1 for i in range(n)]
    status = [int(s) for s in b.status]
    ranges = [[(int(rb.rng_start[j]), int(rb.rng_end[j])) for j in range(int(rb.rng_off[t]), int(rb.rng_off[t + 1]))]
              for t in range(n)]
    keys = [[int(x) for x in b.key_code[int(b.key_off[t]):int(b.key_off[t + 1])]] for t in range(n)]
    cmds = [c for c in range(n) if is_range[c] and status[c] != 7 and ranges[c]]
    dictionary = sorted({r for c in cmds for r in ranges[c]})
    rid = {r: i for i, r in enumerate(dictionary)}
    ei = int(rb.end_inclusive)

    def contains(r, k):
        s, e = r
        return (s < k <= e) if ei else (s <= k < e)

    out = []
    hi = n if query_hi is None else query_hi
    for t in range(n):
        if not (query_lo <= t < hi):
            out.append(([], [], []))
            continue
        wk = WITNESSES[kinds[t]]
        p1 = None if tex[t] == tid[t] else t
        m: dict = {}
        for c in cmds:
            if not (tid[c] < tex[t]) or kinds[c] not in wk or c == p1:
                continue
            for r in ranges[c]:
                if is_range[t]:
                    hit = any(r[0] < q[1] and r[1] > q[0] for q in ranges[t])
                else:
                    hit = any(contains(r, k) for k in keys[t])
                if hit:
                    m.setdefault(rid[r], set()).add(c)
        rids = sorted(m)
        union = sorted({c for cs in m.values() for c in cs}, key=lambda d: tid[d])
        pos = {d: i for i, d in enumerate(union)}
        k2v, end = [], len(rids)
        for r in rids:
            end += len(m[r])
            k2v.append(end)
        for r in rids:
            k2v.extend(pos[d] for d in sorted(m[r], key=lambda d: tid[d]))
        out.append((rids, union, k2v))
    return np.array([r[0] for r in dictionary], np.uint64), np.array([r[1] for r in dictionary], np.uint64), out


def keydeps_mixed(rb, query_lo=0, query_hi=None):
    """KeyDeps of a mixed key/range batch as set definitions. Key txns: as keydeps_batch. A range txn T is no
    CommandsForKey member (SafeCommandStore.updateCommandsForKey registers key txns only) and, as a query, covers
    every CFK key inside its ranges (InMemoryCommandStore.mapReduceForKey :274-289: subMap with the Range bound
    inclusivity), each key's deps being the same set as for a key txn. Returns per txn (key codes, dep txn list,
    keysToTxnIds)."""
    b = rb.keys
    n = b.n_txn
    tid = [ts_key(b.txn_msb[i], b.txn_lsb[i], b.txn_node[i]) for i in range(n)]
    tex = [ts_key(b.exe_msb[i], b.exe_lsb[i], b.exe_node[i]) for i in range(n)]
    kinds = [kind_of(b.txn_lsb[i]) for i in range(n)]
    status = [int(s) for s in b.status]
    by_key: dict[int, list[int]] = {}
    for t in range(n):
        for j in range(int(b.key_off[t]), int(b.key_off[t + 1])):
            by_key.setdefault(int(b.key_code[j]), []).append(t)
    cfk_keys = sorted(by_key)
    ei = int(rb.end_inclusive)
    committed = {4, 5, 6}
    out = []
    hi = n if query_hi is None else query_hi
    for t in range(n):
        if not (query_lo <= t < hi):
            out.append(([], [], []))
            continue
        S = tex[t]
        wk = WITNESSES[kinds[t]]
        p1 = None if tex[t] == tid[t] else t
        qkeys = [int(x) for x in b.key_code[int(b.key_off[t]):int(b.key_off[t + 1])]]
        for j in range(int(rb.rng_off[t]), int(rb.rng_off[t + 1])):
            s_, e_ = int(rb.rng_start[j]), int(rb.rng_end[j])
            qkeys += [k for k in cfk_keys if ((s_ < k <= e_) if ei else (s_ <= k < e_))]
        per_key = []
        for k in sorted(set(qkeys)):
            entries = by_key[k]
            cw = [tex[d] for d in entries if status[d] in committed and kinds[d] == 1 and tex[d] < S]
            M = max(cw) if cw else None
            deps = sorted((d for d in entries
                           if tid[d] < S and kinds[d] in wk and status[d] not in (0, 7)
                           and (status[d] not in committed or M is None or tex[d] >= M)
                           and d != p1), key=lambda d: tid[d])
            if deps:
                per_key.append((k, deps))
        union = sorted({d for _, ds in per_key for d in ds}, key=lambda d: tid[d])
        pos = {d: i for i, d in enumerate(union)}
        k2v, end = [], len(per_key)
        for _, ds in per_key:
            end += len(ds)
            k2v.append(end)
        for _, ds in per_key:
            k2v.extend(pos[d] for d in ds)
        out.append(([k for k, _ in per_key], union, k2v))
    return out


# Kind.witnessedBy() (Txn.java:247-262): EphemeralRead -> Nothing, Read -> WsOrSyncPoints, Write ->
# AnyGloballyVisible, SyncPoint / ExclusiveSyncPoint -> ExclusiveSyncPoints
WITNESSED_BY = {2: set(), 0: {1, 3, 4}, 1: {0, 1, 3, 4}, 3: {4}, 4: {4}}


def map_reduce_full(b, miss_off, miss_txn, queries, started_at, test_dep, test_status, test_kinds=None,
                    exec_after=False):
    """Recovery scans as sets (CommandsForKey.mapReduceFull, CommandsForKey.java:553-612): for query (X, keys) and key
    k, the txns D on k with
      * window: D < X (STARTED_BEFORE), D >= X (STARTED_AFTER, X itself included when it is on k), any (ANY); and when
        X is not on k and test_dep is WITH, nothing;
      * D.kind in X.kind.witnessedBy() (or the explicit mask);
      * status: ACCEPTED/COMMITTED (IS_PROPOSED), STABLE/APPLIED (IS_STABLE), not TRANSITIVELY_KNOWN (ANY_STATUS);
      * unless ANY_DEPS: D has info (ACCEPTED..APPLIED), D.executeAt > X, and (X not in D.missing on k) == WITH;
      * exec_after: D.executeAt > X.
    Returns per query (key_idx list, dep batch indices, keysToTxnIds) like keydeps_batch."""
    n = b.n_txn
    tid = [ts_key(b.txn_msb[i], b.txn_lsb[i], b.txn_node[i]) for i in range(n)]
    tex = [ts_key(b.exe_msb[i], b.exe_lsb[i], b.exe_node[i]) for i in range(n)]
    kinds = [kind_of(b.txn_lsb[i]) for i in range(n)]
    status = [int(s) for s in b.status]
    on_key: dict[int, dict[int, int]] = {}   # key -> {txn: pair index}
    for t in range(n):
        for j in range(int(b.key_off[t]), int(b.key_off[t + 1])):
            on_key.setdefault(int(b.key_code[j]), {})[t] = j
    out = []
    for q in range(len(queries["msb"])):
        X = ts_key(queries["msb"][q], queries["lsb"][q], queries["node"][q])
        mask = WITNESSED_BY[kind_of(queries["lsb"][q])] if test_kinds is None else \
            {k for k in range(8) if (test_kinds >> k) & 1}
        per_key = []
        keys = [int(x) for x in queries["key_code"][int(queries["key_off"][q]):int(queries["key_off"][q + 1])]]
        for ki, k in enumerate(keys):
            members = on_key.get(k, {})
            known = any(tid[d] == X for d in members)
            if not known and test_dep == 0:
                continue
            deps = []
            for d, j in members.items():
                if started_at == 0 and not tid[d] < X:
                    continue
                if started_at == 1 and not tid[d] >= X:
                    continue
                if kinds[d] not in mask:
                    continue
                s = status[d]
                if test_status == 1 and s not in (3, 4):
                    continue
                if test_status == 2 and s not in (5, 6):
                    continue
                if test_status == 0 and s == 0:
                    continue
                if test_dep != 2:
                    if s not in (3, 4, 5, 6) or not tex[d] > X:
                        continue
                    missing = {tid[int(m)] for m in miss_txn[int(miss_off[j]):int(miss_off[j + 1])]}
                    if (X not in missing) != (test_dep == 0):
                        continue
                if exec_after and not tex[d] > X:
                    continue
                deps.append(d)
            if deps:
                per_key.append((ki, sorted(deps, key=lambda d: tid[d])))
        union = sorted({d for _, ds in per_key for d in ds}, key=lambda d: tid[d])
        pos = {d: i for i, d in enumerate(union)}
        k2v, end = [], len(per_key)
        for _, ds in per_key:
            end += len(ds)
            k2v.append(end)
        for _, ds in per_key:
            k2v.extend(pos[d] for d in ds)
        out.append(([ki for ki, _ in per_key], union, k2v))
    return out
