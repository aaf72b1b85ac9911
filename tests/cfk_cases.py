"""Seeded CommandsForKey update sequences with deps — TEST INFRASTRUCTURE.

Commands move through the InternalStatus lifecycle the way SafeCommandStore.updateCommandsForKey sees them
(local/SafeCommandStore.java:217-240; InternalStatus, local/CommandsForKey.java:194-203): PREACCEPTED (no info), then
ACCEPTED with proposed deps, COMMITTED / STABLE with decided deps and an executeAt that may be bumped, APPLIED, or
INVALID_OR_TRUNCATED; some ACCEPTED rounds repeat with a new ballot (acceptedOrCommitted changed). The deps of a command
on key k (its partialDeps().keyDeps.txnIds(k)) are other txns on k below its depsKnownBefore (TxnId for ACCEPTED,
executeAt once committed), including txns the store has not seen yet: CommandsForKey adds those as TRANSITIVELY_KNOWN
and records the ones it knows but the deps lack in missing[].
"""
from __future__ import annotations

import numpy as np

from accord_amd import workload as W

TK, HIST, PRE, ACC, COMMITTED, STABLE, APPLIED, INVALID = range(8)
KINDS = np.array([0, 1, 3, 4])   # Read, Write, SyncPoint, ExclusiveSyncPoint


def empty_snapshot():
    z = lambda dt: np.zeros(0, dt)  # noqa: E731
    return dict(key=z(np.uint64), ent_off=np.zeros(1, np.uint32), emsb=z(np.uint64), elsb=z(np.uint64),
                enode=z(np.int32), xmsb=z(np.uint64), xlsb=z(np.uint64), xnode=z(np.int32), status=z(np.uint8),
                miss_off=np.zeros(1, np.uint32), mmsb=z(np.uint64), mlsb=z(np.uint64), mnode=z(np.int32))


def _ts_key(m, l, n):
    return (m, l >> 16, l & 0x1E, n)


def cfk_case(seed, n_txn=200, n_keys=12, keys_per=3, p_dep=0.5, p_bump=0.5, p_invalid=0.05, p_reaccept=0.15,
             p_noop=0.03, window=40, p_accinv=0.1):
    """The updates in the CFK_UPD layout of oracle.py. Events of different txns interleave; each txn's
    own events stay in lifecycle order."""
    rng = np.random.default_rng(seed)
    kind = rng.choice(KINDS, size=n_txn, p=[0.35, 0.45, 0.1, 0.1])
    tid = [tuple(int(x) for x in W.encode_ts(1, 4 * i + 4, int(kind[i]) << 1, 1 + int(rng.integers(0, 4))))
           for i in range(n_txn)]
    keys = [np.sort(rng.choice(n_keys, size=min(keys_per, n_keys), replace=False)) * 10 + 100 for _ in range(n_txn)]
    on_key = {}
    for i in range(n_txn):
        for k in keys[i]:
            on_key.setdefault(int(k), []).append(i)
    # per txn: its lifecycle events (status, executeAt, ballot flag)
    life = []
    for i in range(n_txn):
        ev = [(PRE, tid[i], 0)]
        if rng.random() < p_invalid:
            ev.append((INVALID, tid[i], 0))
        else:
            ev.append((ACC, tid[i], 0))
            if rng.random() < p_accinv:
                # a recovery's Commands.acceptInvalidate (Commands.java:267-297): AcceptedInvalidateWithDefinition maps
                # to PREACCEPTED, below the CFK's ACCEPTED (flags bit 1: no stale check, no change), then a new Accept
                ev.append((PRE, tid[i], 2))
                ev.append((ACC, tid[i], 1))
            if rng.random() < p_reaccept:
                ev.append((ACC, tid[i], 1))
            ex = tid[i]
            if rng.random() < p_bump:
                ex = tuple(int(x) for x in W.encode_ts(1, 4 * i + 4 + 2 + 4 * int(rng.integers(0, 8)), 0,
                                                         1 + int(rng.integers(0, 4))))
            end = int(rng.integers(0, 4))
            ev.append((COMMITTED, ex, 0))
            if end >= 1:
                ev.append((STABLE, ex, 0))
            if end >= 2:
                ev.append((APPLIED, ex, 0))
        if rng.random() < p_noop:
            ev.insert(1, (0xFF, tid[i], 0))   # a save status with no InternalStatus
        if rng.random() < 0.1:
            ev = ev[1:]                         # first seen already ACCEPTED (or later)
        life.append(ev)
    # interleave: txns start roughly in TxnId order, events spread over a window
    events = []
    for i in range(n_txn):
        t = float(i)
        for e in life[i]:
            t += rng.exponential(window / 4)
            events.append((t, i, e))
    events.sort(key=lambda x: x[0])
    cols = {k: [] for k in ("msb", "lsb", "node", "xmsb", "xlsb", "xnode", "status", "flags")}
    key_off, key_list, dep_off, dm, dl, dn = [0], [], [0], [], [], []
    for _, i, (st, ex, fl) in events:
        m, l, n = tid[i]
        cols["msb"].append(m); cols["lsb"].append(l); cols["node"].append(n)
        cols["xmsb"].append(ex[0]); cols["xlsb"].append(ex[1]); cols["xnode"].append(ex[2])
        cols["status"].append(st); cols["flags"].append(fl)
        dkb = _ts_key(*tid[i]) if st in (PRE, ACC, 0xFF) or ex == tid[i] else _ts_key(*ex)
        for k in keys[i]:
            key_list.append(int(k))
            if st in (ACC, COMMITTED, STABLE, APPLIED):
                cand = [j for j in on_key[int(k)] if j != i and _ts_key(*tid[j]) < dkb]
                near = [j for j in cand if j >= i - window]
                pick = [j for j in near if rng.random() < p_dep]
                for j in sorted(pick, key=lambda j: _ts_key(*tid[j])):
                    dm.append(tid[j][0]); dl.append(tid[j][1]); dn.append(tid[j][2])
            dep_off.append(len(dm))
        key_off.append(len(key_list))
    upd = {k: np.array(v, dt) for (k, v), dt in zip(cols.items(), (np.uint64, np.uint64, np.int32, np.uint64, np.uint64,
                                                                  np.int32, np.uint8, np.uint8))}
    upd.update(key_off=np.array(key_off, np.uint32), key=np.array(key_list, np.uint64),
               dep_off=np.array(dep_off, np.uint32), dmsb=np.array(dm, np.uint64), dlsb=np.array(dl, np.uint64),
               dnode=np.array(dn, np.int32))
    return upd


def split_updates(upd, at):
    """(first `at` updates, the rest) in the CFK_UPD layout"""
    ko, do = upd["key_off"].astype(np.int64), upd["dep_off"].astype(np.int64)
    def part(a, b):
        out = {k: upd[k][a:b] for k in ("msb", "lsb", "node", "xmsb", "xlsb", "xnode", "status", "flags")}
        out["key_off"] = (ko[a:b + 1] - ko[a]).astype(np.uint32)
        out["key"] = upd["key"][ko[a]:ko[b]]
        out["dep_off"] = (do[ko[a]:ko[b] + 1] - do[ko[a]]).astype(np.uint32)
        for f in ("dmsb", "dlsb", "dnode"):
            out[f] = upd[f][do[ko[a]]:do[ko[b]]]
        return out
    n = len(upd["msb"])
    return part(0, at), part(at, n)


def handmade():
    """Three Writes A < B < C on one key, worked through CommandsForKey.java:657-1149 by hand:
      1. B PREACCEPTED                         -> [B PRE]
      2. C ACCEPTED, deps [A] (A unknown)      -> [A TK, B PRE, C ACC missing [B]]   (A added, B missing from C's deps)
      3. A COMMITTED, no deps                  -> [A COMMITTED, B PRE, C ACC [B]]
      4. B ACCEPTED, deps [A]                  -> [A COMMITTED, B ACC, C ACC [B]]
      5. B COMMITTED                           -> [A COMMITTED, B COMMITTED, C ACC]   (removeMissing(B))
    Returns (updates, [(n_updates applied, expected [(hlc, status, [missing hlcs])])])."""
    ts = {h: tuple(int(x) for x in W.encode_ts(1, h, 1 << 1, 1)) for h in (4, 8, 12)}
    steps = [(8, PRE, []), (12, ACC, [4]), (4, COMMITTED, []), (8, ACC, [4]), (8, COMMITTED, [4])]
    cols = {k: [] for k in ("msb", "lsb", "node", "xmsb", "xlsb", "xnode", "status", "flags")}
    key_off, keys, dep_off, dm, dl, dn = [0], [], [0], [], [], []
    for h, st, deps in steps:
        m, l, n = ts[h]
        for k, v in zip(("msb", "lsb", "node", "xmsb", "xlsb", "xnode", "status", "flags"), (m, l, n, m, l, n, st, 0)):
            cols[k].append(v)
        keys.append(500)
        key_off.append(len(keys))
        for d in deps:
            dm.append(ts[d][0]); dl.append(ts[d][1]); dn.append(ts[d][2])
        dep_off.append(len(dm))
    upd = {k: np.array(v, dt) for (k, v), dt in zip(cols.items(), (np.uint64, np.uint64, np.int32, np.uint64, np.uint64,
                                                                  np.int32, np.uint8, np.uint8))}
    upd.update(key_off=np.array(key_off, np.uint32), key=np.array(keys, np.uint64), dep_off=np.array(dep_off, np.uint32),
               dmsb=np.array(dm, np.uint64), dlsb=np.array(dl, np.uint64), dnode=np.array(dn, np.int32))
    expect = [
        (1, [(8, PRE, [])]),
        (2, [(4, TK, []), (8, PRE, []), (12, ACC, [8])]),
        (3, [(4, COMMITTED, []), (8, PRE, []), (12, ACC, [8])]),
        (4, [(4, COMMITTED, []), (8, ACC, []), (12, ACC, [8])]),
        (5, [(4, COMMITTED, []), (8, COMMITTED, []), (12, ACC, [])]),
    ]
    return upd, expect


def describe(snap):
    """key-major snapshot -> [(hlc, status, [missing hlcs])] of its single key"""
    out = []
    for e in range(int(snap["ent_off"][-1])):
        a, b = int(snap["miss_off"][e]), int(snap["miss_off"][e + 1])
        out.append((int(snap["elsb"][e]) >> 16, int(snap["status"][e]), [int(x) >> 16 for x in snap["mlsb"][a:b]]))
    return out


def conflicts_case(seed, n_upd=500, n_query=300, span=4000, p_range=0.3, end_inclusive=1):
    """MaxConflicts updates (executeAt + keys or ranges; distinct executeAts, some bumped past later TxnIds) and
    PreAccept queries (a TxnId + keys or ranges): TxnIds on even hlcs, queries spread so both fast-path outcomes
    occur."""
    rng = np.random.default_rng(seed)
    upd = dict(end_inclusive=end_inclusive)
    xm, xl, xn, ko, keys, ro, rs, re_ = [], [], [], [0], [], [0], [], []
    for i in range(n_upd):
        m, l, n = (int(x) for x in W.encode_ts(1, 2 * int(rng.integers(0, 3 * n_upd)) + 1, 0, 1 + i % 1000))
        xm.append(m); xl.append(l); xn.append(n)
        if rng.random() < p_range:
            pts = sorted(set(int(x) for x in rng.integers(0, span, size=2 * int(rng.integers(1, 3)))))
            prs = [(pts[j], pts[j + 1]) for j in range(0, len(pts) - 1, 2)]
            rs.extend(a for a, _ in prs); re_.extend(b for _, b in prs)
        else:
            keys.extend(sorted(set(int(x) for x in rng.integers(0, span, size=int(rng.integers(1, 6))))))
        ko.append(len(keys)); ro.append(len(rs))
    upd.update(xmsb=np.array(xm, np.uint64), xlsb=np.array(xl, np.uint64), xnode=np.array(xn, np.int32),
               key_off=np.array(ko, np.uint32), key=np.array(keys, np.uint64), rng_off=np.array(ro, np.uint32),
               rng_start=np.array(rs, np.uint64), rng_end=np.array(re_, np.uint64))
    qm, ql, qn, qr, qo, ps, pe = [], [], [], [], [0], [], []
    for _ in range(n_query):
        h = 2 * int(rng.integers(0, 3 * n_upd)) if rng.random() < 0.7 else 2 * int(rng.integers(3 * n_upd, 4 * n_upd))
        m, l, n = (int(x) for x in W.encode_ts(1, h, int(rng.choice(KINDS)) << 1, 1 + int(rng.integers(0, 4))))
        qm.append(m); ql.append(l); qn.append(n)
        if rng.random() < 0.4:
            pts = sorted(set(int(x) for x in rng.integers(0, span, size=2 * int(rng.integers(1, 3)))))
            prs = [(pts[j], pts[j + 1]) for j in range(0, len(pts) - 1, 2)]
            qr.append(1); ps.extend(a for a, _ in prs); pe.extend(b for _, b in prs)
        else:
            ks = sorted(set(int(x) for x in rng.integers(0, span, size=int(rng.integers(1, 8)))))
            qr.append(0); ps.extend(ks); pe.extend([0] * len(ks))
        qo.append(len(ps))
    q = dict(msb=np.array(qm, np.uint64), lsb=np.array(ql, np.uint64), node=np.array(qn, np.int32),
             is_range=np.array(qr, np.uint8), part_off=np.array(qo, np.uint32), part_start=np.array(ps, np.uint64),
             part_end=np.array(pe, np.uint64))
    return upd, q


def conflicts_slice(upd, a, b):
    """updates [a, b) of a conflicts_case update list, same layout"""
    ko, ro = upd["key_off"].astype(np.int64), upd["rng_off"].astype(np.int64)
    return dict(end_inclusive=upd["end_inclusive"], xmsb=upd["xmsb"][a:b], xlsb=upd["xlsb"][a:b], xnode=upd["xnode"][a:b],
                key_off=(ko[a:b + 1] - ko[a]).astype(np.uint32), key=upd["key"][ko[a]:ko[b]],
                rng_off=(ro[a:b + 1] - ro[a]).astype(np.uint32), rng_start=upd["rng_start"][ro[a]:ro[b]],
                rng_end=upd["rng_end"][ro[a]:ro[b]])


def snap_as_batch(snap):
    """The key-major CFK state as the txn-major snapshot acc_map_reduce_full scans, restated on the host (what
    acc_cfk_snap_to_batch builds): one txn per distinct TxnId in TxnId order, its keys = the keys holding it, its
    executeAt / InternalStatus from its first key (all must agree), each pair's missing[] as batch indices.
    Returns (Batch, missing_off, missing_txn)."""
    nk = len(snap["key"])
    off = snap["ent_off"].astype(np.int64)
    owner = np.repeat(np.arange(nk), np.diff(off))
    tk = [_ts_key(int(m), int(l), int(n)) for m, l, n in zip(snap["emsb"], snap["elsb"], snap["enode"])]
    order = sorted(range(len(tk)), key=lambda e: (tk[e], owner[e]))
    first, key_off, key_code, pairs = [], [], [], []
    for i, e in enumerate(order):
        if i == 0 or tk[e] != tk[order[i - 1]]:
            first.append(e)
            key_off.append(i)
        else:
            p = first[-1]
            assert snap["status"][e] == snap["status"][p]
            assert _ts_key(int(snap["xmsb"][e]), int(snap["xlsb"][e]), int(snap["xnode"][e])) == \
                _ts_key(int(snap["xmsb"][p]), int(snap["xlsb"][p]), int(snap["xnode"][p]))
        key_code.append(int(snap["key"][owner[e]]))
        pairs.append(e)
    key_off.append(len(order))
    index = {tk[e]: t for t, e in enumerate(first)}
    mo, mt = [0], []
    for e in pairs:
        for j in range(int(snap["miss_off"][e]), int(snap["miss_off"][e + 1])):
            mt.append(index[_ts_key(int(snap["mmsb"][j]), int(snap["mlsb"][j]), int(snap["mnode"][j]))])
        mo.append(len(mt))
    f = np.array(first, np.int64)
    b = W.Batch(snap["emsb"][f].astype(np.uint64), snap["elsb"][f].astype(np.uint64), snap["enode"][f].astype(np.int32),
                snap["xmsb"][f].astype(np.uint64), snap["xlsb"][f].astype(np.uint64), snap["xnode"][f].astype(np.int32),
                snap["status"][f].astype(np.uint8), np.array(key_off, np.uint32), np.array(key_code, np.uint64))
    return b, np.array(mo, np.uint32), np.array(mt, np.uint32)


def recovery_queries(b, seed, n_query=80):
    """BeginRecovery-style queries over a CFK state: a member's TxnId on its keys (plus maybe another key or one
    without a CFK), a foreign TxnId on an odd hlc, or a bumped executeAt."""
    rng = np.random.default_rng(seed)
    n = b.n_txn
    codes = np.unique(b.key_code) if len(b.key_code) else np.array([100], np.uint64)
    qm, ql, qn, qo, qk = [], [], [], [0], []
    for _ in range(n_query):
        r = rng.random()
        if r < 0.55 and n:
            t = int(rng.integers(0, n))
            m, l, nd = int(b.txn_msb[t]), int(b.txn_lsb[t]), int(b.txn_node[t])
            ks = set(int(x) for x in b.key_code[int(b.key_off[t]):int(b.key_off[t + 1])])
            if rng.random() < 0.4:
                ks.add(int(rng.choice(codes)))
            if rng.random() < 0.2:
                ks.add(7)
        elif r < 0.85 or not n:
            m, l, nd = (int(x) for x in W.encode_ts(1, 2 * int(rng.integers(0, 4 * n + 8)) + 1,
                                                    int(rng.choice(KINDS)) << 1, 1 + int(rng.integers(0, 4))))
            ks = set(int(x) for x in rng.choice(codes, size=min(len(codes), int(rng.integers(1, 5))), replace=False))
        else:
            t = int(rng.integers(0, n))
            m, l, nd = int(b.exe_msb[t]), int(b.exe_lsb[t]), int(b.exe_node[t])
            ks = set(int(x) for x in rng.choice(codes, size=min(len(codes), int(rng.integers(1, 5))), replace=False))
        qm.append(m); ql.append(l); qn.append(nd)
        qk.extend(sorted(ks))
        qo.append(len(qk))
    return dict(msb=np.array(qm, np.uint64), lsb=np.array(ql, np.uint64), node=np.array(qn, np.int32),
                key_off=np.array(qo, np.uint32), key_code=np.array(qk, np.uint64))


def restrict(upd, keyset):
    """The update stream restricted to the keys in `keyset` (CommandsForKey states are per key, so a key's state after
    the restricted stream equals its state after the whole one); updates left without keys are dropped."""
    ko = upd["key_off"].astype(np.int64)
    do = upd["dep_off"].astype(np.int64)
    keep = np.isin(upd["key"], keyset)
    csum = np.concatenate([[0], np.cumsum(keep.astype(np.int64))])
    per = csum[ko[1:]] - csum[ko[:-1]]
    ukeep = per > 0
    out = {k: upd[k][ukeep] for k in ("msb", "lsb", "node", "xmsb", "xlsb", "xnode", "status", "flags")}
    out["key_off"] = np.concatenate([[0], np.cumsum(per[ukeep])]).astype(np.uint32)
    out["key"] = upd["key"][keep]
    out["dep_off"] = np.concatenate([[0], np.cumsum(np.diff(do)[keep])]).astype(np.uint32)
    dsel = np.repeat(keep, np.diff(do))
    for f in ("dmsb", "dlsb", "dnode"):
        out[f] = upd[f][dsel]
    return out


def key_hashes(snap, keys):
    """Per key of `keys` (each present in the key-major snapshot `snap`): a 64-bit hash of its CommandsForKey state --
    every TxnInfo (TxnId, executeAt, status) in order and each one's missing[] TxnIds in order -- plus (entries, missing)
    counts. Vectorised over the selected keys."""
    def mix(x):
        with np.errstate(over="ignore"):
            x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            return x ^ (x >> np.uint64(31))
    k = np.searchsorted(snap["key"], keys)
    assert np.array_equal(snap["key"][k], keys), "a sampled key is missing from the state"
    eo = snap["ent_off"].astype(np.int64)
    mo = snap["miss_off"].astype(np.int64)
    e0, e1 = eo[k], eo[k + 1]
    m0, m1 = mo[e0], mo[e1]

    def seg(cols, a, b, salt):
        n = b - a
        idx = np.repeat(a, n) + (np.arange(int(n.sum())) - np.repeat(np.cumsum(n) - n, n))
        pos = (idx - np.repeat(a, n)).astype(np.uint64)
        with np.errstate(over="ignore"):
            h = np.full(len(idx), np.uint64(salt))
            for c in cols:
                h = mix(h ^ (np.asarray(c)[idx].astype(np.int64).astype(np.uint64) + pos * np.uint64(0x9E3779B97F4A7C15)))
            cs = np.concatenate([[np.uint64(0)], np.cumsum(h, dtype=np.uint64)])
            ends = np.cumsum(n)
            return cs[ends] - cs[ends - n]
    he = seg([snap["emsb"], snap["elsb"], snap["enode"], snap["xmsb"], snap["xlsb"], snap["xnode"], snap["status"],
              np.diff(mo)], e0, e1, 11)
    hm = seg([snap["mmsb"], snap["mlsb"], snap["mnode"]], m0, m1, 13)
    with np.errstate(over="ignore"):
        h = mix(he + np.uint64(0x632BE59BD9B4E019)) ^ mix(hm + (e1 - e0).astype(np.uint64))
    return h, (e1 - e0).astype(np.int64), (m1 - m0).astype(np.int64)
