"""LatestDeps.mergeProposal / mergeCommit restated in Python — TEST INFRASTRUCTURE ONLY (tests/ import it as the
checker of acc_latest_deps_merge; the product never does).

primitives/LatestDeps.java:228-413 and utils/ReducingIntervalMap.java:202-273, 522-575, step for step:
  * each reply is a ReducingRangeMap: starts[] and values[] (None = gap); `Merge(LatestDeps)` converts entries one for
    one (localDeps -> a one-element merge list);
  * the replies are folded left to right with mergeIntervals, reducing overlapping entries with MergeEntry.reduce
    (higher KnownDeps, ballot tie-break in the Accept / Commit phases; when the winner is <= DepsProposed the merged
    entry is built from the arguments as passed: a.known, a.ballot, a.coordinatedDeps, a.merge ++ b.merge), and every
    append coalescing with an equal (same coordinatedDeps / merge list objects) contiguous tail;
  * forProposal / forCommit select deps objects per interval; each is sliced to its interval (KeyDeps.slice /
    RangeDeps.slice + trimUnusedValues, the C restatement in accord_oracle_rmm.c) and the slices of a group are merged
    (KeyDeps.merge / RangeDeps.merge, the LinearMerger fold in accord_oracle_rmm.c).
"""
from __future__ import annotations

import numpy as np

import oracle

DEPS_UNKNOWN, DEPS_PROPOSED, DEPS_COMMITTED, DEPS_ERASED, DEPS_KNOWN, NO_DEPS = range(6)


def _ts_key(t):
    msb, lsb, node = t
    return (int(msb), int(lsb) >> 16, int(lsb) & 0x1E, int(node))


class Entry:
    __slots__ = ("known", "ballot", "coord", "merge")

    def __init__(self, known, ballot, coord, merge):
        self.known, self.ballot, self.coord, self.merge = known, ballot, coord, merge


def _reduce(a: Entry, b: Entry) -> Entry:
    c = (a.known > b.known) - (a.known < b.known)
    if c == 0 and a.known in (DEPS_PROPOSED, DEPS_COMMITTED):   # Phase.Accept / Commit tieBreakWithBallot
        ka, kb = _ts_key(a.ballot), _ts_key(b.ballot)
        c = (ka > kb) - (ka < kb)
    hi = b if c < 0 else a
    if hi.known <= DEPS_PROPOSED:
        return Entry(a.known, a.ballot, a.coord, list(a.merge) + list(b.merge))
    return hi


def _equal(a: Entry, b: Entry) -> bool:
    return a.coord == b.coord and len(a.merge) == len(b.merge) and all(x == y for x, y in zip(a.merge, b.merge))


class _Builder:
    def __init__(self):
        self.starts, self.values, self.prev_end = [], [], None

    def append(self, start, end, v):
        if self.prev_end is not None:
            assert self.prev_end <= start
            if self.prev_end < start:
                self.starts.append(self.prev_end)
                self.values.append(None)
        if self.values and self.values[-1] is not None and _equal(self.values[-1], v):
            pass
        else:
            self.starts.append(start)
            self.values.append(v)
        self.prev_end = end

    def build(self):
        if self.prev_end is not None:
            self.starts.append(self.prev_end)
        return self.starts, self.values


def merge_intervals(left, right):
    ls, lv = left
    rs, rv = right
    if not lv:
        return right
    if not rv:
        return left
    b = _Builder()
    it = {"l": 0, "r": 0}
    maps = {"l": (ls, lv), "r": (rs, rv)}

    def has(k):
        return it[k] < len(maps[k][1])

    def st(k):
        return maps[k][0][it[k]]

    def en(k):
        return maps[k][0][it[k] + 1]

    def val(k):
        return maps[k][1][it[k]]

    first = "l" if st("l") <= st("r") else "r"
    second = "r" if first == "l" else "l"
    while has(first) and en(first) <= st(second):
        if val(first) is not None:
            b.append(st(first), en(first), val(first))
        it[first] += 1
    start = st(second)
    if has(first) and st(first) < start and val(first) is not None:
        b.append(st(first), start, val(first))
    while has("l") and has("r"):
        le, re = en("l"), en("r")
        end = min(le, re)
        a, c = val("l"), val("r")
        v = c if a is None else a if c is None else _reduce(a, c)
        if le <= re:
            it["l"] += 1
        if le >= re:
            it["r"] += 1
        if v is not None:
            b.append(start, end, v)
        start = end
    rem = "l" if has("l") else "r"
    while has(rem):
        end = en(rem)
        if val(rem) is not None:
            b.append(start, end, val(rem))
        start = end
        it[rem] += 1
    return b.build()


def fold_group(replies):
    """replies: list of lists of (start, end, known, ballot, coord, local) -> merged (starts, values)"""
    acc = ([], [])
    for ivs in replies:
        starts, values = [], []
        for (s, e, known, ballot, coord, local) in ivs:
            if starts:
                assert starts[-1] <= s
                if starts[-1] < s:
                    values.append(None)
                    starts.append(s)
            else:
                starts.append(s)
            values.append(Entry(known, ballot, coord, [] if local < 0 else [local]))
            starts.append(e)
        acc = merge_intervals(acc, (starts, values))
    return acc


class InvalidKnownDeps(AssertionError):
    pass


def items_of(merged, commit=False, use_local=False):
    """(items [(deps id, start, end)], sufficientFor [(start, end)]) in stream order."""
    starts, values = merged
    items, suff = [], []
    for i, e in enumerate(values):
        if e is None:
            continue
        s, t = starts[i], starts[i + 1]
        if not commit:
            if e.known == DEPS_PROPOSED:
                if e.coord < 0:
                    raise InvalidKnownDeps("null coordinatedDeps")
                items.append((e.coord, s, t))
            elif e.known == DEPS_UNKNOWN:
                items.extend((d, s, t) for d in e.merge)
            else:
                raise InvalidKnownDeps(e.known)
        else:
            if e.known in (DEPS_UNKNOWN, DEPS_PROPOSED):
                if not use_local:
                    continue
                suff.append((s, t))
                if e.known == DEPS_PROPOSED:
                    if e.coord < 0:
                        raise InvalidKnownDeps("null coordinatedDeps")
                    items.append((e.coord, s, t))
                items.extend((d, s, t) for d in e.merge)
            elif e.known in (DEPS_KNOWN, DEPS_COMMITTED):
                if e.coord < 0:
                    raise InvalidKnownDeps("null coordinatedDeps")
                suff.append((s, t))
                items.append((e.coord, s, t))
            else:
                raise InvalidKnownDeps(e.known)
    return items, suff


def _gather_half(objs: dict, ids, is_range):
    """the deps objects `ids` (in order) of one half as an rmm batch / merge half"""
    key_off, val_off, k2v_off = [0], [0], [0]
    ka, kb, m, l, nd, k2v = [], [], [], [], [], []
    for d in ids:
        k0, k1 = int(objs["key_off"][d]), int(objs["key_off"][d + 1])
        v0, v1 = int(objs["val_off"][d]), int(objs["val_off"][d + 1])
        o0, o1 = int(objs["k2v_off"][d]), int(objs["k2v_off"][d + 1])
        ka.extend(objs["key_a"][k0:k1])
        if is_range:
            kb.extend(objs["key_b"][k0:k1])
        m.extend(objs["msb"][v0:v1]); l.extend(objs["lsb"][v0:v1]); nd.extend(objs["node"][v0:v1])
        k2v.extend(objs["k2v"][o0:o1])
        key_off.append(len(ka)); val_off.append(len(m)); k2v_off.append(len(k2v))
    h = dict(key_off=np.array(key_off, np.uint64), key_a=np.array(ka, np.uint64), val_off=np.array(val_off, np.uint64),
             msb=np.array(m, np.uint64), lsb=np.array(l, np.uint64), node=np.array(nd, np.int32),
             k2v_off=np.array(k2v_off, np.uint64), k2v=np.array(k2v, np.int32))
    if is_range:
        h["key_b"] = np.array(kb, np.uint64)
    return h


def _slice_half(objs, items, is_range, end_inclusive):
    g = _gather_half(objs, [d for d, _, _ in items], is_range)
    n = len(items)
    sl = oracle.rmm_slice(g, np.arange(n + 1, dtype=np.uint64), np.array([s for _, s, _ in items], np.uint64),
                          np.array([e for _, _, e in items], np.uint64), is_range, end_inclusive)
    ko, vo = sl["key_off"].astype(np.int64), sl["val_off"].astype(np.int64)
    ka, kb, m, l, nd = [], [], [], [], []
    for i in range(n):
        k0, v0 = int(g["key_off"][i]), int(g["val_off"][i])
        for x in sl["key_idx"][ko[i]:ko[i + 1]]:
            ka.append(g["key_a"][k0 + int(x)])
            if is_range:
                kb.append(g["key_b"][k0 + int(x)])
        for y in sl["val_idx"][vo[i]:vo[i + 1]]:
            m.append(g["msb"][v0 + int(y)]); l.append(g["lsb"][v0 + int(y)]); nd.append(g["node"][v0 + int(y)])
    h = dict(key_off=sl["key_off"], key_a=np.array(ka, np.uint64), val_off=sl["val_off"], msb=np.array(m, np.uint64),
             lsb=np.array(l, np.uint64), node=np.array(nd, np.int32), k2v_off=sl["k2v_off"], k2v=sl["k2v"])
    if is_range:
        h["key_b"] = np.array(kb, np.uint64)
    return h


def latest_deps_merge(groups, key_objs, range_objs, end_inclusive=True, commit=False, use_local=None):
    """groups: per recovering txn the replies (lists of intervals, see fold_group); key_objs / range_objs: the deps
    objects' halves (merge-half dicts, one slot per deps id). use_local[g] = txnId.equals(executeAt) (commit).
    Returns dict(key=merged half, range=merged half, sufficient=[[(s, e)...] per group], items=[[...] per group])."""
    all_items, grp_off, suff, per = [], [0], [], []
    for g, replies in enumerate(groups):
        its, sf = items_of(fold_group(replies), commit, bool(use_local[g]) if commit else False)
        all_items.extend(its)
        grp_off.append(len(all_items))
        suff.append(sf)
        per.append(its)
    grp = np.array(grp_off, np.uint64)
    kh = _slice_half(key_objs, all_items, False, end_inclusive)
    rh = _slice_half(range_objs, all_items, True, end_inclusive)
    return dict(key=oracle.rmm_merge(grp, kh, False), range=oracle.rmm_merge(grp, rh, True), sufficient=suff, items=per)
