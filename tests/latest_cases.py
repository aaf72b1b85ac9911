"""Seeded LatestDeps recovery cases (primitives/LatestDeps.java, coordinate/Recover.java:295-355) — TEST INFRASTRUCTURE.

Deps objects come from rmm_cases (KeyDepsTest / RangeDepsTest shapes over a 0..1000 key space); each recovering txn gets
2-5 replies, each a LatestDeps of 1-4 RoutingKey intervals with gaps, KnownDeps phases, small ballots (ties exercise
the Accept/Commit ballot tie-break), coordinatedDeps / localDeps ids, and neighbours sharing ids (the builder's
tryMergeEqual coalescing)."""
from __future__ import annotations

import numpy as np

import rmm_cases as RC


def deps_objects(seed, n_deps):
    _, kh = RC.gen_groups(seed, 1, n_deps, is_range=False, n_keys=25, n_txn=40, p_empty=0.1)
    _, rh = RC.gen_groups(seed + 7, 1, n_deps, is_range=True, n_keys=12, n_txn=40, p_empty=0.1)
    return kh, rh


def groups(seed, n_groups, n_deps, phases, span=1000):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n_groups):
        replies = []
        for _ in range(int(rng.integers(1, 6))):
            pts = sorted({int(x) for x in rng.integers(0, span, size=2 * int(rng.integers(1, 5)))})
            if len(pts) < 2:
                pts = [pts[0], pts[0] + 5]
            ivs = []
            # consecutive points make adjacent intervals; skipping one leaves a gap
            i = 0
            prev = None
            while i + 1 < len(pts):
                s, e = pts[i], pts[i + 1]
                known = int(rng.choice(phases))
                ballot = (1 << 15, (int(rng.integers(0, 3)) << 16), int(rng.integers(0, 2)))
                if prev is not None and rng.random() < 0.3 and (known == 0 or prev[4] >= 0):
                    cd, ld = prev[4], prev[5]            # same objects as the neighbour: coalescing candidates
                else:
                    cd = int(rng.integers(0, n_deps)) if (known != 0 or rng.random() < 0.5) else -1
                    ld = int(rng.integers(0, n_deps)) if rng.random() < 0.7 else -1
                iv = (s, e, known, ballot, cd, ld)
                ivs.append(iv)
                prev = iv
                i += 1 if rng.random() < 0.6 else 2
            replies.append(ivs)
        out.append(replies)
    return out


def canonical_union(objs, items, is_range, end_inclusive=True):
    """{key: set of TxnIds} = union over items of the object's relation restricted to the item's range (KeyDeps.slice:
    keys contained; RangeDeps.slice: ranges intersecting), by compareTo identity."""
    out = {}
    for d, s, e in items:
        k0, k1 = int(objs["key_off"][d]), int(objs["key_off"][d + 1])
        v0 = int(objs["val_off"][d])
        o0 = int(objs["k2v_off"][d])
        nk = k1 - k0
        prev = nk
        for i in range(nk):
            end = int(objs["k2v"][o0 + i])
            if is_range:
                key = (int(objs["key_a"][k0 + i]), int(objs["key_b"][k0 + i]))
                inside = key[0] < e and key[1] > s
            else:
                key = int(objs["key_a"][k0 + i])
                inside = (s < key <= e) if end_inclusive else (s <= key < e)
            if inside:
                ids = {RC.ts_key(objs["msb"][v0 + int(x)], objs["lsb"][v0 + int(x)], objs["node"][v0 + int(x)])
                       for x in objs["k2v"][o0 + prev:o0 + end]}
                if ids:
                    out.setdefault(key, set()).update(ids)
            prev = end
    return out


def result_map(half, g, is_range):
    m = RC.as_groups(half, is_range)[g]
    return {k: set(v) for k, v in m[2].items() if v}
