"""CPU: oracle restatements of RelationMultiMap.invert, KeyDeps/RangeDeps.slice + trimUnusedValues and the RangeDeps
stabbing query against independent Python models (no GPU)."""
import numpy as np
import pytest

import oracle
import rmm_cases as RC


@pytest.mark.parametrize("is_range", [False, True])
def test_invert_oracle(is_range):
    _, half = RC.gen_groups(3, 10, 6, is_range=is_range, p_keyonly=0.3)
    m = RC.as_batch(half)
    nk = np.diff(m["key_off"].astype(np.int64)).astype(np.uint64)
    nv = np.diff(m["val_off"].astype(np.int64)).astype(np.uint64)
    off, ints = oracle.invert(m["k2v_off"], m["k2v"], nk, nv)
    ref = RC.py_invert(m)
    for g, r in enumerate(ref):
        assert ints[int(off[g]):int(off[g + 1])].tolist() == r, g


def py_slice(m, g, sel, is_range, end_inclusive):
    """Set model of KeyDeps.slice / RangeDeps.slice + trimUnusedValues with the reference's short cuts."""
    k0, k1 = int(m["key_off"][g]), int(m["key_off"][g + 1])
    nk, nv = k1 - k0, int(m["val_off"][g + 1] - m["val_off"][g])
    h = m["k2v"][int(m["k2v_off"][g]):int(m["k2v_off"][g + 1])].tolist()
    if len(h) == nk:
        return (list(range(nk)) if not is_range else []), list(range(nv)), (h if not is_range else [])
    def hit(k):
        if is_range:
            a, b = int(m["key_a"][k0 + k]), int(m["key_b"][k0 + k])
            return any(a < e and b > s for s, e in sel)
        c = int(m["key_a"][k0 + k])
        return any((s < c <= e) if end_inclusive else (s <= c < e) for s, e in sel)
    ks = [k for k in range(nk) if hit(k)]
    if not ks:
        return [], [], []
    if len(ks) == nk:
        return list(range(nk)), list(range(nv)), h
    lists = [h[(nk if k == 0 else h[k - 1]):h[k]] for k in ks]
    used = sorted({x for l in lists for x in l})
    rm = {v: i for i, v in enumerate(used)}
    hdr, body = [], []
    for l in lists:
        body += [rm[x] for x in l]
        hdr.append(len(ks) + len(body))
    return ks, used, hdr + body


@pytest.mark.parametrize("is_range,end_inclusive", [(False, True), (False, False), (True, True)])
def test_slice_oracle(is_range, end_inclusive):
    _, half = RC.gen_groups(4, 12, 5, is_range=is_range, p_keyonly=0.2)
    m = RC.as_batch(half)
    n = len(m["key_off"]) - 1
    so, ss, se = RC.gen_select(9, n)
    r = oracle.rmm_slice(m, so, ss, se, is_range, end_inclusive)
    for g in range(n):
        sel = list(zip(ss[int(so[g]):int(so[g + 1])].tolist(), se[int(so[g]):int(so[g + 1])].tolist()))
        ks, vs, ints = py_slice(m, g, sel, is_range, end_inclusive)
        assert r["key_idx"][int(r["key_off"][g]):int(r["key_off"][g + 1])].tolist() == ks, g
        assert r["val_idx"][int(r["val_off"][g]):int(r["val_off"][g + 1])].tolist() == vs, g
        assert r["k2v"][int(r["k2v_off"][g]):int(r["k2v_off"][g + 1])].tolist() == ints, g


def test_stab_oracle_full_world():
    """SearchableRangeListTest.fullWorld (tst/utils/SearchableRangeListTest.java:36-59): ranges (i, i+1] for i < 1000;
    the range query (s, e] intersects exactly the ranges s .. e-1 (the Java's counter adds its callback's inclusive end),
    in ascending order."""
    n = 1000
    rs = np.arange(n, dtype=np.uint64)
    re = rs + np.uint64(1)
    qs = np.concatenate([np.arange(n), np.zeros(n)]).astype(np.uint64)
    qe = np.concatenate([np.full(n, n), n - np.arange(n)]).astype(np.uint64)
    off, idx = oracle.rmm_stab(np.zeros(2 * n, np.uint32), qs, qe, False, True, np.array([0, n], np.uint64), rs, re)
    for q in range(2 * n):
        assert idx[int(off[q]):int(off[q + 1])].tolist() == list(range(int(qs[q]), int(qe[q])))
