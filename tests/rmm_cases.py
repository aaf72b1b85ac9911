"""Seeded deps objects (KeyDeps / RangeDeps halves in the SerializerSupport layout) for the Deps.merge, invert, slice and
stabbing tests, plus the canonical set model they are checked against — TEST INFRASTRUCTURE ONLY.

Shapes follow the reference's own generators: KeyDepsTest.Deps.generate (tst/primitives/KeyDepsTest.java:315-374:
TxnIds with epoch < 3, hlc < 500, node < 4, keys and values in random orders), RangeDepsTest.generate /
generateIdenticalTxns / generateNemesisRanges (tst/primitives/RangeDepsTest.java:154-192, 214-268: random ranges,
many txns over identical ranges, heavily overlapping "nemesis" ranges stressing the checkpoints).
"""
from __future__ import annotations

import numpy as np

IDENTITY_LSB = 0xFFFFFFFFFFFF001E
KINDS = (0, 1, 3, 4)   # Read, Write, SyncPoint, ExclusiveSyncPoint


def ts_key(msb, lsb, node):
    """Timestamp.compareTo key (primitives/Timestamp.java:208-217)."""
    return (int(msb), int(lsb) >> 16, int(lsb) & 0x1E, int(node))


def txn_pool(rng, n, wide=False, domain=0):
    """n distinct TxnIds (msb, lsb, node) in compareTo order, KeyDepsTest-style small fields unless `wide`."""
    seen, out = set(), []
    while len(out) < n:
        if wide:
            msb = int(rng.integers(0, 1 << 63)) * 2 + int(rng.integers(0, 2))
            hlc_lo = int(rng.integers(0, 1 << 48))
            node = int(rng.integers(-(1 << 31), 1 << 31))
        else:
            epoch, hlc = int(rng.integers(0, 3)), int(rng.integers(0, 500))
            msb, hlc_lo, node = (epoch << 15) | (hlc >> 48), hlc & ((1 << 48) - 1), int(rng.integers(0, 4))
        kind = int(rng.choice(KINDS))
        lsb = (hlc_lo << 16) | (kind << 1) | domain
        k = ts_key(msb, lsb, node)
        if k in seen:
            continue
        seen.add(k)
        out.append((msb, lsb, node))
    out.sort(key=lambda t: ts_key(*t))
    return out


def flip_bits(rng, t, p):
    """The same TxnId (Timestamp.equals) with different raw flag bits outside IDENTITY_LSB (domain bit, REJECTED 0x8000,
    bits 5..14) with probability p."""
    msb, lsb, node = t
    if rng.random() < p:
        noise = int(rng.integers(0, 1 << 16)) & ~0x1E & 0xFFFF
        lsb = (lsb & ~0xFFFF & 0xFFFFFFFFFFFFFFFF) | (lsb & 0x1E) | noise
    return (msb, lsb, node)


def int_hash_key(key: int) -> int:
    """IntHashKey.hash (tst/impl/IntHashKey.java:255-263): CRC32 over update(key), update(key >> 8), update(key >> 16),
    update(key >> 24) (CRC32.update(int) takes the low byte), masked to 16 bits. IntHashKey.compareTo orders by this
    hash alone (:275-279), so it is the key's order-preserving code and keys with equal hashes compare equal."""
    import zlib
    k = key & 0xFFFFFFFF
    return zlib.crc32(bytes([k & 0xFF, (k >> 8) & 0xFF, (k >> 16) & 0xFF, (k >> 24) & 0xFF])) & 0xFFFF


def int_hash_collisions(limit=1 << 17):
    """pairs (a, b), a < b < limit, of ints whose IntHashKey hashes are equal"""
    seen, out = {}, []
    for k in range(limit):
        h = int_hash_key(k)
        if h in seen:
            out.append((seen[h], k))
        else:
            seen[h] = k
    return out


def random_keys(rng, n, is_range, wide, nemesis=False, identical=False, span=1000, inthash=False):
    """n distinct keys: u64 codes, or ranges (start < end) sorted by Range::compare (start, end). inthash: KeyDepsTest's
    IntHashKey.key(random.nextInt(keyRange)) codes (distinct by compareTo, i.e. by hash)."""
    keys = set()
    if inthash and not is_range:
        while len(keys) < n:
            keys.add(int_hash_key(int(rng.integers(0, max(span, n + 10)))))
        return sorted(keys)
    hi = (1 << 64) - 1 if wide else span
    while len(keys) < n:
        if not is_range:
            keys.add(int(rng.integers(0, hi, dtype=np.uint64)) if wide else int(rng.integers(0, hi)))
            continue
        if identical:
            # generateIdenticalTxns: many txns over a few identical ranges (at most 40 distinct here)
            assert n <= 40
            s = int(rng.integers(0, 10)) * 10
            keys.add((s, s + 10 + int(rng.integers(0, 4))))
        elif nemesis:
            s = int(rng.integers(0, 50))
            keys.add((s, s + int(rng.integers(1, 400))))
        elif wide:
            a, b = sorted(int(x) for x in rng.integers(0, hi, size=2, dtype=np.uint64))
            if a < b:
                keys.add((a, b))
        else:
            s = int(rng.integers(0, span))
            keys.add((s, s + int(rng.integers(1, 64))))
    return sorted(keys)


def build_half(replies, is_range):
    """Concatenate per-reply (keys, [raw TxnIds], {key index: [value index...]}) into the acc_rmm_in layout."""
    key_off, val_off, k2v_off = [0], [0], [0]
    ka, kb, msb, lsb, node, k2v = [], [], [], [], [], []
    for keys, vals, ent in replies:
        hdr, body = [], []
        for i, k in enumerate(keys):
            body.extend(sorted(ent.get(i, [])))
            hdr.append(len(keys) + len(body))
        for k in keys:
            if is_range:
                ka.append(k[0]); kb.append(k[1])
            else:
                ka.append(k)
        for t in vals:
            msb.append(t[0]); lsb.append(t[1]); node.append(t[2])
        k2v.extend(hdr + body)
        key_off.append(len(ka)); val_off.append(len(msb)); k2v_off.append(len(k2v))
    h = dict(key_off=np.array(key_off, np.uint64), key_a=np.array(ka, np.uint64), val_off=np.array(val_off, np.uint64),
             msb=np.array(msb, np.uint64), lsb=np.array(lsb, np.uint64), node=np.array(node, np.int32),
             k2v_off=np.array(k2v_off, np.uint64), k2v=np.array(k2v, np.int32))
    if is_range:
        h["key_b"] = np.array(kb, np.uint64)
    return h


def gen_groups(seed, n_groups, replies, is_range=False, n_keys=12, n_txn=30, p_drop=0.3, p_flip=0.0, p_empty=0.1,
               p_extra=0.1, p_keyonly=0.05, wide=False, nemesis=False, identical=False, max_replies=None, counts=None,
               inthash=False):
    """Groups of replies, each reply a random sub-relation of the group's truth relation (+ unreferenced TxnIds, keys
    without entries, empty replies, raw-bit flips of equal TxnIds). Returns (grp_off, half)."""
    rng = np.random.default_rng(seed)
    grp_off, reps = [0], []
    for _ in range(n_groups):
        pool = txn_pool(rng, n_txn, wide=wide, domain=1 if is_range else 0)
        keys = random_keys(rng, n_keys, is_range, wide, nemesis, identical, inthash=inthash)
        truth = {i: sorted(rng.choice(n_txn, size=int(rng.integers(1, min(n_txn, 8) + 1)), replace=False).tolist())
                 for i in range(len(keys))}
        nr = replies if max_replies is None else int(rng.integers(1, max_replies + 1))
        if counts is not None:
            nr = int(counts[len(grp_off) - 1])
        for _ in range(nr):
            if rng.random() < p_empty:
                # isEmpty(): no entries (possibly keys without entries)
                ks = sorted(rng.choice(len(keys), size=int(rng.integers(0, 3)), replace=False).tolist()) if keys else []
                reps.append(([keys[i] for i in ks], [], {}))
                continue
            ks = sorted(i for i in range(len(keys)) if rng.random() > 0.4)
            if not ks:
                ks = [int(rng.integers(0, len(keys)))]
            ent = {}
            used = set()
            for j, i in enumerate(ks):
                if rng.random() < p_keyonly:
                    continue
                vs = [v for v in truth[i] if rng.random() > p_drop]
                if vs:
                    ent[j] = vs
                    used.update(vs)
            if not used:
                v = truth[ks[0]][0]
                ent[0] = [v]
                used.add(v)
            extra = {int(x) for x in rng.choice(n_txn, size=2, replace=False)} if rng.random() < p_extra else set()
            vals = sorted(used | extra)
            idx = {v: q for q, v in enumerate(vals)}
            ent = {j: [idx[v] for v in vs] for j, vs in ent.items()}
            reps.append(([keys[i] for i in ks], [flip_bits(rng, pool[v], p_flip) for v in vals], ent))
        grp_off.append(len(reps))
    return np.array(grp_off, np.uint64), build_half(reps, is_range)


def canonical_merge(grp_off, half, is_range):
    """Canonical union per group (KeyDepsTest.testMergedProperty, tst/primitives/KeyDepsTest.java:275-283): keys and
    txnIds of the non-empty replies, per key the union of its TxnIds; returns comparable python structures (TxnIds by
    compareTo identity)."""
    out = []
    for g in range(len(grp_off) - 1):
        keys, vals, ent = set(), set(), {}
        for r in range(int(grp_off[g]), int(grp_off[g + 1])):
            k0, k1 = int(half["key_off"][r]), int(half["key_off"][r + 1])
            v0, v1 = int(half["val_off"][r]), int(half["val_off"][r + 1])
            o0, o1 = int(half["k2v_off"][r]), int(half["k2v_off"][r + 1])
            nk = k1 - k0
            if o1 - o0 == nk:
                continue
            rv = [ts_key(half["msb"][v], half["lsb"][v], half["node"][v]) for v in range(v0, v1)]
            vals.update(rv)
            prev = nk
            for i in range(nk):
                key = (int(half["key_a"][k0 + i]), int(half["key_b"][k0 + i])) if is_range else int(half["key_a"][k0 + i])
                keys.add(key)
                end = int(half["k2v"][o0 + i])
                ent.setdefault(key, set()).update(rv[int(x)] for x in half["k2v"][o0 + prev:o0 + end])
                prev = end
        out.append((sorted(keys), sorted(vals), {k: sorted(v) for k, v in ent.items()}))
    return out


def as_groups(res, is_range):
    """Merged CSR (acc_rmm_view host copy or oracle result) -> the canonical_merge structure."""
    out = []
    g = len(res["key_off"]) - 1
    for i in range(g):
        k0, k1 = int(res["key_off"][i]), int(res["key_off"][i + 1])
        v0, v1 = int(res["val_off"][i]), int(res["val_off"][i + 1])
        o0 = int(res["k2v_off"][i])
        keys = [(int(res["key_a"][k]), int(res["key_b"][k])) if is_range else int(res["key_a"][k]) for k in range(k0, k1)]
        vals = [ts_key(res["msb"][v], res["lsb"][v], res["node"][v]) for v in range(v0, v1)]
        ent, prev = {}, len(keys)
        for q, key in enumerate(keys):
            end = int(res["k2v"][o0 + q])
            ent[key] = [vals[int(x)] for x in res["k2v"][o0 + prev:o0 + end]]
            prev = end
        out.append((keys, vals, ent))
    return out


# ---------------------------------------------------------------- invert / slice / stab models

def as_batch(half):
    """One deps object per reply: the acc_rmm_batch dict of a gen_groups half."""
    m = dict(key_off=half["key_off"], key_a=half["key_a"], val_off=half["val_off"], k2v_off=half["k2v_off"], k2v=half["k2v"])
    if "key_b" in half:
        m["key_b"] = half["key_b"]
    return m


def py_invert(m):
    """txnIdsToKeys per group as set lists: for each TxnId index, the ascending key indices referencing it."""
    out = []
    for g in range(len(m["key_off"]) - 1):
        nk = int(m["key_off"][g + 1] - m["key_off"][g])
        nv = int(m["val_off"][g + 1] - m["val_off"][g])
        o0 = int(m["k2v_off"][g])
        h = m["k2v"][o0:int(m["k2v_off"][g + 1])]
        lists = [[] for _ in range(nv)]
        prev = nk
        for k in range(nk):
            for x in h[prev:int(h[k])]:
                lists[int(x)].append(k)
            prev = int(h[k])
        hdr, body = [], []
        for v in range(nv):
            body += lists[v]
            hdr.append(nv + len(body))
        out.append(hdr + body)
    return out


def gen_select(seed, n_groups, span=1000, wide=False, max_ranges=4):
    """Per group select Ranges (sorted, deoverlapped) over the same key space as gen_groups."""
    rng = np.random.default_rng(seed)
    off, s, e = [0], [], []
    hi = (1 << 62) if wide else span
    for _ in range(n_groups):
        pts = sorted({int(x) for x in rng.integers(0, hi, size=2 * int(rng.integers(0, max_ranges + 1)))})
        if len(pts) % 2:
            pts = pts[:-1]
        for i in range(0, len(pts), 2):
            s.append(pts[i]); e.append(pts[i + 1])
        off.append(len(s))
    return np.array(off, np.uint64), np.array(s, np.uint64), np.array(e, np.uint64)


def random_range_list(seed, n, span_lo=0, span_hi=1 << 32, max_w=1000):
    """SearchableRangeListTest.random (tst/utils/SearchableRangeListTest.java:61-115): n ranges with random starts and
    widths in [1, 1000), sorted by start (Range::start only, ties in generation order)."""
    rng = np.random.default_rng(seed)
    st = rng.integers(span_lo, span_hi - max_w, size=n).astype(np.uint64)
    w = rng.integers(1, max_w, size=n).astype(np.uint64)
    order = np.argsort(st, kind="stable")
    return st[order], (st + w)[order]
