"""Maelstrom Deps JSON (accord-maelstrom Json.DEPS_ADAPTER, mael/Json.java:316-398) — TEST INFRASTRUCTURE: a Python
writer in Gson's compact form and the Builder semantics (sorted unique keys by Datum.compareTo, sorted unique TxnIds by
Timestamp.compareTo) over the datum kinds the device path takes (LONG, HASH, null sentinels)."""
from __future__ import annotations

import zlib

import numpy as np

STRING, LONG, DOUBLE, HASH = range(4)   # Datum.Kind ordinals


def _i32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= 1 << 31 else x


def datum_hash(kind, null, value):
    """Datum.hash (mael/Datum.java:188-200): null -> Integer.MAX_VALUE; Hash -> its hash; else CRC32 over the 4 low
    bytes of value.hashCode() (Long.hashCode = (int)(v ^ (v >>> 32)))."""
    if null:
        return 0x7FFFFFFF
    if kind == HASH:
        return _i32(value)
    v = value & 0xFFFFFFFFFFFFFFFF
    i = (v ^ (v >> 32)) & 0xFFFFFFFF
    return _i32(zlib.crc32(bytes([i & 0xFF, (i >> 8) & 0xFF, (i >> 16) & 0xFF, (i >> 24) & 0xFF])))


def datum_order(d):
    """Datum.compareTo (:172-186): hash, kind, null last, value"""
    kind, null, value = d
    return (datum_hash(kind, null, value), kind, 1 if null else 0, 0 if null else value)


def ts_order(t):
    msb, lsb, node = t
    return (msb & 0xFFFFFFFFFFFFFFFF, (lsb & 0xFFFFFFFFFFFFFFFF) >> 16, lsb & 0x1E, node)


def write_datum(d):
    kind, null, value = d
    if null:
        return '["HASH",false]' if kind == HASH else f'["{("STRING", "LONG", "DOUBLE", "HASH")[kind]}"]'
    if kind == HASH:
        return f'["HASH",true,{_i32(value)}]'
    return str(value)


def write_txn(t):
    msb, lsb, node = t
    s = lambda x: x - (1 << 64) if x >= 1 << 63 else x  # noqa: E731  (Java longs)
    nd = "null" if node == 0 else f'"{"c" if node < 0 else "n"}{node}"'
    return f"[{s(msb)},{s(lsb)},{nd}]"


def write_deps(key_entries, range_entries):
    """entries in the order given: [(datum, txn)], [((start, end), txn)]"""
    k = ",".join(f"[{write_datum(d)},{write_txn(t)}]" for d, t in key_entries)
    r = ",".join(f"[{write_datum(a)},{write_datum(b)},{write_txn(t)}]" for (a, b), t in range_entries)
    return ('{"keyDeps":[' + k + '],"rangeDeps":[' + r + "]}").encode()


def build(key_entries, range_entries):
    """KeyDeps / RangeDeps Builder result in DEPS_ADAPTER write order: keys ascending, then each key's TxnIds ascending"""
    km, rm = {}, {}
    for d, t in key_entries:
        km.setdefault(datum_order(d), (d, {}))[1].setdefault(ts_order(t), t)
    for (a, b), t in range_entries:
        rm.setdefault((datum_order(a), datum_order(b)), ((a, b), {}))[1].setdefault(ts_order(t), t)
    ke = [(d, ts[o]) for _, (d, ts) in sorted(km.items()) for o in sorted(ts)]
    re_ = [(r, ts[o]) for _, (r, ts) in sorted(rm.items()) for o in sorted(ts)]
    return ke, re_


def random_datum(rng, p_hash=0.25, p_null=0.03, span=None):
    if rng.random() < p_null:
        return (int(rng.choice([LONG, HASH])), True, 0)
    if rng.random() < p_hash:
        return (HASH, False, int(rng.integers(-(1 << 31), 1 << 31)))
    v = int(rng.integers(-(1 << 62), 1 << 62)) if span is None else int(rng.integers(0, span))
    return (LONG, False, v)


def random_txn(rng):
    epoch, hlc = int(rng.integers(0, 3)), int(rng.integers(0, 500))
    kind = int(rng.choice([0, 1, 3, 4]))
    node = int(rng.choice([0, 1, 2, 3, -2]))
    return ((epoch << 15) | (hlc >> 48), (hlc << 16) | (kind << 1), node)


def random_doc(rng, n_keys=20, n_txn=30, n_entries=60, n_ranges=10, canonical=False):
    keys = [random_datum(rng, span=None if rng.random() < 0.5 else 200) for _ in range(n_keys)]
    txns = [random_txn(rng) for _ in range(n_txn)]
    ke = [(keys[int(rng.integers(0, n_keys))], txns[int(rng.integers(0, n_txn))]) for _ in range(int(rng.integers(0, n_entries)))]
    re_ = []
    for _ in range(int(rng.integers(0, n_ranges))):
        a, b = keys[int(rng.integers(0, n_keys))], keys[int(rng.integers(0, n_keys))]
        if datum_order(a) == datum_order(b):
            continue
        if datum_order(a) > datum_order(b):
            a, b = b, a
        re_.append(((a, b), txns[int(rng.integers(0, n_txn))]))
    if canonical:
        ke, re_ = build(ke, re_)
    return ke, re_
