"""Maelstrom Deps JSON (accord-maelstrom Json.DEPS_ADAPTER, mael/Json.java:316-398) — TEST INFRASTRUCTURE: a Python
writer in Gson's compact form and the Builder semantics (sorted unique keys by Datum.compareTo, sorted unique TxnIds by
Timestamp.compareTo) over every datum kind: LONG, HASH, null sentinels, STRING (ASCII; Gson's HTML-safe escaping) and
DOUBLE (Java's Double.toString, restated with exact rational arithmetic: shortest digits that round back, closest on
ties, the JDK 19 two-digit rule, Java's plain / computerized-scientific layout). A datum is (kind, null, value) with
value an int (LONG, HASH), a str (STRING) or a float (DOUBLE)."""
from __future__ import annotations

import math
import struct
import zlib
from fractions import Fraction

import numpy as np

STRING, LONG, DOUBLE, HASH = range(4)   # Datum.Kind ordinals


def _i32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= 1 << 31 else x


def double_bits(x: float) -> int:
    return struct.unpack(">Q", struct.pack(">d", x))[0]


def string_hash_code(s: str) -> int:
    """String.hashCode over UTF-16 units (ASCII here: one per character)"""
    h = 0
    for ch in s:
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return _i32(h)


def datum_hash(kind, null, value):
    """Datum.hash (mael/Datum.java:188-200): null -> Integer.MAX_VALUE; Hash -> its hash; else CRC32 over the 4 low
    bytes of value.hashCode() (Long.hashCode = (int)(v ^ (v >>> 32)); Double.hashCode the same over the bits)."""
    if null:
        return 0x7FFFFFFF
    if kind == HASH:
        return _i32(value)
    if kind == STRING:
        i = string_hash_code(value) & 0xFFFFFFFF
    else:
        v = double_bits(value) if kind == DOUBLE else value & 0xFFFFFFFFFFFFFFFF
        i = (v ^ (v >> 32)) & 0xFFFFFFFF
    return _i32(zlib.crc32(bytes([i & 0xFF, (i >> 8) & 0xFF, (i >> 16) & 0xFF, (i >> 24) & 0xFF])))


def _value_order(kind, value):
    if kind == DOUBLE:   # Double.compareTo: bit order with -0.0 < 0.0
        b = double_bits(value)
        return (~b & 0xFFFFFFFFFFFFFFFF) if b >> 63 else b | (1 << 63)
    return value


def datum_order(d):
    """Datum.compareTo (:172-186): hash, kind, null last, value"""
    kind, null, value = d
    return (datum_hash(kind, null, value), kind, 1 if null else 0, 0 if null else _value_order(kind, value))


def _rounds_to(q: Fraction, x: float) -> bool:
    try:
        return float(q) == x
    except OverflowError:
        return False


def java_double_to_string(x: float) -> str:
    """Double.toString (JDK >= 19): among the decimals that round to x, the shortest; of those the closest (ties: even
    last digit); if the shortest has one digit, the closest of those with one or two digits. Then Java's layout:
    plain with at least one fraction digit for 1e-3 <= |x| < 1e7, else d.dddE[-]n."""
    if x == 0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    neg = x < 0
    v = Fraction(abs(x))
    # shortest digit count n with some n-digit decimal rounding to x
    best = None
    for n in range(1, 18):
        e = math.floor(math.log10(abs(x)))
        for ee in (e - 1, e, e + 1):   # the decimal exponent of the first digit
            scale = Fraction(10) ** (ee - n + 1)
            q = v / scale
            lo, hi = math.floor(q), math.ceil(q)
            cands = []
            for c in {lo, hi}:
                if 10 ** (n - 1) <= c < 10 ** n and _rounds_to(Fraction(c) * scale, abs(x)):
                    cands.append((abs(Fraction(c) * scale - v), c % 2, c, ee))
            if cands:
                cands.sort()
                if best is None or cands[0][:2] < best[0][:2]:
                    best = (cands[0][0], cands[0][1]), cands[0][2], cands[0][3], n
        if best is not None:
            if n == 1:   # JDK 19: a closer two-digit decimal wins over the one-digit one
                _, c1, ee1, _ = best
                scale = Fraction(10) ** (ee1 - 1)
                for c in (math.floor(v / scale), math.ceil(v / scale)):
                    if 10 <= c < 100 and float(Fraction(c) * scale) == abs(x) and \
                            abs(Fraction(c) * scale - v) < abs(Fraction(c1) * Fraction(10) ** ee1 - v):
                        best = (None, c, ee1, 2)
                        break
            break
    _, c, ee, n = best
    digits = str(c).rstrip("0") or "0"
    k = ee   # value = 0.d1d2.. * 10^(k+1) = d1.d2.. * 10^k
    if -3 <= k < 7:
        if k < 0:
            s = "0." + "0" * (-k - 1) + digits
        else:
            ip = digits[:k + 1].ljust(k + 1, "0")
            fp = digits[k + 1:] or "0"
            s = ip + "." + fp
    else:
        s = digits[0] + "." + (digits[1:] or "0") + "E" + str(k)
    return ("-" if neg else "") + s


def gson_string(t: str) -> str:
    """JsonWriter.string with Gson's default HTML-safe replacement table"""
    out = ['"']
    for ch in t:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch in "\t\b\n\r\f":
            out.append({"\t": "\\t", "\b": "\\b", "\n": "\\n", "\r": "\\r", "\f": "\\f"}[ch])
        elif o < 0x20 or ch in "<>&='":
            out.append("\\u%04x" % o)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def ts_order(t):
    msb, lsb, node = t
    return (msb & 0xFFFFFFFFFFFFFFFF, (lsb & 0xFFFFFFFFFFFFFFFF) >> 16, lsb & 0x1E, node)


def write_datum(d):
    kind, null, value = d
    if null:
        return '["HASH",false]' if kind == HASH else f'["{("STRING", "LONG", "DOUBLE", "HASH")[kind]}"]'
    if kind == HASH:
        return f'["HASH",true,{_i32(value)}]'
    if kind == STRING:
        return gson_string(value)
    if kind == DOUBLE:
        return java_double_to_string(value)
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


_ALPHABET = "abcXYZ019 <>&='\"\\/\t\n-_.~"


def random_double(rng):
    """a non-integral double (an integral one is read back as LONG): random bits over the whole range, or short decimals"""
    while True:
        if rng.random() < 0.5:
            x = struct.unpack(">d", struct.pack(">Q", int(rng.integers(0, 1 << 63))))[0]
            if rng.random() < 0.5:
                x = -x
        else:
            x = float(f"{int(rng.integers(-10**6, 10**6))}e{int(rng.integers(-12, 12))}")
        if math.isfinite(x) and x != math.floor(x):
            return x


def random_datum(rng, p_hash=0.25, p_null=0.03, span=None, p_string=0.0, p_double=0.0):
    if rng.random() < p_null:
        return (int(rng.choice([LONG, HASH, STRING, DOUBLE] if p_string or p_double else [LONG, HASH])), True, 0)
    if rng.random() < p_hash:
        return (HASH, False, int(rng.integers(-(1 << 31), 1 << 31)))
    if rng.random() < p_string:
        n = int(rng.integers(0, 24))
        return (STRING, False, "".join(_ALPHABET[int(i)] for i in rng.integers(0, len(_ALPHABET), size=n)))
    if rng.random() < p_double:
        return (DOUBLE, False, random_double(rng))
    v = int(rng.integers(-(1 << 62), 1 << 62)) if span is None else int(rng.integers(0, span))
    return (LONG, False, v)


def random_txn(rng):
    epoch, hlc = int(rng.integers(0, 3)), int(rng.integers(0, 500))
    kind = int(rng.choice([0, 1, 3, 4]))
    node = int(rng.choice([0, 1, 2, 3, -2]))
    return ((epoch << 15) | (hlc >> 48), (hlc << 16) | (kind << 1), node)


def random_doc(rng, n_keys=20, n_txn=30, n_entries=60, n_ranges=10, canonical=False, p_string=0.0, p_double=0.0):
    keys = [random_datum(rng, span=None if rng.random() < 0.5 else 200, p_string=p_string, p_double=p_double)
            for _ in range(n_keys)]
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
