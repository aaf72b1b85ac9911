"""Ranges algebra through the C ABI (acc_ranges_*: host code of libaccord_amd.so, no GPU context needed).

Mirrors accord.primitives.Ranges (primitives/Ranges.java, AbstractRanges.java): an immutable, sorted, deoverlapped
list of Range (start, end) u64 key codes of one bound type (end_inclusive 1 = Range.EndInclusive (s, e],
0 = Range.StartInclusive [s, e); Range.java:40-138). Method names follow the reference (`with_` for `with`).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .deps import IllegalArgumentException


class RList(C.Structure):
    _fields_ = [("start", C.c_void_p), ("end", C.c_void_p), ("n", C.c_uint32), ("reserved", C.c_uint32)]


_OUT = [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]
_SET = False


def _lib():
    global _SET
    lib = L.load()
    if not _SET:
        P = C.POINTER(RList)
        lib.acc_ranges_of.argtypes = [P] + _OUT
        lib.acc_ranges_with.argtypes = [P, P] + _OUT
        lib.acc_ranges_subtract.argtypes = [P, P] + _OUT
        lib.acc_ranges_merge_touching.argtypes = [P] + _OUT
        lib.acc_ranges_select.argtypes = [P, C.c_void_p, C.c_uint32] + _OUT
        lib.acc_ranges_index_of.argtypes = [P, C.c_uint32, C.c_uint64, C.POINTER(C.c_int64)]
        lib.acc_ranges_contains_all_keys.argtypes = [P, C.c_uint32, C.c_void_p, C.c_uint32, C.POINTER(C.c_int32)]
        lib.acc_ranges_contains_all.argtypes = [P, P, C.POINTER(C.c_int32)]
        lib.acc_rangedeps_is_covered_by.argtypes = [P, P, C.POINTER(C.c_int32)]
        for f in ("acc_ranges_of", "acc_ranges_with", "acc_ranges_subtract", "acc_ranges_merge_touching",
                  "acc_ranges_select", "acc_ranges_index_of", "acc_ranges_contains_all_keys", "acc_ranges_contains_all",
                  "acc_rangedeps_is_covered_by"):
            getattr(lib, f).restype = C.c_int
        _SET = True
    return lib


def _check(rc):
    if rc == L.ACC_E_ARG:
        raise IllegalArgumentException("Ranges: invalid argument (not sorted / deoverlapped, or out of range)")
    if rc != L.ACC_OK:
        raise RuntimeError(f"acc_ranges_*: error {rc}")


class Ranges:
    """A sorted, deoverlapped Ranges (Ranges.ofSortedAndDeoverlapped) of one bound type."""

    def __init__(self, start, end, end_inclusive: int = 1):
        self.start = np.ascontiguousarray(start, dtype=np.uint64)
        self.end = np.ascontiguousarray(end, dtype=np.uint64)
        self.end_inclusive = int(end_inclusive)

    # -- construction
    @classmethod
    def of(cls, *ranges, end_inclusive: int = 1) -> "Ranges":
        """Ranges.of(Range...): sorted by Range::compare, overlapping ranges merged (AbstractRanges.java:689-707)."""
        s = np.array([r[0] for r in ranges], np.uint64)
        e = np.array([r[1] for r in ranges], np.uint64)
        return cls._call(lambda o: _lib().acc_ranges_of(C.byref(cls._rl(s, e)), *o), len(ranges), end_inclusive)

    EMPTY = None   # set below

    @staticmethod
    def _rl(s, e):
        return RList(s.ctypes.data if len(s) else None, e.ctypes.data if len(e) else None, len(s), 0)

    def _self(self):
        return self._rl(self.start, self.end)

    @classmethod
    def _call(cls, fn, cap, ei):
        cap = max(int(cap), 1)
        s = np.zeros(cap, np.uint64)
        e = np.zeros(cap, np.uint64)
        n = C.c_uint32(0)
        _check(fn([s.ctypes.data, e.ctypes.data, cap, C.byref(n)]))
        return cls(s[:n.value].copy(), e[:n.value].copy(), ei)

    # -- algebra
    def with_(self, that: "Ranges") -> "Ranges":
        a, b = self._self(), that._self()
        return self._call(lambda o: _lib().acc_ranges_with(C.byref(a), C.byref(b), *o), len(self) + len(that),
                          self.end_inclusive)

    def subtract(self, that: "Ranges") -> "Ranges":
        a, b = self._self(), that._self()
        return self._call(lambda o: _lib().acc_ranges_subtract(C.byref(a), C.byref(b), *o), len(self) + len(that),
                          self.end_inclusive)

    def merge_touching(self) -> "Ranges":
        a = self._self()
        return self._call(lambda o: _lib().acc_ranges_merge_touching(C.byref(a), *o), len(self), self.end_inclusive)

    def select(self, indexes) -> "Ranges":
        a = self._self()
        idx = np.ascontiguousarray(indexes, dtype=np.uint32)
        return self._call(lambda o: _lib().acc_ranges_select(C.byref(a), idx.ctypes.data if len(idx) else None,
                                                             len(idx), *o), len(idx), self.end_inclusive)

    def index_of(self, key: int) -> int:
        a = self._self()
        out = C.c_int64(0)
        _check(_lib().acc_ranges_index_of(C.byref(a), self.end_inclusive, int(key), C.byref(out)))
        return out.value

    def contains(self, key: int) -> bool:
        return self.index_of(key) >= 0

    def contains_all_keys(self, keys) -> bool:
        a = self._self()
        k = np.ascontiguousarray(keys, dtype=np.uint64)
        out = C.c_int32(0)
        _check(_lib().acc_ranges_contains_all_keys(C.byref(a), self.end_inclusive, k.ctypes.data if len(k) else None,
                                                   len(k), C.byref(out)))
        return bool(out.value)

    def contains_all(self, that: "Ranges") -> bool:
        a, b = self._self(), that._self()
        out = C.c_int32(0)
        _check(_lib().acc_ranges_contains_all(C.byref(a), C.byref(b), C.byref(out)))
        return bool(out.value)

    # -- value semantics
    def __len__(self):
        return len(self.start)

    def __iter__(self):
        return iter(zip((int(x) for x in self.start), (int(x) for x in self.end)))

    def __eq__(self, other):
        return (isinstance(other, Ranges) and np.array_equal(self.start, other.start)
                and np.array_equal(self.end, other.end))

    def __repr__(self):
        o, c = ("(", "]") if self.end_inclusive else ("[", ")")
        return "[" + ", ".join(f"{o}{s},{e}{c}" for s, e in self) + "]"


Ranges.EMPTY = Ranges(np.zeros(0, np.uint64), np.zeros(0, np.uint64))


def range_deps_is_covered_by(rd_start, rd_end, covering: Ranges) -> bool:
    """RangeDeps.isCoveredBy(covering) over a RangeDeps' ranges (primitives/RangeDeps.java:595-613)."""
    s = np.ascontiguousarray(rd_start, dtype=np.uint64)
    e = np.ascontiguousarray(rd_end, dtype=np.uint64)
    a, b = Ranges._rl(s, e), covering._self()
    out = C.c_int32(0)
    _check(_lib().acc_rangedeps_is_covered_by(C.byref(a), C.byref(b), C.byref(out)))
    return bool(out.value)


def ranges_to_string(start, end, prefix, start_inclusive=True, end_inclusive=False) -> str:
    """AbstractRanges.toString (AbstractRanges.java:589-617) for keys carrying a prefix (e.g. a table): consecutive
    ranges whose end shares the first range's prefix are grouped as `prefix:[r1, r2]`, each range as
    Range.toSuffixString (Range.java:446-449). Without prefixes: Arrays.toString of the ranges."""
    o, c = ("[" if start_inclusive else "("), ("]" if end_inclusive else ")")
    sfx = [f"{o}{int(s)},{int(e)}{c}" for s, e in zip(start, end)]
    if len(sfx) == 0:
        return "[]"
    if prefix is None or prefix[0] is None:
        return "[" + ", ".join(sfx) + "]"
    out, i = [], 0
    while i < len(sfx):
        p = prefix[i]
        j = i + 1
        while j < len(sfx) and prefix[j] == p:   # the reference compares the next range's end prefix
            j += 1
        out.append(f"{p}:[" + ", ".join(sfx[i:j]) + "]")
        i = j
    return "[" + ", ".join(out) + "]"
