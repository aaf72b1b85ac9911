"""ctypes binding of the C restatement (oracle/accord_oracle.c) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module. It is the
checker, never the thing measured or shipped.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

u64p = C.POINTER(C.c_uint64)
u32p = C.POINTER(C.c_uint32)
i32p = C.POINTER(C.c_int32)
u8p = C.POINTER(C.c_uint8)


class KeydepsResult(C.Structure):
    _fields_ = [("n_txn", C.c_uint32),
                ("arena_off", u64p), ("arena", i32p),
                ("kd_off", u64p), ("key_idx", u32p),
                ("u_off", u64p), ("dep_txn", u32p),
                ("total_edges", C.c_uint64), ("visited", C.c_uint64),
                ("queried_pairs", C.c_uint64), ("build_s", C.c_double), ("query_s", C.c_double),
                ("error", C.c_int), ("message", C.c_char * 256), ("kd_key", u64p)]


class MergeResult(C.Structure):
    _fields_ = [("n_groups", C.c_uint32),
                ("key_off", u64p), ("key_code", u64p),
                ("val_off", u64p), ("txn_rank", u32p),
                ("k2v_off", u64p), ("k2v", i32p),
                ("error", C.c_int), ("message", C.c_char * 256)]


class RmmMergeResult(C.Structure):
    _fields_ = [("n_groups", C.c_uint32),
                ("key_off", u64p), ("key_a", u64p), ("key_b", u64p),
                ("val_off", u64p), ("val_src", u64p), ("val_msb", u64p), ("val_lsb", u64p), ("val_node", i32p),
                ("k2v_off", u64p), ("k2v", i32p), ("error", C.c_int), ("message", C.c_char * 256)]


class SliceResult(C.Structure):
    _fields_ = [("n_groups", C.c_uint32), ("key_off", u64p), ("key_idx", u32p), ("val_off", u64p), ("val_idx", u32p),
                ("k2v_off", u64p), ("k2v", i32p)]


class StabResult(C.Structure):
    _fields_ = [("off", u64p), ("idx", u32p)]


class RangedepsResult(C.Structure):
    _fields_ = [("n_txn", C.c_uint32),
                ("n_ranges", C.c_uint32), ("rng_start", u64p), ("rng_end", u64p),
                ("arena_off", u64p), ("arena", i32p),
                ("rd_off", u64p), ("range_id", u32p),
                ("u_off", u64p), ("dep_txn", u32p),
                ("total_edges", C.c_uint64), ("visited", C.c_uint64), ("queried", C.c_uint64),
                ("query_s", C.c_double), ("error", C.c_int), ("message", C.c_char * 256)]


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_keydeps_batch.restype = C.POINTER(KeydepsResult)
        L.orc_keydeps_batch.argtypes = [C.c_uint32, u64p, u64p, i32p, u64p, u64p, i32p, u8p, u32p, u64p,
                                        C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
        L.orc_keydeps_free.argtypes = [C.POINTER(KeydepsResult)]
        L.orc_keydeps_batch_qmask.restype = C.POINTER(KeydepsResult)
        L.orc_keydeps_batch_qmask.argtypes = [C.c_uint32, u64p, u64p, i32p, u64p, u64p, i32p, u8p, u32p, u64p, u8p]
        L.orc_keydeps_mixed.restype = C.POINTER(KeydepsResult)
        L.orc_keydeps_mixed.argtypes = [C.c_uint32, u64p, u64p, i32p, u64p, u64p, i32p, u8p, u32p, u64p,
                                        u32p, u64p, u64p, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
        L.orc_keydeps_mixed_qmask.restype = C.POINTER(KeydepsResult)
        L.orc_keydeps_mixed_qmask.argtypes = [C.c_uint32, u64p, u64p, i32p, u64p, u64p, i32p, u8p, u32p, u64p,
                                              u32p, u64p, u64p, C.c_int, u8p]
        L.orc_rangedeps_batch_qmask.restype = C.POINTER(RangedepsResult)
        L.orc_rangedeps_batch_qmask.argtypes = [C.c_uint32, u64p, u64p, i32p, u64p, u64p, i32p, u8p, u32p, u64p,
                                                u32p, u64p, u64p, C.c_int, u8p]
        L.orc_keydeps_merge.restype = C.POINTER(MergeResult)
        L.orc_keydeps_merge.argtypes = [C.c_uint32, u64p, u64p, u64p, u64p, u32p, u64p, i32p]
        L.orc_merge_free.argtypes = [C.POINTER(MergeResult)]
        L.orc_levelise.restype = C.c_int
        L.orc_levelise.argtypes = [C.c_uint32, u64p, u32p, u32p, u32p, u32p, u32p]
        L.orc_rangedeps_batch.restype = C.POINTER(RangedepsResult)
        L.orc_rangedeps_batch.argtypes = [C.c_uint32, u64p, u64p, i32p, u64p, u64p, i32p, u8p, u32p, u64p,
                                          u32p, u64p, u64p, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32]
        L.orc_rangedeps_free.argtypes = [C.POINTER(RangedepsResult)]
        L.orc_rmm_merge.restype = C.POINTER(RmmMergeResult)
        L.orc_rmm_merge.argtypes = [C.c_uint32, u64p, C.c_int, u64p, u64p, u64p, u64p, u64p, u64p, i32p, u64p, i32p]
        L.orc_rmm_merge_free.argtypes = [C.POINTER(RmmMergeResult)]
        L.orc_invert.restype = C.c_int
        L.orc_invert.argtypes = [C.c_uint32, u64p, i32p, u64p, u64p, u64p, i32p]
        L.orc_rmm_slice.restype = C.POINTER(SliceResult)
        L.orc_rmm_slice.argtypes = [C.c_uint32, C.c_int, C.c_int, u64p, u64p, u64p, u64p, u64p, i32p, u64p, u64p, u64p]
        L.orc_slice_free.argtypes = [C.POINTER(SliceResult)]
        L.orc_rmm_without.restype = C.POINTER(SliceResult)
        L.orc_rmm_without.argtypes = [C.c_uint32, u64p, u64p, u64p, i32p, u64p, u64p, i32p,
                                      u64p, u64p, u64p, i32p, u64p, u64p, u64p, i32p, u8p]
        L.orc_rmm_stab.restype = C.POINTER(StabResult)
        L.orc_rmm_stab.argtypes = [C.c_uint32, u32p, u64p, u64p, C.c_int, C.c_int, u64p, u64p, u64p]
        L.orc_stab_free.argtypes = [C.POINTER(StabResult)]
        L.orc_map_reduce_full_ranges.restype = C.POINTER(RangedepsResult)
        L.orc_map_reduce_full_ranges.argtypes = ([C.c_uint32, u64p, u64p, i32p, u64p, u64p, i32p, u8p, u8p, u32p, u64p, u64p,
                                                  C.c_int, u32p, u64p, u64p, i32p, u64p, u64p, u8p, C.c_uint32, u64p, u64p,
                                                  i32p, u8p, u32p, u64p, u64p] + [C.c_int] * 5)
        L.orc_map_reduce_full.restype = C.POINTER(KeydepsResult)
        L.orc_map_reduce_full.argtypes = [C.c_uint32, u64p, u64p, i32p, u64p, u64p, i32p, u8p, u32p, u64p, u32p, u32p,
                                          C.c_uint32, u64p, u64p, i32p, u32p, u64p,
                                          C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
        L.orc_ts_compare.restype = C.c_int
        L.orc_ts_compare.argtypes = [C.c_uint64, C.c_uint64, C.c_int32, C.c_uint64, C.c_uint64, C.c_int32]
        _lib = L
    return _lib


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(t)


@dataclass
class KeyDepsBatchOut:
    """Per-txn results in the acc_keydeps_view layout (host numpy arrays)."""
    arena_off: np.ndarray
    arena: np.ndarray
    kd_off: np.ndarray
    key_idx: np.ndarray
    u_off: np.ndarray
    dep_txn: np.ndarray
    total_edges: int = 0
    visited: int = 0
    queried_pairs: int = 0
    build_s: float = 0.0
    query_s: float = 0.0
    kd_key: np.ndarray | None = None   # KeyDeps.keys as key codes (every txn)

    def txn(self, t: int):
        a = self.arena[self.arena_off[t]:self.arena_off[t + 1]]
        k = self.key_idx[self.kd_off[t]:self.kd_off[t + 1]]
        d = self.dep_txn[self.u_off[t]:self.u_off[t + 1]]
        return k, d, a


class OracleError(RuntimeError):
    def __init__(self, code, message):
        super().__init__(f"oracle error {code}: {message}")
        self.code = code


def keydeps_batch(batch, n_shards: int = 1, query_lo: int = 0, query_hi: int | None = None,
                  query_stride: int = 1, queries=None) -> KeyDepsBatchOut:
    """orc_keydeps_batch; `queries` (txn indices) selects an explicit query set instead of lo/hi/stride."""
    L = lib()
    n = batch.n_txn
    if queries is not None:
        mask = np.zeros(max(n, 1), np.uint8)
        mask[np.asarray(queries, dtype=np.int64)] = 1
        arrs = [np.ascontiguousarray(x) for x in (batch.txn_msb.astype(np.uint64), batch.txn_lsb.astype(np.uint64),
                                                  batch.txn_node.astype(np.int32), batch.exe_msb.astype(np.uint64),
                                                  batch.exe_lsb.astype(np.uint64), batch.exe_node.astype(np.int32),
                                                  batch.status.astype(np.uint8), batch.key_off.astype(np.uint32),
                                                  batch.key_code.astype(np.uint64), mask)]
        types = [u64p, u64p, i32p, u64p, u64p, i32p, u8p, u32p, u64p, u8p]
        return _keydeps_out(L, L.orc_keydeps_batch_qmask(n, *[_p(a, t) for a, t in zip(arrs, types)]), n)
    arrs = [np.ascontiguousarray(x) for x in (batch.txn_msb.astype(np.uint64), batch.txn_lsb.astype(np.uint64),
                                              batch.txn_node.astype(np.int32), batch.exe_msb.astype(np.uint64),
                                              batch.exe_lsb.astype(np.uint64), batch.exe_node.astype(np.int32),
                                              batch.status.astype(np.uint8), batch.key_off.astype(np.uint32),
                                              batch.key_code.astype(np.uint64))]
    types = [u64p, u64p, i32p, u64p, u64p, i32p, u8p, u32p, u64p]
    r = L.orc_keydeps_batch(n, *[_p(a, t) for a, t in zip(arrs, types)], n_shards, query_lo,
                            n if query_hi is None else query_hi, query_stride)
    return _keydeps_out(L, r, n)


def keydeps_mixed(rb, n_shards: int = 1, query_lo: int = 0, query_hi: int | None = None,
                  query_stride: int = 1) -> KeyDepsBatchOut:
    """KeyDeps of every queried txn of a mixed key/range batch (accord_oracle.c orc_keydeps_mixed): key txns as
    keydeps_batch, range txns scan the CommandsForKey of every key inside their ranges."""
    L = lib()
    b = rb.keys
    n = b.n_txn
    arrs = [np.ascontiguousarray(x) for x in (b.txn_msb.astype(np.uint64), b.txn_lsb.astype(np.uint64),
                                              b.txn_node.astype(np.int32), b.exe_msb.astype(np.uint64),
                                              b.exe_lsb.astype(np.uint64), b.exe_node.astype(np.int32),
                                              b.status.astype(np.uint8), b.key_off.astype(np.uint32),
                                              b.key_code.astype(np.uint64), rb.rng_off.astype(np.uint32),
                                              rb.rng_start.astype(np.uint64), rb.rng_end.astype(np.uint64))]
    types = [u64p, u64p, i32p, u64p, u64p, i32p, u8p, u32p, u64p, u32p, u64p, u64p]
    r = L.orc_keydeps_mixed(n, *[_p(a, t) for a, t in zip(arrs, types)], int(rb.end_inclusive), n_shards,
                            query_lo, n if query_hi is None else query_hi, query_stride)
    return _keydeps_out(L, r, n)


def _mixed_arrays(rb):
    b = rb.keys
    arrs = [np.ascontiguousarray(x) for x in (b.txn_msb.astype(np.uint64), b.txn_lsb.astype(np.uint64),
                                              b.txn_node.astype(np.int32), b.exe_msb.astype(np.uint64),
                                              b.exe_lsb.astype(np.uint64), b.exe_node.astype(np.int32),
                                              b.status.astype(np.uint8), b.key_off.astype(np.uint32),
                                              b.key_code.astype(np.uint64), rb.rng_off.astype(np.uint32),
                                              rb.rng_start.astype(np.uint64), rb.rng_end.astype(np.uint64))]
    types = [u64p, u64p, i32p, u64p, u64p, i32p, u8p, u32p, u64p, u32p, u64p, u64p]
    return [_p(a, t) for a, t in zip(arrs, types)], arrs


def _qmask(n, queries):
    mask = np.zeros(max(n, 1), np.uint8)
    mask[np.asarray(queries, dtype=np.int64)] = 1
    return mask


def keydeps_mixed_queries(rb, queries) -> KeyDepsBatchOut:
    """keydeps_mixed on an explicit query set (txn indices), one snapshot build (orc_keydeps_mixed_qmask)."""
    L = lib()
    n = rb.n_txn
    ptrs, keep = _mixed_arrays(rb)
    mask = _qmask(n, queries)
    return _keydeps_out(L, L.orc_keydeps_mixed_qmask(n, *ptrs, int(rb.end_inclusive), _p(mask, u8p)), n)


def rangedeps_batch_queries(rb, queries) -> "RangeDepsBatchOut":
    """rangedeps_batch on an explicit query set (txn indices), one table build (orc_rangedeps_batch_qmask)."""
    L = lib()
    n = rb.n_txn
    ptrs, keep = _mixed_arrays(rb)
    mask = _qmask(n, queries)
    return _rangedeps_out(L, L.orc_rangedeps_batch_qmask(n, *ptrs, int(rb.end_inclusive), _p(mask, u8p)), n)


def map_reduce_full(batch, miss_off, miss_txn, queries, started_at: int, test_dep: int, test_status: int,
                    test_kinds: int = -1, exec_after: bool = False) -> KeyDepsBatchOut:
    """orc_map_reduce_full: CommandsForKey.mapReduceFull (CommandsForKey.java:553-612) per key of each recovery query,
    into a Deps.Builder (BeginRecovery.java:334-378). queries = dict(msb, lsb, node, key_off, key_code); results per
    query in the acc_keydeps_view layout (dep_txn = batch indices)."""
    L = lib()
    n = batch.n_txn
    nq = len(queries["msb"])
    arrs = [np.ascontiguousarray(x) for x in (batch.txn_msb.astype(np.uint64), batch.txn_lsb.astype(np.uint64),
                                              batch.txn_node.astype(np.int32), batch.exe_msb.astype(np.uint64),
                                              batch.exe_lsb.astype(np.uint64), batch.exe_node.astype(np.int32),
                                              batch.status.astype(np.uint8), batch.key_off.astype(np.uint32),
                                              batch.key_code.astype(np.uint64), np.asarray(miss_off, np.uint32),
                                              np.append(np.asarray(miss_txn, np.uint32), np.uint32(0)))]
    types = [u64p, u64p, i32p, u64p, u64p, i32p, u8p, u32p, u64p, u32p, u32p]
    qa = [np.ascontiguousarray(np.append(np.asarray(queries[k], dt), dt(0))) if k != "key_off" else
          np.ascontiguousarray(np.asarray(queries[k], dt))
          for k, dt in (("msb", np.uint64), ("lsb", np.uint64), ("node", np.int32), ("key_off", np.uint32),
                        ("key_code", np.uint64))]
    qt = [u64p, u64p, i32p, u32p, u64p]
    r = L.orc_map_reduce_full(n, *[_p(a, t) for a, t in zip(arrs, types)], nq, *[_p(a, t) for a, t in zip(qa, qt)],
                              started_at, test_dep, test_status, test_kinds, int(exec_after))
    return _keydeps_out(L, r, nq)


def _keydeps_out(L, r, n) -> KeyDepsBatchOut:
    try:
        R = r.contents
        if R.error:
            raise OracleError(R.error, R.message.decode())
        arena_off = np.ctypeslib.as_array(R.arena_off, (n + 1,)).copy()
        kd_off = np.ctypeslib.as_array(R.kd_off, (n + 1,)).copy()
        u_off = np.ctypeslib.as_array(R.u_off, (n + 1,)).copy()
        na, nk, nd = int(arena_off[-1]), int(kd_off[-1]), int(u_off[-1])
        out = KeyDepsBatchOut(arena_off, np.ctypeslib.as_array(R.arena, (max(na, 1),))[:na].copy(), kd_off,
                              np.ctypeslib.as_array(R.key_idx, (max(nk, 1),))[:nk].copy(), u_off,
                              np.ctypeslib.as_array(R.dep_txn, (max(nd, 1),))[:nd].copy(),
                              int(R.total_edges), int(R.visited), int(R.queried_pairs), float(R.build_s),
                              float(R.query_s),
                              np.ctypeslib.as_array(R.kd_key, (max(nk, 1),))[:nk].copy() if R.kd_key else None)
    finally:
        L.orc_keydeps_free(r)
    return out


@dataclass
class RangeDepsBatchOut:
    """Per-txn RangeDeps in the acc_rangedeps_view layout: ranges as ids into the dictionary of distinct stored
    ranges (sorted by Range.compare), rangesToTxnIds per txn, txnIds as batch indices."""
    rng_start: np.ndarray
    rng_end: np.ndarray
    arena_off: np.ndarray
    arena: np.ndarray
    rd_off: np.ndarray
    range_id: np.ndarray
    u_off: np.ndarray
    dep_txn: np.ndarray
    total_edges: int = 0
    visited: int = 0
    queried: int = 0
    query_s: float = 0.0

    def txn(self, t: int):
        a = self.arena[self.arena_off[t]:self.arena_off[t + 1]]
        r = self.range_id[self.rd_off[t]:self.rd_off[t + 1]]
        d = self.dep_txn[self.u_off[t]:self.u_off[t + 1]]
        return r, d, a


def rangedeps_batch(rb, query_lo: int = 0, query_hi: int | None = None, query_stride: int = 1) -> RangeDepsBatchOut:
    """RangeDeps of every queried txn of a mixed key/range batch (accord_oracle.c orc_rangedeps_batch)."""
    L = lib()
    b = rb.keys
    n = b.n_txn
    arrs = [np.ascontiguousarray(x) for x in (b.txn_msb.astype(np.uint64), b.txn_lsb.astype(np.uint64),
                                              b.txn_node.astype(np.int32), b.exe_msb.astype(np.uint64),
                                              b.exe_lsb.astype(np.uint64), b.exe_node.astype(np.int32),
                                              b.status.astype(np.uint8), b.key_off.astype(np.uint32),
                                              b.key_code.astype(np.uint64), rb.rng_off.astype(np.uint32),
                                              rb.rng_start.astype(np.uint64), rb.rng_end.astype(np.uint64))]
    types = [u64p, u64p, i32p, u64p, u64p, i32p, u8p, u32p, u64p, u32p, u64p, u64p]
    r = L.orc_rangedeps_batch(n, *[_p(a, t) for a, t in zip(arrs, types)], int(rb.end_inclusive), query_lo,
                              n if query_hi is None else query_hi, query_stride)
    return _rangedeps_out(L, r, n)


def _rangedeps_out(L, r, n) -> RangeDepsBatchOut:
    try:
        R = r.contents
        if R.error:
            raise OracleError(R.error, R.message.decode())
        nr = int(R.n_ranges)
        arena_off = np.ctypeslib.as_array(R.arena_off, (n + 1,)).copy()
        rd_off = np.ctypeslib.as_array(R.rd_off, (n + 1,)).copy()
        u_off = np.ctypeslib.as_array(R.u_off, (n + 1,)).copy()
        na, nk, nd = int(arena_off[-1]), int(rd_off[-1]), int(u_off[-1])
        out = RangeDepsBatchOut(np.ctypeslib.as_array(R.rng_start, (max(nr, 1),))[:nr].copy(),
                                np.ctypeslib.as_array(R.rng_end, (max(nr, 1),))[:nr].copy(),
                                arena_off, np.ctypeslib.as_array(R.arena, (max(na, 1),))[:na].copy(),
                                rd_off, np.ctypeslib.as_array(R.range_id, (max(nk, 1),))[:nk].copy(),
                                u_off, np.ctypeslib.as_array(R.dep_txn, (max(nd, 1),))[:nd].copy(),
                                int(R.total_edges), int(R.visited), int(R.queried), float(R.query_s))
    finally:
        L.orc_rangedeps_free(r)
    return out


RCMD_FIELDS = (("txn_msb", np.uint64), ("txn_lsb", np.uint64), ("txn_node", np.int32), ("exe_msb", np.uint64),
               ("exe_lsb", np.uint64), ("exe_node", np.int32), ("status", np.uint8), ("flags", np.uint8),
               ("rng_off", np.uint32), ("rng_start", np.uint64), ("rng_end", np.uint64))
RCMD_DEP_FIELDS = (("dep_off", np.uint32), ("dep_msb", np.uint64), ("dep_lsb", np.uint64), ("dep_node", np.int32),
                   ("dep_start", np.uint64), ("dep_end", np.uint64), ("dep_is_key", np.uint8))
RQ_FIELDS = (("msb", np.uint64), ("lsb", np.uint64), ("node", np.int32), ("is_range", np.uint8), ("part_off", np.uint32),
             ("part_start", np.uint64), ("part_end", np.uint64))
_CT = {np.uint64: u64p, np.uint32: u32p, np.int32: i32p, np.uint8: u8p}


def map_reduce_full_ranges(cmds: dict, queries: dict, started_at: int, test_dep: int, test_status: int,
                           test_kinds: int = -1, exec_after: bool = False) -> RangeDepsBatchOut:
    """orc_map_reduce_full_ranges: InMemorySafeStore.mapReduceRangesInternal (impl/InMemoryCommandStore.java:883-1016)
    per recovery query into a Deps.Builder (BeginRecovery.java:334-378). cmds / queries: dicts of the RCMD_FIELDS /
    RCMD_DEP_FIELDS / RQ_FIELDS arrays plus cmds["end_inclusive"]; results per query in the rangedeps layout."""
    L = lib()
    n = len(cmds["txn_msb"])
    nq = len(queries["msb"])
    pad = lambda k, dt, src: np.ascontiguousarray(np.append(np.asarray(src[k], dt), dt(0)))  # noqa: E731
    a1 = [pad(k, dt, cmds) for k, dt in RCMD_FIELDS]
    a2 = [pad(k, dt, cmds) for k, dt in RCMD_DEP_FIELDS]
    aq = [pad(k, dt, queries) for k, dt in RQ_FIELDS]
    r = L.orc_map_reduce_full_ranges(n, *[_p(a, _CT[dt]) for a, (_, dt) in zip(a1, RCMD_FIELDS)], int(cmds["end_inclusive"]),
                                     *[_p(a, _CT[dt]) for a, (_, dt) in zip(a2, RCMD_DEP_FIELDS)], nq,
                                     *[_p(a, _CT[dt]) for a, (_, dt) in zip(aq, RQ_FIELDS)],
                                     started_at, test_dep, test_status, test_kinds, int(exec_after))
    return _rangedeps_out(L, r, nq)


CFK_SNAP = (("key", np.uint64), ("ent_off", np.uint32), ("emsb", np.uint64), ("elsb", np.uint64), ("enode", np.int32),
            ("xmsb", np.uint64), ("xlsb", np.uint64), ("xnode", np.int32), ("status", np.uint8), ("miss_off", np.uint32),
            ("mmsb", np.uint64), ("mlsb", np.uint64), ("mnode", np.int32))
CFK_UPD = (("msb", np.uint64), ("lsb", np.uint64), ("node", np.int32), ("xmsb", np.uint64), ("xlsb", np.uint64),
           ("xnode", np.int32), ("status", np.uint8), ("flags", np.uint8), ("key_off", np.uint32), ("key", np.uint64),
           ("dep_off", np.uint32), ("dmsb", np.uint64), ("dlsb", np.uint64), ("dnode", np.int32))


class CfkResult(C.Structure):
    _fields_ = [("n_keys", C.c_uint32), ("key", u64p), ("ent_off", u32p), ("emsb", u64p), ("elsb", u64p),
                ("enode", i32p), ("xmsb", u64p), ("xlsb", u64p), ("xnode", i32p), ("status", u8p), ("miss_off", u32p),
                ("mmsb", u64p), ("mlsb", u64p), ("mnode", i32p), ("n_entries", C.c_uint64), ("n_missing", C.c_uint64),
                ("error", C.c_int), ("message", C.c_char * 256)]


def cfk_apply(snap: dict, upd: dict) -> dict:
    """orc_cfk_apply: CommandsForKey.update with each command's deps (local/CommandsForKey.java:657-1149) for a batch of
    updates against a key-major snapshot (CFK_SNAP arrays; empty: key of length 0 and ent_off = [0]). Returns the
    new key-major snapshot as a dict of the same arrays."""
    L = lib()
    if not hasattr(L.orc_cfk_apply, "_set"):
        L.orc_cfk_apply.restype = C.POINTER(CfkResult)
        L.orc_cfk_apply.argtypes = ([C.c_uint32] + [_CT[dt] for _, dt in CFK_SNAP] + [C.c_uint32] +
                                    [_CT[dt] for _, dt in CFK_UPD])
        L.orc_cfk_free.argtypes = [C.POINTER(CfkResult)]
        L.orc_cfk_apply._set = True
    pad = lambda src, k, dt: np.ascontiguousarray(np.append(np.asarray(src[k], dt), dt(0)))  # noqa: E731
    sa = [pad(snap, k, dt) for k, dt in CFK_SNAP]
    ua = [pad(upd, k, dt) for k, dt in CFK_UPD]
    nk = len(snap["key"])
    nu = len(upd["msb"])
    r = L.orc_cfk_apply(nk, *[_p(a, _CT[dt]) for a, (_, dt) in zip(sa, CFK_SNAP)], nu,
                        *[_p(a, _CT[dt]) for a, (_, dt) in zip(ua, CFK_UPD)])
    try:
        R = r.contents
        if R.error:
            raise OracleError(R.error, R.message.decode())
        k, ne, nm = int(R.n_keys), int(R.n_entries), int(R.n_missing)
        arr = lambda p, n, dt: np.ctypeslib.as_array(p, (max(n, 1),))[:n].astype(dt).copy()  # noqa: E731
        out = dict(key=arr(R.key, k, np.uint64), ent_off=arr(R.ent_off, k + 1, np.uint32))
        for f, dt in (("emsb", np.uint64), ("elsb", np.uint64), ("enode", np.int32), ("xmsb", np.uint64),
                      ("xlsb", np.uint64), ("xnode", np.int32), ("status", np.uint8)):
            out[f] = arr(getattr(R, f), ne, dt)
        out["miss_off"] = arr(R.miss_off, ne + 1, np.uint32)
        for f, dt in (("mmsb", np.uint64), ("mlsb", np.uint64), ("mnode", np.int32)):
            out[f] = arr(getattr(R, f), nm, dt)
    finally:
        L.orc_cfk_free(r)
    return out


MC_UPD = (("xmsb", np.uint64), ("xlsb", np.uint64), ("xnode", np.int32), ("key_off", np.uint32), ("key", np.uint64),
          ("rng_off", np.uint32), ("rng_start", np.uint64), ("rng_end", np.uint64))
MC_Q = (("msb", np.uint64), ("lsb", np.uint64), ("node", np.int32), ("is_range", np.uint8), ("part_off", np.uint32),
        ("part_start", np.uint64), ("part_end", np.uint64))


def max_conflicts(upd: dict, q: dict) -> dict:
    """orc_max_conflicts: MaxConflicts.get(keys) over the updates (local/MaxConflicts.java:31-96) and the fast-path
    test of CommandStore.preaccept (local/CommandStore.java:320-345) per query: dict(msb, lsb, node, fast)."""
    L = lib()
    if not hasattr(L.orc_max_conflicts, "_set"):
        L.orc_max_conflicts.restype = C.c_int
        L.orc_max_conflicts.argtypes = ([C.c_uint32] + [_CT[dt] for _, dt in MC_UPD] + [C.c_int, C.c_uint32] +
                                        [_CT[dt] for _, dt in MC_Q] + [u64p, u64p, i32p, u8p])
        L.orc_max_conflicts._set = True
    pad = lambda src, k, dt: np.ascontiguousarray(np.append(np.asarray(src[k], dt), dt(0)))  # noqa: E731
    ua = [pad(upd, k, dt) for k, dt in MC_UPD]
    qa = [pad(q, k, dt) for k, dt in MC_Q]
    nq = len(q["msb"])
    out = dict(msb=np.zeros(nq + 1, np.uint64), lsb=np.zeros(nq + 1, np.uint64), node=np.zeros(nq + 1, np.int32),
               fast=np.zeros(nq + 1, np.uint8))
    L.orc_max_conflicts(len(upd["xmsb"]), *[_p(a, _CT[dt]) for a, (_, dt) in zip(ua, MC_UPD)], int(upd["end_inclusive"]),
                        nq, *[_p(a, _CT[dt]) for a, (_, dt) in zip(qa, MC_Q)], _p(out["msb"], u64p), _p(out["lsb"], u64p),
                        _p(out["node"], i32p), _p(out["fast"], u8p))
    return {k: v[:nq] for k, v in out.items()}


def keydeps_merge(m: dict) -> dict:
    """KeyDeps.merge per group over the acc_merge_in layout dict (grp_off, key_off, key_code, val_off,
    txn_rank, k2v_off, k2v). Returns the same-named merged arrays per group."""
    L = lib()
    g = len(m["grp_off"]) - 1
    a = {k: np.ascontiguousarray(v) for k, v in m.items()}
    r = L.orc_keydeps_merge(g, _p(a["grp_off"], u64p), _p(a["key_off"], u64p), _p(a["key_code"], u64p),
                            _p(a["val_off"], u64p), _p(a["txn_rank"], u32p), _p(a["k2v_off"], u64p),
                            _p(a["k2v"], i32p))
    try:
        R = r.contents
        if R.error:
            raise OracleError(R.error, R.message.decode())
        ko = np.ctypeslib.as_array(R.key_off, (g + 1,)).copy()
        vo = np.ctypeslib.as_array(R.val_off, (g + 1,)).copy()
        oo = np.ctypeslib.as_array(R.k2v_off, (g + 1,)).copy()
        out = dict(key_off=ko, val_off=vo, k2v_off=oo,
                   key_code=np.ctypeslib.as_array(R.key_code, (max(int(ko[-1]), 1),))[:int(ko[-1])].copy(),
                   txn_rank=np.ctypeslib.as_array(R.txn_rank, (max(int(vo[-1]), 1),))[:int(vo[-1])].copy(),
                   k2v=np.ctypeslib.as_array(R.k2v, (max(int(oo[-1]), 1),))[:int(oo[-1])].copy())
    finally:
        L.orc_merge_free(r)
    return out


def levelise(off: np.ndarray, dep: np.ndarray, exec_rank: np.ndarray):
    L = lib()
    n = len(exec_rank)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    dep = np.ascontiguousarray(dep, dtype=np.uint32)
    er = np.ascontiguousarray(exec_rank, dtype=np.uint32)
    level = np.zeros(n, dtype=np.uint32)
    order = np.zeros(n, dtype=np.uint32)
    nl = np.zeros(1, dtype=np.uint32)
    rc = L.orc_levelise(n, _p(off, u64p), _p(dep, u32p), _p(er, u32p), _p(level, u32p), _p(order, u32p),
                        _p(nl, u32p))
    if rc:
        raise OracleError(rc, "levelise: dep out of range")
    return level, order, int(nl[0])


def ts_compare(a, b) -> int:
    return lib().orc_ts_compare(*a, *b)


def _arr(ptr, n, dt):
    return np.ctypeslib.as_array(ptr, (max(int(n), 1),))[:int(n)].astype(dt, copy=True)


def rmm_merge(grp_off, half: dict, is_range: bool) -> dict:
    """KeyDeps.merge / RangeDeps.merge per group over raw TxnIds (accord_oracle_rmm.c orc_rmm_merge). `half` holds
    key_off, key_a, [key_b], val_off, msb, lsb, node, k2v_off, k2v (the acc_rmm_in layout)."""
    L = lib()
    grp_off = np.ascontiguousarray(grp_off, dtype=np.uint64)
    g = len(grp_off) - 1
    a = {k: np.ascontiguousarray(half[k], dtype=dt) for k, dt in
         (("key_off", np.uint64), ("key_a", np.uint64), ("val_off", np.uint64), ("msb", np.uint64), ("lsb", np.uint64),
          ("node", np.int32), ("k2v_off", np.uint64), ("k2v", np.int32))}
    kb = np.ascontiguousarray(half["key_b"], dtype=np.uint64) if is_range else None
    r = L.orc_rmm_merge(g, _p(grp_off, u64p), int(is_range), _p(a["key_off"], u64p), _p(a["key_a"], u64p),
                        _p(kb, u64p) if kb is not None else None, _p(a["val_off"], u64p), _p(a["msb"], u64p),
                        _p(a["lsb"], u64p), _p(a["node"], i32p), _p(a["k2v_off"], u64p), _p(a["k2v"], i32p))
    try:
        R = r.contents
        if R.error:
            raise OracleError(R.error, R.message.decode())
        ko = _arr(R.key_off, g + 1, np.uint64)
        vo = _arr(R.val_off, g + 1, np.uint64)
        oo = _arr(R.k2v_off, g + 1, np.uint64)
        nk, nv, no = int(ko[-1]), int(vo[-1]), int(oo[-1])
        out = dict(key_off=ko, val_off=vo, k2v_off=oo, key_a=_arr(R.key_a, nk, np.uint64),
                   src=_arr(R.val_src, nv, np.uint64), msb=_arr(R.val_msb, nv, np.uint64),
                   lsb=_arr(R.val_lsb, nv, np.uint64), node=_arr(R.val_node, nv, np.int32), k2v=_arr(R.k2v, no, np.int32))
        if is_range:
            out["key_b"] = _arr(R.key_b, nk, np.uint64)
    finally:
        L.orc_rmm_merge_free(r)
    return out


def invert(src_off, src, nsrc, ntrg):
    """RelationMultiMap.invert per group (accord_oracle_rmm.c orc_invert): returns (trg_off, trg)."""
    L = lib()
    src_off = np.ascontiguousarray(src_off, dtype=np.uint64)
    src = np.ascontiguousarray(src, dtype=np.int32)
    nsrc = np.ascontiguousarray(nsrc, dtype=np.uint64)
    ntrg = np.ascontiguousarray(ntrg, dtype=np.uint64)
    g = len(src_off) - 1
    total = int(ntrg.sum()) + int(src_off[-1]) - int(nsrc.sum())
    trg_off = np.zeros(g + 1, np.uint64)
    trg = np.zeros(max(total, 1), np.int32)
    rc = L.orc_invert(g, _p(src_off, u64p), _p(src, i32p), _p(nsrc, u64p), _p(ntrg, u64p), _p(trg_off, u64p),
                      _p(trg, i32p))
    if rc:
        raise OracleError(rc, "invert: entry out of range")
    return trg_off, trg[:total]


def rmm_slice(m: dict, sel_off, sel_s, sel_e, is_range: bool, end_inclusive: bool) -> dict:
    """KeyDeps.slice / RangeDeps.slice + trimUnusedValues per group (accord_oracle_rmm.c orc_rmm_slice)."""
    L = lib()
    a = {k: np.ascontiguousarray(m[k], dtype=dt) for k, dt in
         (("key_off", np.uint64), ("key_a", np.uint64), ("val_off", np.uint64), ("k2v_off", np.uint64), ("k2v", np.int32))}
    kb = np.ascontiguousarray(m["key_b"], dtype=np.uint64) if is_range else None
    so, ss, se = (np.ascontiguousarray(x, dtype=np.uint64) for x in (sel_off, sel_s, sel_e))
    g = len(a["key_off"]) - 1
    r = L.orc_rmm_slice(g, int(is_range), int(end_inclusive), _p(a["key_off"], u64p), _p(a["key_a"], u64p),
                        _p(kb, u64p) if kb is not None else None, _p(a["val_off"], u64p), _p(a["k2v_off"], u64p),
                        _p(a["k2v"], i32p), _p(so, u64p), _p(ss, u64p), _p(se, u64p))
    try:
        R = r.contents
        ko, vo, oo = (_arr(x, g + 1, np.uint64) for x in (R.key_off, R.val_off, R.k2v_off))
        out = dict(key_off=ko, val_off=vo, k2v_off=oo, key_idx=_arr(R.key_idx, ko[-1], np.uint32),
                   val_idx=_arr(R.val_idx, vo[-1], np.uint32), k2v=_arr(R.k2v, oo[-1], np.int32))
    finally:
        L.orc_slice_free(r)
    return out


def rmm_without(m: dict, set_a=None, set_b=None) -> dict:
    """RelationMultiMap.remove = KeyDeps/RangeDeps.without per group (accord_oracle_rmm.c orc_rmm_without). m: one deps
    half per group (key_off, val_off, k2v_off, k2v, msb, lsb, node); set_a / set_b: dict(off, msb, lsb, node) or None.
    Returns the slice-shaped result plus kind[g] (0 from, 1 none, 2 rebuilt)."""
    L = lib()
    a = {k: np.ascontiguousarray(m[k], dtype=dt) for k, dt in
         (("key_off", np.uint64), ("val_off", np.uint64), ("k2v_off", np.uint64), ("k2v", np.int32),
          ("msb", np.uint64), ("lsb", np.uint64), ("node", np.int32))}
    g = len(a["key_off"]) - 1

    def sp(x):
        if x is None:
            return (None,) * 4, None
        y = {k: np.ascontiguousarray(x[k], dtype=dt) for k, dt in
             (("off", np.uint64), ("msb", np.uint64), ("lsb", np.uint64), ("node", np.int32))}
        return (_p(y["off"], u64p), _p(y["msb"], u64p), _p(y["lsb"], u64p), _p(y["node"], i32p)), y
    pa, ka = sp(set_a)
    pb, kb = sp(set_b)
    kind = np.zeros(max(g, 1), np.uint8)
    r = L.orc_rmm_without(g, _p(a["key_off"], u64p), _p(a["val_off"], u64p), _p(a["k2v_off"], u64p), _p(a["k2v"], i32p),
                          _p(a["msb"], u64p), _p(a["lsb"], u64p), _p(a["node"], i32p), *pa, *pb, _p(kind, u8p))
    try:
        R = r.contents
        ko, vo, oo = (_arr(x, g + 1, np.uint64) for x in (R.key_off, R.val_off, R.k2v_off))
        out = dict(key_off=ko, val_off=vo, k2v_off=oo, key_idx=_arr(R.key_idx, ko[-1], np.uint32),
                   val_idx=_arr(R.val_idx, vo[-1], np.uint32), k2v=_arr(R.k2v, oo[-1], np.int32), kind=kind[:g].copy())
    finally:
        L.orc_slice_free(r)
    del ka, kb
    return out


def rmm_stab(grp, qs, qe, is_key_query: bool, end_inclusive: bool, rng_off, rs, re):
    """Stabbing queries over built RangeDeps (accord_oracle_rmm.c orc_rmm_stab): (off, ascending range indices)."""
    L = lib()
    grp = np.ascontiguousarray(grp, dtype=np.uint32)
    qs = np.ascontiguousarray(qs, dtype=np.uint64)
    qe = np.ascontiguousarray(qe if qe is not None else qs, dtype=np.uint64)
    ro, rs_, re_ = (np.ascontiguousarray(x, dtype=np.uint64) for x in (rng_off, rs, re))
    n = len(grp)
    r = L.orc_rmm_stab(n, _p(grp, u32p), _p(qs, u64p), _p(qe, u64p), int(is_key_query), int(end_inclusive),
                       _p(ro, u64p), _p(rs_, u64p), _p(re_, u64p))
    try:
        R = r.contents
        off = _arr(R.off, n + 1, np.uint64)
        idx = _arr(R.idx, off[-1], np.uint32)
    finally:
        L.orc_stab_free(r)
    return off, idx
