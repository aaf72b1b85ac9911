"""Host-side mirror of the reference deps API over the C ABI (include/accord_amd.h).

Names and error behaviour follow accord-core: ``KeyDeps`` (primitives/KeyDeps.java) with the Java
three-array layout, ``calculate_partial_deps`` for a whole batch (messages/PreAccept.java:245-265 over
local/CommandsForKey.java:614-650), ``KeyDeps.merge`` (primitives/KeyDeps.java:115-135). Errors map to
``IllegalArgumentException`` / ``IllegalStateException`` like utils/Invariants.java:98-205.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L


class AccordError(RuntimeError):
    code = None


class IllegalArgumentException(AccordError):
    code = L.ACC_E_ARG


class IllegalStateException(AccordError):
    code = L.ACC_E_STATE


class DeviceError(AccordError):
    code = L.ACC_E_DEVICE


class CapacityError(AccordError):
    code = L.ACC_E_CAP


_ERRORS = {L.ACC_E_ARG: IllegalArgumentException, L.ACC_E_STATE: IllegalStateException,
           L.ACC_E_DEVICE: DeviceError, L.ACC_E_NOMEM: DeviceError, L.ACC_E_CAP: CapacityError}


def _ptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data)


class Context:
    """One acc_ctx: a HIP stream plus device scratch (one per host thread / CommandStore)."""

    LV_TIERS = {"auto": 0, "lds": 1, "windowed": 2, "waves": 3}

    def __init__(self, device: int = 0, timing: bool = False, force_replay: bool = False, *, cfk_hot: int = 0,
                 lv_tier: str = "auto", lv_chunk: int = 0, no_window_tier: bool = False, rd_wide_sort: bool = False,
                 pd_serial: bool = False):
        """acc_opts, fixed for the context's life (the library reads no environment): timing = per-kernel HIP events;
        the rest force code paths for tests (force_replay: the exact replay scan; cfk_hot: the closed-form threshold of
        acc_cfk_apply; lv_tier / lv_chunk: the levelise walk; no_window_tier: the KeyDeps sorting tiers; rd_wide_sort:
        RangeDeps 64-bit sort keys) or trade speed for memory (pd_serial: acc_partial_deps_batch on one buffer set)."""
        self.timing_enabled = timing
        self.device = device
        self._lib = L.load()
        h = C.c_void_p()
        flags = ((L.ACC_OPT_TIMING if timing else 0) | (L.ACC_OPT_FORCE_REPLAY if force_replay else 0) |
                 (L.ACC_OPT_NO_WINDOW_TIER if no_window_tier else 0) | (L.ACC_OPT_RD_WIDE_SORT if rd_wide_sort else 0) |
                 (L.ACC_OPT_PD_SERIAL if pd_serial else 0))
        opts = L.Opts(flags, 0, int(cfk_hot), self.LV_TIERS[lv_tier], int(lv_chunk), 0)
        rc = self._lib.acc_create(device, C.byref(opts), C.byref(h))
        if rc != L.ACC_OK:
            raise _ERRORS.get(rc, AccordError)(f"acc_create failed ({rc})")
        self._h = h
        self._keep = []

    def close(self):
        if getattr(self, "_h", None):
            self._lib.acc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    @property
    def stream(self) -> int:
        return int(self._lib.acc_stream(self._h) or 0)

    def check(self, rc: int):
        if rc != L.ACC_OK:
            msg = (self._lib.acc_last_error(self._h) or b"").decode()
            raise _ERRORS.get(rc, AccordError)(msg)

    def sync(self):
        self.check(self._lib.acc_sync(self._h))

    # ---- timing
    def timing(self) -> dict:
        n = self._lib.acc_timing_count(self._h)
        out = {}
        for i in range(max(n, 0)):
            name = C.c_char_p()
            ms = C.c_double()
            cnt = C.c_uint64()
            self._lib.acc_timing_get(self._h, i, C.byref(name), C.byref(ms), C.byref(cnt))
            out[name.value.decode()] = (ms.value, cnt.value)
        return out

    def stats(self) -> dict:
        out = {}
        for i in range(max(self._lib.acc_stats_count(self._h), 0)):
            name = C.c_char_p()
            val = C.c_uint64()
            self._lib.acc_stats_get(self._h, i, C.byref(name), C.byref(val))
            out[name.value.decode()] = val.value
        return out

    def timing_reset(self):
        self._lib.acc_timing_reset(self._h)

    def timing_filter(self, tags=None):
        """Time only the launches with these tags (None: every launch; ACC_OPT_TIMING contexts)."""
        self.check(self._lib.acc_timing_filter(self._h, ",".join(tags).encode() if tags else None))

    # ---- KeyDeps batch
    def keydeps_batch_raw(self, batch_in: "L.BatchIn") -> "L.KeydepsView":
        view = L.KeydepsView()
        self.check(self._lib.acc_keydeps_batch(self._h, C.byref(batch_in), C.byref(view)))
        return view

    def calculate_partial_deps(self, batch) -> "BatchKeyDeps":
        """PreAccept.calculatePartialDeps for every txn of `batch` (host numpy arrays in, host out)."""
        arrs = dict(tm=np.ascontiguousarray(batch.txn_msb, dtype=np.uint64),
                    tl=np.ascontiguousarray(batch.txn_lsb, dtype=np.uint64),
                    tn=np.ascontiguousarray(batch.txn_node, dtype=np.int32),
                    em=np.ascontiguousarray(batch.exe_msb, dtype=np.uint64),
                    el=np.ascontiguousarray(batch.exe_lsb, dtype=np.uint64),
                    en=np.ascontiguousarray(batch.exe_node, dtype=np.int32),
                    st=np.ascontiguousarray(batch.status, dtype=np.uint8),
                    ko=np.ascontiguousarray(batch.key_off, dtype=np.uint32),
                    kc=np.ascontiguousarray(batch.key_code, dtype=np.uint64))
        n = int(arrs["st"].shape[0])
        bi = L.BatchIn(n, L.ACC_MEM_HOST, int(arrs["ko"][-1]) if n else 0,
                       L.TsCols(arrs["tm"].ctypes.data, arrs["tl"].ctypes.data, arrs["tn"].ctypes.data),
                       L.TsCols(arrs["em"].ctypes.data, arrs["el"].ctypes.data, arrs["en"].ctypes.data),
                       arrs["st"].ctypes.data, arrs["ko"].ctypes.data, arrs["kc"].ctypes.data)
        view = self.keydeps_batch_raw(bi)
        return self.copy_out(view, batch)

    # ---- RangeDeps batch
    def range_batch_in(self, rb, keep: list) -> "L.RangeBatchIn":
        b = rb.keys
        a = dict(tm=np.ascontiguousarray(b.txn_msb, dtype=np.uint64), tl=np.ascontiguousarray(b.txn_lsb, dtype=np.uint64),
                 tn=np.ascontiguousarray(b.txn_node, dtype=np.int32), em=np.ascontiguousarray(b.exe_msb, dtype=np.uint64),
                 el=np.ascontiguousarray(b.exe_lsb, dtype=np.uint64), en=np.ascontiguousarray(b.exe_node, dtype=np.int32),
                 st=np.ascontiguousarray(b.status, dtype=np.uint8), ko=np.ascontiguousarray(b.key_off, dtype=np.uint32),
                 kc=np.ascontiguousarray(b.key_code, dtype=np.uint64), ro=np.ascontiguousarray(rb.rng_off, dtype=np.uint32),
                 rs=np.ascontiguousarray(rb.rng_start, dtype=np.uint64), re=np.ascontiguousarray(rb.rng_end, dtype=np.uint64))
        keep.append(a)
        n = int(a["st"].shape[0])
        p = lambda k: a[k].ctypes.data  # noqa: E731
        return L.RangeBatchIn(n, L.ACC_MEM_HOST, int(a["ko"][-1]) if n else 0, int(a["ro"][-1]) if n else 0,
                              L.TsCols(p("tm"), p("tl"), p("tn")), L.TsCols(p("em"), p("el"), p("en")),
                              p("st"), p("ko"), p("kc"), p("ro"), p("rs"), p("re"), int(rb.end_inclusive), 0)

    def rangedeps_batch_raw(self, batch_in: "L.RangeBatchIn") -> "L.RangedepsView":
        view = L.RangedepsView()
        self.check(self._lib.acc_rangedeps_batch(self._h, C.byref(batch_in), C.byref(view)))
        return view

    def calculate_partial_range_deps(self, rb) -> "BatchRangeDeps":
        """PartialDeps.rangeDeps of PreAccept.calculatePartialDeps for every txn of a mixed key/range batch
        (InMemoryCommandStore.mapReduceRangesInternal, impl/InMemoryCommandStore.java:883-1016)."""
        keep = []
        view = self.rangedeps_batch_raw(self.range_batch_in(rb, keep))
        return self.copy_out_range(view)

    def keydeps_mixed_raw(self, batch_in: "L.RangeBatchIn") -> "L.KeydepsView":
        view = L.KeydepsView()
        self.check(self._lib.acc_keydeps_mixed(self._h, C.byref(batch_in), C.byref(view)))
        return view

    def calculate_partial_key_deps_mixed(self, rb) -> "BatchKeyDeps":
        """PartialDeps.keyDeps of PreAccept.calculatePartialDeps for every txn of a mixed key/range batch: key txns as
        calculate_partial_deps, range txns over every CommandsForKey inside their ranges
        (InMemoryCommandStore.mapReduceForKey, impl/InMemoryCommandStore.java:274-289). kd_key holds the key codes."""
        keep = []
        view = self.keydeps_mixed_raw(self.range_batch_in(rb, keep))
        return self.copy_out(view, rb.keys)

    def map_reduce_full(self, batch, missing_off, missing_txn, queries: dict, started_at: int, test_dep: int,
                        test_status: int, test_kinds: int = -1, executes_after: bool = False) -> "BatchKeyDeps":
        """SafeCommandStore.mapReduceFull (local/CommandsForKey.java:553-612 per key) for a batch of recovery queries
        against the CommandsForKey snapshot `batch` (acc_map_reduce_full). queries = dict(msb, lsb, node, key_off,
        key_code): the testTxnId and keys of each query; missing_off / missing_txn: per input pair of `batch`, the
        entry's missing[] TxnIds as batch indices sorted by TxnId. Tests are TestStartedAt / TestDep / TestStatus
        ordinals (ACC_STARTED_* / ACC_DEP_* / ACC_STATUS_*). Returns the per-query Deps.Builder KeyDeps."""
        keep = []
        a = dict(tm=np.ascontiguousarray(batch.txn_msb, dtype=np.uint64), tl=np.ascontiguousarray(batch.txn_lsb, dtype=np.uint64),
                 tn=np.ascontiguousarray(batch.txn_node, dtype=np.int32), em=np.ascontiguousarray(batch.exe_msb, dtype=np.uint64),
                 el=np.ascontiguousarray(batch.exe_lsb, dtype=np.uint64), en=np.ascontiguousarray(batch.exe_node, dtype=np.int32),
                 st=np.ascontiguousarray(batch.status, dtype=np.uint8), ko=np.ascontiguousarray(batch.key_off, dtype=np.uint32),
                 kc=np.ascontiguousarray(batch.key_code, dtype=np.uint64),
                 mo=np.ascontiguousarray(missing_off, dtype=np.uint32), mt=np.ascontiguousarray(missing_txn, dtype=np.uint32),
                 qm=np.ascontiguousarray(queries["msb"], dtype=np.uint64), ql=np.ascontiguousarray(queries["lsb"], dtype=np.uint64),
                 qn=np.ascontiguousarray(queries["node"], dtype=np.int32),
                 qo=np.ascontiguousarray(queries["key_off"], dtype=np.uint32),
                 qk=np.ascontiguousarray(queries["key_code"], dtype=np.uint64))
        keep.append(a)
        p = lambda k: a[k].ctypes.data  # noqa: E731
        n = int(a["st"].shape[0])
        bi = L.BatchIn(n, L.ACC_MEM_HOST, int(a["ko"][-1]) if n else 0, L.TsCols(p("tm"), p("tl"), p("tn")),
                       L.TsCols(p("em"), p("el"), p("en")), p("st"), p("ko"), p("kc"))
        ri = L.RecoveryIn(len(a["qm"]), L.ACC_MEM_HOST, L.TsCols(p("qm"), p("ql"), p("qn")), p("qo"), p("qk"), p("mo"),
                          p("mt"), len(a["mt"]), started_at, test_dep, test_status,
                          L.ACC_FULL_EXECUTES_AFTER if executes_after else 0, test_kinds)
        view = L.KeydepsView()
        self.check(self._lib.acc_map_reduce_full(self._h, C.byref(bi), C.byref(ri), C.byref(view)))
        return self.copy_out(view, None)

    def map_reduce_full_ranges(self, cmds: dict, queries: dict, started_at: int, test_dep: int, test_status: int,
                               test_kinds: int = -1, executes_after: bool = False) -> "BatchRangeDeps":
        """The range-command half of SafeCommandStore.mapReduceFull: InMemorySafeStore.mapReduceRangesInternal
        (impl/InMemoryCommandStore.java:883-1016) for a batch of recovery queries (acc_map_reduce_full_ranges).
        cmds: the store's range-command table sorted by TxnId (txn_*, exe_*, status = Status ordinals, flags =
        ACC_RCMD_*, rng_off/rng_start/rng_end, dep_off/dep_msb/dep_lsb/dep_node/dep_start/dep_end/dep_is_key =
        each command's PartialDeps as (TxnId, participant) pairs sorted by TxnId, end_inclusive); queries: msb, lsb,
        node, is_range, part_off, part_start, part_end (the sliced keys or ranges). Returns per query the Deps.Builder
        RangeDeps (dep_txn = first table index of the TxnId)."""
        def arr(src, k, dt):
            return np.ascontiguousarray(np.asarray(src[k], dtype=dt))
        c = {k: arr(cmds, k, dt) for k, dt in (("txn_msb", np.uint64), ("txn_lsb", np.uint64), ("txn_node", np.int32),
                                               ("exe_msb", np.uint64), ("exe_lsb", np.uint64), ("exe_node", np.int32),
                                               ("status", np.uint8), ("flags", np.uint8), ("rng_off", np.uint32),
                                               ("rng_start", np.uint64), ("rng_end", np.uint64), ("dep_off", np.uint32),
                                               ("dep_msb", np.uint64), ("dep_lsb", np.uint64), ("dep_node", np.int32),
                                               ("dep_start", np.uint64), ("dep_end", np.uint64), ("dep_is_key", np.uint8))}
        q = {k: arr(queries, k, dt) for k, dt in (("msb", np.uint64), ("lsb", np.uint64), ("node", np.int32),
                                                  ("is_range", np.uint8), ("part_off", np.uint32),
                                                  ("part_start", np.uint64), ("part_end", np.uint64))}
        p = lambda d, k: d[k].ctypes.data  # noqa: E731
        ci = L.RangeCmdsIn(len(c["txn_msb"]), L.ACC_MEM_HOST, int(cmds["end_inclusive"]),
                           L.TsCols(p(c, "txn_msb"), p(c, "txn_lsb"), p(c, "txn_node")),
                           L.TsCols(p(c, "exe_msb"), p(c, "exe_lsb"), p(c, "exe_node")), p(c, "status"), p(c, "flags"),
                           p(c, "rng_off"), p(c, "rng_start"), p(c, "rng_end"), p(c, "dep_off"),
                           L.TsCols(p(c, "dep_msb"), p(c, "dep_lsb"), p(c, "dep_node")), p(c, "dep_start"),
                           p(c, "dep_end"), p(c, "dep_is_key"))
        ri = L.RecoveryRangesIn(len(q["msb"]), L.ACC_MEM_HOST, L.TsCols(p(q, "msb"), p(q, "lsb"), p(q, "node")),
                                p(q, "is_range"), p(q, "part_off"), p(q, "part_start"), p(q, "part_end"), started_at,
                                test_dep, test_status, L.ACC_FULL_EXECUTES_AFTER if executes_after else 0, test_kinds)
        view = L.RangedepsView()
        self.check(self._lib.acc_map_reduce_full_ranges(self._h, C.byref(ci), C.byref(ri), C.byref(view)))
        return self.copy_out_range(view)

    def partial_deps_batch_raw(self, batch_in: "L.RangeBatchIn"):
        kv, rv = L.KeydepsView(), L.RangedepsView()
        self.check(self._lib.acc_partial_deps_batch(self._h, C.byref(batch_in), C.byref(kv), C.byref(rv)))
        return kv, rv

    def calculate_partial_deps_mixed(self, rb):
        """The whole PartialDeps (KeyDeps, RangeDeps) of every txn of a mixed key/range batch in one call
        (acc_partial_deps_batch): PreAccept.calculatePartialDeps through PartialDeps.Builder."""
        keep = []
        kv, rv = self.partial_deps_batch_raw(self.range_batch_in(rb, keep))
        return self.copy_out(kv, rb.keys), self.copy_out_range(rv)

    def copy_out_range(self, view: "L.RangedepsView") -> "BatchRangeDeps":
        n = view.n_txn
        out = L.RangedepsOut()
        out.mem = L.ACC_MEM_HOST
        rc = self._lib.acc_rangedeps_copy_out(self._h, C.byref(out))
        if rc not in (L.ACC_OK, L.ACC_E_CAP):
            self.check(rc)
        r = dict(arena_off=np.zeros(n + 1, np.uint64), rd_off=np.zeros(n + 1, np.uint64), u_off=np.zeros(n + 1, np.uint64),
                 arena=np.zeros(max(out.need_arena, 1), np.int32), range_id=np.zeros(max(out.need_ranges, 1), np.uint32),
                 dep_txn=np.zeros(max(out.need_deps, 1), np.uint32), rng_start=np.zeros(max(out.need_dict, 1), np.uint64),
                 rng_end=np.zeros(max(out.need_dict, 1), np.uint64))
        out.cap_arena, out.cap_ranges, out.cap_deps, out.cap_dict = (out.need_arena, out.need_ranges, out.need_deps,
                                                                     out.need_dict)
        for k, v in r.items():
            setattr(out, k, v.ctypes.data)
        self.check(self._lib.acc_rangedeps_copy_out(self._h, C.byref(out)))
        return BatchRangeDeps(r["rng_start"][:out.need_dict], r["rng_end"][:out.need_dict], r["arena_off"],
                              r["arena"][:out.need_arena], r["rd_off"], r["range_id"][:out.need_ranges], r["u_off"],
                              r["dep_txn"][:out.need_deps], int(view.total_edges))

    def copy_out(self, view: "L.KeydepsView", batch=None) -> "BatchKeyDeps":
        n = view.n_txn
        out = L.KeydepsOut()
        out.mem = L.ACC_MEM_HOST
        # first call: sizing (ACC_E_CAP with need_* filled)
        rc = self._lib.acc_keydeps_copy_out(self._h, C.byref(out))
        if rc not in (L.ACC_OK, L.ACC_E_CAP):
            self.check(rc)
        arena_off = np.zeros(n + 1, np.uint64)
        kd_off = np.zeros(n + 1, np.uint64)
        u_off = np.zeros(n + 1, np.uint64)
        arena = np.zeros(max(out.need_arena, 1), np.int32)
        key_idx = np.zeros(max(out.need_keys, 1), np.uint32)
        dep_txn = np.zeros(max(out.need_deps, 1), np.uint32)
        out.cap_arena, out.cap_keys, out.cap_deps = out.need_arena, out.need_keys, out.need_deps
        out.arena_off, out.kd_off, out.u_off = arena_off.ctypes.data, kd_off.ctypes.data, u_off.ctypes.data
        out.arena, out.key_idx, out.dep_txn = arena.ctypes.data, key_idx.ctypes.data, dep_txn.ctypes.data
        kd_key = None
        if view.kd_key:
            kd_key = np.zeros(max(out.need_keys, 1), np.uint64)
            out.kd_key = kd_key.ctypes.data
        self.check(self._lib.acc_keydeps_copy_out(self._h, C.byref(out)))
        return BatchKeyDeps(arena_off, arena[:out.need_arena], kd_off, key_idx[:out.need_keys], u_off,
                            dep_txn[:out.need_deps], int(view.total_edges), batch,
                            None if kd_key is None else kd_key[:out.need_keys])


@dataclass
class BatchRangeDeps:
    """Per-txn PartialDeps.rangeDeps of a mixed batch in the acc_rangedeps_view layout: ranges as ids into the
    dictionary (rng_start, rng_end) of distinct stored ranges sorted by Range::compare."""
    rng_start: np.ndarray
    rng_end: np.ndarray
    arena_off: np.ndarray
    arena: np.ndarray
    rd_off: np.ndarray
    range_id: np.ndarray
    u_off: np.ndarray
    dep_txn: np.ndarray
    total_edges: int

    def txn(self, t: int):
        a = self.arena[self.arena_off[t]:self.arena_off[t + 1]]
        r = self.range_id[self.rd_off[t]:self.rd_off[t + 1]]
        d = self.dep_txn[self.u_off[t]:self.u_off[t + 1]]
        return r, d, a

    def range_deps(self, t: int):
        """{(start, end): [dep batch index ...]} of txn t (RangeDeps.forEach over its ranges)."""
        r, d, a = self.txn(t)
        out, start = {}, len(r)
        for i, rid in enumerate(r):
            end = int(a[i])
            out[(int(self.rng_start[rid]), int(self.rng_end[rid]))] = [int(d[x]) for x in a[start:end]]
            start = end
        return out


@dataclass
class BatchKeyDeps:
    """Per-txn PartialDeps.keyDeps of a batch in the acc_keydeps_view layout."""
    arena_off: np.ndarray
    arena: np.ndarray
    kd_off: np.ndarray
    key_idx: np.ndarray
    u_off: np.ndarray
    dep_txn: np.ndarray
    total_edges: int
    batch: object = None
    kd_key: np.ndarray | None = None   # key codes (acc_keydeps_mixed)

    def txn(self, t: int):
        a = self.arena[self.arena_off[t]:self.arena_off[t + 1]]
        k = self.key_idx[self.kd_off[t]:self.kd_off[t + 1]]
        d = self.dep_txn[self.u_off[t]:self.u_off[t + 1]]
        return k, d, a

    def key_deps(self, t: int) -> "KeyDeps":
        """KeyDeps of txn t with real key codes and TxnId tuples (needs the input batch)."""
        k, d, a = self.txn(t)
        b = self.batch
        if self.kd_key is not None:
            keys = self.kd_key[self.kd_off[t]:self.kd_off[t + 1]]
        else:
            keys = b.key_code[int(b.key_off[t]) + k.astype(np.int64)]
        txn_ids = [TxnId(int(b.txn_msb[x]), int(b.txn_lsb[x]), int(b.txn_node[x])) for x in d]
        return KeyDeps(keys, txn_ids, a)


class TxnId(tuple):
    """(msb, lsb, node) with Timestamp.compareTo/equals semantics (primitives/Timestamp.java:208-249)."""

    def __new__(cls, msb, lsb, node):
        return super().__new__(cls, (int(msb), int(lsb), int(node)))

    def order_key(self):
        msb, lsb, node = self
        return (msb, lsb >> 16, lsb & 0x1E, node)

    @property
    def epoch(self):
        return self[0] >> 15

    @property
    def hlc(self):
        return ((self[0] & 0x7FFF) << 48) | (self[1] >> 16)

    @property
    def flags(self):
        return self[1] & 0xFFFF

    def __str__(self):  # TxnId.toString (TxnId.java:119-122) without the kind/domain short names
        return f"[{self.epoch},{self.hlc},{self.flags},{self[2]}]"


class KeyDeps:
    """KeyDeps in the reference layout (primitives/KeyDeps.java:150-172): keys (sorted unique codes),
    txnIds (sorted unique), keysToTxnIds (Java int[]: end offsets from keys.length, then indices)."""

    def __init__(self, keys, txn_ids, keys_to_txn_ids):
        self.keys = np.asarray(keys, dtype=np.uint64)
        self.txn_ids = list(txn_ids)
        self.keys_to_txn_ids = np.asarray(keys_to_txn_ids, dtype=np.int32)
        nk = len(self.keys)
        # KeyDeps ctor check (KeyDeps.java:184-185)
        if nk and int(self.keys_to_txn_ids[nk - 1]) != len(self.keys_to_txn_ids):
            raise IllegalArgumentException("Last key in keyToTxnId does not point to the end of the array")

    def is_empty(self):
        return len(self.keys) == 0

    def txn_id_count(self):
        return len(self.txn_ids)

    def for_each(self, key):
        """TxnIds depended on for `key` (KeyDeps.forEach(key, ...))."""
        i = int(np.searchsorted(self.keys, np.uint64(key)))
        if i >= len(self.keys) or int(self.keys[i]) != int(key):
            return []
        start = len(self.keys) if i == 0 else int(self.keys_to_txn_ids[i - 1])
        end = int(self.keys_to_txn_ids[i])
        return [self.txn_ids[int(x)] for x in self.keys_to_txn_ids[start:end]]

    def canonical(self):
        return {int(k): self.for_each(k) for k in self.keys}

    def __eq__(self, other):  # RelationMultiMap.testEquality (:1027-1036)
        return (isinstance(other, KeyDeps) and np.array_equal(self.keys, other.keys)
                and self.txn_ids == other.txn_ids
                and np.array_equal(self.keys_to_txn_ids, other.keys_to_txn_ids))

    def __str__(self):
        return "{" + ", ".join(f"{k}:[{', '.join(str(t) for t in v)}]" for k, v in self.canonical().items()) + "}"


def _merge_in(m: dict, keep: list) -> "L.MergeIn":
    a = {k: np.ascontiguousarray(v, dtype=dt) for (k, dt), v in
         zip([("grp_off", np.uint64), ("key_off", np.uint64), ("key_code", np.uint64), ("val_off", np.uint64),
              ("txn_rank", np.uint32), ("k2v_off", np.uint64), ("k2v", np.int32)],
             [m["grp_off"], m["key_off"], m["key_code"], m["val_off"], m["txn_rank"], m["k2v_off"], m["k2v"]])}
    keep.append(a)
    ng = len(a["grp_off"]) - 1
    nr = len(a["key_off"]) - 1
    return L.MergeIn(L.ACC_MEM_HOST, ng, nr, *(a[k].ctypes.data for k in
                                               ("grp_off", "key_off", "key_code", "val_off", "txn_rank", "k2v_off", "k2v")))


def keydeps_merge(ctx: Context, m: dict) -> dict:
    """KeyDeps.merge for every group of replies (primitives/KeyDeps.java:115-135) on the GPU.
    `m` uses the acc_merge_in layout (grp_off, key_off, key_code, val_off, txn_rank, k2v_off, k2v)."""
    keep = []
    mi = _merge_in(m, keep)
    view = L.MergeView()
    ctx.check(ctx._lib.acc_keydeps_merge(ctx.handle, C.byref(mi), C.byref(view)))
    return merge_copy_out(ctx, view)


def merge_copy_out(ctx: Context, view) -> dict:
    """Host copy of the last merge result on ctx (acc_merge_copy_out, two-call sizing)."""
    out = L.MergeOut()
    out.mem = L.ACC_MEM_HOST
    rc = ctx._lib.acc_merge_copy_out(ctx.handle, C.byref(out))
    if rc not in (L.ACC_OK, L.ACC_E_CAP):
        ctx.check(rc)
    ng = view.n_groups
    r = dict(key_off=np.zeros(ng + 1, np.uint64), val_off=np.zeros(ng + 1, np.uint64),
             k2v_off=np.zeros(ng + 1, np.uint64), key_code=np.zeros(max(out.need_keys, 1), np.uint64),
             txn_rank=np.zeros(max(out.need_vals, 1), np.uint32), k2v=np.zeros(max(out.need_k2v, 1), np.int32))
    out.cap_keys, out.cap_vals, out.cap_k2v = out.need_keys, out.need_vals, out.need_k2v
    for k in r:
        setattr(out, k, r[k].ctypes.data)
    ctx.check(ctx._lib.acc_merge_copy_out(ctx.handle, C.byref(out)))
    r["key_code"] = r["key_code"][:out.need_keys]
    r["txn_rank"] = r["txn_rank"][:out.need_vals]
    r["k2v"] = r["k2v"][:out.need_k2v]
    return r


def levelise(ctx: Context, off, dep, exec_rank):
    """Execution-order levels of a deps graph (restatement of Commands.updateWaitingOn ordering,
    local/Commands.java:776-830): returns (level[n], order[n], n_levels)."""
    off = np.ascontiguousarray(off, dtype=np.uint64)
    dep = np.ascontiguousarray(dep, dtype=np.uint32)
    er = np.ascontiguousarray(exec_rank, dtype=np.uint32)
    n = len(er)
    level = np.zeros(max(n, 1), np.uint32)
    order = np.zeros(max(n, 1), np.uint32)
    nl = np.zeros(1, np.uint32)
    gi = L.GraphIn(L.ACC_MEM_HOST, n, off.ctypes.data, dep.ctypes.data if len(dep) else 0, er.ctypes.data)
    ctx.check(ctx._lib.acc_levelise(ctx.handle, C.byref(gi), level.ctypes.data_as(L.u32p), order.ctypes.data_as(L.u32p),
                                    nl.ctypes.data_as(L.u32p)))
    return level[:n], order[:n], int(nl[0])


def merge_levelise_device(ctx: Context, mi: "L.MergeIn", exec_rank_ptr: int, level_ptr: int, order_ptr: int):
    """The coordinator path of config 5 on device: KeyDeps.merge of every txn's replies (acc_keydeps_merge,
    primitives/KeyDeps.java:115-135), then levelisation of the merged graph (deps of txn t = its merged TxnIds, as
    batch indices) by executeAt (acc_levelise, local/Commands.java:776-830). `mi` and the three pointers are device
    memory; the merged view stays device-resident on ctx. Returns (merge view, n_levels)."""
    view = L.MergeView()
    ctx.check(ctx._lib.acc_keydeps_merge(ctx.handle, C.byref(mi), C.byref(view)))
    gi = L.GraphIn(L.ACC_MEM_DEVICE, view.n_groups, view.val_off, view.txn_rank, exec_rank_ptr)
    nl = np.zeros(1, np.uint32)
    ctx.check(ctx._lib.acc_levelise(ctx.handle, C.byref(gi), C.cast(level_ptr, L.u32p), C.cast(order_ptr, L.u32p),
                                    nl.ctypes.data_as(L.u32p)))
    return view, int(nl[0])


# ---------------------------------------------------------------- Deps.merge over raw deps objects

RMM_FIELDS = (("key_off", np.uint64), ("key_a", np.uint64), ("key_b", np.uint64), ("val_off", np.uint64),
              ("msb", np.uint64), ("lsb", np.uint64), ("node", np.int32), ("k2v_off", np.uint64), ("k2v", np.int32))


def _rmm_in(half, keep: list) -> "L.RmmIn":
    """acc_rmm_in over host arrays of one half: dict(key_off, key_a, [key_b], val_off, msb, lsb, node, k2v_off, k2v)."""
    if half is None:
        return L.RmmIn()
    a = {k: np.ascontiguousarray(half[k], dtype=dt) for k, dt in RMM_FIELDS if half.get(k) is not None}
    keep.append(a)
    p = lambda k: a[k].ctypes.data if k in a and a[k].size else (a[k].ctypes.data if k in a else None)  # noqa: E731
    return L.RmmIn(p("key_off"), p("key_a"), p("key_b"), p("val_off"), L.TsCols(p("msb"), p("lsb"), p("node")),
                   p("k2v_off"), p("k2v"))


def rmm_copy_out(ctx: Context, n_groups: int, view: "L.RmmView", with_b: bool) -> dict:
    """Host copy of one acc_rmm_view (acc_rmm_copy_out, two-call sizing)."""
    out = L.RmmOut()
    out.mem = L.ACC_MEM_HOST
    rc = ctx._lib.acc_rmm_copy_out(ctx.handle, n_groups, C.byref(view), C.byref(out))
    if rc not in (L.ACC_OK, L.ACC_E_CAP):
        ctx.check(rc)
    nk, nv, no = out.need_keys, out.need_vals, out.need_k2v
    r = dict(key_off=np.zeros(n_groups + 1, np.uint64), val_off=np.zeros(n_groups + 1, np.uint64),
             k2v_off=np.zeros(n_groups + 1, np.uint64), key_a=np.zeros(max(nk, 1), np.uint64),
             msb=np.zeros(max(nv, 1), np.uint64), lsb=np.zeros(max(nv, 1), np.uint64), node=np.zeros(max(nv, 1), np.int32),
             src=np.zeros(max(nv, 1), np.uint32), k2v=np.zeros(max(no, 1), np.int32))
    if with_b:
        r["key_b"] = np.zeros(max(nk, 1), np.uint64)
    out.cap_keys, out.cap_vals, out.cap_k2v = nk, nv, no
    for f, k in (("key_off", "key_off"), ("val_off", "val_off"), ("k2v_off", "k2v_off"), ("key_a", "key_a"),
                 ("txn_msb", "msb"), ("txn_lsb", "lsb"), ("txn_node", "node"), ("txn_src", "src"), ("k2v", "k2v")):
        setattr(out, f, r[k].ctypes.data)
    if with_b:
        out.key_b = r["key_b"].ctypes.data
    ctx.check(ctx._lib.acc_rmm_copy_out(ctx.handle, n_groups, C.byref(view), C.byref(out)))
    for k, n in (("key_a", nk), ("key_b", nk), ("msb", nv), ("lsb", nv), ("node", nv), ("src", nv), ("k2v", no)):
        if k in r:
            r[k] = r[k][:n]
    return r


def deps_merge(ctx: Context, m: dict) -> dict:
    """Deps.merge (primitives/Deps.java:256-260) of every group's replies on the GPU. `m` = dict(grp_off, key=half|None,
    range=half|None) with halves in the SerializerSupport layout (see _rmm_in); returns dict(key=..., range=...) of
    merged halves (per-group CSR: key_off/key_a[/key_b], val_off/msb/lsb/node/src, k2v_off/k2v)."""
    keep = []
    grp_off = np.ascontiguousarray(m["grp_off"], dtype=np.uint64)
    keep.append(grp_off)
    ng = len(grp_off) - 1
    nr = int(grp_off[-1]) if ng >= 0 else 0
    di = L.DepsMergeIn(L.ACC_MEM_HOST, ng, nr, grp_off.ctypes.data, _rmm_in(m.get("key"), keep),
                       _rmm_in(m.get("range"), keep))
    view = L.DepsMergeView()
    ctx.check(ctx._lib.acc_deps_merge(ctx.handle, C.byref(di), C.byref(view)))
    return dict(key=rmm_copy_out(ctx, ng, view.key_deps, False), range=rmm_copy_out(ctx, ng, view.range_deps, True),
                total_in_entries=int(view.total_in_entries))


# ---------------------------------------------------------------- RelationMultiMap helpers (invert, slice, stab)

def device_array(ctx: Context, ptr, n: int, dtype) -> np.ndarray:
    """Host copy of n elements at a device pointer of a result view (acc_copy_out)."""
    out = np.zeros(max(int(n), 1), dtype=dtype)
    if n:
        ctx.check(ctx._lib.acc_copy_out(ctx.handle, out.ctypes.data, ptr, int(n) * out.itemsize, L.ACC_MEM_HOST))
    return out[:int(n)]


def _rmm_batch(m: dict, keep: list) -> "L.RmmBatch":
    """acc_rmm_batch over host arrays: dict(key_off, key_a, [key_b], val_off, k2v_off, k2v)."""
    a = {k: np.ascontiguousarray(m[k], dtype=dt) for k, dt in
         (("key_off", np.uint64), ("key_a", np.uint64), ("key_b", np.uint64), ("val_off", np.uint64),
          ("k2v_off", np.uint64), ("k2v", np.int32)) if m.get(k) is not None}
    keep.append(a)
    p = lambda k: a[k].ctypes.data if k in a else None  # noqa: E731
    return L.RmmBatch(L.ACC_MEM_HOST, len(a["key_off"]) - 1, p("key_off"), p("key_a"), p("key_b"), p("val_off"),
                      p("k2v_off"), p("k2v"))


def rmm_invert(ctx: Context, m: dict):
    """RelationMultiMap.invert of every group (acc_rmm_invert): (off[n_groups+1], ints) = txnIdsToKeys per group."""
    keep = []
    b = _rmm_batch(m, keep)
    v = L.CsrView()
    ctx.check(ctx._lib.acc_rmm_invert(ctx.handle, C.byref(b), C.byref(v)))
    return device_array(ctx, v.off, v.n_groups + 1, np.uint64), device_array(ctx, v.ints, v.total, np.int32)


def rmm_slice(ctx: Context, m: dict, sel_off, sel_start, sel_end, end_inclusive: bool = True) -> dict:
    """KeyDeps.slice / RangeDeps.slice (+ trimUnusedValues) of every group against its own select Ranges."""
    keep = []
    b = _rmm_batch(m, keep)
    so, ss, se = (np.ascontiguousarray(x, dtype=np.uint64) for x in (sel_off, sel_start, sel_end))
    keep.append((so, ss, se))
    sel = L.RangesIn(so.ctypes.data, ss.ctypes.data, se.ctypes.data, int(end_inclusive), 0)
    v = L.SliceView()
    ctx.check(ctx._lib.acc_rmm_slice(ctx.handle, C.byref(b), C.byref(sel), C.byref(v)))
    g = v.n_groups + 1
    return dict(key_off=device_array(ctx, v.key_off, g, np.uint64), key_idx=device_array(ctx, v.key_idx, v.total_keys, np.uint32),
                val_off=device_array(ctx, v.val_off, g, np.uint64), val_idx=device_array(ctx, v.val_idx, v.total_vals, np.uint32),
                k2v_off=device_array(ctx, v.k2v_off, g, np.uint64), k2v=device_array(ctx, v.k2v, v.total_k2v, np.int32))


def _slice_copy(ctx: Context, v) -> dict:
    g = v.n_groups + 1
    return dict(key_off=device_array(ctx, v.key_off, g, np.uint64), key_idx=device_array(ctx, v.key_idx, v.total_keys, np.uint32),
                val_off=device_array(ctx, v.val_off, g, np.uint64), val_idx=device_array(ctx, v.val_idx, v.total_vals, np.uint32),
                k2v_off=device_array(ctx, v.k2v_off, g, np.uint64), k2v=device_array(ctx, v.k2v, v.total_k2v, np.int32))


def _without_copy(ctx: Context, w) -> dict:
    out = _slice_copy(ctx, w.sl)
    out["kind"] = device_array(ctx, w.kind, w.sl.n_groups, np.uint8)
    out["counts"] = (int(w.n_from), int(w.n_none), int(w.n_new))
    return out


def _txn_sets(x, keep: list) -> "L.TxnSets | None":
    if x is None:
        return None
    a = {k: np.ascontiguousarray(x[k], dtype=dt) for k, dt in
         (("off", np.uint64), ("msb", np.uint64), ("lsb", np.uint64), ("node", np.int32))}
    keep.append(a)
    return L.TxnSets(a["off"].ctypes.data, L.TsCols(a["msb"].ctypes.data, a["lsb"].ctypes.data, a["node"].ctypes.data))


def rmm_without(ctx: Context, m: dict, set_a=None, set_b=None) -> dict:
    """KeyDeps.without / RangeDeps.without (RelationMultiMap.remove, utils/RelationMultiMap.java:843-905) of every group
    with remove = membership in the group's sorted TxnId set(s) (Deps::contains). `m`: one deps half per group (the
    acc_rmm_batch dict + its TxnIds msb/lsb/node); sets: dict(off, msb, lsb, node) or None. Returns the slice-shaped
    result (kept key / TxnId indices, the new int[]) with kind[g] = ACC_WITHOUT_FROM / _NONE / _NEW."""
    keep = []
    b = _rmm_batch(m, keep)
    t = {k: np.ascontiguousarray(m[k], dtype=dt) for k, dt in (("msb", np.uint64), ("lsb", np.uint64), ("node", np.int32))}
    keep.append(t)
    txn = L.TsCols(t["msb"].ctypes.data, t["lsb"].ctypes.data, t["node"].ctypes.data)
    sa, sb = _txn_sets(set_a, keep), _txn_sets(set_b, keep)
    v = L.WithoutView()
    ctx.check(ctx._lib.acc_rmm_without(ctx.handle, C.byref(b), C.byref(txn), C.byref(sa) if sa is not None else None,
                                       C.byref(sb) if sb is not None else None, C.byref(v)))
    return _without_copy(ctx, v)


def recovery_deps_reduce(ctx: Context, committed: dict, accepted: dict) -> dict:
    """The recovery coordinator's reduce of the replies' recovery deps (coordinate/Recover.java:320-322,
    messages/BeginRecovery.java:180-183; acc_recovery_deps_reduce): earlierCommittedWitness = Deps.merge(...),
    earlierAcceptedNoWitness = Deps.merge(...).without(earlierCommittedWitness::contains). Inputs as deps_merge's `m`
    (same grp_off). Returns dict(committed=merged halves, accepted_merged=merged halves, accepted_key / accepted_range =
    the without results over accepted_merged's halves)."""
    keep = []

    def dmi(m):
        grp_off = np.ascontiguousarray(m["grp_off"], dtype=np.uint64)
        keep.append(grp_off)
        ng = len(grp_off) - 1
        return L.DepsMergeIn(L.ACC_MEM_HOST, ng, int(grp_off[-1]) if ng >= 0 else 0, grp_off.ctypes.data,
                             _rmm_in(m.get("key"), keep), _rmm_in(m.get("range"), keep)), ng
    ci, ng = dmi(committed)
    ai, ng2 = dmi(accepted)
    v = L.RecoveryDepsView()
    ctx.check(ctx._lib.acc_recovery_deps_reduce(ctx.handle, C.byref(ci), C.byref(ai), C.byref(v)))
    return dict(committed=dict(key=rmm_copy_out(ctx, ng, v.committed.key_deps, False),
                               range=rmm_copy_out(ctx, ng, v.committed.range_deps, True)),
                accepted_merged=dict(key=rmm_copy_out(ctx, ng, v.accepted_merged.key_deps, False),
                                     range=rmm_copy_out(ctx, ng, v.accepted_merged.range_deps, True)),
                accepted_key=_without_copy(ctx, v.accepted_key), accepted_range=_without_copy(ctx, v.accepted_range))


def rangedeps_stab(ctx: Context, m: dict, grp, q_start, q_end=None, end_inclusive: bool = True, want_txns: bool = True):
    """Stabbing queries over built RangeDeps (acc_rangedeps_stab): per query the ascending range indices (and, with
    want_txns, the sorted unique TxnId indices = RangeDeps.computeTxnIds)."""
    keep = []
    b = _rmm_batch(m, keep)
    grp = np.ascontiguousarray(grp, dtype=np.uint32)
    qs = np.ascontiguousarray(q_start, dtype=np.uint64)
    qe = np.ascontiguousarray(q_end, dtype=np.uint64) if q_end is not None else None
    keep.append((grp, qs, qe))
    qi = L.StabIn(L.ACC_MEM_HOST, len(grp), grp.ctypes.data, qs.ctypes.data, qe.ctypes.data if qe is not None else None,
                  int(end_inclusive), int(want_txns))
    v = L.StabView()
    ctx.check(ctx._lib.acc_rangedeps_stab(ctx.handle, C.byref(b), C.byref(qi), C.byref(v)))
    n = v.n_queries + 1
    out = dict(range_off=device_array(ctx, v.range_off, n, np.uint64),
               range_idx=device_array(ctx, v.range_idx, v.total_ranges, np.uint32))
    if want_txns:
        out["txn_off"] = device_array(ctx, v.txn_off, n, np.uint64)
        out["txn_idx"] = device_array(ctx, v.txn_idx, v.total_txns, np.uint32)
    return out


# ---------------------------------------------------------------- LatestDeps (recovery merge)

def latest_deps_merge(ctx: Context, groups, key_objs: dict | None, range_objs: dict | None, end_inclusive: bool = True,
                      commit: bool = False, txn_ids=None, execute_ats=None) -> dict:
    """LatestDeps.mergeProposal / mergeCommit (primitives/LatestDeps.java:306-326) for every recovering txn
    (acc_latest_deps_merge). groups[g] = the replies, each a list of intervals (start, end, KnownDeps ordinal,
    ballot (msb, lsb, node), coordinatedDeps id, localDeps id) with ids into the deps objects (-1 = null); key_objs /
    range_objs = the objects' halves in the Deps.merge layout (one slot per id). Returns dict(key=..., range=...,
    sufficient=[[(start, end)...] per group])."""
    keep = []
    grp_off, iv_off = [0], [0]
    cols = {k: [] for k in ("s", "e", "known", "bm", "bl", "bn", "cd", "ld")}
    for replies in groups:
        for ivs in replies:
            for (s, e, known, ballot, cd, ld) in ivs:
                for k, v in zip(("s", "e", "known", "bm", "bl", "bn", "cd", "ld"), (s, e, known, *ballot, cd, ld)):
                    cols[k].append(v)
            iv_off.append(len(cols["s"]))
        grp_off.append(len(iv_off) - 1)
    a = dict(grp=np.array(grp_off, np.uint32), ivo=np.array(iv_off, np.uint32), s=np.array(cols["s"], np.uint64),
             e=np.array(cols["e"], np.uint64), known=np.array(cols["known"], np.uint8), bm=np.array(cols["bm"], np.uint64),
             bl=np.array(cols["bl"], np.uint64), bn=np.array(cols["bn"], np.int32), cd=np.array(cols["cd"], np.int32),
             ld=np.array(cols["ld"], np.int32))
    ng = len(groups)
    tid = [np.ascontiguousarray([t[i] for t in (txn_ids or [])] or [0], dtype=dt) for i, dt in
           enumerate((np.uint64, np.uint64, np.int32))]
    exe = [np.ascontiguousarray([t[i] for t in (execute_ats or [])] or [0], dtype=dt) for i, dt in
           enumerate((np.uint64, np.uint64, np.int32))]
    keep += [a, tid, exe]
    p = lambda x: x.ctypes.data  # noqa: E731
    nd = max(len(key_objs["key_off"]) - 1 if key_objs else 0, len(range_objs["key_off"]) - 1 if range_objs else 0)
    li = L.LatestIn(ng, L.ACC_LATEST_COMMIT if commit else L.ACC_LATEST_PROPOSAL, p(a["grp"]), p(a["ivo"]), p(a["s"]),
                    p(a["e"]), p(a["known"]), L.TsCols(p(a["bm"]), p(a["bl"]), p(a["bn"])), p(a["cd"]), p(a["ld"]),
                    L.TsCols(*(p(x) for x in tid)), L.TsCols(*(p(x) for x in exe)), int(end_inclusive), L.ACC_MEM_HOST,
                    nd, _rmm_in(key_objs, keep), _rmm_in(range_objs, keep))
    v = L.LatestView()
    ctx.check(ctx._lib.acc_latest_deps_merge(ctx.handle, C.byref(li), C.byref(v)))
    ns = int(v.total_sufficient)
    so = np.ctypeslib.as_array(v.sufficient_off, (ng + 1,)).copy() if ng else np.zeros(1, np.uint64)
    ss = np.ctypeslib.as_array(v.sufficient_start, (ns,)).copy() if ns else np.zeros(0, np.uint64)
    se = np.ctypeslib.as_array(v.sufficient_end, (ns,)).copy() if ns else np.zeros(0, np.uint64)
    suff = [[(int(ss[x]), int(se[x])) for x in range(int(so[g]), int(so[g + 1]))] for g in range(ng)]
    return dict(key=rmm_copy_out(ctx, ng, v.deps.key_deps, False), range=rmm_copy_out(ctx, ng, v.deps.range_deps, True),
                sufficient=suff)


# ---------------------------------------------------------------- Deps wire format (Maelstrom JSON)

def deps_from_json(ctx: Context, docs: list[bytes], with_view: bool = False):
    """Json.DEPS_ADAPTER.read of every document on device (acc_deps_from_json): dict(key=..., range=...) per-document
    Deps halves (key codes = dictionary ranks) and the dictionary (kind, null, value, hash per rank)."""
    blob = np.frombuffer(b"".join(docs), dtype=np.uint8) if docs else np.zeros(0, np.uint8)
    off = np.zeros(len(docs) + 1, np.uint64)
    if docs:
        np.cumsum([len(x) for x in docs], out=off[1:])
    blob = np.ascontiguousarray(blob)
    ji = L.JsonIn(L.ACC_MEM_HOST, len(docs), blob.ctypes.data if blob.size else None, off.ctypes.data)
    v = L.JsonDepsView()
    ctx.check(ctx._lib.acc_deps_from_json(ctx.handle, C.byref(ji), C.byref(v)))
    nd = int(v.n_dict)
    out = dict(key=rmm_copy_out(ctx, len(docs), v.deps.key_deps, False),
               range=rmm_copy_out(ctx, len(docs), v.deps.range_deps, True),
               dict_kind=device_array(ctx, v.dict_kind, nd, np.uint8), dict_null=device_array(ctx, v.dict_null, nd, np.uint8),
               dict_value=device_array(ctx, v.dict_value, nd, np.uint64), dict_hash=device_array(ctx, v.dict_hash, nd, np.int32),
               dict_len=device_array(ctx, v.dict_len, nd, np.uint32))
    # STRING texts: dict_str[value : value + len] of every STRING rank
    total = int(max((int(o) + int(n) for o, n, k in zip(out["dict_value"], out["dict_len"], out["dict_kind"]) if k == 0),
                    default=0))
    out["dict_str"] = device_array(ctx, v.dict_str, total, np.uint8)
    if with_view:
        out["view"] = v
    return out


def deps_to_json(ctx: Context, view) -> list[bytes]:
    """Json.DEPS_ADAPTER.write of every document of an acc_json_deps_view on device (acc_deps_to_json)."""
    oi = L.JsonOutIn(view.n_docs, view.deps.key_deps, view.deps.range_deps, view.n_dict, view.dict_kind, view.dict_null,
                     view.dict_value, view.dict_len, view.dict_str)
    o = L.JsonOut()
    o.mem = L.ACC_MEM_HOST
    rc = ctx._lib.acc_deps_to_json(ctx.handle, C.byref(oi), C.byref(o))
    if rc not in (L.ACC_OK, L.ACC_E_CAP):
        ctx.check(rc)
    buf = np.zeros(max(int(o.need_bytes), 1), np.uint8)
    off = np.zeros(view.n_docs + 1, np.uint64)
    o.cap_bytes, o.bytes, o.doc_off = int(o.need_bytes), buf.ctypes.data, off.ctypes.data
    ctx.check(ctx._lib.acc_deps_to_json(ctx.handle, C.byref(oi), C.byref(o)))
    raw = buf.tobytes()
    return [raw[int(off[i]):int(off[i + 1])] for i in range(view.n_docs)]


# ---------------------------------------------------------------- CommandsForKey.update with deps (key-major)

def _cfk_updates_host(upd: dict) -> dict:
    return {k: np.ascontiguousarray(np.asarray(upd[k], dt)) for k, dt in (
        ("msb", np.uint64), ("lsb", np.uint64), ("node", np.int32), ("xmsb", np.uint64), ("xlsb", np.uint64),
        ("xnode", np.int32), ("status", np.uint8), ("flags", np.uint8), ("key_off", np.uint32), ("key", np.uint64),
        ("dep_off", np.uint32), ("dmsb", np.uint64), ("dlsb", np.uint64), ("dnode", np.int32))}


def _cfk_updates_in(b: dict) -> "L.CfkUpdates":
    p = lambda k: b[k].ctypes.data  # noqa: E731
    return L.CfkUpdates(L.ACC_MEM_HOST, len(b["msb"]), len(b["key"]), len(b["dmsb"]),
                        L.TsCols(p("msb"), p("lsb"), p("node")), L.TsCols(p("xmsb"), p("xlsb"), p("xnode")),
                        p("status"), p("flags"), p("key_off"), p("key"), p("dep_off"),
                        L.TsCols(p("dmsb"), p("dlsb"), p("dnode")))


def _snap_host(ctx: Context, v) -> dict:
    nk, ne, nm = int(v.n_keys), int(v.n_entries), int(v.n_missing)
    return dict(key=device_array(ctx, v.key, nk, np.uint64), ent_off=device_array(ctx, v.ent_off, nk + 1, np.uint32),
                emsb=device_array(ctx, v.txn_id.msb, ne, np.uint64), elsb=device_array(ctx, v.txn_id.lsb, ne, np.uint64),
                enode=device_array(ctx, v.txn_id.node, ne, np.int32), xmsb=device_array(ctx, v.execute_at.msb, ne, np.uint64),
                xlsb=device_array(ctx, v.execute_at.lsb, ne, np.uint64), xnode=device_array(ctx, v.execute_at.node, ne, np.int32),
                status=device_array(ctx, v.status, ne, np.uint8), miss_off=device_array(ctx, v.miss_off, ne + 1, np.uint32),
                mmsb=device_array(ctx, v.missing.msb, nm, np.uint64), mlsb=device_array(ctx, v.missing.lsb, nm, np.uint64),
                mnode=device_array(ctx, v.missing.node, nm, np.int32))


def cfk_apply(ctx: Context, snap: dict, upd: dict, keep_device: bool = False):
    """CommandsForKey.update(prev, next) with each command's deps (local/CommandsForKey.java:657-1149) for a batch of
    updates against a key-major snapshot (acc_cfk_apply): missing[] maintenance and TRANSITIVELY_KNOWN additions.
    snap: key, ent_off, emsb/elsb/enode (TxnIds), xmsb/xlsb/xnode (executeAts), status, miss_off, mmsb/mlsb/mnode;
    upd: msb/lsb/node, xmsb/xlsb/xnode, status, flags, key_off, key, dep_off, dmsb/dlsb/dnode. Returns the new
    snapshot in the same layout (host copies), or with keep_device its device-resident acc_cfk_snap_view."""
    a = {k: np.ascontiguousarray(np.asarray(snap[k], dt)) for k, dt in (
        ("key", np.uint64), ("ent_off", np.uint32), ("emsb", np.uint64), ("elsb", np.uint64), ("enode", np.int32),
        ("xmsb", np.uint64), ("xlsb", np.uint64), ("xnode", np.int32), ("status", np.uint8), ("miss_off", np.uint32),
        ("mmsb", np.uint64), ("mlsb", np.uint64), ("mnode", np.int32))}
    b = _cfk_updates_host(upd)
    p = lambda d, k: d[k].ctypes.data  # noqa: E731
    si = L.CfkSnap(L.ACC_MEM_HOST, len(a["key"]), len(a["status"]), len(a["mmsb"]), p(a, "key"), p(a, "ent_off"),
                   L.TsCols(p(a, "emsb"), p(a, "elsb"), p(a, "enode")), L.TsCols(p(a, "xmsb"), p(a, "xlsb"), p(a, "xnode")),
                   p(a, "status"), p(a, "miss_off"), L.TsCols(p(a, "mmsb"), p(a, "mlsb"), p(a, "mnode")))
    ui = _cfk_updates_in(b)
    v = L.CfkSnapView()
    ctx.check(ctx._lib.acc_cfk_apply(ctx.handle, C.byref(si), C.byref(ui), C.byref(v)))
    if keep_device:
        return v
    return _snap_host(ctx, v)


def _view_as_snap(v) -> "L.CfkSnap":
    return L.CfkSnap(L.ACC_MEM_DEVICE, v.n_keys, v.n_entries, v.n_missing, v.key, v.ent_off, v.txn_id, v.execute_at,
                     v.status, v.miss_off, v.missing)


def cfk_snap_to_batch(ctx: Context, snap) -> "L.CfkBatchView":
    """acc_cfk_snap_to_batch: the txn-major snapshot and per-pair missing[] batch indices acc_map_reduce_full reads,
    in HBM. snap: a device-resident acc_cfk_snap_view (cfk_apply(..., keep_device=True)) or a host dict in the
    cfk_apply snapshot layout."""
    out = L.CfkBatchView()
    if isinstance(snap, dict):
        a = {k: np.ascontiguousarray(np.asarray(snap[k], dt)) for k, dt in (
            ("key", np.uint64), ("ent_off", np.uint32), ("emsb", np.uint64), ("elsb", np.uint64), ("enode", np.int32),
            ("xmsb", np.uint64), ("xlsb", np.uint64), ("xnode", np.int32), ("status", np.uint8),
            ("miss_off", np.uint32), ("mmsb", np.uint64), ("mlsb", np.uint64), ("mnode", np.int32))}
        p = lambda k: a[k].ctypes.data  # noqa: E731
        si = L.CfkSnap(L.ACC_MEM_HOST, len(a["key"]), len(a["status"]), len(a["mmsb"]), p("key"), p("ent_off"),
                       L.TsCols(p("emsb"), p("elsb"), p("enode")), L.TsCols(p("xmsb"), p("xlsb"), p("xnode")),
                       p("status"), p("miss_off"), L.TsCols(p("mmsb"), p("mlsb"), p("mnode")))
    else:
        si = _view_as_snap(snap)
    ctx.check(ctx._lib.acc_cfk_snap_to_batch(ctx.handle, C.byref(si), C.byref(out)))
    return out


def cfk_batch_host(ctx: Context, bv) -> tuple:
    """Host copies of an acc_cfk_batch_view: (Batch, missing_off, missing_txn)."""
    b = bv.batch
    n, p = int(b.n_txn), int(b.n_pairs)
    from .workload import Batch
    batch = Batch(device_array(ctx, b.txn_id.msb, n, np.uint64), device_array(ctx, b.txn_id.lsb, n, np.uint64),
                  device_array(ctx, b.txn_id.node, n, np.int32), device_array(ctx, b.execute_at.msb, n, np.uint64),
                  device_array(ctx, b.execute_at.lsb, n, np.uint64), device_array(ctx, b.execute_at.node, n, np.int32),
                  device_array(ctx, b.status, n, np.uint8), device_array(ctx, b.key_off, n + 1, np.uint32),
                  device_array(ctx, b.key_code, p, np.uint64))
    return (batch, device_array(ctx, bv.missing_off, p + 1, np.uint32),
            device_array(ctx, bv.missing_txn, int(bv.n_missing), np.uint32))


def cfk_map_reduce_full(ctx: Context, bv, queries: dict, started_at: int, test_dep: int, test_status: int,
                        test_kinds: int = -1, executes_after: bool = False) -> "BatchKeyDeps":
    """SafeCommandStore.mapReduceFull over the store's CommandsForKey state in place: acc_map_reduce_full reading the
    acc_cfk_batch_view bv (cfk_snap_to_batch) straight from HBM. The query arrays are uploaded with torch (the
    acc_recovery_in arrays share the missing[] placement, ACC_MEM_DEVICE)."""
    import torch
    dev = torch.device("cuda", ctx.device)
    t = {k: torch.from_numpy(np.ascontiguousarray(queries[k], dtype=dt)).to(dev) for k, dt in (
        ("msb", np.uint64), ("lsb", np.uint64), ("node", np.int32), ("key_off", np.uint32), ("key_code", np.uint64))}
    torch.cuda.synchronize(dev)
    p = lambda k: t[k].data_ptr()  # noqa: E731
    ri = L.RecoveryIn(int(t["msb"].shape[0]), L.ACC_MEM_DEVICE, L.TsCols(p("msb"), p("lsb"), p("node")), p("key_off"),
                      p("key_code"), bv.missing_off, bv.missing_txn, int(bv.n_missing), started_at, test_dep,
                      test_status, L.ACC_FULL_EXECUTES_AFTER if executes_after else 0, test_kinds)
    view = L.KeydepsView()
    ctx.check(ctx._lib.acc_map_reduce_full(ctx.handle, C.byref(bv.batch), C.byref(ri), C.byref(view)))
    out = ctx.copy_out(view, None)
    del t
    return out


def _conflicts_in(upd: dict, keep: list) -> "L.ConflictsIn":
    a = {k: np.ascontiguousarray(np.asarray(upd[k], dt)) for k, dt in (
        ("xmsb", np.uint64), ("xlsb", np.uint64), ("xnode", np.int32), ("key_off", np.uint32), ("key", np.uint64),
        ("rng_off", np.uint32), ("rng_start", np.uint64), ("rng_end", np.uint64))}
    keep.append(a)
    p = lambda k: a[k].ctypes.data  # noqa: E731
    return L.ConflictsIn(L.ACC_MEM_HOST, len(a["xmsb"]), int(upd["end_inclusive"]), len(a["key"]), len(a["rng_start"]),
                         L.TsCols(p("xmsb"), p("xlsb"), p("xnode")), p("key_off"), p("key"), p("rng_off"), p("rng_start"),
                         p("rng_end"))


def _preaccept_io(q: dict, keep: list):
    b = {k: np.ascontiguousarray(np.asarray(q[k], dt)) for k, dt in (
        ("msb", np.uint64), ("lsb", np.uint64), ("node", np.int32), ("is_range", np.uint8), ("part_off", np.uint32),
        ("part_start", np.uint64), ("part_end", np.uint64))}
    keep.append(b)
    p = lambda k: b[k].ctypes.data  # noqa: E731
    nq = len(b["msb"])
    qi = L.PreacceptIn(L.ACC_MEM_HOST, nq, len(b["part_start"]), L.TsCols(p("msb"), p("lsb"), p("node")),
                       p("is_range"), p("part_off"), p("part_start"), p("part_end"))
    out = dict(msb=np.zeros(max(nq, 1), np.uint64), lsb=np.zeros(max(nq, 1), np.uint64),
               node=np.zeros(max(nq, 1), np.int32), fast=np.zeros(max(nq, 1), np.uint8))
    o = L.PreacceptOut(L.ACC_MEM_HOST, out["msb"].ctypes.data, out["lsb"].ctypes.data, out["node"].ctypes.data,
                       out["fast"].ctypes.data)
    return qi, o, out, nq


def max_conflicts(ctx: Context, upd: dict, q: dict) -> dict:
    """MaxConflicts.get(keys) per PreAccept query and the fast-path test (acc_max_conflicts; local/MaxConflicts.java,
    local/CommandStore.java:320-345). upd: xmsb/xlsb/xnode (executeAt), key_off/key, rng_off/rng_start/rng_end,
    end_inclusive; q: msb/lsb/node (TxnId), is_range, part_off, part_start, part_end. Returns dict(msb, lsb, node,
    fast)."""
    keep = []
    ui = _conflicts_in(upd, keep)
    qi, o, out, nq = _preaccept_io(q, keep)
    ctx.check(ctx._lib.acc_max_conflicts(ctx.handle, C.byref(ui), C.byref(qi), C.byref(o)))
    return {k: v[:nq] for k, v in out.items()}


class MaxConflictsMap:
    """A CommandStore's MaxConflicts kept on the device (acc_maxconflicts_*): update() merges a batch of commands'
    (keysOrRanges, executeAt), get() answers PreAccept queries (MaxConflicts.get + the fast-path test)."""

    def __init__(self, ctx: Context, end_inclusive: int = 1):
        self.ctx = ctx
        h = C.c_void_p()
        ctx.check(ctx._lib.acc_maxconflicts_create(ctx.handle, int(end_inclusive), C.byref(h)))
        self.h = h

    def update(self, upd: dict):
        keep = []
        ui = _conflicts_in(upd, keep)
        self.ctx.check(self.ctx._lib.acc_maxconflicts_update(self.ctx.handle, self.h, C.byref(ui)))

    def get(self, q: dict) -> dict:
        keep = []
        qi, o, out, nq = _preaccept_io(q, keep)
        self.ctx.check(self.ctx._lib.acc_maxconflicts_get(self.ctx.handle, self.h, C.byref(qi), C.byref(o)))
        return {k: v[:nq] for k, v in out.items()}

    def size(self) -> int:
        return int(self.ctx._lib.acc_maxconflicts_size(self.h))

    def close(self):
        if self.h:
            self.ctx._lib.acc_maxconflicts_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


# ---------------------------------------------------------------- device-resident CommandsForKey store

class CfkStore:
    """A CommandsForKey store kept in HBM and updated by batches of commands (acc_cfk_*): CommandsForKey.update for
    every key of every command (local/CommandsForKey.java:652-706)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        h = C.c_void_p()
        ctx.check(ctx._lib.acc_cfk_create(ctx.handle, C.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self.ctx._lib.acc_cfk_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def update(self, batch):
        """Apply a batch of commands (host arrays in the acc_batch_in layout)."""
        a = dict(tm=np.ascontiguousarray(batch.txn_msb, dtype=np.uint64), tl=np.ascontiguousarray(batch.txn_lsb, dtype=np.uint64),
                 tn=np.ascontiguousarray(batch.txn_node, dtype=np.int32), em=np.ascontiguousarray(batch.exe_msb, dtype=np.uint64),
                 el=np.ascontiguousarray(batch.exe_lsb, dtype=np.uint64), en=np.ascontiguousarray(batch.exe_node, dtype=np.int32),
                 st=np.ascontiguousarray(batch.status, dtype=np.uint8), ko=np.ascontiguousarray(batch.key_off, dtype=np.uint32),
                 kc=np.ascontiguousarray(batch.key_code, dtype=np.uint64))
        p = lambda k: a[k].ctypes.data  # noqa: E731
        n = int(a["st"].shape[0])
        bi = L.BatchIn(n, L.ACC_MEM_HOST, int(a["ko"][-1]) if n else 0, L.TsCols(p("tm"), p("tl"), p("tn")),
                       L.TsCols(p("em"), p("el"), p("en")), p("st"), p("ko"), p("kc"))
        self.ctx.check(self.ctx._lib.acc_cfk_update(self.ctx.handle, self._h, C.byref(bi)))

    def view(self) -> "L.BatchIn":
        """The store as an acc_batch_in of device pointers (valid until the next update)."""
        v = L.BatchIn()
        self.ctx.check(self.ctx._lib.acc_cfk_view(self.ctx.handle, self._h, C.byref(v)))
        return v

    def snapshot(self):
        """Host copy of the store (a workload.Batch)."""
        from .workload import Batch
        v = self.view()
        n, P = int(v.n_txn), int(v.n_pairs)
        g = lambda ptr, cnt, dt: device_array(self.ctx, ptr, cnt, dt)  # noqa: E731
        return Batch(g(v.txn_id.msb, n, np.uint64), g(v.txn_id.lsb, n, np.uint64), g(v.txn_id.node, n, np.int32),
                     g(v.execute_at.msb, n, np.uint64), g(v.execute_at.lsb, n, np.uint64), g(v.execute_at.node, n, np.int32),
                     g(v.status, n, np.uint8), g(v.key_off, n + 1, np.uint32), g(v.key_code, P, np.uint64))

    def calculate_partial_deps(self) -> "BatchKeyDeps":
        """PreAccept.calculatePartialDeps for every txn of the store, read in place (no host round trip)."""
        view = self.ctx.keydeps_batch_raw(self.view())
        return self.ctx.copy_out(view, None)

    def apply_deps(self, upd: dict):
        """CommandsForKey.update with each command's deps on the store itself (acc_cfk_apply_deps; the cfk_apply
        update layout): missing[] maintained, the txn-major view and its missing[] indices rebuilt."""
        b = _cfk_updates_host(upd)
        self.ctx.check(self.ctx._lib.acc_cfk_apply_deps(self.ctx.handle, self._h, C.byref(_cfk_updates_in(b))))

    def state(self) -> dict:
        """Host copy of the key-major CommandsForKey state (the cfk_apply snapshot layout)."""
        s = L.CfkSnap()
        self.ctx.check(self.ctx._lib.acc_cfk_state(self.ctx.handle, self._h, C.byref(s)))
        return _snap_host(self.ctx, s)

    def missing_view(self) -> "L.CfkBatchView":
        """The store's txn-major view with each pair's missing[] as txn indices (device), for cfk_map_reduce_full."""
        bv = L.CfkBatchView()
        self.ctx.check(self.ctx._lib.acc_cfk_missing(self.ctx.handle, self._h, C.byref(bv)))
        return bv


class ReplicaStore:
    """A replica CommandStore's PreAccept path on device-resident state (SURVEY.md §8(f) N4 in steady state): per batch
    of commands, the store's MaxConflicts proposes each new txn's executeAt (CommandStore.preaccept,
    local/CommandStore.java:320-345), the batch's executeAts merge into it (updateMaxConflicts, :280-290), every key's
    CommandsForKey takes the updates with deps (CommandsForKey.update, local/CommandsForKey.java:652-706, through
    acc_cfk_apply_deps: the key-major state and the txn-major view with missing[] indices stay in HBM), and the KeyDeps
    scan reads the updated store in place (PreAccept.calculatePartialDeps, messages/PreAccept.java:107-138). A batch's
    commands are concurrent: its proposals see MaxConflicts as of the previous batch."""

    def __init__(self, ctx: Context, end_inclusive: int = 1):
        self.ctx = ctx
        self.end_inclusive = int(end_inclusive)
        self.cfk = CfkStore(ctx)
        self.mc = MaxConflictsMap(ctx, end_inclusive)

    def preaccept_batch(self, part: dict, queries: dict | None = None, scan: bool = True) -> dict:
        """part: the batch's updates (cfk_update_stream layout); queries: its PreAccept queries (default: one per
        command first seen in part). Returns dict(propose = MaxConflicts.get + fast path per query, keydeps = the
        KeyDeps of every txn of the store after the batch, when scan)."""
        from . import workload as W
        q = W.preaccept_queries(part) if queries is None else queries
        out = dict(propose=self.mc.get(q))
        self.mc.update(W.conflicts_updates(part, self.end_inclusive))
        self.cfk.apply_deps(part)
        if scan:
            out["keydeps"] = self.cfk.calculate_partial_deps()
        return out

    def close(self):
        self.cfk.close()
        self.mc.close()
