"""ctypes binding of include/accord_amd.h (libaccord_amd.so, built for gfx950).

The product path has no CPU fallback: if the HIP library is missing or cannot be loaded this module
raises, and every op fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# ACC_LIB_PATH: another build of the same library (A/B timing of two kernel variants in one GPU session)
LIB_PATH = os.environ.get("ACC_LIB_PATH") or os.path.join(HERE, "libaccord_amd.so")

ACC_OK, ACC_E_ARG, ACC_E_STATE, ACC_E_NOMEM, ACC_E_DEVICE, ACC_E_CAP = 0, -1, -2, -3, -4, -5
ACC_MEM_HOST, ACC_MEM_DEVICE = 0, 1
ACC_OPT_TIMING = 1
ACC_OPT_FORCE_REPLAY = 2
ACC_OPT_NO_WINDOW_TIER = 4
ACC_OPT_RD_WIDE_SORT = 8
ACC_OPT_PD_SERIAL = 16
ACC_LV_AUTO, ACC_LV_LDS_WALK, ACC_LV_WINDOWED, ACC_LV_WAVES = 0, 1, 2, 3
# SafeCommandStore.TestStartedAt / TestDep / TestStatus ordinals (local/SafeCommandStore.java:63-70)
ACC_STARTED_BEFORE, ACC_STARTED_AFTER, ACC_STARTED_ANY = 0, 1, 2
ACC_DEP_WITH, ACC_DEP_WITHOUT, ACC_DEP_ANY = 0, 1, 2
ACC_STATUS_ANY, ACC_STATUS_IS_PROPOSED, ACC_STATUS_IS_STABLE = 0, 1, 2
ACC_FULL_EXECUTES_AFTER = 1
ACC_LATEST_PROPOSAL, ACC_LATEST_COMMIT = 0, 1
# the four BeginRecovery scans (messages/BeginRecovery.java:334-378): (started_at, test_dep, test_status, executes_after)
RECOVERY_SCANS = {
    "acceptedOrCommittedStartedBeforeWithoutWitnessing": (ACC_STARTED_BEFORE, ACC_DEP_WITHOUT, ACC_STATUS_IS_PROPOSED, True),
    "stableStartedBeforeAndWitnessed": (ACC_STARTED_BEFORE, ACC_DEP_WITH, ACC_STATUS_IS_STABLE, False),
    "hasAcceptedOrCommittedStartedAfterWithoutWitnessing": (ACC_STARTED_AFTER, ACC_DEP_WITHOUT, ACC_STATUS_IS_PROPOSED, False),
    "hasStableExecutesAfterWithoutWitnessing": (ACC_STARTED_ANY, ACC_DEP_WITHOUT, ACC_STATUS_IS_STABLE, False),
}

u64p = C.POINTER(C.c_uint64)
u32p = C.POINTER(C.c_uint32)
i32p = C.POINTER(C.c_int32)
u8p = C.POINTER(C.c_uint8)

# Every symbol declared in include/accord_amd.h (tests check the library exports all of them).
EXPORTS = ["acc_create", "acc_destroy", "acc_last_error", "acc_sync", "acc_stream", "acc_version",
           "acc_keydeps_batch", "acc_keydeps_copy_out", "acc_keydeps_mixed", "acc_rangedeps_batch", "acc_rangedeps_copy_out",
           "acc_shard_pack", "acc_shard_merge", "acc_keydeps_merge", "acc_merge_copy_out", "acc_levelise",
           "acc_timing_count", "acc_timing_get", "acc_timing_reset", "acc_timing_filter", "acc_stats_count", "acc_stats_get",
           "acc_deps_merge", "acc_rmm_copy_out", "acc_rmm_invert", "acc_rmm_slice", "acc_rangedeps_stab", "acc_copy_out", "acc_comm_unique_id", "acc_comm_init_rccl", "acc_comm_init_host", "acc_comm_destroy", "acc_partial_deps_reduce", "acc_shard_reduce",
           "acc_map_reduce_full", "acc_map_reduce_full_ranges", "acc_latest_deps_merge", "acc_partial_deps_batch",
           "acc_deps_from_json", "acc_deps_to_json",
           "acc_cfk_create", "acc_cfk_destroy", "acc_cfk_update", "acc_cfk_view", "acc_cfk_apply", "acc_cfk_snap_to_batch",
           "acc_cfk_apply_deps", "acc_cfk_state", "acc_cfk_missing", "acc_max_conflicts",
           "acc_maxconflicts_create", "acc_maxconflicts_destroy", "acc_maxconflicts_update", "acc_maxconflicts_get",
           "acc_maxconflicts_size",
           "acc_ranges_of", "acc_ranges_with", "acc_ranges_subtract", "acc_ranges_merge_touching", "acc_ranges_select",
           "acc_ranges_index_of", "acc_ranges_contains_all_keys", "acc_ranges_contains_all", "acc_rangedeps_is_covered_by",
           "acc_partial_deps_covering", "acc_rmm_without", "acc_recovery_deps_reduce"]


class Opts(C.Structure):
    _fields_ = [("flags", C.c_uint32), ("reserved", C.c_uint32), ("cfk_hot", C.c_uint32), ("lv_tier", C.c_uint32),
                ("lv_chunk", C.c_uint32), ("reserved2", C.c_uint32)]


class TsCols(C.Structure):
    _fields_ = [("msb", C.c_void_p), ("lsb", C.c_void_p), ("node", C.c_void_p)]


class BatchIn(C.Structure):
    _fields_ = [("n_txn", C.c_uint32), ("mem", C.c_uint32), ("n_pairs", C.c_uint64),
                ("txn_id", TsCols), ("execute_at", TsCols),
                ("status", C.c_void_p), ("key_off", C.c_void_p), ("key_code", C.c_void_p)]


class KeydepsView(C.Structure):
    _fields_ = [("n_txn", C.c_uint32),
                ("total_arena", C.c_uint64), ("total_keys", C.c_uint64), ("total_deps", C.c_uint64),
                ("total_edges", C.c_uint64),
                ("arena_off", C.c_void_p), ("arena", C.c_void_p), ("kd_off", C.c_void_p),
                ("key_idx", C.c_void_p), ("u_off", C.c_void_p), ("dep_txn", C.c_void_p), ("kd_key", C.c_void_p)]


class KeydepsOut(C.Structure):
    _fields_ = [("mem", C.c_uint32),
                ("cap_arena", C.c_uint64), ("cap_keys", C.c_uint64), ("cap_deps", C.c_uint64),
                ("need_arena", C.c_uint64), ("need_keys", C.c_uint64), ("need_deps", C.c_uint64),
                ("arena_off", C.c_void_p), ("arena", C.c_void_p), ("kd_off", C.c_void_p),
                ("key_idx", C.c_void_p), ("u_off", C.c_void_p), ("dep_txn", C.c_void_p), ("kd_key", C.c_void_p)]


class RangeBatchIn(C.Structure):
    _fields_ = [("n_txn", C.c_uint32), ("mem", C.c_uint32), ("n_pairs", C.c_uint64), ("n_ranges", C.c_uint64),
                ("txn_id", TsCols), ("execute_at", TsCols),
                ("status", C.c_void_p), ("key_off", C.c_void_p), ("key_code", C.c_void_p),
                ("rng_off", C.c_void_p), ("rng_start", C.c_void_p), ("rng_end", C.c_void_p),
                ("end_inclusive", C.c_uint32), ("reserved", C.c_uint32)]


class RangedepsView(C.Structure):
    _fields_ = [("n_txn", C.c_uint32), ("n_ranges", C.c_uint32),
                ("total_arena", C.c_uint64), ("total_ranges", C.c_uint64), ("total_deps", C.c_uint64),
                ("total_edges", C.c_uint64),
                ("rng_start", C.c_void_p), ("rng_end", C.c_void_p),
                ("arena_off", C.c_void_p), ("arena", C.c_void_p), ("rd_off", C.c_void_p),
                ("range_id", C.c_void_p), ("u_off", C.c_void_p), ("dep_txn", C.c_void_p)]


class RangedepsOut(C.Structure):
    _fields_ = [("mem", C.c_uint32),
                ("cap_arena", C.c_uint64), ("cap_ranges", C.c_uint64), ("cap_deps", C.c_uint64), ("cap_dict", C.c_uint64),
                ("need_arena", C.c_uint64), ("need_ranges", C.c_uint64), ("need_deps", C.c_uint64),
                ("need_dict", C.c_uint64),
                ("rng_start", C.c_void_p), ("rng_end", C.c_void_p),
                ("arena_off", C.c_void_p), ("arena", C.c_void_p), ("rd_off", C.c_void_p),
                ("range_id", C.c_void_p), ("u_off", C.c_void_p), ("dep_txn", C.c_void_p)]


class MergeIn(C.Structure):
    _fields_ = [("mem", C.c_uint32), ("n_groups", C.c_uint32), ("n_replies", C.c_uint64),
                ("grp_off", C.c_void_p), ("key_off", C.c_void_p), ("key_code", C.c_void_p),
                ("val_off", C.c_void_p), ("txn_rank", C.c_void_p), ("k2v_off", C.c_void_p),
                ("k2v", C.c_void_p)]


class MergeView(C.Structure):
    _fields_ = [("n_groups", C.c_uint32),
                ("total_keys", C.c_uint64), ("total_vals", C.c_uint64), ("total_k2v", C.c_uint64),
                ("total_in_entries", C.c_uint64),
                ("key_off", C.c_void_p), ("key_code", C.c_void_p),
                ("val_off", C.c_void_p), ("txn_rank", C.c_void_p),
                ("k2v_off", C.c_void_p), ("k2v", C.c_void_p)]


class MergeOut(C.Structure):
    _fields_ = [("mem", C.c_uint32),
                ("cap_keys", C.c_uint64), ("cap_vals", C.c_uint64), ("cap_k2v", C.c_uint64),
                ("need_keys", C.c_uint64), ("need_vals", C.c_uint64), ("need_k2v", C.c_uint64),
                ("key_off", C.c_void_p), ("key_code", C.c_void_p),
                ("val_off", C.c_void_p), ("txn_rank", C.c_void_p),
                ("k2v_off", C.c_void_p), ("k2v", C.c_void_p)]


class FragStreams(C.Structure):
    _fields_ = [("world", C.c_uint32), ("mem", C.c_uint32),
                ("cap_frag", C.c_uint64), ("cap_keys", C.c_uint64), ("cap_vals", C.c_uint64), ("cap_k2v", C.c_uint64),
                ("hdr", C.c_void_p), ("keys", C.c_void_p), ("vals", C.c_void_p), ("k2v", C.c_void_p),
                ("frag_off", C.c_void_p), ("key_off", C.c_void_p), ("val_off", C.c_void_p), ("k2v_off", C.c_void_p),
                ("txn_global", C.c_void_p)]


class FragRecv(C.Structure):
    _fields_ = [("mem", C.c_uint32), ("world", C.c_uint32), ("rank", C.c_uint32), ("n_txn", C.c_uint32),
                ("n_frag", C.c_void_p), ("n_keys", C.c_void_p), ("n_vals", C.c_void_p), ("n_k2v", C.c_void_p),
                ("hdr", C.c_void_p), ("keys", C.c_void_p), ("vals", C.c_void_p), ("k2v", C.c_void_p)]


class RmmIn(C.Structure):
    _fields_ = [("key_off", C.c_void_p), ("key_a", C.c_void_p), ("key_b", C.c_void_p), ("val_off", C.c_void_p),
                ("txn", TsCols), ("k2v_off", C.c_void_p), ("k2v", C.c_void_p)]


class DepsMergeIn(C.Structure):
    _fields_ = [("mem", C.c_uint32), ("n_groups", C.c_uint32), ("n_replies", C.c_uint64), ("grp_off", C.c_void_p),
                ("key_deps", RmmIn), ("range_deps", RmmIn)]


class RmmView(C.Structure):
    _fields_ = [("total_keys", C.c_uint64), ("total_vals", C.c_uint64), ("total_k2v", C.c_uint64),
                ("key_off", C.c_void_p), ("key_a", C.c_void_p), ("key_b", C.c_void_p),
                ("val_off", C.c_void_p), ("txn_msb", C.c_void_p), ("txn_lsb", C.c_void_p), ("txn_node", C.c_void_p),
                ("txn_src", C.c_void_p), ("k2v_off", C.c_void_p), ("k2v", C.c_void_p)]


class DepsMergeView(C.Structure):
    _fields_ = [("n_groups", C.c_uint32), ("total_in_entries", C.c_uint64), ("key_deps", RmmView),
                ("range_deps", RmmView)]


class RList(C.Structure):
    """acc_rlist: a Ranges as parallel (start, end) code arrays"""
    _fields_ = [("start", C.c_void_p), ("end", C.c_void_p), ("n", C.c_uint32), ("reserved", C.c_uint32)]


class CoveringView(C.Structure):
    _fields_ = [("n_groups", C.c_uint32), ("n_coverings", C.c_uint32), ("cov_id", C.c_void_p), ("cov_off", C.c_void_p),
                ("cov_start", C.c_void_p), ("cov_end", C.c_void_p), ("store_mask", C.c_void_p),
                ("total_ranges", C.c_uint64)]


class RmmOut(C.Structure):
    _fields_ = [("mem", C.c_uint32),
                ("cap_keys", C.c_uint64), ("cap_vals", C.c_uint64), ("cap_k2v", C.c_uint64),
                ("need_keys", C.c_uint64), ("need_vals", C.c_uint64), ("need_k2v", C.c_uint64),
                ("key_off", C.c_void_p), ("key_a", C.c_void_p), ("key_b", C.c_void_p),
                ("val_off", C.c_void_p), ("txn_msb", C.c_void_p), ("txn_lsb", C.c_void_p), ("txn_node", C.c_void_p),
                ("txn_src", C.c_void_p), ("k2v_off", C.c_void_p), ("k2v", C.c_void_p)]


class RmmBatch(C.Structure):
    _fields_ = [("mem", C.c_uint32), ("n_groups", C.c_uint32), ("key_off", C.c_void_p), ("key_a", C.c_void_p),
                ("key_b", C.c_void_p), ("val_off", C.c_void_p), ("k2v_off", C.c_void_p), ("k2v", C.c_void_p)]


class CsrView(C.Structure):
    _fields_ = [("n_groups", C.c_uint32), ("total", C.c_uint64), ("off", C.c_void_p), ("ints", C.c_void_p)]


class RangesIn(C.Structure):
    _fields_ = [("off", C.c_void_p), ("start", C.c_void_p), ("end", C.c_void_p), ("end_inclusive", C.c_uint32),
                ("reserved", C.c_uint32)]


class SliceView(C.Structure):
    _fields_ = [("n_groups", C.c_uint32), ("total_keys", C.c_uint64), ("total_vals", C.c_uint64),
                ("total_k2v", C.c_uint64), ("key_off", C.c_void_p), ("key_idx", C.c_void_p), ("val_off", C.c_void_p),
                ("val_idx", C.c_void_p), ("k2v_off", C.c_void_p), ("k2v", C.c_void_p)]


ACC_WITHOUT_FROM, ACC_WITHOUT_NONE, ACC_WITHOUT_NEW = 0, 1, 2


class TxnSets(C.Structure):
    _fields_ = [("off", C.c_void_p), ("txn", TsCols)]


class WithoutView(C.Structure):
    _fields_ = [("sl", SliceView), ("kind", C.c_void_p), ("n_from", C.c_uint64), ("n_none", C.c_uint64),
                ("n_new", C.c_uint64)]


class RecoveryDepsView(C.Structure):
    _fields_ = [("committed", DepsMergeView), ("accepted_merged", DepsMergeView), ("accepted_key", WithoutView),
                ("accepted_range", WithoutView)]


class StabIn(C.Structure):
    _fields_ = [("mem", C.c_uint32), ("n_queries", C.c_uint32), ("grp", C.c_void_p), ("q_start", C.c_void_p),
                ("q_end", C.c_void_p), ("end_inclusive", C.c_uint32), ("want_txns", C.c_uint32)]


class StabView(C.Structure):
    _fields_ = [("n_queries", C.c_uint32), ("total_ranges", C.c_uint64), ("total_txns", C.c_uint64),
                ("range_off", C.c_void_p), ("range_idx", C.c_void_p), ("txn_off", C.c_void_p), ("txn_idx", C.c_void_p)]


class RecoveryIn(C.Structure):
    _fields_ = [("n_query", C.c_uint32), ("mem", C.c_uint32), ("test_txn", TsCols), ("key_off", C.c_void_p),
                ("key_code", C.c_void_p), ("missing_off", C.c_void_p), ("missing_txn", C.c_void_p),
                ("n_missing", C.c_uint64), ("started_at", C.c_uint8), ("test_dep", C.c_uint8),
                ("test_status", C.c_uint8), ("flags", C.c_uint8), ("test_kinds", C.c_int32)]


ACC_RCMD_ERASED, ACC_RCMD_HAS_DEPS, ACC_RCMD_HISTORICAL = 1, 2, 4


class RangeCmdsIn(C.Structure):
    _fields_ = [("n_cmd", C.c_uint32), ("mem", C.c_uint32), ("end_inclusive", C.c_uint32), ("txn_id", TsCols),
                ("execute_at", TsCols), ("status", C.c_void_p), ("flags", C.c_void_p), ("rng_off", C.c_void_p),
                ("rng_start", C.c_void_p), ("rng_end", C.c_void_p), ("dep_off", C.c_void_p), ("dep_txn", TsCols),
                ("dep_start", C.c_void_p), ("dep_end", C.c_void_p), ("dep_is_key", C.c_void_p)]


class RecoveryRangesIn(C.Structure):
    _fields_ = [("n_query", C.c_uint32), ("mem", C.c_uint32), ("test_txn", TsCols), ("part_is_range", C.c_void_p),
                ("part_off", C.c_void_p), ("part_start", C.c_void_p), ("part_end", C.c_void_p),
                ("started_at", C.c_uint8), ("test_dep", C.c_uint8), ("test_status", C.c_uint8), ("flags", C.c_uint8),
                ("test_kinds", C.c_int32)]


class CfkSnap(C.Structure):
    _fields_ = [("mem", C.c_uint32), ("n_keys", C.c_uint32), ("n_entries", C.c_uint64), ("n_missing", C.c_uint64),
                ("key", C.c_void_p), ("ent_off", C.c_void_p), ("txn_id", TsCols), ("execute_at", TsCols),
                ("status", C.c_void_p), ("miss_off", C.c_void_p), ("missing", TsCols)]


class CfkUpdates(C.Structure):
    _fields_ = [("mem", C.c_uint32), ("n_upd", C.c_uint32), ("n_pairs", C.c_uint64), ("n_deps", C.c_uint64),
                ("txn_id", TsCols), ("execute_at", TsCols), ("status", C.c_void_p), ("flags", C.c_void_p),
                ("key_off", C.c_void_p), ("key", C.c_void_p), ("dep_off", C.c_void_p), ("deps", TsCols)]


class CfkSnapView(C.Structure):
    _fields_ = [("n_keys", C.c_uint32), ("n_entries", C.c_uint64), ("n_missing", C.c_uint64), ("key", C.c_void_p),
                ("ent_off", C.c_void_p), ("txn_id", TsCols), ("execute_at", TsCols), ("status", C.c_void_p),
                ("miss_off", C.c_void_p), ("missing", TsCols)]


class CfkBatchView(C.Structure):
    _fields_ = [("batch", BatchIn), ("missing_off", C.c_void_p), ("missing_txn", C.c_void_p), ("n_missing", C.c_uint64)]


class ConflictsIn(C.Structure):
    _fields_ = [("mem", C.c_uint32), ("n_upd", C.c_uint32), ("end_inclusive", C.c_uint32), ("n_keys", C.c_uint64),
                ("n_ranges", C.c_uint64), ("execute_at", TsCols), ("key_off", C.c_void_p), ("key", C.c_void_p),
                ("rng_off", C.c_void_p), ("rng_start", C.c_void_p), ("rng_end", C.c_void_p)]


class PreacceptIn(C.Structure):
    _fields_ = [("mem", C.c_uint32), ("n_query", C.c_uint32), ("n_parts", C.c_uint64), ("txn_id", TsCols),
                ("is_range", C.c_void_p), ("part_off", C.c_void_p), ("part_start", C.c_void_p), ("part_end", C.c_void_p)]


class PreacceptOut(C.Structure):
    _fields_ = [("mem", C.c_uint32), ("max_msb", C.c_void_p), ("max_lsb", C.c_void_p), ("max_node", C.c_void_p),
                ("fast_path", C.c_void_p)]


class LatestIn(C.Structure):
    _fields_ = [("n_groups", C.c_uint32), ("mode", C.c_uint32), ("grp_off", C.c_void_p), ("iv_off", C.c_void_p),
                ("iv_start", C.c_void_p), ("iv_end", C.c_void_p), ("known", C.c_void_p), ("ballot", TsCols),
                ("coord_deps", C.c_void_p), ("local_deps", C.c_void_p), ("txn_id", TsCols), ("execute_at", TsCols),
                ("end_inclusive", C.c_uint32), ("deps_mem", C.c_uint32), ("n_deps", C.c_uint32),
                ("key_deps", RmmIn), ("range_deps", RmmIn)]


class LatestView(C.Structure):
    _fields_ = [("deps", DepsMergeView), ("total_sufficient", C.c_uint64), ("sufficient_off", u64p),
                ("sufficient_start", u64p), ("sufficient_end", u64p)]


class JsonIn(C.Structure):
    _fields_ = [("mem", C.c_uint32), ("n_docs", C.c_uint32), ("bytes", C.c_void_p), ("doc_off", C.c_void_p)]


class JsonDepsView(C.Structure):
    _fields_ = [("n_docs", C.c_uint32), ("deps", DepsMergeView), ("n_dict", C.c_uint64), ("dict_kind", C.c_void_p),
                ("dict_null", C.c_void_p), ("dict_value", C.c_void_p), ("dict_hash", C.c_void_p),
                ("dict_len", C.c_void_p), ("dict_str", C.c_void_p)]


class JsonOutIn(C.Structure):
    _fields_ = [("n_groups", C.c_uint32), ("key_deps", RmmView), ("range_deps", RmmView), ("n_dict", C.c_uint64),
                ("dict_kind", C.c_void_p), ("dict_null", C.c_void_p), ("dict_value", C.c_void_p),
                ("dict_len", C.c_void_p), ("dict_str", C.c_void_p)]


class JsonOut(C.Structure):
    _fields_ = [("mem", C.c_uint32), ("cap_bytes", C.c_uint64), ("need_bytes", C.c_uint64), ("bytes", C.c_void_p),
                ("doc_off", C.c_void_p)]


class GraphIn(C.Structure):
    _fields_ = [("mem", C.c_uint32), ("n", C.c_uint32),
                ("off", C.c_void_p), ("dep", C.c_void_p), ("exec_rank", C.c_void_p)]


# acc_alltoallv_fn: int (*)(void *user, const void *send, const uint64_t *send_bytes, void *recv, const uint64_t *recv_bytes)
AllToAllvFn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_void_p, C.POINTER(C.c_uint64))
ACC_COMM_ID_BYTES = 128

_lib = None


class _Tolerant:
    """A tuning build (ACC_LIB_PATH, e.g. an older library timed beside the current one) may lack the newest entry
    points: their signatures are skipped, and calling one fails with the library's own AttributeError."""

    class _Skip:
        """A missing acc_* symbol: signature assignments land here harmlessly; a call raises AttributeError."""

        def __init__(self, name):
            object.__setattr__(self, "_name", name)

        def __call__(self, *args, **kwargs):
            raise AttributeError(f"{self._name} not exported by {LIB_PATH}")

    def __init__(self, lib):
        object.__setattr__(self, "_l", lib)

    def __getattr__(self, name):
        try:
            return getattr(self._l, name)
        except AttributeError:
            if name.startswith("acc_"):
                return _Tolerant._Skip(name)
            raise


def load():
    """Load libaccord_amd.so; raises if it is missing (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"accord_amd: HIP library not built ({LIB_PATH}); run __graft_entry__.build()")
    # torch bundles its own libamdhip64.so.7 (same soname as /opt/rocm's). Whichever is loaded first serves the
    # whole process; if ours came first, torch's device init later fails ("No HIP GPUs are available"). Load
    # torch's first so the library and torch share one HIP runtime (and device buffers) when both are used.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    if os.environ.get("ACC_LIB_PATH"):
        L = _Tolerant(L)
    L.acc_create.argtypes = [C.c_int, C.POINTER(Opts), C.POINTER(C.c_void_p)]
    L.acc_create.restype = C.c_int
    L.acc_destroy.argtypes = [C.c_void_p]
    L.acc_destroy.restype = None
    L.acc_last_error.argtypes = [C.c_void_p]
    L.acc_last_error.restype = C.c_char_p
    L.acc_sync.argtypes = [C.c_void_p]
    L.acc_sync.restype = C.c_int
    L.acc_stream.argtypes = [C.c_void_p]
    L.acc_stream.restype = C.c_void_p
    L.acc_version.argtypes = []
    L.acc_version.restype = C.c_char_p
    L.acc_keydeps_batch.argtypes = [C.c_void_p, C.POINTER(BatchIn), C.POINTER(KeydepsView)]
    L.acc_keydeps_batch.restype = C.c_int
    L.acc_keydeps_copy_out.argtypes = [C.c_void_p, C.POINTER(KeydepsOut)]
    L.acc_keydeps_copy_out.restype = C.c_int
    L.acc_keydeps_mixed.argtypes = [C.c_void_p, C.POINTER(RangeBatchIn), C.POINTER(KeydepsView)]
    L.acc_keydeps_mixed.restype = C.c_int
    L.acc_rangedeps_batch.argtypes = [C.c_void_p, C.POINTER(RangeBatchIn), C.POINTER(RangedepsView)]
    L.acc_rangedeps_batch.restype = C.c_int
    L.acc_partial_deps_batch.argtypes = [C.c_void_p, C.POINTER(RangeBatchIn), C.POINTER(KeydepsView), C.POINTER(RangedepsView)]
    L.acc_partial_deps_batch.restype = C.c_int
    L.acc_rangedeps_copy_out.argtypes = [C.c_void_p, C.POINTER(RangedepsOut)]
    L.acc_rangedeps_copy_out.restype = C.c_int
    L.acc_shard_pack.argtypes = [C.c_void_p, C.POINTER(BatchIn), C.POINTER(FragStreams)]
    L.acc_shard_pack.restype = C.c_int
    L.acc_shard_merge.argtypes = [C.c_void_p, C.POINTER(FragRecv), C.POINTER(MergeView)]
    L.acc_shard_merge.restype = C.c_int
    L.acc_keydeps_merge.argtypes = [C.c_void_p, C.POINTER(MergeIn), C.POINTER(MergeView)]
    L.acc_keydeps_merge.restype = C.c_int
    L.acc_merge_copy_out.argtypes = [C.c_void_p, C.POINTER(MergeOut)]
    L.acc_merge_copy_out.restype = C.c_int
    L.acc_levelise.argtypes = [C.c_void_p, C.POINTER(GraphIn), u32p, u32p, u32p]
    L.acc_levelise.restype = C.c_int
    L.acc_deps_merge.argtypes = [C.c_void_p, C.POINTER(DepsMergeIn), C.POINTER(DepsMergeView)]
    L.acc_deps_merge.restype = C.c_int
    L.acc_rmm_copy_out.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(RmmView), C.POINTER(RmmOut)]
    L.acc_rmm_copy_out.restype = C.c_int
    L.acc_rmm_invert.argtypes = [C.c_void_p, C.POINTER(RmmBatch), C.POINTER(CsrView)]
    L.acc_rmm_invert.restype = C.c_int
    L.acc_rmm_slice.argtypes = [C.c_void_p, C.POINTER(RmmBatch), C.POINTER(RangesIn), C.POINTER(SliceView)]
    L.acc_rmm_slice.restype = C.c_int
    L.acc_rmm_without.argtypes = [C.c_void_p, C.POINTER(RmmBatch), C.POINTER(TsCols), C.POINTER(TxnSets),
                                  C.POINTER(TxnSets), C.POINTER(WithoutView)]
    L.acc_rmm_without.restype = C.c_int
    L.acc_recovery_deps_reduce.argtypes = [C.c_void_p, C.POINTER(DepsMergeIn), C.POINTER(DepsMergeIn),
                                           C.POINTER(RecoveryDepsView)]
    L.acc_recovery_deps_reduce.restype = C.c_int
    L.acc_rangedeps_stab.argtypes = [C.c_void_p, C.POINTER(RmmBatch), C.POINTER(StabIn), C.POINTER(StabView)]
    L.acc_rangedeps_stab.restype = C.c_int
    L.acc_comm_unique_id.argtypes = [C.c_void_p]
    L.acc_comm_unique_id.restype = C.c_int
    L.acc_comm_init_rccl.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.POINTER(C.c_void_p)]
    L.acc_comm_init_rccl.restype = C.c_int
    L.acc_comm_init_host.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, AllToAllvFn, C.c_void_p, C.POINTER(C.c_void_p)]
    L.acc_comm_init_host.restype = C.c_int
    L.acc_comm_destroy.argtypes = [C.c_void_p]
    L.acc_comm_destroy.restype = None
    L.acc_shard_reduce.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(BatchIn), C.c_void_p, C.c_uint32, C.POINTER(MergeView)]
    L.acc_shard_reduce.restype = C.c_int
    L.acc_partial_deps_reduce.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(RangeBatchIn), C.c_void_p, C.c_uint32,
                                          C.POINTER(RList), C.POINTER(MergeView), C.POINTER(DepsMergeView),
                                          C.POINTER(CoveringView)]
    L.acc_partial_deps_reduce.restype = C.c_int
    L.acc_partial_deps_covering.argtypes = [C.c_void_p, C.POINTER(RangeBatchIn), C.POINTER(RList)]
    L.acc_partial_deps_covering.restype = C.c_int
    L.acc_map_reduce_full.argtypes = [C.c_void_p, C.POINTER(BatchIn), C.POINTER(RecoveryIn), C.POINTER(KeydepsView)]
    L.acc_map_reduce_full.restype = C.c_int
    L.acc_map_reduce_full_ranges.argtypes = [C.c_void_p, C.POINTER(RangeCmdsIn), C.POINTER(RecoveryRangesIn),
                                             C.POINTER(RangedepsView)]
    L.acc_map_reduce_full_ranges.restype = C.c_int
    L.acc_latest_deps_merge.argtypes = [C.c_void_p, C.POINTER(LatestIn), C.POINTER(LatestView)]
    L.acc_latest_deps_merge.restype = C.c_int
    L.acc_deps_from_json.argtypes = [C.c_void_p, C.POINTER(JsonIn), C.POINTER(JsonDepsView)]
    L.acc_deps_from_json.restype = C.c_int
    L.acc_deps_to_json.argtypes = [C.c_void_p, C.POINTER(JsonOutIn), C.POINTER(JsonOut)]
    L.acc_deps_to_json.restype = C.c_int
    L.acc_cfk_create.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
    L.acc_cfk_create.restype = C.c_int
    L.acc_cfk_destroy.argtypes = [C.c_void_p]
    L.acc_cfk_destroy.restype = None
    L.acc_cfk_update.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(BatchIn)]
    L.acc_cfk_update.restype = C.c_int
    L.acc_cfk_view.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(BatchIn)]
    L.acc_cfk_view.restype = C.c_int
    L.acc_cfk_apply.argtypes = [C.c_void_p, C.POINTER(CfkSnap), C.POINTER(CfkUpdates), C.POINTER(CfkSnapView)]
    L.acc_cfk_apply.restype = C.c_int
    L.acc_cfk_snap_to_batch.argtypes = [C.c_void_p, C.POINTER(CfkSnap), C.POINTER(CfkBatchView)]
    L.acc_cfk_snap_to_batch.restype = C.c_int
    L.acc_max_conflicts.argtypes = [C.c_void_p, C.POINTER(ConflictsIn), C.POINTER(PreacceptIn), C.POINTER(PreacceptOut)]
    L.acc_max_conflicts.restype = C.c_int
    try:
        L.acc_cfk_apply_deps.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(CfkUpdates)]
        L.acc_cfk_apply_deps.restype = C.c_int
        L.acc_cfk_state.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(CfkSnap)]
        L.acc_cfk_state.restype = C.c_int
        L.acc_cfk_missing.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(CfkBatchView)]
        L.acc_cfk_missing.restype = C.c_int
        L.acc_maxconflicts_create.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_void_p)]
        L.acc_maxconflicts_create.restype = C.c_int
        L.acc_maxconflicts_destroy.argtypes = [C.c_void_p]
        L.acc_maxconflicts_destroy.restype = None
        L.acc_maxconflicts_update.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(ConflictsIn)]
        L.acc_maxconflicts_update.restype = C.c_int
        L.acc_maxconflicts_get.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(PreacceptIn), C.POINTER(PreacceptOut)]
        L.acc_maxconflicts_get.restype = C.c_int
        L.acc_maxconflicts_size.argtypes = [C.c_void_p]
        L.acc_maxconflicts_size.restype = C.c_uint64
    except AttributeError:
        if not os.environ.get("ACC_LIB_PATH"):   # an older tuning build (A/B runs) may lack them; the product may not
            raise
    L.acc_copy_out.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32]
    L.acc_copy_out.restype = C.c_int
    L.acc_timing_count.argtypes = [C.c_void_p]
    L.acc_timing_count.restype = C.c_int
    L.acc_timing_get.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_double),
                                 C.POINTER(C.c_uint64)]
    L.acc_timing_get.restype = C.c_int
    L.acc_timing_reset.argtypes = [C.c_void_p]
    L.acc_timing_reset.restype = None
    L.acc_timing_filter.argtypes = [C.c_void_p, C.c_char_p]
    L.acc_timing_filter.restype = C.c_int
    L.acc_stats_count.argtypes = [C.c_void_p]
    L.acc_stats_count.restype = C.c_int
    L.acc_stats_get.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_uint64)]
    L.acc_stats_get.restype = C.c_int
    _lib = L
    return L
