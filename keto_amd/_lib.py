"""ctypes binding of libketogpu.so (include/ketogpu.h).  Fails loudly when the HIP library is
missing -- there is no CPU fallback on the product path."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# KG_LIB_PATH: another build of the same library (A/B runs of bench.py on one box)
LIB_PATH = os.environ.get("KG_LIB_PATH") or os.path.join(HERE, "lib", "libketogpu.so")

KG_SUBJECT_ID = 0xFFFFFFFF
KG_NOT_MEMBER, KG_IS_MEMBER, KG_ERROR = 0, 1, 2
KG_FREC_HIT = 0xFFFFFFFF
KG_FREC_ERR = 0xFFFFFFFE
KG_SHARD_MAX_RANKS = 64
KG_ERR_NONE, KG_ERR_RELATION_NOT_FOUND, KG_ERR_NOT_IMPLEMENTED, KG_ERR_REWRITE_CYCLE, KG_ERR_RESOURCE = 0, 1, 2, 3, 4


KG_PACK_ID_MAX = 4094
KG_PACK_SUBJECT_ID = 4095


def pack_queries(q: "np.ndarray") -> "np.ndarray":
    """kg_pack_query (include/ketogpu.h) over an (n, 7) uint32 kg_query array: (n, 4) uint32 kg_query_packed
    rows.  Raises ValueError when an id does not fit (namespace / relation ids <= KG_PACK_ID_MAX)."""
    import numpy as np
    q = np.ascontiguousarray(q, dtype=np.uint32).reshape(-1, 7)
    sid = q[:, 3] == 0xFFFFFFFF
    sns = np.where(sid, KG_PACK_SUBJECT_ID, q[:, 3]).astype(np.uint64)
    srel = np.where(sid, 0, q[:, 5]).astype(np.uint64)
    d = q[:, 6].view(np.int32).astype(np.int64)
    d = np.clip(d, 0, 65535).astype(np.uint64)
    if (q[:, 0] > KG_PACK_ID_MAX).any() or (q[:, 2] > KG_PACK_ID_MAX).any() or \
            ((sns > KG_PACK_ID_MAX) & ~sid).any() or (srel > KG_PACK_ID_MAX).any():
        raise ValueError("an id does not fit kg_query_packed (use kg_check_batch)")
    out = np.empty((len(q), 4), np.uint32)
    out[:, 0] = q[:, 1]
    out[:, 1] = q[:, 4]
    out[:, 2] = (q[:, 0].astype(np.uint64) | (q[:, 2].astype(np.uint64) << 12) | ((sns & 0xFF) << 24)).astype(np.uint32)
    out[:, 3] = ((sns >> 8) | (srel << 4) | (d << 16)).astype(np.uint32)
    return out


class kg_tuple(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("ns", "obj", "rel", "sns", "sobj", "srel")]


class kg_query(C.Structure):
    _fields_ = [("t", kg_tuple), ("max_depth", C.c_int32)]


class kg_set(C.Structure):
    _fields_ = [("sns", C.c_uint32), ("sobj", C.c_uint32), ("srel", C.c_uint32), ("max_depth", C.c_int32)]


class kg_dict(C.Structure):
    _fields_ = [("n_namespaces", C.c_uint32), ("n_relations", C.c_uint32), ("wildcard_rel", C.c_uint32)]


class kg_rw_node(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("kind", "rel", "crel", "first", "count")]


class kg_rewrite_prog(C.Structure):
    _fields_ = [("n_ns", C.c_uint32), ("ns_has_rel", C.c_void_p), ("n_rel", C.c_uint32), ("rel_ns", C.c_void_p),
                ("rel_rel", C.c_void_p), ("rel_root", C.c_void_p), ("n_rw", C.c_uint32), ("rw", C.c_void_p),
                ("n_child", C.c_uint32), ("child", C.c_void_p)]


class kg_stats(C.Structure):
    _fields_ = [("rows_opened", C.c_uint64), ("edges_read", C.c_uint64), ("direct_probes", C.c_uint64),
                ("frontier_hbm", C.c_uint64), ("n_light", C.c_uint64), ("n_heavy", C.c_uint64),
                ("n_general", C.c_uint64), ("n_medium", C.c_uint64), ("light_rows_opened", C.c_uint64), ("light_edges_read", C.c_uint64),
                ("light_probes", C.c_uint64), ("kernel_ms", C.c_double), ("light_ms", C.c_double),
                ("n_wide", C.c_uint64), ("n_grid", C.c_uint64),
                ("n_back", C.c_uint64), ("n_no_holder", C.c_uint64), ("back_rows", C.c_uint64),
                ("back_edges", C.c_uint64), ("light_steps", C.c_uint64), ("light_waves", C.c_uint64),
                ("light_wave_ticks", C.c_uint64),
                ("light_span_ticks", C.c_uint64), ("light_wave_max_ticks", C.c_uint64),
                ("tail_ms", C.c_double), ("tail_launches", C.c_uint64), ("tail_kind", C.c_uint64),
                ("tail_rows", C.c_uint64), ("tail_edges", C.c_uint64), ("tail_probes", C.c_uint64),
                ("tail_logged", C.c_uint64), ("ms_edges_loaded", C.c_uint64), ("ms_words_active", C.c_uint64),
                ("split_ms", C.c_double)]

    def as_dict(self) -> dict:
        return {n: getattr(self, n) for n, _ in self._fields_}


class kg_tree_node(C.Structure):
    _fields_ = [("type", C.c_uint8), ("is_set", C.c_uint8), ("pad", C.c_uint16), ("ns", C.c_uint32),
                ("obj", C.c_uint32), ("rel", C.c_uint32), ("n_children", C.c_uint32)]


class kg_tree_buf(C.Structure):
    _fields_ = [("nodes", C.POINTER(kg_tree_node)), ("n_nodes", C.c_uint64), ("root_off", C.POINTER(C.c_uint64)),
                ("n_roots", C.c_uint64), ("kernel_ms", C.c_double), ("pinned", C.c_uint64)]


class kg_synth_params(C.Structure):
    _fields_ = [("n_tuples_target", C.c_uint64), ("seed", C.c_uint64), ("n_layers", C.c_uint32),
                ("max_degree", C.c_uint32), ("set_fraction", C.c_float), ("doc_set_fraction", C.c_float),
                ("preset", C.c_uint32), ("doc_alpha", C.c_float), ("group_alpha", C.c_float)]


# every symbol include/ketogpu.h declares
EXPORTS = ["kg_snapshot_create", "kg_snapshot_create_on", "kg_snapshot_synthetic", "kg_snapshot_synthetic_on",
           "kg_snapshot_replicas", "kg_snapshot_destroy", "kg_snapshot_info", "kg_snapshot_materialized", "kg_snapshot_tune", "kg_synth_ids",
           "kg_snapshot_create_ordered", "kg_snapshot_apply",
           "kg_snapshot_export", "kg_snapshot_rows", "kg_snapshot_export_csr", "kg_check_batch", "kg_check_batch_device", "kg_check_batch_packed_device", "kg_pack_queries_device", "kg_synth_queries",
           "kg_expand_batch", "kg_expand_batch_device", "kg_tree_free", "kg_last_error", "kg_version", "kg_check_batch_packed", "kg_shard_owner", "kg_snapshot_create_shard",
           "kg_snapshot_synthetic_shard", "kg_shard_seed", "kg_shard_level", "kg_shard_level_seg", "kg_shard_finish",
           "kg_shard_done", "kg_shard_levels", "kg_shard_back_list", "kg_shard_back_seed", "kg_shard_back_level", "kg_shard_refwd_seed",
           "kg_shard_held_words", "kg_shard_held", "kg_shard_result_slots", "kg_shard_bad_nodes", "kg_batcher_create", "kg_batcher_check", "kg_batcher_stats", "kg_batcher_reset_stats", "kg_batcher_destroy",
           "kg_shard_unique_id", "kg_shard_comm_init", "kg_shard_transport_attach", "kg_shard_comm_release",
           "kg_shard_comm_stats", "kg_shard_comm_stats_ex", "kg_shard_comm_levels", "kg_check_tree"]

KG_SHARD_UNIQUE_ID_BYTES = 128
# kg_shard_transport callbacks (include/ketogpu.h): collective over the ranks, 0 = success
ALLTOALL2_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t,
                           C.c_void_p)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t, C.c_void_p)


class kg_check_node(C.Structure):
    _fields_ = [("type", C.c_uint8), ("has_tuple", C.c_uint8), ("pad", C.c_uint16), ("n_children", C.c_uint32),
                ("t", kg_tuple)]


KG_CTREE = {1: "leaf", 2: "union", 3: "intersection", 4: "computed_subject_set", 5: "tuple_to_subject_set", 6: "not"}


class kg_shard_transport(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("rank", C.c_int32), ("world", C.c_int32), ("host_memory", C.c_int32),
                ("alltoall2", ALLTOALL2_FN), ("allgather", ALLGATHER_FN), ("allreduce_max_u64", ALLREDUCE_FN)]


class kg_batcher_stats_t(C.Structure):
    _fields_ = [("batches", C.c_uint64), ("checks", C.c_uint64), ("batch_p50_ms", C.c_double),
                ("batch_p99_ms", C.c_double), ("call_p50_ms", C.c_double), ("call_p99_ms", C.c_double)]


class KetoGPUError(RuntimeError):
    pass


_lib = None


def load(path: str = LIB_PATH):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise KetoGPUError(f"libketogpu.so not found at {path}: build it with `python -m keto_amd.build` "
                           "(there is no CPU fallback)")
    L = C.CDLL(path)
    vp, sz, i32, u32, u64 = C.c_void_p, C.c_size_t, C.c_int32, C.c_uint32, C.c_uint64
    L.kg_snapshot_create.argtypes = [vp, sz, C.POINTER(kg_dict), C.POINTER(kg_rewrite_prog), C.c_int, C.POINTER(vp)]
    L.kg_snapshot_create_on.argtypes = [vp, sz, C.POINTER(kg_dict), C.POINTER(kg_rewrite_prog), vp, C.c_int,
                                        C.POINTER(vp)]
    L.kg_snapshot_synthetic.argtypes = [C.POINTER(kg_synth_params), C.POINTER(kg_rewrite_prog), C.c_int,
                                        C.POINTER(vp)]
    L.kg_snapshot_synthetic_on.argtypes = [C.POINTER(kg_synth_params), C.POINTER(kg_rewrite_prog), vp, C.c_int,
                                           C.POINTER(vp)]
    L.kg_snapshot_replicas.argtypes = [vp, vp, C.c_int]
    L.kg_snapshot_destroy.argtypes = [vp]
    L.kg_snapshot_destroy.restype = None
    L.kg_snapshot_info.argtypes = [vp, vp]
    L.kg_snapshot_create_ordered.argtypes = [vp, vp, sz, vp, vp, vp, C.c_int, vp]
    L.kg_snapshot_apply.argtypes = [vp, vp, vp, sz, vp, sz, vp, vp, vp]
    L.kg_snapshot_materialized.argtypes = [vp, vp]
    L.kg_synth_ids.argtypes = [vp, vp]
    L.kg_snapshot_tune.argtypes = [vp, C.c_char_p, C.c_int64]
    L.kg_snapshot_export.argtypes = [vp, vp, u64]
    L.kg_snapshot_export.restype = C.c_int64
    L.kg_snapshot_rows.argtypes = [vp, vp, sz, vp, vp, u64]
    L.kg_snapshot_rows.restype = C.c_int64
    L.kg_snapshot_export_csr.argtypes = [vp, vp, vp, vp, vp, vp]
    L.kg_snapshot_export_csr.restype = C.c_int
    L.kg_check_batch.argtypes = [vp, vp, sz, i32, vp, vp, C.POINTER(kg_stats)]
    L.kg_check_batch_device.argtypes = [vp, vp, sz, i32, vp, vp, C.POINTER(kg_stats), vp]
    L.kg_check_batch_packed.argtypes = [vp, vp, sz, i32, vp, vp, vp, sz, C.POINTER(sz), C.POINTER(kg_stats)]
    L.kg_check_batch_packed_device.argtypes = [vp, vp, sz, i32, vp, vp, C.POINTER(kg_stats), vp]
    L.kg_pack_queries_device.argtypes = [vp, vp, sz, vp, vp]
    L.kg_synth_queries.argtypes = [vp, u64, sz, vp]
    L.kg_expand_batch.argtypes = [vp, vp, sz, i32, C.POINTER(kg_tree_buf)]
    L.kg_expand_batch_device.argtypes = [vp, vp, sz, i32, C.POINTER(kg_tree_buf), vp]
    L.kg_tree_free.argtypes = [C.POINTER(kg_tree_buf)]
    L.kg_tree_free.restype = None
    L.kg_last_error.argtypes = [C.c_char_p, sz]
    L.kg_last_error.restype = sz
    L.kg_version.restype = C.c_char_p
    L.kg_shard_owner.argtypes = [u32, u32, u32]
    L.kg_shard_owner.restype = u32
    L.kg_snapshot_create_shard.argtypes = [vp, sz, C.POINTER(kg_dict), C.POINTER(kg_rewrite_prog), C.c_int, u32, u32,
                                           C.POINTER(vp)]
    L.kg_snapshot_synthetic_shard.argtypes = [C.POINTER(kg_synth_params), C.POINTER(kg_rewrite_prog), C.c_int, u32,
                                              u32, C.POINTER(vp)]
    L.kg_shard_seed.argtypes = [vp, vp, sz, i32, vp, sz, vp, vp, vp, vp]
    L.kg_shard_level.argtypes = [vp, vp, sz, vp, vp, sz, vp, vp, vp, vp, C.c_uint32, vp]
    L.kg_shard_level_seg.argtypes = [vp, vp, C.c_uint32, sz, vp, vp, sz, vp, vp, vp, vp, C.c_uint32, vp]
    L.kg_shard_level_seg.restype = C.c_int
    L.kg_shard_done.argtypes = [vp, sz, vp, vp, C.c_int, vp, C.c_uint32, vp]
    L.kg_shard_levels.argtypes = [vp, i32, vp, vp, sz, vp, vp, i32, vp, vp, sz, i32, C.POINTER(i32), vp]
    L.kg_shard_levels.restype = C.c_int
    L.kg_shard_back_list.argtypes = [vp, sz, vp, vp, vp, sz, vp, vp]
    L.kg_shard_back_seed.argtypes = [vp, vp, sz, vp, vp, sz, vp, vp]
    L.kg_shard_back_level.argtypes = [vp, vp, sz, vp, vp, sz, vp, vp, vp, vp, C.c_uint32, vp]
    L.kg_shard_refwd_seed.argtypes = [vp, sz, vp, vp, vp, sz, vp, vp]
    L.kg_shard_held_words.argtypes = [vp, vp]
    L.kg_shard_held.argtypes = [vp, vp, sz, C.c_int, vp]
    L.kg_shard_bad_nodes.argtypes = [vp, vp]
    L.kg_shard_result_slots.argtypes = [vp, sz]
    L.kg_shard_result_slots.restype = sz
    L.kg_shard_finish.argtypes = [vp, sz, vp, vp, vp]
    L.kg_shard_unique_id.argtypes = [vp]
    L.kg_shard_comm_init.argtypes = [vp, vp, C.c_int, C.c_int, vp]
    L.kg_shard_transport_attach.argtypes = [vp, C.POINTER(kg_shard_transport), vp]
    L.kg_shard_comm_release.argtypes = [vp, vp]
    L.kg_shard_comm_stats.argtypes = [vp, vp, vp]
    L.kg_shard_comm_stats_ex.argtypes = [vp, vp, vp, sz]
    L.kg_shard_comm_levels.argtypes = [vp, vp, vp, sz]
    L.kg_shard_comm_levels.restype = C.c_int64
    L.kg_check_tree.argtypes = [vp, vp, i32, vp, sz, vp, sz, C.POINTER(sz), C.POINTER(C.c_uint8), C.POINTER(u32)]
    L.kg_batcher_create.argtypes = [vp, i32, sz, u32, C.c_int, C.POINTER(vp)]
    L.kg_batcher_check.argtypes = [vp, vp, sz, vp, vp]
    L.kg_batcher_stats.argtypes = [vp, C.POINTER(kg_batcher_stats_t)]
    L.kg_batcher_reset_stats.argtypes = [vp]
    L.kg_batcher_reset_stats.restype = None
    L.kg_batcher_destroy.argtypes = [vp]
    L.kg_batcher_destroy.restype = None
    for name in ("kg_snapshot_create", "kg_snapshot_create_on", "kg_snapshot_synthetic", "kg_snapshot_synthetic_on",
                 "kg_snapshot_replicas", "kg_snapshot_info", "kg_snapshot_materialized", "kg_snapshot_tune",
                 "kg_snapshot_create_ordered", "kg_snapshot_apply", "kg_synth_ids", "kg_check_batch", "kg_check_batch_packed",
                 "kg_check_batch_device", "kg_check_batch_packed_device", "kg_pack_queries_device", "kg_synth_queries",
                 "kg_expand_batch", "kg_expand_batch_device", "kg_snapshot_create_shard",
                 "kg_snapshot_synthetic_shard", "kg_shard_seed", "kg_shard_level", "kg_shard_level_seg", "kg_shard_finish",
                 "kg_shard_done", "kg_shard_levels", "kg_shard_back_list", "kg_shard_back_seed", "kg_shard_back_level", "kg_shard_refwd_seed",
                 "kg_shard_held_words", "kg_shard_held", "kg_batcher_create", "kg_batcher_check", "kg_batcher_stats",
                 "kg_shard_unique_id", "kg_shard_comm_init", "kg_shard_transport_attach", "kg_shard_comm_release",
                 "kg_shard_comm_stats", "kg_shard_comm_stats_ex", "kg_check_tree"):
        getattr(L, name).restype = C.c_int
    _lib = L
    return L


_hip = None


def device_to_host(dst: np.ndarray, src, nbytes: int) -> None:
    """hipMemcpy of nbytes from a device pointer the library returned (kg_expand_batch_device trees)
    into a host array: test and bench plumbing."""
    global _hip
    if nbytes == 0:
        return
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so")
        _hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        _hip.hipMemcpy.restype = C.c_int
    assert dst.nbytes >= nbytes
    rc = _hip.hipMemcpy(dst.ctypes.data_as(C.c_void_p), C.cast(src, C.c_void_p), nbytes, 2)  # hipMemcpyDeviceToHost
    if rc != 0:
        raise KetoGPUError(f"hipMemcpy device->host failed ({rc})")


def last_error() -> str:
    buf = C.create_string_buffer(2048)
    load().kg_last_error(buf, 2048)
    return buf.value.decode(errors="replace")


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise KetoGPUError(f"{what} failed ({rc}): {last_error()}")
