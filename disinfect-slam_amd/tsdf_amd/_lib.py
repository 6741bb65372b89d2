"""ctypes binding of libdisinfect_tsdf.so (include/disinfect_tsdf.h).

The HIP engine is the only implementation: if the shared library is missing or cannot be loaded
this module raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_DIR, "libdisinfect_tsdf.so")

TSDF_OK = 0
TSDF_ERR_CAPACITY = 4
TSDF_MEM_HOST = 0
TSDF_MEM_DEVICE = 1
STATUS_POOL_EXHAUSTED = 1
STATUS_NEWKEY_OVERFLOW = 2
STATUS_DDA_OVERFLOW = 4
STATUS_RESOLVE_ABORT = 8
STATUS_SHARD_OVERFLOW = 16
STATUS_SHARD_ABORTED = 32
STATUS_PIPELINE_TIMEOUT = 64
TSDF_ERR_PIPELINE = 6
SHARD_RECORD_BYTES = 16


class Config(C.Structure):
    _fields_ = [
        ("voxel_size", C.c_float),
        ("truncation", C.c_float),
        ("max_width", C.c_int),
        ("max_height", C.c_int),
        ("num_block_bits", C.c_int),
        ("shard_index", C.c_int),
        ("shard_count", C.c_int),
        ("stream", C.c_void_p),
        ("use_stream", C.c_int),
    ]


class Intrinsics(C.Structure):
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float)]


class Pose(C.Structure):
    _fields_ = [(n, C.c_float) for n in ("qx", "qy", "qz", "qw", "tx", "ty", "tz")]


class Frame(C.Structure):
    _fields_ = [
        ("width", C.c_int),
        ("height", C.c_int),
        ("rgb", C.c_void_p),
        ("depth", C.c_void_p),
        ("ht", C.c_void_p),
        ("lt", C.c_void_p),
        ("mem_kind", C.c_int),
    ]


class Stats(C.Structure):
    _fields_ = [
        ("frames", C.c_int64),
        ("active_blocks", C.c_int32),
        ("free_blocks", C.c_int32),
        ("last_num_visible", C.c_int32),
        ("last_num_alloc", C.c_int32),
        ("last_num_deleted", C.c_int32),
        ("last_num_new_keys", C.c_int32),
        ("last_num_updated", C.c_int64),
        ("total_visible", C.c_int64),
        ("total_updated", C.c_int64),
        ("total_alloc", C.c_int64),
        ("total_deleted", C.c_int64),
        ("status", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


class Profile(C.Structure):
    _fields_ = [
        ("frames", C.c_int64),
        ("ms_allocate", C.c_double),
        ("ms_visible", C.c_double),
        ("ms_integrate", C.c_double),
        ("ms_carve", C.c_double),
        ("sum_visible", C.c_int64),
        ("sum_updated", C.c_int64),
        ("ms_integrate_device", C.c_double),
        ("calls", C.c_int64),
        ("ms_ingest_device", C.c_double),
        ("ms_resolve_alloc_device", C.c_double),
        ("ms_resolve_delete_device", C.c_double),
        ("pipelined", C.c_int64),
    ]


EXPORTS = [
    "tsdf_config_default", "tsdf_create", "tsdf_destroy", "tsdf_integrate", "tsdf_raycast",
    "tsdf_query", "tsdf_extract_mesh", "tsdf_get_stats", "tsdf_synchronize", "tsdf_flush", "tsdf_profile_begin", "tsdf_profile_end",
    "tsdf_debug_dump", "tsdf_debug_stamps", "tsdf_num_entries", "tsdf_num_blocks", "tsdf_hash_allocate",
    "tsdf_hash_delete", "tsdf_hash_retrieve", "tsdf_hash_assign", "tsdf_num_active_blocks",
    "tsdf_pool_acquire", "tsdf_pool_release", "tsdf_pool_set_weight", "tsdf_pool_get_weights",
    "tsdf_hash_block", "tsdf_block_owner", "tsdf_error_string", "tsdf_last_error",
    "tsdf_shard_slot_bytes", "tsdf_integrate_shard_begin", "tsdf_integrate_shard_update",
    "tsdf_integrate_shard_end", "tsdf_integrate_shard_abort", "tsdf_stream_wait", "tsdf_stream_signal", "tsdf_get_stream",
    "tsdf_feed_rgbd_frame", "tsdf_rgbd_half", "tsdf_graph_create", "tsdf_graph_create_deferred", "tsdf_graph_frame", "tsdf_graph_destroy",
    "tsdf_snapshot_bytes", "tsdf_snapshot_save", "tsdf_snapshot_load",
    "tsdf_render_blocks", "tsdf_import_blocks", "tsdf_reset", "tsdf_pack_blocks",
    "tsdf_raycast_rows", "tsdf_raycast_deferred", "tsdf_render_bands", "tsdf_pack_halo", "tsdf_extract_mesh_owned",
    "tsdf_graph_create_shard", "tsdf_graph_shard_begin", "tsdf_graph_shard_update", "tsdf_graph_shard_end",
    "tsdf_integrate_shard_pipe",
    "tsdf_graph_create_batch",
    "tsdf_group_create", "tsdf_group_destroy", "tsdf_group_size", "tsdf_group_integrate", "tsdf_group_flush",
    "tsdf_group_synchronize", "tsdf_group_shard", "tsdf_group_get_stats", "tsdf_group_query", "tsdf_group_raycast",
    "tsdf_group_stream_signal",
]

_lib = None


def load(path: str | None = None):
    """Load (once) and type the engine library. Raises OSError if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    # TSDF_AMD_LIB selects an alternative build of the same ABI (e.g. the DIAG=1 stamp variant)
    path = path or os.environ.get("TSDF_AMD_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise OSError(f"HIP engine library not built: {path} (run __graft_entry__.build())")
    L = C.CDLL(path)
    P = C.c_void_p
    i, i64, f = C.c_int, C.c_int64, C.c_float
    L.tsdf_config_default.argtypes = [C.POINTER(Config)]
    L.tsdf_create.argtypes = [C.POINTER(Config), i, C.POINTER(P)]
    L.tsdf_destroy.argtypes = [P]
    L.tsdf_integrate.argtypes = [P, C.POINTER(Frame), C.POINTER(Intrinsics), C.POINTER(Pose), f]
    L.tsdf_raycast.argtypes = [P, C.POINTER(Intrinsics), i, i, C.POINTER(Pose), f, P, P, i]
    L.tsdf_shard_slot_bytes.restype = C.c_int64
    L.tsdf_shard_slot_bytes.argtypes = [C.c_int32]
    L.tsdf_integrate_shard_begin.argtypes = [P, C.POINTER(Frame), C.POINTER(Intrinsics), C.POINTER(Pose), f,
                                             C.c_int32, C.c_int32, P, C.c_int32]
    L.tsdf_integrate_shard_update.argtypes = [P, P, C.c_int32, P, C.c_int32]
    L.tsdf_integrate_shard_end.argtypes = [P, P, C.c_int32]
    L.tsdf_integrate_shard_abort.argtypes = [P]
    L.tsdf_integrate_shard_pipe.argtypes = [P, C.POINTER(Frame), C.POINTER(Intrinsics), C.POINTER(Pose), f, P, P,
                                            C.c_int32, C.POINTER(C.c_int32)]
    L.tsdf_group_create.argtypes = [C.POINTER(Config), C.POINTER(i), i, C.POINTER(P)]
    L.tsdf_group_destroy.argtypes = [P]
    L.tsdf_group_size.argtypes = [P]
    L.tsdf_group_integrate.argtypes = [P, C.POINTER(Frame), C.POINTER(Intrinsics), C.POINTER(Pose), f]
    L.tsdf_group_flush.argtypes = [P]
    L.tsdf_group_synchronize.argtypes = [P]
    L.tsdf_group_shard.argtypes = [P, i, C.POINTER(P)]
    L.tsdf_group_get_stats.argtypes = [P, C.POINTER(Stats), i]
    L.tsdf_group_query.argtypes = [P, P, P, i64, C.POINTER(i64)]
    L.tsdf_group_raycast.argtypes = [P, C.POINTER(Intrinsics), i, i, C.POINTER(Pose), f, P, P, i]
    L.tsdf_group_stream_signal.argtypes = [P, P]
    L.tsdf_stream_wait.argtypes = [P, P]
    L.tsdf_stream_signal.argtypes = [P, P]
    L.tsdf_get_stream.argtypes = [P, C.POINTER(P)]
    L.tsdf_feed_rgbd_frame.argtypes = [P, P, P, P, i, i, f, C.POINTER(Intrinsics), C.POINTER(Pose), f, i]
    L.tsdf_rgbd_half.argtypes = [P, P, P, P, i, i, f, P, P, i]
    L.tsdf_graph_create.argtypes = [P, i, i, i, i, C.POINTER(P)]
    L.tsdf_graph_create_deferred.argtypes = [P, i, i, i, i, C.POINTER(P)]
    L.tsdf_graph_create_batch.argtypes = [P, i, i, i, i, i, i, C.POINTER(P)]
    L.tsdf_graph_frame.argtypes = [P, C.POINTER(Frame), C.POINTER(Intrinsics), C.POINTER(Pose), f,
                                   C.POINTER(Intrinsics), C.POINTER(Pose), P, P]
    L.tsdf_graph_destroy.argtypes = [P]
    L.tsdf_graph_create_shard.argtypes = [P, i, i, i, i, C.POINTER(P)]
    L.tsdf_graph_shard_begin.argtypes = [P, C.POINTER(Frame), C.POINTER(Intrinsics), C.POINTER(Pose), f,
                                         P, P, C.c_int32, P, P, C.c_int32]
    L.tsdf_graph_shard_update.argtypes = [P]
    L.tsdf_graph_shard_end.argtypes = [P]
    L.tsdf_snapshot_bytes.argtypes = [P, C.POINTER(i64)]
    L.tsdf_snapshot_save.argtypes = [P, P, i64]
    L.tsdf_snapshot_load.argtypes = [P, P, i64]
    L.tsdf_render_blocks.argtypes = [P, C.POINTER(Intrinsics), i, i, C.POINTER(Pose), f, P, i64,
                                     C.POINTER(i64), i]
    L.tsdf_import_blocks.argtypes = [P, P, i64, i, i]
    L.tsdf_raycast_rows.argtypes = [P, C.POINTER(Intrinsics), i, i, C.POINTER(Pose), f, i, i, P, P, i]
    L.tsdf_raycast_deferred.argtypes = [P, C.POINTER(Intrinsics), i, i, C.POINTER(Pose), f, P, P]
    L.tsdf_render_bands.argtypes = [P, C.POINTER(Intrinsics), i, i, C.POINTER(Pose), f, i, P, P, i64,
                                    P, i]
    L.tsdf_pack_halo.argtypes = [P, P, i64, P, i]
    L.tsdf_extract_mesh_owned.argtypes = [P, P, f, i, i, i, P, i64, C.POINTER(i64), i]
    L.tsdf_reset.argtypes = [P]
    L.tsdf_pack_blocks.argtypes = [P, P, P, i64, C.POINTER(i64), i]
    L.tsdf_query.argtypes = [P, P, P, i64, C.POINTER(i64)]
    L.tsdf_extract_mesh.argtypes = [P, P, f, i, P, i64, C.POINTER(i64), i]
    L.tsdf_get_stats.argtypes = [P, C.POINTER(Stats), i]
    L.tsdf_synchronize.argtypes = [P]
    L.tsdf_flush.argtypes = [P]
    L.tsdf_profile_begin.argtypes = [P, i, i]
    L.tsdf_profile_end.argtypes = [P, C.POINTER(Profile)]
    L.tsdf_debug_dump.argtypes = [P, P, P, P, P, P, P, P]
    L.tsdf_debug_stamps.argtypes = [P, P, i64, C.POINTER(i)]
    L.tsdf_num_entries.restype = C.c_int32
    L.tsdf_num_entries.argtypes = []
    L.tsdf_num_blocks.restype = C.c_int32
    L.tsdf_num_blocks.argtypes = [P]
    L.tsdf_hash_allocate.argtypes = [P, P, i]
    L.tsdf_hash_delete.argtypes = [P, P, i]
    L.tsdf_hash_retrieve.argtypes = [P, P, i, P, P, P, P, P]
    L.tsdf_hash_assign.argtypes = [P, P, i, P, C.POINTER(i)]
    L.tsdf_num_active_blocks.argtypes = [P, C.POINTER(C.c_int32)]
    L.tsdf_pool_acquire.argtypes = [P, i, P]
    L.tsdf_pool_release.argtypes = [P, P, i]
    L.tsdf_pool_set_weight.argtypes = [P, C.c_int32, C.c_uint8]
    L.tsdf_pool_get_weights.argtypes = [P, C.c_int32, P]
    L.tsdf_hash_block.restype = C.c_uint32
    L.tsdf_hash_block.argtypes = [C.c_int16, C.c_int16, C.c_int16]
    L.tsdf_block_owner.restype = C.c_int32
    L.tsdf_block_owner.argtypes = [C.c_int16, C.c_int16, C.c_int16, C.c_int32]
    L.tsdf_error_string.restype = C.c_char_p
    L.tsdf_error_string.argtypes = [i]
    L.tsdf_last_error.restype = C.c_char_p
    L.tsdf_last_error.argtypes = []
    for name in ("tsdf_create", "tsdf_destroy", "tsdf_integrate", "tsdf_raycast", "tsdf_query",
                 "tsdf_integrate_shard_begin", "tsdf_integrate_shard_update", "tsdf_integrate_shard_end",
                 "tsdf_integrate_shard_abort", "tsdf_stream_wait", "tsdf_stream_signal", "tsdf_get_stream",
                 "tsdf_feed_rgbd_frame", "tsdf_rgbd_half", "tsdf_graph_create", "tsdf_graph_create_deferred", "tsdf_graph_frame",
                 "tsdf_graph_destroy", "tsdf_snapshot_bytes", "tsdf_snapshot_save", "tsdf_snapshot_load",
                 "tsdf_extract_mesh", "tsdf_raycast_rows", "tsdf_raycast_deferred", "tsdf_render_bands", "tsdf_pack_halo",
                 "tsdf_extract_mesh_owned", "tsdf_render_blocks", "tsdf_import_blocks", "tsdf_reset",
                 "tsdf_pack_blocks", "tsdf_graph_create_shard", "tsdf_graph_shard_begin",
                 "tsdf_graph_shard_update", "tsdf_graph_shard_end", "tsdf_integrate_shard_pipe",
                 "tsdf_get_stats", "tsdf_synchronize", "tsdf_flush", "tsdf_profile_begin", "tsdf_profile_end",
                 "tsdf_debug_dump", "tsdf_debug_stamps", "tsdf_hash_allocate", "tsdf_hash_delete",
                 "tsdf_hash_retrieve",
                 "tsdf_hash_assign", "tsdf_num_active_blocks", "tsdf_pool_acquire",
                 "tsdf_pool_release", "tsdf_pool_set_weight", "tsdf_pool_get_weights",
                 "tsdf_graph_create_batch",
                 "tsdf_group_create", "tsdf_group_destroy", "tsdf_group_size", "tsdf_group_integrate",
                 "tsdf_group_flush", "tsdf_group_synchronize", "tsdf_group_shard", "tsdf_group_get_stats",
                 "tsdf_group_query", "tsdf_group_raycast", "tsdf_group_stream_signal"):
        getattr(L, name).restype = C.c_int
    _lib = L
    return L


class TSDFError(RuntimeError):
    pass


def check(rc: int, what: str):
    if rc != TSDF_OK:
        L = load()
        raise TSDFError(f"{what}: {L.tsdf_error_string(rc).decode()} "
                        f"({L.tsdf_last_error().decode()})")
