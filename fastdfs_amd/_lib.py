"""ctypes binding of libfdfs_gpu (include/fdfs_gpu.h).

There is no fallback: if the gfx950 library is missing this module raises,
and every compute entry point goes through the HIP kernels.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libfdfs_gpu.so")
# Measurement scripts (scripts/) may point this at the probe build
# (`make -C fastdfs_amd/csrc probes` -> lib/probes/libfdfs_gpu.so, whose
# FDFS_GPU_* knobs change results); the production library reads no
# environment.
if os.environ.get("FDFS_GPU_PROBE_LIB") == "1":
    LIB_PATH = os.path.join(_HERE, "lib", "probes", "libfdfs_gpu.so")
elif os.environ.get("FDFS_GPU_PROBE_LIB") == "ab":  # `make ab`: the previous form of a kernel, for A/B runs
    LIB_PATH = os.path.join(_HERE, "lib", "ab", "libfdfs_gpu.so")
elif os.environ.get("FDFS_GPU_PROBE_LIB", "").startswith("var:"):  # `make variant NAME=<x> EXTRA=...`
    LIB_PATH = os.path.join(_HERE, "lib", "var", os.environ["FDFS_GPU_PROBE_LIB"][4:], "libfdfs_gpu.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "fdfs_gpu.h")
# The test-hooks build (`make test-hooks`, part of `make all`): the same
# objects with fdfs_api.cpp compiled with FDFS_TEST_HOOKS, which adds
# fdfs_gpu_inject_error (fastdfs_amd/csrc/fdfs_test_hooks.h).  The shipped
# library does not export it; only the error-path tests load this one.
TEST_HOOKS_LIB_PATH = os.path.join(_HERE, "lib", "test", "libfdfs_gpu.so")

SIG_CRC_ONLY = 0
SIG_HASH = 1
SIG_MD5 = 2
FLAG_UNSIGNED_HASH = 0x1
FILE_SIGNATURE_SIZE = 24

# Every entry point declared in include/fdfs_gpu.h.
EXPORTS = (
    "fdfs_gpu_abi_version",
    "fdfs_gpu_open",
    "fdfs_gpu_close",
    "fdfs_gpu_reserve",
    "fdfs_gpu_sig_batch",
    "fdfs_gpu_dedup",
    "fdfs_gpu_dedup_bucket",
    "fdfs_gpu_dedup_group",
    "fdfs_gpu_set_timing",
    "fdfs_gpu_read_timing",
    "fdfs_gpu_crc_lane_min_files",
    "fdfs_gpu_file_ids",
    "fdfs_gpu_parse_file_ids",
    "fdfs_gpu_trunk_pack",
    "fdfs_gpu_trunk_unpack",
    "fdfs_gpu_fdht_route",
    "fdfs_gpu_fdht_route_keys",
    "fdfs_gpu_recovery_batch",
    "fdfs_gpu_sig_batch_host",
    "fdfs_gpu_scrub",
    "fdfs_gpu_last_error",
    "fdfs_gpu_state_init",
    "fdfs_gpu_update_batch",
    "fdfs_gpu_final_batch",
    "fdfs_gpu_crc_combine",
    "fdfs_gpu_dedup_packed",
    "fdfs_gpu_dedup_global",
    "fdfs_gpu_dedup_global_local",
    "fdfs_gpu_dedup_global_stats",
    "fdfs_gpu_crc_batch_global",
    "fdfs_gpu_crc_batch_global_local",
    "fdfs_gpu_comm_unique_id",
    "fdfs_gpu_comm_init",
    "fdfs_gpu_comm_destroy",
    "fdfs_gpu_index_create",
    "fdfs_gpu_index_destroy",
    "fdfs_gpu_index_ingest",
    "fdfs_gpu_index_stats",
    "fdfs_gpu_index_slots",
)
COMM_ID_BYTES = 128
FILE_STATE_SIZE = 128  # sizeof(fdfs_gpu_file_state)
KERNEL_SIG_LANE = 0
KERNEL_CRC_SEG = 1
KERNEL_DEDUP = 2
KERNEL_BUCKET = 3


class FdfsGpuBatch(ctypes.Structure):
    _fields_ = [
        ("base", ctypes.c_void_p),
        ("offset", ctypes.c_void_p),
        ("size", ctypes.c_void_p),
        ("n", ctypes.c_uint32),
    ]


class FdfsGpuRouted(ctypes.Structure):
    _fields_ = [(f, ctypes.c_void_p) for f in
                ("index", "key_hash", "group", "server", "order", "group_start")]


class FdfsGpuRecoveryOut(ctypes.Structure):
    _fields_ = [("crc", ctypes.c_void_p), ("sig", ctypes.c_void_p), ("rep", ctypes.c_void_p),
                ("ref", ctypes.c_void_p), ("nsources", ctypes.c_void_p),
                ("fid", FdfsGpuRouted), ("ref_rec", FdfsGpuRouted), ("sig_rec", FdfsGpuRouted)]


_lib = None


def load() -> ctypes.CDLL:
    """Load libfdfs_gpu.so; raises if it has not been built."""
    global _lib
    if _lib is None:
        _lib = _bind(LIB_PATH)
    return _lib


_hooks = None


def load_test_hooks() -> ctypes.CDLL:
    """The test-hooks build of the library (a second copy of every entry
    point plus fdfs_gpu_inject_error), for the error-path tests only."""
    global _hooks
    if _hooks is None:
        L = _bind(TEST_HOOKS_LIB_PATH)
        L.fdfs_gpu_inject_error.restype = ctypes.c_int
        L.fdfs_gpu_inject_error.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        _hooks = L
    return _hooks


def _bind(path: str) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise RuntimeError(
            f"{os.path.basename(path)} not found at {path}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    L = ctypes.CDLL(path)
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    L.fdfs_gpu_abi_version.restype = i32
    L.fdfs_gpu_abi_version.argtypes = []
    L.fdfs_gpu_open.restype = i32
    L.fdfs_gpu_open.argtypes = [i32, ctypes.c_uint, ctypes.POINTER(vp)]
    L.fdfs_gpu_close.restype = i32
    L.fdfs_gpu_close.argtypes = [vp]
    L.fdfs_gpu_reserve.restype = i32
    L.fdfs_gpu_reserve.argtypes = [vp, u64, u64]
    L.fdfs_gpu_sig_batch.restype = i32
    L.fdfs_gpu_sig_batch.argtypes = [vp, ctypes.POINTER(FdfsGpuBatch), i32, vp, vp, vp, vp]
    L.fdfs_gpu_dedup.restype = i32
    L.fdfs_gpu_dedup.argtypes = [vp, vp, vp, u64, vp, vp, vp]
    L.fdfs_gpu_dedup_bucket.restype = i32
    L.fdfs_gpu_dedup_bucket.argtypes = [vp, vp, vp, u64, u32, vp, vp, vp, vp]
    L.fdfs_gpu_dedup_group.restype = i32
    L.fdfs_gpu_dedup_group.argtypes = [vp, vp, u64, vp, vp, vp]
    L.fdfs_gpu_set_timing.restype = i32
    L.fdfs_gpu_set_timing.argtypes = [vp, i32]
    if hasattr(L, "fdfs_gpu_crc_lane_min_files"):  # (absent from A/B builds of round 5)
        L.fdfs_gpu_crc_lane_min_files.restype = i32
        L.fdfs_gpu_crc_lane_min_files.argtypes = [vp, vp]
    L.fdfs_gpu_read_timing.restype = i32
    L.fdfs_gpu_read_timing.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(ctypes.c_uint64)]
    L.fdfs_gpu_file_ids.restype = i32
    L.fdfs_gpu_file_ids.argtypes = [vp, u32, vp, vp, vp, vp, u32, u32, vp, vp, vp]
    L.fdfs_gpu_parse_file_ids.restype = i32
    L.fdfs_gpu_parse_file_ids.argtypes = [vp, vp, u32, vp, vp, vp, vp, vp]
    L.fdfs_gpu_trunk_pack.restype = i32
    L.fdfs_gpu_trunk_pack.argtypes = [vp, vp, vp, vp, vp, vp, vp, u32, vp, vp]
    L.fdfs_gpu_trunk_unpack.restype = i32
    L.fdfs_gpu_trunk_unpack.argtypes = [vp, vp, u32, vp, vp, vp, vp, vp, vp, vp]
    L.fdfs_gpu_fdht_route.restype = i32
    L.fdfs_gpu_fdht_route.argtypes = [vp, vp, u64, ctypes.c_char_p, i32, u32, vp, vp, vp, vp, vp,
                                      vp, vp]
    L.fdfs_gpu_fdht_route_keys.restype = i32
    L.fdfs_gpu_fdht_route_keys.argtypes = [vp, vp, u32, vp, u64, ctypes.c_char_p, i32, u32, vp, vp,
                                           vp, vp, vp, vp, vp]
    L.fdfs_gpu_recovery_batch.restype = i32
    L.fdfs_gpu_recovery_batch.argtypes = [vp, ctypes.POINTER(FdfsGpuBatch), i32, vp, u32, vp,
                                          ctypes.c_char_p, i32, u32, vp,
                                          ctypes.POINTER(FdfsGpuRecoveryOut), vp]
    L.fdfs_gpu_sig_batch_host.restype = i32
    L.fdfs_gpu_sig_batch_host.argtypes = [vp, ctypes.POINTER(FdfsGpuBatch), i32, vp, vp, vp, u64]
    L.fdfs_gpu_scrub.restype = i32
    L.fdfs_gpu_scrub.argtypes = [vp, ctypes.POINTER(FdfsGpuBatch), vp, vp, vp, vp, vp]
    L.fdfs_gpu_last_error.restype = ctypes.c_char_p
    L.fdfs_gpu_last_error.argtypes = [vp]
    L.fdfs_gpu_state_init.restype = i32
    L.fdfs_gpu_state_init.argtypes = [vp, vp, u32, vp]
    L.fdfs_gpu_update_batch.restype = i32
    L.fdfs_gpu_update_batch.argtypes = [vp, ctypes.POINTER(FdfsGpuBatch), vp, i32, vp, vp]
    L.fdfs_gpu_final_batch.restype = i32
    L.fdfs_gpu_final_batch.argtypes = [vp, vp, vp, u32, i32, vp, vp, vp, vp]
    L.fdfs_gpu_crc_combine.restype = i32
    L.fdfs_gpu_crc_combine.argtypes = [vp, vp, vp, vp, u32, vp, vp]
    L.fdfs_gpu_dedup_packed.restype = i32
    L.fdfs_gpu_dedup_packed.argtypes = [vp, vp, vp, u64, vp, vp]
    L.fdfs_gpu_dedup_global.restype = i32
    L.fdfs_gpu_dedup_global.argtypes = [vp, vp, vp, vp, u64, vp, vp, vp]
    L.fdfs_gpu_dedup_global_local.restype = i32
    L.fdfs_gpu_dedup_global_local.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp]
    if hasattr(L, "fdfs_gpu_dedup_global_stats"):  # (absent from A/B builds of round 5)
        L.fdfs_gpu_dedup_global_stats.restype = i32
        L.fdfs_gpu_dedup_global_stats.argtypes = [vp, vp, vp]
    L.fdfs_gpu_crc_batch_global.restype = i32
    L.fdfs_gpu_crc_batch_global.argtypes = [vp, vp, ctypes.POINTER(FdfsGpuBatch), vp, vp, vp, u64, vp, vp]
    L.fdfs_gpu_crc_batch_global_local.restype = i32
    L.fdfs_gpu_crc_batch_global_local.argtypes = [vp, i32, ctypes.POINTER(FdfsGpuBatch), vp, vp, vp, u64, vp, vp]
    L.fdfs_gpu_comm_unique_id.restype = i32
    L.fdfs_gpu_comm_unique_id.argtypes = [ctypes.c_char_p]
    L.fdfs_gpu_comm_init.restype = i32
    L.fdfs_gpu_comm_init.argtypes = [vp, ctypes.c_char_p, i32, i32, ctypes.POINTER(vp)]
    L.fdfs_gpu_comm_destroy.restype = i32
    L.fdfs_gpu_comm_destroy.argtypes = [vp]
    L.fdfs_gpu_index_create.restype = i32
    L.fdfs_gpu_index_create.argtypes = [vp, u64, ctypes.POINTER(vp)]
    L.fdfs_gpu_index_destroy.restype = i32
    L.fdfs_gpu_index_destroy.argtypes = [vp]
    L.fdfs_gpu_index_ingest.restype = i32
    L.fdfs_gpu_index_ingest.argtypes = [vp, vp, vp, vp, u64, vp, vp, vp]
    L.fdfs_gpu_index_stats.restype = i32
    L.fdfs_gpu_index_stats.argtypes = [vp, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u64)]
    L.fdfs_gpu_index_slots.restype = i32
    L.fdfs_gpu_index_slots.argtypes = [vp, ctypes.POINTER(u64)]
    return L
