"""fastdfs_amd -- MI355X-native FastDFS upload-path CRC32 / dedup signature.

The product is libfdfs_gpu (C ABI in include/fdfs_gpu.h, HIP kernels in
fastdfs_amd/csrc).  This package is the thin host layer used by the tests and
bench: ctypes binding, torch-resident batches, multi-GPU orchestration.
"""
from ._lib import (FILE_SIGNATURE_SIZE, FLAG_UNSIGNED_HASH, LIB_PATH, SIG_CRC_ONLY, SIG_HASH,
                   SIG_MD5)
from .api import Context, FdfsGpuError

__all__ = ["Context", "FdfsGpuError", "SIG_CRC_ONLY", "SIG_HASH", "SIG_MD5",
           "FLAG_UNSIGNED_HASH", "FILE_SIGNATURE_SIZE", "LIB_PATH"]
