"""CPU: the C-ABI library builds for gfx950, loads, and exports exactly what
include/fdfs_gpu.h declares.  No compute calls (there is no GPU here)."""
import ctypes
import errno
import os
import re
import subprocess

import pytest

from fastdfs_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(_lib.HEADER_PATH).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fdfs_gpu_\w+)\s*\(", src)))


def test_header_and_binding_agree():
    assert _declared() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    for name in _declared():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (fdfs_gpu_\w+)", out))
    assert exported == set(_declared())


def test_gfx950_code_object_embedded():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    for k in (b"sig_hash_kernel", b"md5_stage_kernel", b"crc_seg_kernel", b"dp_group_kernel"):
        assert k in data, k


def test_abi_version():
    assert _lib.load().fdfs_gpu_abi_version() == 1


def test_argument_errors_without_device():
    L = _lib.load()
    assert L.fdfs_gpu_open(0, 0, None) == errno.EINVAL
    assert L.fdfs_gpu_close(None) == errno.EINVAL
    assert L.fdfs_gpu_sig_batch(None, None, 1, None, None, None, None) == errno.EINVAL
    assert L.fdfs_gpu_dedup_bucket(None, None, None, 0, 0, None, None, None, None) == errno.EINVAL
    assert L.fdfs_gpu_last_error(None) == b"null context"


def test_open_fails_loudly_without_gpu():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    h = ctypes.c_void_p()
    rc = _lib.load().fdfs_gpu_open(0, 0, ctypes.byref(h))
    assert rc == errno.ENODEV and not h.value


def test_context_refuses_cpu_tensors():
    import torch
    from fastdfs_amd.api import _check_dev
    with pytest.raises(ValueError, match="no CPU path"):
        _check_dev(torch.zeros(4, dtype=torch.uint8), "data", torch.uint8)
