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


def test_production_library_reads_no_environment():
    """No environment variable can change a result: the production .so does
    not import getenv/secure_getenv (the probe knobs live in `make probes`)."""
    out = subprocess.run(["nm", "-D", "--undefined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    assert not re.search(r"\b(secure_)?getenv\b", out)


def test_file_state_layout_matches_storage_file_context():
    """fdfs_gpu_file_state mirrors StorageFileContext's hash fields
    (storage/storage_nio.h:94-96: int crc32; int file_hash_codes[4];
    MD5_CTX {UINT4 state[4]; UINT4 count[2]; unsigned char buffer[64]}),
    compiled by the host C compiler from the public header."""
    import tempfile
    src = r'''
#include <stddef.h>
#include <stdio.h>
#include "fdfs_gpu.h"
int main(void) {
    printf("%zu %zu %zu %zu %zu %zu\n", sizeof(fdfs_gpu_file_state),
           offsetof(fdfs_gpu_file_state, crc32), offsetof(fdfs_gpu_file_state, hash_codes),
           offsetof(fdfs_gpu_file_state, md5_state), offsetof(fdfs_gpu_file_state, md5_count),
           offsetof(fdfs_gpu_file_state, md5_buffer));
    return 0;
}
'''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.run(["gcc", "-std=c99", "-I", os.path.dirname(_lib.HEADER_PATH), "-o", exe, c],
                       check=True)
        got = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()
    assert [int(x) for x in got] == [_lib.FILE_STATE_SIZE, 0, 4, 20, 36, 44]


def test_stream_api_argument_errors():
    L = _lib.load()
    assert L.fdfs_gpu_state_init(None, None, 1, None) == errno.EINVAL
    assert L.fdfs_gpu_update_batch(None, None, None, 0, None, None) == errno.EINVAL
    assert L.fdfs_gpu_final_batch(None, None, None, 1, 0, None, None, None, None) == errno.EINVAL
    assert L.fdfs_gpu_crc_combine(None, None, None, None, 1, None, None) == errno.EINVAL


def test_tools_read_no_environment():
    """The drop-in C tools select the hash variant by a -u flag, never by an
    environment variable: neither imports getenv."""
    for tool in ("fdfs_crc32_gpu", "fdfs_dio_sim"):
        path = os.path.join(os.path.dirname(_lib.LIB_PATH), tool)
        out = subprocess.run(["nm", "-D", "--undefined-only", path], capture_output=True, text=True,
                             check=True).stdout
        assert not re.search(r"\b(secure_)?getenv\b", out), tool
