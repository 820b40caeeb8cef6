"""ctypes wrapper over the C oracle (oracle/fdfs_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker / CPU baseline and never
as the thing measured or shipped.  The product library (libfdfs_gpu) does not
link or call any of this.

Parity status: MD5 pinned by RFC 1321 vectors; the unsigned CRC32 variant
pinned by zlib; the signed (libfastcommon-as-declared) CRC32/ELF variant is
PARITY UNPINNED -- libfastcommon is not vendored in the reference and no
reference test pins a value ("Oracle").
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle.so")

VARIANT_SIGNED = 0
VARIANT_UNSIGNED = 1
METHOD_CRC_ONLY = 0
METHOD_HASH = 1
METHOD_MD5 = 2

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        u8p = ctypes.c_void_p
        L.orc_crc32_ex.restype = ctypes.c_int32
        L.orc_crc32_ex.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int32, ctypes.c_int]
        L.orc_crc32_final.restype = ctypes.c_int32
        L.orc_crc32_final.argtypes = [ctypes.c_int32]
        L.orc_elf_ex.restype = ctypes.c_int32
        L.orc_elf_ex.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int32, ctypes.c_int]
        L.orc_simple_ex.restype = ctypes.c_int32
        L.orc_simple_ex.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int32]
        L.orc_time33_ex.restype = ctypes.c_int32
        L.orc_time33_ex.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int32]
        L.orc_crc_table_entry.restype = ctypes.c_uint32
        L.orc_crc_table_entry.argtypes = [ctypes.c_int]
        L.orc_dio_file.restype = None
        L.orc_dio_file.argtypes = [u8p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_int, u8p, u8p, u8p]
        L.orc_dio_batch.restype = ctypes.c_int
        L.orc_dio_batch.argtypes = [u8p, u8p, u8p, ctypes.c_uint64, ctypes.c_size_t,
                                    ctypes.c_int, ctypes.c_int, u8p, u8p, ctypes.c_int]
        L.orc_gen_files_total.restype = ctypes.c_uint64
        L.orc_gen_files.restype = None
        L.orc_gen_files.argtypes = [u8p]
        L.orc_dedup.restype = ctypes.c_int
        L.orc_dedup.argtypes = [u8p, ctypes.c_uint64, u8p, u8p]
        L.orc_dedup_mt.restype = ctypes.c_int
        L.orc_dedup_mt.argtypes = [u8p, ctypes.c_uint64, u8p, u8p, ctypes.c_int]
        L.orc_md5_init.argtypes = [u8p]
        L.orc_md5_update.argtypes = [u8p, u8p, ctypes.c_size_t]
        L.orc_md5_final.argtypes = [u8p, u8p]
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _u8(data) -> np.ndarray:
    if isinstance(data, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(data), dtype=np.uint8)
    return np.ascontiguousarray(data, dtype=np.uint8)


def crc32_ex(data, init: int = -1, variant: int = VARIANT_SIGNED) -> int:
    a = _u8(data)
    return lib().orc_crc32_ex(_ptr(a), a.size, ctypes.c_int32(init).value, variant)


def crc32(data, variant: int = VARIANT_SIGNED) -> int:
    """CRC32_XINIT -> CRC32_ex -> CRC32_FINAL, as an unsigned 32-bit value
    (what fdfs_crc32 prints with %u, client/fdfs_crc32.c:100)."""
    return lib().orc_crc32_final(crc32_ex(data, -1, variant)) & 0xFFFFFFFF


def elf_ex(data, init: int = 0, variant: int = VARIANT_SIGNED) -> int:
    a = _u8(data)
    return lib().orc_elf_ex(_ptr(a), a.size, init, variant)


def simple_ex(data, init: int = 0) -> int:
    a = _u8(data)
    return lib().orc_simple_ex(_ptr(a), a.size, init)


def time33_ex(data, init: int = 0) -> int:
    a = _u8(data)
    return lib().orc_time33_ex(_ptr(a), a.size, init)


def md5(data) -> bytes:
    a = _u8(data)
    ctx = ctypes.create_string_buffer(128)
    out = ctypes.create_string_buffer(16)
    L = lib()
    L.orc_md5_init(ctypes.addressof(ctx))
    L.orc_md5_update(ctypes.addressof(ctx), _ptr(a), a.size)
    L.orc_md5_final(ctypes.addressof(out), ctypes.addressof(ctx))
    return out.raw


def dio_file(data, method: int, variant: int = VARIANT_SIGNED, chunk: int = 256 * 1024):
    """Returns (crc32 unsigned, sig24 bytes or None, hash codes (4 int32) or None)."""
    a = _u8(data)
    crc = np.zeros(1, np.uint32)
    sig = np.zeros(24, np.uint8)
    codes = np.zeros(4, np.int32)
    lib().orc_dio_file(_ptr(a), a.size, chunk, method, variant, _ptr(crc), _ptr(sig),
                       _ptr(codes))
    if method == METHOD_CRC_ONLY:
        return int(crc[0]), None, None
    return int(crc[0]), sig.tobytes(), [int(x) for x in codes]


def dio_batch(base: np.ndarray, offset: np.ndarray, size: np.ndarray, method: int,
              variant: int = VARIANT_SIGNED, chunk: int = 256 * 1024, nthreads: int = 1):
    """Oracle over a batch; returns (crc uint32[n], sig uint8[n,24])."""
    base = np.ascontiguousarray(base, dtype=np.uint8)
    offset = np.ascontiguousarray(offset, dtype=np.uint64)
    size = np.ascontiguousarray(size, dtype=np.uint64)
    n = offset.size
    crc = np.zeros(n, np.uint32)
    sig = np.zeros((n, 24), np.uint8)
    rc = lib().orc_dio_batch(_ptr(base), _ptr(offset), _ptr(size), n, chunk, method, variant,
                             _ptr(crc), _ptr(sig), nthreads)
    assert rc == 0
    return crc, sig


def gen_files() -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """test/gen_files.c corpus: (bytes, offsets, sizes) of the 6 files."""
    L = lib()
    total = L.orc_gen_files_total()
    buf = np.empty(total, np.uint8)
    L.orc_gen_files(_ptr(buf))
    sizes = np.array([5 << 10, 50 << 10, 200 << 10, 1 << 20, 10 << 20, 100 << 20], np.uint64)
    offs = np.zeros(6, np.uint64)
    offs[1:] = np.cumsum(sizes)[:-1]
    return buf, offs, sizes


def dedup(sig: np.ndarray, nthreads: int = 1, partitioned: bool = False) -> tuple[np.ndarray, np.ndarray]:
    """(rep uint64[n], ref uint32[n]) with the sequential FastDHT semantics
    (nthreads > 1 or partitioned: the hash-partitioned form, same answers)."""
    sig = np.ascontiguousarray(sig, dtype=np.uint8).reshape(-1, 24)
    n = sig.shape[0]
    rep = np.zeros(n, np.uint64)
    ref = np.zeros(n, np.uint32)
    if nthreads > 1 or partitioned:
        assert lib().orc_dedup_mt(_ptr(sig), n, _ptr(rep), _ptr(ref), nthreads) == 0
    else:
        assert lib().orc_dedup(_ptr(sig), n, _ptr(rep), _ptr(ref)) == 0
    return rep, ref


# ---- formats that consume the CRC, FastDHT routing ----------

def _fmt_lib():
    L = lib()
    if not getattr(L, "_fmt_ready", False):
        vp, i32, u32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint32
        L.orc_pjw_hash.restype = i32
        L.orc_pjw_hash.argtypes = [vp, ctypes.c_size_t, ctypes.c_int]
        L.orc_base64_encode.restype = ctypes.c_int
        L.orc_base64_encode.argtypes = [vp, ctypes.c_int, vp]
        L.orc_base64_decode.restype = ctypes.c_int
        L.orc_base64_decode.argtypes = [vp, ctypes.c_int, vp]
        L.orc_file_id.restype = None
        L.orc_file_id.argtypes = [u32, i32, ctypes.c_int64, u32, u32, ctypes.c_int, ctypes.c_int,
                                  vp, vp]
        L.orc_parse_file_id.restype = None
        L.orc_parse_file_id.argtypes = [vp, vp, vp, vp, vp]
        L.orc_trunk_pack.restype = None
        L.orc_trunk_pack.argtypes = [ctypes.c_uint8, i32, i32, u32, i32, vp, vp]
        L.orc_fdht_route.restype = None
        L.orc_fdht_route.argtypes = [ctypes.c_char_p, ctypes.c_int, vp, u32, u32, ctypes.c_int,
                                     vp, vp, vp]
        L.orc_fdht_route_key.restype = None
        L.orc_fdht_route_key.argtypes = [ctypes.c_char_p, ctypes.c_int, vp, ctypes.c_int, u32, u32,
                                         ctypes.c_int, vp, vp, vp]
        L._fmt_ready = True
    return L


def pjw_hash(data: bytes, variant: int = VARIANT_SIGNED) -> int:
    return _fmt_lib().orc_pjw_hash(data, len(data), variant)


def base64_encode(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(4 * len(data) // 3 + 4)
    n = _fmt_lib().orc_base64_encode(data, len(data), out)
    return out.raw[:n]


def base64_decode(text: bytes) -> bytes:
    out = ctypes.create_string_buffer(len(text))
    n = _fmt_lib().orc_base64_decode(text, len(text), out)
    return out.raw[:n]


def file_ids(server_id: int, crc32, file_size, timestamp, rnd, subdir_count: int = 256,
             variant: int = VARIANT_SIGNED):
    """(names uint8[n,27], sub_path uint8[n,2]) for a batch."""
    n = len(crc32)
    names = np.zeros((n, 27), np.uint8)
    sub = np.zeros((n, 2), np.uint8)
    L = _fmt_lib()
    for i in range(n):
        L.orc_file_id(server_id, int(timestamp[i]), int(file_size[i]), int(crc32[i]),
                      int(rnd[i]), subdir_count, variant, names[i].ctypes.data,
                      sub[i].ctypes.data)
    return names, sub


def parse_file_ids(names):
    """(server_id u32, timestamp i32, file_size i64, crc32 u32) arrays."""
    names = np.ascontiguousarray(names, np.uint8).reshape(-1, 27)
    n = names.shape[0]
    sid, ts = np.zeros(n, np.uint32), np.zeros(n, np.int32)
    sz, crc = np.zeros(n, np.int64), np.zeros(n, np.uint32)
    L = _fmt_lib()
    for i in range(n):
        L.orc_parse_file_id(names[i].ctypes.data, sid[i:].ctypes.data, ts[i:].ctypes.data,
                            sz[i:].ctypes.data, crc[i:].ctypes.data)
    return sid, ts, sz, crc


def trunk_pack(file_type, alloc_size, file_size, crc32, mtime, ext):
    """uint8[n,24] trunk headers."""
    n = len(crc32)
    ext = np.ascontiguousarray(ext, np.uint8).reshape(n, 7)
    out = np.zeros((n, 24), np.uint8)
    L = _fmt_lib()
    for i in range(n):
        L.orc_trunk_pack(int(file_type[i]), int(alloc_size[i]), int(file_size[i]),
                         int(crc32[i]), int(mtime[i]), ext[i].ctypes.data, out[i].ctypes.data)
    return out


def fdht_route(ns: bytes, sig, group_count: int, servers_per_group,
               variant: int = VARIANT_SIGNED):
    """(key_hash i32, group u32, server u32) per signature."""
    sig = np.ascontiguousarray(sig, np.uint8).reshape(-1, 24)
    n = sig.shape[0]
    kh, grp, srv = np.zeros(n, np.int32), np.zeros(n, np.uint32), np.zeros(n, np.uint32)
    L = _fmt_lib()
    for i in range(n):
        g = ctypes.c_uint32()
        L.orc_fdht_route(ns, len(ns), sig[i].ctypes.data, group_count, 1, variant,
                         kh[i:].ctypes.data, ctypes.byref(g), srv[i:].ctypes.data)
        grp[i] = g.value
        L.orc_fdht_route(ns, len(ns), sig[i].ctypes.data, group_count,
                         int(servers_per_group[g.value]), variant, kh[i:].ctypes.data,
                         grp[i:].ctypes.data, srv[i:].ctypes.data)
    return kh, grp, srv


def fdht_route_keys(ns: bytes, keys, lens, group_count: int, servers_per_group,
                    variant: int = VARIANT_SIGNED):
    """(key_hash i32, group u32, server u32) for obj ids keys[i, :lens[i]]."""
    keys = np.ascontiguousarray(keys, np.uint8)
    n = keys.shape[0]
    kh, grp, srv = np.zeros(n, np.int32), np.zeros(n, np.uint32), np.zeros(n, np.uint32)
    L = _fmt_lib()
    for i in range(n):
        g = ctypes.c_uint32()
        row = np.ascontiguousarray(keys[i])
        L.orc_fdht_route_key(ns, len(ns), row.ctypes.data, int(lens[i]), group_count, 1, variant,
                             kh[i:].ctypes.data, ctypes.byref(g), srv[i:].ctypes.data)
        grp[i] = g.value
        L.orc_fdht_route_key(ns, len(ns), row.ctypes.data, int(lens[i]), group_count,
                             int(servers_per_group[g.value]), variant, kh[i:].ctypes.data,
                             grp[i:].ctypes.data, srv[i:].ctypes.data)
    return kh, grp, srv
