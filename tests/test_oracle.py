"""CPU: pin the oracle (oracle/fdfs_oracle.c) against the golden vectors.

These are the checks that make the oracle trustworthy as the GPU parity
checker: RFC 1321 for MD5, zlib for the unsigned CRC, the survey's recorded
corpus values for both CRC/ELF shift semantics, simple and Time33.
"""
import hashlib
import zlib

import numpy as np
import pytest


def _random_buffers(kat):
    rng = np.random.default_rng(kat["random"][0]["seed"])
    for v in kat["random"]:
        buf = rng.integers(0, 256, size=v["len"], dtype=np.uint8).tobytes()
        if v["hex"] is not None:
            assert buf.hex() == v["hex"]
        yield v, buf


def test_md5_rfc1321(oracle, kat):
    for msg, digest in kat["rfc1321"]:
        assert oracle.md5(msg.encode()).hex() == digest


def test_md5_random_vs_hashlib(oracle, kat):
    for v, buf in _random_buffers(kat):
        assert oracle.md5(buf).hex() == v["md5"], v["len"]


def test_crc_unsigned_vs_zlib(oracle, kat):
    for v, buf in _random_buffers(kat):
        assert "%08X" % oracle.crc32(buf, oracle.VARIANT_UNSIGNED) == v["crc_unsigned"], v["len"]


def test_crc_check_value(oracle, kat):
    c = kat["check"]
    assert "%08X" % oracle.crc32(c["input"].encode()) == c["crc_signed"]
    assert "%08X" % oracle.crc32(c["input"].encode(), oracle.VARIANT_UNSIGNED) == c["crc_unsigned"]


def test_crc_table_is_reflected_edb88320(oracle):
    assert oracle.lib().orc_crc_table_entry(1) == 0x77073096
    assert oracle.lib().orc_crc_table_entry(255) == 0x2D02EF8D


def test_gen_files_corpus(oracle, kat, corpus):
    buf, offs, sizes = corpus
    k = kat["corpus"]
    assert [int(s) for s in sizes] == k["sizes"]
    assert buf.size == sum(k["sizes"])
    for i in range(6):
        d = buf[int(offs[i]): int(offs[i] + sizes[i])]
        assert np.all(d[-1024:] == 0xFF)  # test/gen_files.c:64-65
        crc_s, sig_s, codes_s = oracle.dio_file(d, oracle.METHOD_HASH, oracle.VARIANT_SIGNED)
        crc_u, _, codes_u = oracle.dio_file(d, oracle.METHOD_HASH, oracle.VARIANT_UNSIGNED)
        assert "%08X" % crc_s == k["crc_signed"][i]
        assert "%08X" % crc_u == k["crc_unsigned"][i]
        assert "%08X" % (codes_s[2] & 0xFFFFFFFF) == k["simple"][i]
        assert "%08X" % (codes_s[3] & 0xFFFFFFFF) == k["time33"][i]
        assert codes_s[2] == codes_u[2] and codes_s[3] == codes_u[3]
        if str(i) in k["elf_signed"]:
            assert "%08X" % (codes_s[1] & 0xFFFFFFFF) == k["elf_signed"][str(i)]
            assert "%08X" % (codes_u[1] & 0xFFFFFFFF) == k["elf_unsigned"][str(i)]
        if i < 5:  # hashlib on the 100 MB file is covered by the GPU tests
            assert oracle.md5(d).hex() == k["md5"][i]
            assert hashlib.md5(d.tobytes()).hexdigest() == k["md5"][i]


@pytest.mark.parametrize("variant", [0, 1])
def test_chunking_invariance(oracle, variant):
    """dio_write_file feeds <= buff_size chunks (storage/storage_dio.c:439);
    fdfs_crc32 uses 512 KiB (client/fdfs_crc32.c:28): results must not depend on it."""
    rng = np.random.default_rng(7)
    d = rng.integers(0, 256, size=300_001, dtype=np.uint8)
    ref = oracle.dio_file(d, oracle.METHOD_HASH, variant, chunk=len(d))
    for chunk in (1, 3, 4096, 65536, 256 * 1024, 512 * 1024):
        assert oracle.dio_file(d, oracle.METHOD_HASH, variant, chunk=chunk) == ref
    m = oracle.dio_file(d, oracle.METHOD_MD5, variant, chunk=len(d))
    for chunk in (1, 63, 64, 65, 256 * 1024):
        assert oracle.dio_file(d, oracle.METHOD_MD5, variant, chunk=chunk) == m


@pytest.mark.parametrize("variant", [0, 1])
def test_crc_split_identity(oracle, variant):
    """What the segmented kernels and md5_pair_kernel's two-chain CRC rely
    on: CRC32_ex (storage/storage_dio.c:467) is linear in (state, data) for
    both shift variants, so crc(c, A || B) = M^|B| crc(c, A) ^ crc(0, B), with
    M^n x = crc(x, n zero bytes) (the zero-data CRC from state 0 is 0)."""
    rng = np.random.default_rng(11 + variant)
    zeros = np.zeros(4096, np.uint8)
    for _ in range(200):
        la, lb = (int(x) for x in rng.integers(0, 300, 2))
        a = rng.integers(0, 256, la, dtype=np.uint8)
        b = rng.integers(0, 256, lb, dtype=np.uint8)
        c = int(rng.integers(-2**31, 2**31))
        whole = oracle.crc32_ex(np.concatenate([a, b]), c, variant)
        adv = oracle.crc32_ex(zeros[:lb], oracle.crc32_ex(a, c, variant), variant)
        assert whole == adv ^ oracle.crc32_ex(b, 0, variant)
    assert oracle.crc32_ex(zeros, 0, variant) == 0


def test_sig_pack_layout(oracle):
    """STORAGE_GEN_FILE_SIGNATURE: be64 size, then be32 x4 (hash) / raw md5."""
    d = np.frombuffer(b"hello fastdfs", dtype=np.uint8)
    crc, sig, codes = oracle.dio_file(d, oracle.METHOD_HASH)
    assert sig[:8] == len(d).to_bytes(8, "big")
    for k in range(4):
        assert sig[8 + 4 * k: 12 + 4 * k] == (codes[k] & 0xFFFFFFFF).to_bytes(4, "big")
    assert codes[0] & 0xFFFFFFFF == crc  # h[0] is the file CRC
    crc2, sig2, _ = oracle.dio_file(d, oracle.METHOD_MD5)
    assert crc2 == crc
    assert sig2[8:] == hashlib.md5(b"hello fastdfs").digest()


def test_crc_signed_differs_from_zlib_only_when_sign_set(oracle):
    # a state never reaching bit 31 would make the variants agree; they must
    # differ on ordinary data and agree on the empty input.
    assert oracle.crc32(b"") == 0 == zlib.crc32(b"")
    assert oracle.crc32(b"fastdfs") != zlib.crc32(b"fastdfs")


def test_dedup_oracle_vs_dict(oracle):
    rng = np.random.default_rng(3)
    base = rng.integers(0, 256, size=(50, 24), dtype=np.uint8)
    pick = rng.integers(0, 50, size=400)
    sig = base[pick]
    rep, ref = oracle.dedup(sig)
    first, cnt = {}, {}
    for i, row in enumerate(sig):
        k = row.tobytes()
        first.setdefault(k, i)
        cnt[k] = cnt.get(k, 0) + 1
    for i, row in enumerate(sig):
        k = row.tobytes()
        assert rep[i] == first[k] and ref[i] == cnt[k]
