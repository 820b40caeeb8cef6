"""Generates tests/golden/kat.json -- the known-answer vectors that pin the oracle.

Sources, all independent of the oracle under test:
  * RFC 1321 appendix A.5 MD5 test suite (literal strings/digests below);
  * Python's hashlib.md5 and zlib.crc32 on seeded random buffers (zlib is the
    unsigned/logical-shift CRC-32, i.e. the "unsigned" variant);
  * the gen_files corpus values recorded in SURVEY.md section 8(c) (computed
    during the survey by an independent restatement, before this repo
    existed) for both CRC shift semantics, ELF, simple, Time33 and MD5.

The reference itself holds no such vectors: libfastcommon,
which owns CRC32_ex/ELFHash_ex/simple_hash_ex/Time33Hash_ex, is not vendored,
so the signed-variant values are pinned only by the survey's record
("parity unpinned" w.r.t. a real libfastcommon build).

Run:  python tests/golden/make_golden.py
"""
import base64
import hashlib
import json
import os
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

RFC1321 = [
    ("", "d41d8cd98f00b204e9800998ecf8427e"),
    ("a", "0cc175b9c0f1b6a831c399e269772661"),
    ("abc", "900150983cd24fb0d6963f7d28e17f72"),
    ("message digest", "f96b697d7cb7938d525a2f31aaf161d0"),
    ("abcdefghijklmnopqrstuvwxyz", "c3fcd3d76192e4007dfb496cca67e13b"),
    ("ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789",
     "d174ab98d277d9f5a5611c2c9f419d9f"),
    ("1234567890" * 8, "57edf4a22be3c955ac49da2e2107b67a"),
]

# gen_files corpus (test/gen_files.c, seed test/test_types.h:19)
CORPUS = {
    "sizes": [5120, 51200, 204800, 1048576, 10485760, 104857600],
    "crc_signed": ["1AD1FD78", "550662AE", "2C35A61C", "DE538268", "AC81EB35", "BF7B7BEA"],
    "crc_unsigned": ["6EF879CB", "BB159108", "16F39D2B", "BF860922", "2899705B", "33EFE191"],
    "simple": ["8301BEC8", "5C2605CA", "64D5F219", "D0936718", "8C5D8201", "6CE6EA09"],
    "time33": ["0990F240", "0BDCCD2A", "6F8A7AB7", "CFB617A8", "E9156C27", "1EAE1805"],
    # ELF recorded for the first and last file only
    "elf_signed": {"0": "5147574F", "5": "59C3044F"},
    "elf_unsigned": {"0": "04B04B5F", "5": "0EE0FABF"},
    "md5": ["1e34c11406c4c7b9379dfc72891ac53c", "aa5ca666544b1faaa4c2c7877da7c477",
            "d5ee2da2645cc403a133bc6443644852", "3d9182c9b697bfddd7f264e3a8dbb78c",
            "094ecd5e085cc2483cc64fb74576022e", "253e521daf87876882f45be35a73be9c"],
}

CHECK = {"input": "123456789", "crc_signed": "206AF85B", "crc_unsigned": "CBF43926"}

# Real FastDFS file ids held by the reference's own PHP client tests
# (php_client/fastdfs_test.php:3,9, php_client/fastdfs_test1.php:6).  Their
# 27-char core is the storage_gen_filename encoding (storage/storage_service.c:
# 2145-2202) of an older daemon (no COMBINE_RAND_FILE_SIZE mask); the second
# one is a trunk file (size field carries FDFS_TRUNK_FILE_MARK_SIZE).
FILE_IDS = [
    ("php_client/fastdfs_test.php:9", "M00/00/02/wKjRbExc_qIAAAAAAABtNw6hsnM56585.part2.c"),
    ("php_client/fastdfs_test1.php:6", "M00/01/14/wKgAxU5n9gUIAAAAAAAD8uiojuUAAAAEgP_8YAAAAQK66492"),
    ("php_client/fastdfs_test.php:3", "M00/28/E3/U6Q-CkrMFUgAAAAAAAAIEBucRWc5452.h"),
]


def decode_file_id(core: str) -> dict:
    """Independent restatement of fdfs_get_file_info_ex's decode
    (client/storage_client.c:2133-2214) with Python's urlsafe base64 (the
    FastDFS alphabet: A-Z a-z 0-9 - _)."""
    b = base64.urlsafe_b64decode(core + "=")
    sid = int.from_bytes(b[0:4], "little")          # ntohl(buff2int(buff))
    ts = int.from_bytes(b[4:8], "big", signed=True)
    size = int.from_bytes(b[8:16], "big", signed=True)
    crc = int.from_bytes(b[16:20], "big")
    if size & (1 << 58):                            # IS_APPENDER_FILE
        size, crc = -1, 0
    elif (size >> 63) != 0 or size & (1 << 59):     # masked / trunk: low 32 bits
        size &= 0xFFFFFFFF
    return {"server_id": sid, "ip": ".".join(str(x) for x in b[0:4]), "timestamp": ts,
            "file_size": size, "crc32": "%08X" % crc, "raw_hex": b.hex()}


def main():
    rng = np.random.default_rng(20261015)
    rand_vectors = []
    for n in [0, 1, 2, 3, 4, 5, 15, 16, 17, 63, 64, 65, 255, 1000, 4096, 65535, 65536, 65537,
              200003]:
        buf = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        rand_vectors.append({
            "seed": 20261015, "len": n,
            "hex": buf.hex() if n <= 1000 else None,
            "crc_unsigned": "%08X" % zlib.crc32(buf),
            "md5": hashlib.md5(buf).hexdigest(),
        })
    file_ids = []
    for src, fid in FILE_IDS:
        core = fid[10:10 + 27]  # FDFS_LOGIC_FILE_PATH_LEN, FDFS_FILENAME_BASE64_LENGTH
        file_ids.append({"source": src, "file_id": fid, "core": core, **decode_file_id(core)})
    b64 = []
    for n in [0, 1, 2, 3, 4, 5, 19, 20, 21, 64]:
        raw = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        b64.append({"hex": raw.hex(),
                    "enc": base64.urlsafe_b64encode(raw).decode().rstrip("=")})
    out = {"rfc1321": RFC1321, "check": CHECK, "corpus": CORPUS, "random": rand_vectors,
           "file_ids": file_ids, "base64": b64,
           "random_note": "buffers with len > 1000 are regenerated from numpy "
                          "default_rng(20261015) in list order"}
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
