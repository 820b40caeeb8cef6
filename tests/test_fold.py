"""CPU: the sparse fold of crc_seg_kernel (fdfs_tables.hpp fold_exp, DESIGN.md
4.1), checked independently of the library.  For each shift variant, with A =
the CRC32_ex advance by 16 zero bytes, S(A) = sum_k A^e_k must vanish, the
gap between the top two exponents must let 64 consecutive vectors fold at
once, and the fold itself (c_j = x_j ^ sum_k c_{j - (D - e_k)}, D the top
exponent, positions <= n - 1 - D passing on, crc0 of the last D vectors)
must give the byte loop's crc0 on random runs of every length class the
kernel distinguishes."""
import os
import random
import re

import pytest

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "fastdfs_amd", "csrc", "fdfs_tables.hpp")


def exponents():
    """(sar, lsr) exponent lists parsed from kFoldTerms / fold_exp in the header."""
    src = open(HDR).read()
    t = int(re.search(r"constexpr int kFoldTerms = (\d+);", src).group(1))
    terms = (t, t)
    body = src[src.index("constexpr int fold_exp"):]
    body = body[:body.index("}")]
    out = []
    for part in re.findall(r"\(k == 0 \? 0 :(.*?)\)", body):
        out.append([0] + [int(x) for x in re.findall(r"(\d+)", part)[1::2]] + [int(re.findall(r"(\d+)", part)[-1])])
    assert len(out) == 2 and (len(out[0]), len(out[1])) == terms, out
    return out[0], out[1]


def crc_table():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (0xEDB88320 ^ (c >> 1)) if (c & 1) else (c >> 1)
        t.append(c)
    return t


T = crc_table()


def step(c, b, sar):
    sh = (c >> 8) | (0xFF000000 if (sar and (c & 0x80000000)) else 0)
    return (T[(c ^ b) & 0xFF] ^ sh) & 0xFFFFFFFF


def crc0(data, sar):
    c = 0
    for b in data:
        c = step(c, b, sar)
    return c


@pytest.fixture(scope="module")
def exps():
    sar, lsr = exponents()
    return {True: sar, False: lsr}


@pytest.mark.parametrize("sar", [True, False])
def test_relation_and_gap(exps, sar):
    e = exps[sar]
    assert e == sorted(e) and e[0] == 0
    assert e[-1] - e[-2] >= 64, "a step's 64 vectors must not feed each other"
    for i in range(32):
        acc, cur, k = 0, 1 << i, 0
        for p in range(e[-1] + 1):
            if p == e[k]:
                acc ^= cur
                k += 1
            for _ in range(16):
                cur = step(cur, 0, sar)
        assert acc == 0, (sar, i)


@pytest.mark.parametrize("sar", [True, False])
def test_fold_matches_byte_loop(exps, sar):
    e = exps[sar]
    d = e[-1]
    delays = [d - x for x in e[:-1]]
    rng = random.Random(11)
    for n in (1, 63, 64, d - 1, d, d + 1, d + 64, 3 * d + 17, 700):
        data = bytes(rng.getrandbits(8) for _ in range(16 * n))
        lim = n - 1 - d
        c = []
        for j in range(n):
            x = int.from_bytes(data[16 * j:16 * j + 16], "little")
            for dl in delays:
                if 0 <= j - dl <= lim:
                    x ^= c[j - dl]
            c.append(x)
        rem = b"".join(v.to_bytes(16, "little") for v in c[max(0, n - d):])
        assert crc0(rem, sar) == crc0(data, sar), (sar, n)
