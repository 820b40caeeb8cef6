"""CPU: the sparse fold of crc_seg_kernel (fdfs_tables.hpp fold_exp, DESIGN.md
4.1), checked independently of the library.  For each shift variant, with A =
the CRC32_ex advance by 16 zero bytes, S(A) = sum_k A^e_k must vanish, the
gap between the top two exponents must let 64 consecutive vectors fold at
once, and the fold itself (c_j = x_j ^ sum_k c_{j - (D - e_k)}, D the top
exponent, positions <= n - 1 - D passing on, crc0 of the last D vectors)
must give the byte loop's crc0 on random runs of every length class the
kernel distinguishes.  The same for the lane fold of the lane-per-file
kernels (fdfs_tables.hpp lane_fold_exp, below)."""
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


# ---- the lane fold of sig_hash_kernel / md5_pair_kernel (fdfs_tables.hpp
# lane_fold_exp, fdfs_device.hpp lane_fold_dw / lane_fold_finish): the
# minimal polynomial R of A4 = the advance by 4 zero bytes, a 32-dword
# register ring per lane, the state so far entering as the first dword
# (with Y4 for the arithmetic shift), the in-window correction at the end.

def lane_exponents():
    src = open(HDR).read()
    terms = [int(x) for x in re.search(r"lane_fold_terms\(bool sar\) \{ return sar \? (\d+) : (\d+); \}", src).groups()]
    es = [int(x) for x in re.search(r"constexpr int es\[\d+\] = \{([^}]*)\}", src).group(1).split(",")]
    el = [int(x) for x in re.search(r"constexpr int el\[\d+\] = \{([^}]*)\}", src).group(1).split(",")]
    assert (len(es), len(el)) == tuple(terms)
    return {True: es, False: el}


def crc_state(c, data, sar):
    for b in data:
        c = step(c, b, sar)
    return c


def y4(sar):
    """The dword y with crc0(y) = M^4(e_31) ^ crc0(e_31) (fdfs_tables.cpp)."""
    k4 = crc_state(0x80000000, b"\0" * 4, sar) ^ crc0((0x80000000).to_bytes(4, "little"), sar)
    basis = {}
    for i in range(32):  # eliminate on the images of the unit dwords
        val, comb = crc0((1 << i).to_bytes(4, "little"), sar), 1 << i
        while val:
            hb = val.bit_length() - 1
            if hb not in basis:
                basis[hb] = (val, comb)
                break
            val, comb = val ^ basis[hb][0], comb ^ basis[hb][1]
    assert len(basis) == 32, "crc0 of 4 bytes is a bijection"
    y, val = 0, k4
    while val:
        bv, bc = basis[val.bit_length() - 1]
        val, y = val ^ bv, y ^ bc
    return y


@pytest.mark.parametrize("sar", [True, False])
def test_lane_relation(sar):
    e = lane_exponents()[sar]
    assert e == sorted(e) and e[0] == 0 and e[-1] == 32
    for i in range(32):
        acc, cur, k = 0, 1 << i, 0
        for p in range(33):
            if p == e[k]:
                acc ^= cur
                k += 1
            cur = crc_state(cur, b"\0" * 4, sar)
        assert acc == 0, (sar, i)


@pytest.mark.parametrize("sar", [True, False])
def test_lane_fold_matches_byte_loop(sar):
    """The kernels' lane fold, step by step: 32-dword steps (md5_pair_kernel:
    64-byte blocks, so a run may end mid-ring), from a random state."""
    e = lane_exponents()[sar]
    lags = [32 - x for x in e[:-1]]
    Y = y4(sar)
    rng = random.Random(5)
    for ndw in (16, 32, 48, 64, 96, 112, 160, 1024):
        cpre = rng.getrandbits(32)
        data = bytes(rng.getrandbits(8) for _ in range(4 * ndw))
        ring = [0] * 32
        zin = cpre ^ (Y if (sar and cpre & 0x80000000) else 0)
        for j in range(ndw):
            x = int.from_bytes(data[4 * j:4 * j + 4], "little") ^ (zin if j == 0 else 0)
            for lag in lags:  # ring[(j - lag) & 31] holds c'_{j - lag} (0 before the run)
                x ^= ring[(j - lag) & 31]
            ring[j & 31] = x
        u = [ring[(ndw - 32 + i) & 31] for i in range(32)]  # positions ndw - 32 .. ndw - 1
        for i in range(31, -1, -1):
            for lag in lags:
                if i - lag >= 0:
                    u[i] ^= u[i - lag]
        got = crc0(b"".join(v.to_bytes(4, "little") for v in u), sar)
        assert got == crc_state(cpre, data, sar), (sar, ndw)
