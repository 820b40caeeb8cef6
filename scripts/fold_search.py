"""Search for the sparse fold of crc_seg_kernel (fdfs_tables.hpp fold_exp).

A = the advance of the CRC32_ex state by 16 zero bytes (one 16-byte vector),
for the arithmetic-shift (signed state) or logical-shift variant.  Wanted: a
polynomial S(y) = 1 + y^e1 + ... + y^e5 + y^D with S(A) = 0, D small, and
D - e5 >= GAP (so GAP consecutive vectors never feed each other).  With a
cyclic start vector s0, S(A) s0 = 0 is a 32-bit condition; meet in the middle:
pairs y^a + y^b on one side, 1 + y^c + y^d + y^D on the other (the 7-term
search) -- a few seconds per D for D < 200.  Every hit is verified on the
32 basis vectors; build_crc_tables verifies the chosen one again at open.

usage: python3 scripts/fold_search.py sar|lsr [Dmax] [GAP] [TERMS=6|7]
       python3 scripts/fold_search.py lane sar|lsr [unit bytes, default 4]
The lane mode prints the minimal polynomial of A4 = the advance by 4 zero
bytes (Gaussian elimination over A4^e s0, e = 0..32, then verified on the
basis): the relation of the kernels' lane fold (fdfs_tables.hpp
lane_fold_exp; sar 13 terms, lsr 15).
(the shipped exponents: sar 0 20 22 41 53 56 135, lsr 0 37 68 69 77 93 161)
"""
import random
import sys

import numpy as np


def crc_table():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (0xEDB88320 ^ (c >> 1)) if (c & 1) else (c >> 1)
        t.append(c)
    return t


T = crc_table()


def zero_byte(c, sar):
    sh = (c >> 8) | (0xFF000000 if (sar and (c & 0x80000000)) else 0)
    return (T[c & 0xFF] ^ sh) & 0xFFFFFFFF


def lane(sar, unit=4):
    cols = []
    for i in range(32):
        c = 1 << i
        for _ in range(unit):
            c = zero_byte(c, sar)
        cols.append(c)

    def apply(v):
        r = 0
        for i in range(32):
            if (v >> i) & 1:
                r ^= cols[i]
        return r

    random.seed(11)
    p = [random.getrandbits(32)]
    for _ in range(40):
        p.append(apply(p[-1]))
    basis = {}
    for e in range(41):
        val, comb = p[e], 1 << e
        while val:
            hb = val.bit_length() - 1
            if hb not in basis:
                basis[hb] = (val, comb)
                break
            val, comb = val ^ basis[hb][0], comb ^ basis[hb][1]
        if not val:
            ex = [i for i in range(e + 1) if (comb >> i) & 1]
            for i in range(32):  # R(A4) e_i == 0
                cur, acc = 1 << i, 0
                for k in range(ex[-1] + 1):
                    if k in ex:
                        acc ^= cur
                    cur = apply(cur)
                assert acc == 0
            print("degree", e, "terms", len(ex), "exponents", ex)
            return


def main():
    if sys.argv[1] == "lane":
        return lane(sys.argv[2] == "sar", int(sys.argv[3]) if len(sys.argv) > 3 else 4)
    sar = sys.argv[1] == "sar"
    dmax = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    gap = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    terms = int(sys.argv[4]) if len(sys.argv) > 4 else 7
    cols = []
    for i in range(32):
        c = 1 << i
        for _ in range(16):
            c = zero_byte(c, sar)
        cols.append(c)

    def apply(v):
        r = 0
        for i in range(32):
            if (v >> i) & 1:
                r ^= cols[i]
        return r

    def holds(ex):  # S(A) e_i == 0 for every basis vector
        for i in range(32):
            cur, acc, pw = 1 << i, 0, {}
            pw[0] = cur
            for e in range(1, max(ex) + 1):
                cur = apply(cur)
                pw[e] = cur
            for e in ex:
                acc ^= pw[e]
            if acc:
                return False
        return True

    random.seed(7)
    p = [random.getrandbits(32)]
    for _ in range(dmax):
        p.append(apply(p[-1]))
    p = np.array(p, dtype=np.uint64)
    inner = terms - 2
    for d in range(gap + inner, dmax + 1):
        h = d - gap
        a, b = np.triu_indices(h, 1)
        a, b = a + 1, b + 1
        left = p[a] ^ p[b]
        order = np.argsort(left)
        ls = left[order]
        rights = [(None, left ^ p[0] ^ p[d])] if inner == 4 else \
                 [(c, left ^ p[0] ^ p[d] ^ p[c]) for c in range(1, h + 1)]
        for c, r in rights:
            pos = np.searchsorted(ls, r)
            hit = (pos < len(ls)) & (ls[np.minimum(pos, len(ls) - 1)] == r)
            for i in np.nonzero(hit)[0]:
                j = order[pos[i]]
                ex = {0, d, int(a[i]), int(b[i]), int(a[j]), int(b[j])} | ({c} if c else set())
                if len(ex) == terms and holds(sorted(ex)):
                    print("D", d, "exponents", sorted(ex))
                    return


if __name__ == "__main__":
    main()
