"""Does the ELFHash state forget its start?  If it did, a long file's chain
could be split into chunks, each started from an arbitrary state after a
warm-up over the previous chunk's tail.  Feeds the same random bytes to many
random 28-bit start states (both shift variants, fdfs_kernels.hpp elf step)
and counts the distinct states left.  Result: 198,810 of
200,000 after two bytes and still 198,810 after 4096 bytes, i.e. past the
first bytes the update is injective on the reachable states; no split.

usage: python3 scripts/elf_converge.py
"""
import numpy as np


def step(h, b, sar):
    t = ((h << np.uint32(4)) + np.uint32(b)).astype(np.uint32)
    x = t & np.uint32(0xF0000000)
    sx = ((x.astype(np.int32) >> 24).astype(np.uint32) if sar else x >> np.uint32(24))
    return ((t ^ sx) & ~x).astype(np.uint32)


def main():
    rng = np.random.default_rng(1)
    for sar in (False, True):
        h = rng.integers(0, 1 << 28, 200000, dtype=np.uint64).astype(np.uint32)
        data = rng.integers(0, 256, 4096, dtype=np.uint64)
        out = []
        for k, b in enumerate(data, 1):
            h = step(h, b, sar)
            if k & (k - 1) == 0:
                out.append((k, len(np.unique(h))))
        print("sar" if sar else "lsr", out)


if __name__ == "__main__":
    main()
