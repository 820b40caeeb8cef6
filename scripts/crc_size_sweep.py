"""CRC-only batches of uniform file sizes (~4 GiB each): the kernel time of
fdfs_gpu_sig_batch(FDFS_SIG_CRC_ONLY) per size, HIP events
(KERNEL_CRC_SEG), median of REPS calls after a warm-up.  Run once with the
production library and once with FDFS_GPU_PROBE_LIB=ab (e.g. `make ab
AB_REV=8201397`: the slice-by-8 kernel for every size) to place the split
between crc_tab_kernel and the sparse fold (kFoldMinBytes).

usage: [FDFS_GPU_PROBE_LIB=ab] python3 scripts/crc_size_sweep.py [--total GiB] [--reps N] [--kib 32,64,...]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import fastdfs_amd as F  # noqa: E402
from fastdfs_amd import _lib, corpus as C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total", type=float, default=4.0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--kib", default="32,64,128,192,256,384,512,1024,4096", help="file sizes (KiB)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = F.Context(0)
    ctx.set_timing(True)
    for kib in [int(x) for x in a.kib.split(",")]:
        size = kib << 10
        n = max(1, int(a.total * (1 << 30)) // size)
        sizes = np.full(n, size, dtype=np.int64)
        data, offs, szs = C.device_batch(sizes, seed=5, device=dev, align=16)
        ctx.sig_batch(data, offs, szs, method=F.SIG_CRC_ONLY, check_bounds=False)
        torch.cuda.synchronize()
        ctx.read_timing(_lib.KERNEL_CRC_SEG)
        t = []
        for _ in range(a.reps):
            ctx.sig_batch(data, offs, szs, method=F.SIG_CRC_ONLY, check_bounds=False)
            torch.cuda.synchronize()
            ms, _ = ctx.read_timing(_lib.KERNEL_CRC_SEG)
            t.append(ms)
        ms = float(np.median(t))
        print(json.dumps({"file_kib": kib, "files": n, "kernel_ms": round(ms, 4),
                          "tb_per_s": round(n * size / ms / 1e9, 3),
                          "lib": os.environ.get("FDFS_GPU_PROBE_LIB", "production")}), flush=True)
        del data, offs, szs
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main()
