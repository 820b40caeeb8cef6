"""Does address locality of a wave's files matter to sig_hash_kernel?

Config 2's 1M files (U[4, 64] KiB) laid out three ways, same sizes and bytes
in total: as generated (a size-sorted wave's 64 files are scattered over the
34.8 GB buffer), sorted by size descending (the lane order is then the
address order: a wave's files are adjacent), and in windows (sorted by size
within windows of --window consecutive files).  Prints kernel ms per layout
(HIP events around K calls of fdfs_gpu_sig_batch, HASH).  With
FDFS_GPU_PROBE_LIB=1 FDFS_GPU_HASH_MODE=1 it times the loads alone.

    python scripts/locality_probe.py [--files 1000000] [--iters 10]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastdfs_amd import api, corpus as C  # noqa: E402


def run(ctx, sizes, iters, dev):
    data, offs, sz = C.device_batch(sizes, seed=2, device=dev)
    crc = torch.empty(len(sizes), dtype=torch.int32, device=dev)
    sig = torch.empty((len(sizes), 24), dtype=torch.uint8, device=dev)
    for _ in range(2):
        ctx.sig_batch(data, offs, sz, method=1, crc_out=crc, sig_out=sig, check_bounds=False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        ctx.sig_batch(data, offs, sz, method=1, crc_out=crc, sig_out=sig, check_bounds=False)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / iters
    out = (int(crc[:1000].double().sum().item()),)
    del data
    torch.cuda.empty_cache()
    return ms, int(sizes.sum()), out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--window", type=int, default=4096)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = api.Context(0)
    base = C.small_files_sizes(a.files)
    w = a.window
    windowed = np.concatenate([np.sort(base[i:i + w])[::-1] for i in range(0, len(base), w)])
    for name, sizes in [("as_generated", base), ("size_sorted", np.sort(base)[::-1].copy()),
                        (f"window_{w}", windowed)]:
        ms, nbytes, chk = run(ctx, sizes, a.iters, dev)
        print(json.dumps({"layout": name, "ms": round(ms, 3), "GB_s": round(nbytes / ms / 1e6, 1),
                          "bytes": nbytes, "mode": os.environ.get("FDFS_GPU_HASH_MODE", "0"),
                          "lane_window": os.environ.get("FDFS_GPU_LANE_WINDOW", "0"), "check": chk[0]}), flush=True)


if __name__ == "__main__":
    main()
