"""Is the lane kernel limited by address locality?  Same sizes/bytes, files
laid out (a) in random size order (bench layout: a wave's 64 size-sorted
files are scattered over the whole buffer) vs (b) in descending size order
(the size sort then keeps a wave's files adjacent in memory)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import fastdfs_amd as F
from fastdfs_amd import _lib, corpus as C
ctx = F.Context(0)
ctx.set_timing(True)
cases = [("hash", F.SIG_HASH, C.small_files_sizes(int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000, seed=1)),
         ("md5", F.SIG_MD5, C.photo_sizes(24000, seed=3))]
for name, method, sizes in cases:
    for layout in ("random", "sorted"):
        s = sizes if layout == "random" else np.sort(sizes)[::-1].copy()
        data, offs, sz = C.device_batch(s, seed=2, device="cuda")
        ctx.sig_batch(data, offs, sz, method=method); torch.cuda.synchronize()
        ctx.read_timing(_lib.KERNEL_SIG_LANE)
        for _ in range(3):
            ctx.sig_batch(data, offs, sz, method=method)
        torch.cuda.synchronize()
        ms, k = ctx.read_timing(_lib.KERNEL_SIG_LANE); ms /= k
        print(f"{name} {layout}: {ms:.2f} ms, {s.sum()/ms/1e6:.0f} GB/s", flush=True)
        del data, offs, sz; torch.cuda.empty_cache()
