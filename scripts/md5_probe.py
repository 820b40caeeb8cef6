"""Probe the MD5 lane kernel: every file aliases the same 4 MiB (cache
resident) vs distinct files, to separate compute latency from memory."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import fastdfs_amd as F
from fastdfs_amd import _lib
ctx = F.Context(0)
ctx.set_timing(True)
for nfiles in (1024, 8192, 24000, 65536):
    size = 4 << 20
    data = torch.randint(0, 256, (size,), dtype=torch.uint8, device="cuda")
    offs = torch.zeros(nfiles, dtype=torch.int64, device="cuda")
    sizes = torch.full((nfiles,), size, dtype=torch.int64, device="cuda")
    ctx.sig_batch(data, offs, sizes, method=F.SIG_MD5)
    torch.cuda.synchronize(); ctx.read_timing(_lib.KERNEL_SIG_LANE)
    for _ in range(2):
        ctx.sig_batch(data, offs, sizes, method=F.SIG_MD5)
    torch.cuda.synchronize()
    ms, n = ctx.read_timing(_lib.KERNEL_SIG_LANE)
    ms /= n
    per_lane = size / (ms * 1e-3) / 1e6
    print(f"aliased files={nfiles}: {ms:.2f} ms, {nfiles*size/ms/1e6:.1f} GB/s, per lane {per_lane:.1f} MB/s, cycles/64B@2.4GHz {2.4e9*64/(per_lane*1e6):.0f}", flush=True)
