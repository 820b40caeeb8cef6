"""Is the MD5 lane kernel limited by address-translation reach?  Same work
(16384 files x 1 MiB), files packed vs spread at a large stride."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import fastdfs_amd as F
from fastdfs_amd import _lib
ctx = F.Context(0)
ctx.set_timing(True)
nf, size = 16384, 1 << 20
for stride_mb in (1, 2, 4, 8):
    span = nf * stride_mb << 20
    data = torch.empty(span, dtype=torch.uint8, device="cuda")
    data.view(torch.int64).random_()
    offs = torch.arange(nf, dtype=torch.int64, device="cuda") * (stride_mb << 20)
    sizes = torch.full((nf,), size, dtype=torch.int64, device="cuda")
    ctx.sig_batch(data, offs, sizes, method=F.SIG_MD5); torch.cuda.synchronize(); ctx.read_timing(_lib.KERNEL_SIG_LANE)
    for _ in range(2):
        ctx.sig_batch(data, offs, sizes, method=F.SIG_MD5)
    torch.cuda.synchronize()
    ms, n = ctx.read_timing(_lib.KERNEL_SIG_LANE); ms /= n
    print(f"stride {stride_mb} MiB (span {span/1e9:.0f} GB): {ms:.2f} ms, {nf*size/ms/1e6:.0f} GB/s", flush=True)
    del data; torch.cuda.empty_cache()
