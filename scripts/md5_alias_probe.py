"""Config-3 MD5 kernel with every file aliasing one cache-resident 4 MiB
buffer (same sizes and order as the bench) against the real batch: separates
HBM/load latency from the MD5 chain and issue limits."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fastdfs_amd as F  # noqa: E402
from fastdfs_amd import _lib, corpus as C  # noqa: E402

ctx = F.Context(0)
n = 100_000
sizes = C.photo_sizes(n, seed=3)
dev = torch.device("cuda", 0)
buf = torch.randint(0, 256, (4 << 20,), dtype=torch.uint8, device=dev)
offs_t = torch.zeros(n, dtype=torch.int64, device=dev)
sizes_t = torch.from_numpy(sizes).to(dev)
ctx.set_timing(True)
for label, (data, o, s) in (("aliased", (buf, offs_t, sizes_t)),):
    ctx.sig_batch(data, o, s, method=F.SIG_MD5)
    torch.cuda.synchronize()
    ctx.read_timing(_lib.KERNEL_SIG_LANE)
    for _ in range(3):
        ctx.sig_batch(data, o, s, method=F.SIG_MD5)
    torch.cuda.synchronize()
    ms, k = ctx.read_timing(_lib.KERNEL_SIG_LANE)
    print(f"{label}: MD5 lane kernel {ms / k:.2f} ms over {int(sizes.sum()) / 1e9:.1f} GB "
          f"(FDFS_GPU_PROBE_LIB={os.environ.get('FDFS_GPU_PROBE_LIB', '')} "
          f"FDFS_GPU_MD5_PAIR={os.environ.get('FDFS_GPU_MD5_PAIR', '')})", flush=True)
