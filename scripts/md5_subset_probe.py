"""Config-3 MD5 kernel over the real batch, all 100K files vs only the 64K
largest (one heavy wave per SIMD, no light waves sharing the SIMDs): does
the light waves' concurrent footprint slow the heavy ones?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import fastdfs_amd as F  # noqa: E402
from fastdfs_amd import _lib, corpus as C  # noqa: E402

ctx = F.Context(0)
n = 100_000
sizes = C.photo_sizes(n, seed=3)
dev = torch.device("cuda", 0)
data, offs_t, sizes_t = C.device_batch(sizes, seed=5, device=dev)
big = np.argsort(-sizes, kind="stable")[:65536]
sets = {"all 100K": (offs_t, sizes_t),
        "largest 64K": (offs_t[torch.from_numpy(big).to(dev)].contiguous(),
                        sizes_t[torch.from_numpy(big).to(dev)].contiguous())}
ctx.set_timing(True)
for label, (o, s) in sets.items():
    ctx.sig_batch(data, o, s, method=F.SIG_MD5)
    torch.cuda.synchronize()
    ctx.read_timing(_lib.KERNEL_SIG_LANE)
    for _ in range(3):
        ctx.sig_batch(data, o, s, method=F.SIG_MD5)
    torch.cuda.synchronize()
    ms, k = ctx.read_timing(_lib.KERNEL_SIG_LANE)
    gb = float(s.sum().item()) / 1e9
    print(f"{label}: md5_stage_kernel {ms / k:.2f} ms over {gb:.1f} GB", flush=True)
