"""PCIe-inclusive rate of the host-batch path (fdfs_gpu_sig_batch_host):
a config-2-shaped batch (U[4,64] KiB files, hash signature) in pinned and in
pageable host memory, streamed in double-buffered windows and hashed on the
GPU; results back in host memory.  Reported in DESIGN.md (never `value`)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fastdfs_amd as F  # noqa: E402
from fastdfs_amd import corpus as C  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
sizes = C.small_files_sizes(n, seed=1)
offs, total = C.layout(sizes)
ctx = F.Context(0)
rng = np.random.default_rng(2)
pageable = rng.integers(0, 256, size=total, dtype=np.uint8)
pinned = torch.from_numpy(pageable).pin_memory()
for name, buf in (("pinned", pinned), ("pageable", pageable)):
    for chunk in (64 << 20, 256 << 20):
        ctx.sig_batch_host(buf, offs, sizes, method=F.SIG_HASH, chunk_bytes=chunk)  # warm
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            ctx.sig_batch_host(buf, offs, sizes, method=F.SIG_HASH, chunk_bytes=chunk)
        dt = (time.perf_counter() - t0) / reps
        print(f"{name:8s} window {chunk >> 20:4d} MiB: {total / dt / 1e9:6.1f} GB/s "
              f"({n} files, {total / 1e9:.2f} GB, {dt * 1e3:.0f} ms)", flush=True)
ctx.close()
