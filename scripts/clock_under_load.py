"""Shader clock while a config's signature batches run back to back:
scripts/probes/clock_probe (one wave, s_memtime over s_memrealtime) runs as a
child process beside `secs` seconds of ctx.sig_batch on the config's batch.

python scripts/clock_under_load.py c3 20
"""
import os
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fastdfs_amd as F  # noqa: E402
from fastdfs_amd import corpus as C  # noqa: E402


def main(cfg, secs):
    dev = torch.device("cuda", 0)
    if cfg == "c3":
        sizes, method = C.photo_sizes(100_000, seed=3), F.SIG_MD5
    elif cfg == "c2":
        sizes, method = C.small_files_sizes(1_000_000, seed=1), F.SIG_HASH
    else:
        raise SystemExit("c2 or c3")
    data, offs, sz = C.device_batch(sizes, seed=2, device=dev)
    ctx = F.Context(0)
    ctx.reserve(len(sizes), 0)
    ctx.sig_batch(data, offs, sz, method=method, check_bounds=False)
    torch.cuda.synchronize()
    n = int(secs / 0.4)
    probe = subprocess.Popen([os.path.join(ROOT, "scripts/probes/clock_probe"), str(n), "380", "20"])
    t0, k = time.time(), 0
    while time.time() - t0 < secs:
        ctx.sig_batch(data, offs, sz, method=method, check_bounds=False)
        torch.cuda.synchronize()
        k += 1
    print(f"{cfg}: {k} batches in {time.time() - t0:.1f} s", flush=True)
    sys.exit(probe.wait())


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]))
