"""Round-2 hipGraph fault, closed out from the captured graph itself.

Captures the upload-path step (HASH sig_batch of 3,000 files incl. a few
5 MiB ones + dedup of the signatures, the shape of tests/test_gpu_graph.py)
with torch.cuda.graph in debug mode and writes hipGraphDebugDotPrint's dump,
once with the library's zeroing kernels and once with round 2's
hipMemsetAsync zeroing (probe build, FDFS_GPU_MEMSET=1: run this script with
FDFS_GPU_PROBE_LIB=1).  No replay: the dumps are read for the memset nodes'
dependencies (scripts/graph_dot_edges.py).
Usage: FDFS_GPU_PROBE_LIB=1 [FDFS_GPU_MEMSET=1] python3 scripts/graph_memset_probe.py OUT.dot
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fastdfs_amd as F  # noqa: E402


def main():
    out_path = sys.argv[1]
    rng = np.random.default_rng(4243)
    n = 3000
    sizes = rng.integers(0, 70_000, n).astype(np.int64)
    sizes[::97] = 5 << 20
    offs = np.zeros(n, np.int64)
    offs[1:] = np.cumsum((sizes + 15) // 16 * 16)[:-1]
    total = int(offs[-1] + sizes[-1])
    dev = torch.device("cuda", 0)
    data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev)
    offs_t, sizes_t = torch.from_numpy(offs).to(dev), torch.from_numpy(sizes).to(dev)
    ctx = F.Context(0)
    ctx.reserve(n, n)

    def step():
        crc, sig, _ = ctx.sig_batch(data, offs_t, sizes_t, method=F.SIG_HASH, check_bounds=False)
        rep, ref = ctx.dedup(sig)
        return crc, sig, rep, ref

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    g.enable_debug_mode()
    with torch.cuda.graph(g):
        step()
    g.debug_dump(out_path)
    print("dumped", out_path, os.path.getsize(out_path), "bytes")


if __name__ == "__main__":
    main()
