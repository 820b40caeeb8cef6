"""Per-call cost of the chunked (dio_write_file-shaped) path at daemon batch sizes.

The storage daemon's dio thread advances every upload that received a chunk
since its last wakeup (<= buff_size = 256 KiB each, conf/storage.conf:52) in
one fdfs_gpu_update_batch call.  A wakeup carries from a handful to thousands
of chunks, so the fixed cost of a call (its launches) matters as much as the
kernel's streaming rate.  Prints one JSON line per (method, n): mean us per
call, GB/s, and the same with the calls captured in a hipGraph.

    python scripts/chunk_sweep.py [--chunk 262144] [--calls 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastdfs_amd import api  # noqa: E402


def time_calls(fn, calls, stream):
    with torch.cuda.stream(stream):
        for _ in range(3):
            fn()
    stream.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    with torch.cuda.stream(stream):
        for _ in range(calls):
            fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / calls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunk", type=int, default=256 << 10)
    ap.add_argument("--calls", type=int, default=50)
    ap.add_argument("--ns", default="1,16,64,256,1024,4096,16384")
    ap.add_argument("--methods", default="0,1,2")
    ap.add_argument("--graph", type=int, default=1)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = api.Context(0)
    ns = [int(x) for x in a.ns.split(",")]
    nmax = max(ns)
    ctx.reserve(nmax, 0)
    g = torch.Generator(device=dev).manual_seed(1)
    data = torch.randint(0, 256, (nmax * a.chunk,), dtype=torch.uint8, device=dev, generator=g)
    stream = torch.cuda.Stream(dev)
    for m in [int(x) for x in a.methods.split(",")]:
        for n in ns:
            offs = torch.arange(n, dtype=torch.int64, device=dev) * a.chunk
            sizes = torch.full((n,), a.chunk, dtype=torch.int64, device=dev)
            states = ctx.new_states(n, stream=stream)

            def call():
                ctx.update_batch(states, data, offs, sizes, method=m, stream=stream, check_bounds=False)

            us = time_calls(call, a.calls, stream)
            row = {"method": m, "n": n, "chunk": a.chunk, "us_per_call": round(us, 2),
                   "GB_s": round(n * a.chunk / us / 1e3, 1)}
            if a.graph:
                try:
                    stream.synchronize()
                    graph = torch.cuda.CUDAGraph()
                    reps = 10
                    with torch.cuda.graph(graph, stream=stream):
                        for _ in range(reps):
                            call()
                    ug = time_calls(graph.replay, max(1, a.calls // reps), stream) / reps
                    row["graph_us_per_call"] = round(ug, 2)
                    row["graph_GB_s"] = round(n * a.chunk / ug / 1e3, 1)
                except Exception as e:  # capture is optional; report why it failed
                    row["graph_error"] = str(e)[:200]
            print(json.dumps(row), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
