"""Round-2 hipGraph fault, closed out from the captured graph itself.

Captures the upload-path step (HASH sig_batch of 3,000 files incl. a few
5 MiB ones + dedup of the signatures, the shape of tests/test_gpu_graph.py)
on one stream with the HIP stream-capture API (ctypes on libamdhip64),
writes hipGraphDebugDotPrint's dump and lists every node with its type and
its dependencies (hipGraphGetNodes / hipGraphNodeGetDependencies).  Run once
with the library's zeroing kernels and once with round 2's hipMemsetAsync
zeroing (probe build, FDFS_GPU_MEMSET=1; FDFS_GPU_PROBE_LIB=1 in both
cases).  No replay.
Usage: FDFS_GPU_PROBE_LIB=1 [FDFS_GPU_MEMSET=1] python3 scripts/graph_memset_probe.py OUT_PREFIX
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fastdfs_amd as F  # noqa: E402

NODE_TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty", 6: "wait_event",
              7: "event_record", 8: "ext_sem_signal", 9: "ext_sem_wait", 10: "mem_alloc", 11: "mem_free",
              12: "memcpy_from_symbol", 13: "memcpy_to_symbol"}


def main():
    prefix = os.path.abspath(sys.argv[1])
    hip = ctypes.CDLL("libamdhip64.so")
    vp = ctypes.c_void_p
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
    crc = torch.empty(n, dtype=torch.int32, device=dev)
    sig = torch.empty((n, 24), dtype=torch.uint8, device=dev)
    rep = torch.empty(n, dtype=torch.int64, device=dev)
    ref = torch.empty(n, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream()

    def step():
        ctx.sig_batch(data, offs_t, sizes_t, method=F.SIG_HASH, crc_out=crc, sig_out=sig, check_bounds=False,
                      stream=s)
        L = ctx._L
        ctx._rc(L.fdfs_gpu_dedup(ctx._h, sig.data_ptr(), None, n, rep.data_ptr(), ref.data_ptr(),
                                 s.cuda_stream), "dedup")

    step()
    torch.cuda.synchronize()
    graph = vp()
    assert hip.hipStreamBeginCapture(vp(s.cuda_stream), 0) == 0  # hipStreamCaptureModeGlobal
    step()
    assert hip.hipStreamEndCapture(vp(s.cuda_stream), ctypes.byref(graph)) == 0
    rc = hip.hipGraphDebugDotPrint(graph, (prefix + ".dot").encode(), ctypes.c_uint(0xFFFF))
    count = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(graph, None, ctypes.byref(count)) == 0
    nodes = (vp * count.value)()
    assert hip.hipGraphGetNodes(graph, nodes, ctypes.byref(count)) == 0
    index = {nodes[i]: i for i in range(count.value)}
    listing = []
    for i in range(count.value):
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(vp(nodes[i]), ctypes.byref(t))
        nd = ctypes.c_size_t(0)
        hip.hipGraphNodeGetDependencies(vp(nodes[i]), None, ctypes.byref(nd))
        deps = (vp * max(nd.value, 1))()
        hip.hipGraphNodeGetDependencies(vp(nodes[i]), deps, ctypes.byref(nd))
        item = {"node": i, "type": NODE_TYPES.get(t.value, t.value),
                "deps": [index.get(deps[k], -1) for k in range(nd.value)]}
        if t.value == 2:  # memset: its parameters
            class MemsetParams(ctypes.Structure):
                _fields_ = [("dst", vp), ("elementSize", ctypes.c_uint), ("height", ctypes.c_size_t),
                            ("pitch", ctypes.c_size_t), ("value", ctypes.c_uint), ("width", ctypes.c_size_t)]
            p = MemsetParams()
            if hip.hipGraphMemsetNodeGetParams(vp(nodes[i]), ctypes.byref(p)) == 0:
                item["memset"] = {"elementSize": p.elementSize, "width": p.width, "height": p.height,
                                  "pitch": p.pitch, "value": p.value}
        listing.append(item)
    json.dump({"dot_rc": rc, "nodes": listing}, open(prefix + ".json", "w"), indent=1)
    print("nodes", count.value, "dot rc", rc, "memset nodes",
          [x for x in listing if x["type"] == "memset"])
    hip.hipGraphDestroy(graph)


if __name__ == "__main__":
    main()
