"""Config 3 pair timeline (probe build with csrc/probes/pair_timeline.patch,
FDFS_GPU_PROBE_LIB=1): when each workgroup of the MD5 kernel that ran the
batch (md5_pair_kernel's chunk queue, the production form, or with
FDFS_GPU_MD5_PACK=1 the lane-packed md5_pack_kernel, one chunk per pair)
ends, how many chunks and 128-byte rounds it ran, and where it sat (HW_ID /
XCC_ID).  Answers whether the batch ends with a few workgroups (a tail that
idle SIMDs could fill) or all together.

Usage: FDFS_GPU_PROBE_LIB=1 [FDFS_GPU_MD5_PACK=1] python3 scripts/pair_timeline.py [--files N]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import fastdfs_amd as F  # noqa: E402
from fastdfs_amd import _lib, corpus as C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    assert os.environ.get("FDFS_GPU_PROBE_LIB") == "1"
    dev = torch.device("cuda", 0)
    sizes = C.photo_sizes(a.files, seed=3)
    data, offs, szs = C.device_batch(sizes, seed=2, device=dev, align=16)
    ctx = F.Context(0)
    L = _lib.load()
    L.fdfs_gpu_probe_pairs.restype = ctypes.c_int
    L.fdfs_gpu_probe_pairs.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    nwg = min(4 * ncu, (a.files + 63) // 64)  # the grid of either kernel
    hz = 100e6  # s_memrealtime
    res = []
    for rep in range(a.reps):
        ctx.set_timing(True)
        ctx.read_timing(_lib.KERNEL_SIG_LANE)
        ctx.sig_batch(data, offs, szs, method=F.SIG_MD5, check_bounds=False)
        torch.cuda.synchronize()
        kms, _ = ctx.read_timing(_lib.KERNEL_SIG_LANE)
        buf = np.zeros(4 * nwg, np.uint64)
        assert L.fdfs_gpu_probe_pairs(buf.ctypes.data, buf.size) == 0
        r = buf.reshape(nwg, 4)
        t0 = r[:, 0].astype(np.float64)
        t1 = r[:, 1].astype(np.float64)
        base = t0.min()
        end_ms = (t1 - base) / hz * 1e3
        start_ms = (t0 - base) / hz * 1e3
        chunks = (r[:, 2] & ((1 << 20) - 1)).astype(np.int64)
        rounds = (r[:, 2] >> 20).astype(np.int64)
        hw = (r[:, 3] & 0xFFFFFFFF).astype(np.int64)
        xcc = (r[:, 3] >> 32).astype(np.int64) & 0xF
        cu = (hw >> 8) & 0xF
        se = (hw >> 13) & 0x7
        simd = (hw >> 4) & 0x3
        q = lambda x: [round(float(v), 3) for v in np.quantile(x, [0, 0.01, 0.1, 0.5, 0.9, 0.99, 1.0])]  # noqa: E731
        # per CU (xcc, se, cu): the sum of its workgroups' rounds and its last end
        key = xcc * 1000 + se * 100 + cu
        cus = {}
        for k, e, rr in zip(key.tolist(), end_ms.tolist(), rounds.tolist()):
            c = cus.setdefault(k, [0.0, 0])
            c[0] = max(c[0], e)
            c[1] += rr
        cu_end = np.array([v[0] for v in cus.values()])
        cu_rounds = np.array([v[1] for v in cus.values()])
        # time-weighted idleness: SIMD-pair time lost after each workgroup's end
        kend = end_ms.max()
        idle_frac = float(np.mean(kend - end_ms) / kend)
        d = {"rep": rep, "kernel_ms_events": round(kms, 3), "span_ms": round(float(kend), 3),
             "workgroups": int(nwg), "start_ms_q": q(start_ms), "end_ms_q": q(end_ms),
             "chunks_q": q(chunks), "rounds_q": q(rounds), "rounds_total": int(rounds.sum()),
             "idle_after_end_frac": round(idle_frac, 4),
             "last_10_workgroups": [int(i) for i in np.argsort(end_ms)[-10:]],
             "cus": len(cus), "cu_end_ms_q": q(cu_end), "cu_rounds_q": q(cu_rounds),
             "corr_end_vs_rounds": round(float(np.corrcoef(end_ms, rounds)[0, 1]), 4),
             "simd_hist": np.bincount(simd, minlength=4).tolist(),
             "xcc_hist": np.bincount(xcc, minlength=8).tolist()}
        res.append(d)
        print(json.dumps(d), flush=True)
        if a.out and rep == a.reps - 1:
            np.savez_compressed(a.out, start_ms=start_ms, end_ms=end_ms, chunks=chunks, rounds=rounds,
                                hw=hw, xcc=xcc)
    ctx.close()


if __name__ == "__main__":
    main()
