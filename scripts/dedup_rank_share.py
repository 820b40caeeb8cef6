"""Config 5's dedup at one rank's share of an N-GPU run.

The bench's 100M-record set is split as `bench.py --gpus N` splits it
(corpus.c5_signatures); this times rank 0's local work at that share:

  --mode rccl    fdfs_gpu_dedup_global over a one-rank RCCL communicator on
                 rank 0's share: bucket, announcement all-gather + host read,
                 self copy, owner group of the 32-byte rows, answers back,
                 gather -- every step of the N-GPU call except the xGMI moves;
  --mode local   fdfs_gpu_dedup_global_local with N virtual ranks (all of
                 them on this GPU, one after another: per-rank kernels);
  --mode single  fdfs_gpu_dedup (one-GPU API) on rank 0's share.

Prints one JSON line: wall ms per call (host-timed, synchronised), and the
library's HIP-event time of its bucket / group kernels per call.  Run under
`rocprofv3 --kernel-trace --stats` for the per-kernel breakdown
(scripts/kernel_share.py summarises the trace per call).
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fastdfs_amd as F  # noqa: E402
from fastdfs_amd import _lib, corpus as C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["rccl", "local", "single"], default="rccl")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--total", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = F.Context(0)
    comm = None
    if a.mode == "local":
        shares = [C.c5_signatures(a.total, a.world, r, dev) for r in range(a.world)]
        fn = lambda: ctx.dedup_global_local([s for s, _ in shares], [g for _, g in shares])  # noqa: E731
        n0 = shares[0][0].shape[0]
    else:
        sig, gidx = C.c5_signatures(a.total, a.world, 0, dev)
        n0 = sig.shape[0]
        if a.mode == "rccl":
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
            comm = F.api.Comm(ctx)
            fn = lambda: ctx.dedup_global(comm, sig, gidx)  # noqa: E731
        else:
            ctx.reserve(0, n0)
            fn = lambda: ctx.dedup(sig, gidx)  # noqa: E731
    for _ in range(a.warmup):
        fn()
    torch.cuda.synchronize()
    ctx.set_timing(True)
    for k in (_lib.KERNEL_BUCKET, _lib.KERNEL_DEDUP):
        ctx.read_timing(k)
    t0 = time.perf_counter()
    for _ in range(a.reps):
        fn()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.reps * 1e3
    bms, bn = ctx.read_timing(_lib.KERNEL_BUCKET)
    gms, gn = ctx.read_timing(_lib.KERNEL_DEDUP)
    ctx.set_timing(False)
    rec = {"mode": a.mode, "world": a.world, "records_rank0": n0, "reps": a.reps,
           "wall_ms_per_call": round(wall, 4),
           "bucket_ms_per_call": round(bms / a.reps, 4), "bucket_launches": bn,
           "group_ms_per_call": round(gms / a.reps, 4), "group_launches": gn}
    if a.mode != "single" and hasattr(ctx._L, "fdfs_gpu_dedup_global_stats"):
        # bytes between ranks per call (all virtual ranks for --mode local);
        # the round-5 protocol returned a 16-byte answer for every row it
        # received, i.e. half the row bytes
        b = ctx.dedup_global_stats()
        rec.update({"row_bytes": b["row_bytes"], "answer_bytes": b["answer_bytes"],
                    "answer_bytes_round5_protocol": b["row_bytes"] // 2,
                    "answer_ratio_vs_round5": round(b["answer_bytes"] / max(b["row_bytes"] // 2, 1), 4)})
    print(json.dumps(rec), flush=True)
    if comm is not None:
        comm.close()
    ctx.close()
    if a.mode == "rccl":
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
