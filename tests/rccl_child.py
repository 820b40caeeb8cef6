"""One rank of tests/test_gpu_rccl.py: a fresh process per GPU (started by
the test before it makes any GPU call), joined over RCCL.

It runs libfdfs_gpu's two multi-GPU C entry points on its share of seeded
inputs that every rank regenerates identically, and checks its own answers
against the oracle over the concatenation:

* fdfs_gpu_dedup_global (replaces the per-file fdht_get_ex1 / fdht_set_ex /
  fdht_inc_ex round trips, storage/storage_service.c:2652,2714,2734,2984):
  shares of uneven size (one empty when world > 2), duplicates across ranks,
  ingest indices with gaps;
* fdfs_gpu_crc_batch_global (recovery of files spread over ranks,
  storage/storage_disk_recovery.c:512-761): files cut into pieces by
  plan_crc_pieces, so the large ones span ranks, both shift variants; and the
  same plan through the torch.distributed form for comparison.

Prints one line "RANK r OK ..." and exits 0, or prints the mismatch and
exits 1.  Test infrastructure: the oracle is the checker here.
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def shares(n: int, world: int, seed: int) -> list[tuple[int, int]]:
    import numpy as np
    rng = np.random.default_rng(seed)
    cuts = sorted(rng.choice(np.arange(1, n), world - 1, replace=False).tolist()) if world > 1 else []
    b = [0] + cuts + [n]
    if world > 2:
        b[2] = b[1]  # rank 1 holds nothing
    return [(b[p], b[p + 1]) for p in range(world)]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--records", type=int, default=600_000)
    a = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist

    import fastdfs_amd as F
    from fastdfs_amd.api import Comm
    from fastdfs_amd.dist import crc_batch_global, dedup_global, plan_crc_pieces
    from oracle import oracle

    rank, world = a.rank, a.world
    dev = torch.device("cuda", rank)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{a.port}", rank=rank,
                            world_size=world, device_id=dev)
    errs = []
    ctxs = [F.Context(rank), F.Context(rank, unsigned_hash=True)]
    comms = [Comm(c) for c in ctxs]
    try:
        # ---- dedup_global: 600K records, ~40% of them duplicates of others
        n = a.records
        rng = np.random.default_rng(2024)
        base = rng.integers(0, 256, size=(n * 3 // 5, 24), dtype=np.uint8)
        sig = base[rng.integers(0, len(base), size=n)]
        gidx = np.cumsum(rng.integers(1, 4, n)).astype(np.int64)
        orep, oref = oracle.dedup(sig)
        lo, hi = shares(n, world, 99)[rank]
        rep, ref = dedup_global(ctxs[0], torch.from_numpy(sig[lo:hi].copy()).to(dev),
                                torch.from_numpy(gidx[lo:hi].copy()).to(dev), comm=comms[0])
        torch.cuda.synchronize()
        if not np.array_equal(rep.cpu().numpy(), gidx[orep[lo:hi].astype(np.int64)]):
            errs.append(f"dedup_global rep ({hi - lo} records)")
        if not np.array_equal(ref.cpu().numpy(), oref[lo:hi].astype(np.int32)):
            errs.append(f"dedup_global ref ({hi - lo} records)")
        # ---- crc_batch_global: files cut over the ranks in byte order
        frng = np.random.default_rng(7)
        sizes = np.array([0, 5, (48 << 20) + 3, 70_001, (3 << 20) + 11, 1 << 20, 17], np.int64)
        files = [frng.integers(0, 256, size=int(s), dtype=np.uint8) for s in sizes]
        plan = plan_crc_pieces(sizes, world)
        mine = plan[rank]
        offs, pos, chunks = [], 0, []
        for f, s0, ln in mine:
            pos += int(frng.integers(0, 9))  # any alignment
            offs.append(pos)
            chunks.append((pos, files[f][s0:s0 + ln]))
            pos += ln
        buf = np.zeros(pos + 1, np.uint8)
        for p0, b in chunks:
            buf[p0:p0 + len(b)] = b
        data = torch.from_numpy(buf).to(dev)
        offs_t = torch.tensor(offs, dtype=torch.int64, device=dev)
        for v in (0, 1):
            want = [oracle.crc32(f, v) for f in files]
            for c in (comms[v], None):  # the C ABI over RCCL, then the torch.distributed form
                crc = crc_batch_global(ctxs[v], sizes, plan, data, offs_t, comm=c)
                got = [int(x) for x in crc.cpu().numpy().view(np.uint32)]
                if got != want:
                    errs.append(f"crc_batch_global variant {v} {'C ABI' if c is not None else 'torch'}")
    finally:
        for c in comms:
            c.close()
        for c in ctxs:
            c.close()
        dist.destroy_process_group()
    if errs:
        print(f"RANK {rank} FAIL: " + "; ".join(errs), flush=True)
        return 1
    print(f"RANK {rank} OK world={world} records={hi - lo}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
