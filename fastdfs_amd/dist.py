"""Multi-GPU orchestration: one process per GPU over torch.distributed (RCCL).

* Signature work shards with no exchange: files are independent, so ranks
  take disjoint file sets (shard_lpt balances bytes).
* Dedup has exactly one exchange step, replacing the per-file FastDHT
  lookups of storage/storage_service.c:2652-2785: every rank buckets its
  signatures by owner = hash(sig) mod world (the analogue of the FastDHT key
  partition, storage/fdht_client/fdht_client.c:301-305), one all-to-all moves
  the 32-byte rows to their owners over xGMI, owners group locally, and a
  second all-to-all returns {rep, ref} to the ranks that hold the files.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def shard_lpt(sizes: np.ndarray, nranks: int) -> list[np.ndarray]:
    """Longest-processing-time greedy split of files by bytes.

    Returns per-rank file index arrays (each sorted ascending, so a rank's
    files keep their ingest order)."""
    sizes = np.asarray(sizes, dtype=np.int64)
    order = np.argsort(-sizes, kind="stable")
    load = np.zeros(nranks, dtype=np.int64)
    owner = np.empty(sizes.size, dtype=np.int64)
    # heap-free greedy: nranks is small (<= 8 GPUs per node)
    for i in order:
        r = int(np.argmin(load))
        owner[i] = r
        load[r] += max(int(sizes[i]), 1)
    return [np.nonzero(owner == r)[0] for r in range(nranks)]


def plan_crc_pieces(sizes, nranks: int) -> list[list[tuple[int, int, int]]]:
    """CRC-only work split by bytes: the files' concatenated
    byte stream is cut into nranks contiguous shares of equal size, so a
    file larger than a share (or straddling a cut) is split into pieces on
    consecutive ranks, in byte order.  CRC32 is linear over GF(2), so the
    pieces are hashed independently and joined by crc32_combine; ELFHash and
    MD5 are not splittable and use shard_lpt.  Returns, per rank, its
    (file, start, length) pieces; every rank computes the same plan."""
    sizes = np.asarray(sizes, dtype=np.int64)
    total = int(sizes.sum())
    share = -(-total // nranks) if total else 0
    plan: list[list[tuple[int, int, int]]] = [[] for _ in range(nranks)]
    r, room = 0, share
    for f, sz in enumerate(sizes.tolist()):
        a = 0
        while a < sz:
            while room == 0 and r < nranks - 1:
                r, room = r + 1, share
            take = sz - a if r == nranks - 1 else min(sz - a, room)
            plan[r].append((f, a, take))
            a += take
            room -= take
    return plan


def crc_batch_global(kernels, sizes, plan, data: torch.Tensor, offsets: torch.Tensor, group=None, comm=None):
    """CRC32 of files whose bytes are spread over the ranks as `plan`
    (plan_crc_pieces) says: this rank holds its pieces in `data` at
    `offsets` (int64, one per piece of plan[rank], in plan order).

    Each rank hashes its pieces from a zero state (fdfs_gpu_update_batch on
    zeroed states: CRC32_ex(piece, 0)), one all-gather moves the 4-byte
    partial states, and every rank folds each file's pieces in byte order:
    acc = M^|piece| acc ^ part (fdfs_gpu_crc_combine), from CRC32_XINIT; the
    file CRC is CRC32_FINAL(acc).  Returns uint32 CRCs (int32 bit patterns)
    of all files on every rank.  kernels: a fastdfs_amd.Context (tests
    substitute a CPU double).

    comm: a fastdfs_amd.api.Comm -> the whole step runs inside libfdfs_gpu
    (fdfs_gpu_crc_batch_global: each piece's term advanced to its file's
    end, one ncclAllGather of 20 bytes per file, the fold on the device),
    the C recovery caller's path; this function then only builds the piece
    arrays from the plan."""
    if comm is not None:
        dev = data.device
        mine = plan[comm.rank]
        pf = torch.tensor([p[0] for p in mine], dtype=torch.int64, device=dev)
        ps = torch.tensor([p[1] for p in mine], dtype=torch.int64, device=dev)
        lens = torch.tensor([p[2] for p in mine], dtype=torch.int64, device=dev)
        fs = torch.from_numpy(np.asarray(sizes, dtype=np.int64)).to(dev)
        return kernels.crc_batch_global(comm, data, offsets, lens, pf, ps, fs)
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = data.device
    sizes = np.asarray(sizes, dtype=np.int64)
    nfiles = sizes.size
    mine = plan[rank]
    m = len(mine)
    lens = torch.tensor([p[2] for p in mine], dtype=torch.int64, device=dev)
    part = torch.zeros(max(m, 1), dtype=torch.int32, device=dev)
    if m:
        states = torch.zeros((m, 128), dtype=torch.uint8, device=dev)  # crc32 = 0, count = 0
        kernels.update_batch(states, data, offsets, lens, method=0)
        part[:m] = states[:, :4].contiguous().view(torch.int32).view(-1)
    # 4 bytes per piece to every rank (padded to the longest piece list)
    mp = max(max(len(p) for p in plan), 1)
    send = torch.zeros(mp, dtype=torch.int32, device=dev)
    send[:m] = part[:m]
    gathered = [torch.empty_like(send) for _ in range(world)]
    dist.all_gather(gathered, send, group=group)
    # piece k of every file, byte order = rank order then plan order
    per_file: list[list[tuple[int, int, int]]] = [[] for _ in range(nfiles)]
    for r in range(world):
        for j, (f, a, ln) in enumerate(plan[r]):
            per_file[f].append((a, r * mp + j, ln))
    for pcs in per_file:
        pcs.sort()
    kmax = max((len(p) for p in per_file), default=0)
    flat = torch.cat(gathered)
    acc = torch.full((nfiles,), -1, dtype=torch.int32, device=dev)  # CRC32_XINIT
    for k in range(kmax):
        idx = np.zeros(nfiles, np.int64)
        ln = np.zeros(nfiles, np.int64)
        has = np.zeros(nfiles, bool)
        for f, pcs in enumerate(per_file):
            if k < len(pcs):
                _, idx[f], ln[f] = pcs[k]
                has[f] = True
        b = torch.where(torch.from_numpy(has).to(dev), flat[torch.from_numpy(idx).to(dev)],
                        torch.zeros((), dtype=torch.int32, device=dev))
        # missing piece: length 0 and part 0 leave acc unchanged
        acc = kernels.crc_combine(acc, b.contiguous(), torch.from_numpy(ln).to(dev))
    return acc ^ -1  # CRC32_FINAL


def dedup_global(kernels, sig: torch.Tensor, gidx: torch.Tensor, group=None, stats=None, comm=None):
    """Dedup across all ranks of `group`.

    comm: a fastdfs_amd.api.Comm -> the whole exchange runs inside
    libfdfs_gpu (fdfs_gpu_dedup_global over RCCL, the C daemon's path); this
    function is then a thin caller.  Without it the same steps run here over
    torch.distributed collectives (the gloo tests use that form with a CPU
    double of the kernels).

    kernels: a fastdfs_amd.Context (the HIP kernels); tests substitute a
    CPU double to exercise the exchange over gloo.
    sig: uint8 [n, 24] this rank's signatures; gidx: int64 [n] their global
    ingest indices.  Returns (rep int64[n], ref int32[n]) for this rank's
    files, identical to single-process dedup over the concatenated input.
    stats: optional dict; "peer_bytes" accumulates the bytes this rank sent
    to other ranks, "row_bytes" / "answer_bytes" its two parts: with comm,
    the 32-byte rows to the other owners and the 16-byte answer records of
    multi-member classes back to their senders (fdfs_gpu_dedup_global_stats);
    in the torch form 32 bytes per row out and a 16-byte answer per row back.
    """
    if comm is not None:
        out = kernels.dedup_global(comm, sig, gidx)
        if stats is not None:
            b = kernels.dedup_global_stats()
            for k, v in (("row_bytes", b["row_bytes"]), ("answer_bytes", b["answer_bytes"]),
                         ("peer_bytes", b["row_bytes"] + b["answer_bytes"])):
                stats[k] = stats.get(k, 0) + v
        return out
    world = dist.get_world_size(group)
    dev = sig.device
    rows, counts, row_of = kernels.dedup_bucket(sig, gidx, world)
    recv_counts = torch.empty_like(counts)
    dist.all_to_all_single(recv_counts, counts, group=group)
    send = counts.cpu().tolist()
    recv = recv_counts.cpu().tolist()
    if stats is not None:
        me = dist.get_rank(group)
        rb, ab = 32 * (sum(send) - send[me]), 16 * (sum(recv) - recv[me])
        for k, v in (("row_bytes", rb), ("answer_bytes", ab), ("peer_bytes", rb + ab)):
            stats[k] = stats.get(k, 0) + v
    m = int(sum(recv))
    rows_in = torch.empty((m, 32), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(rows_in, rows, output_split_sizes=recv, input_split_sizes=send,
                           group=group)
    rep_in, ref_in = kernels.dedup_group(rows_in)
    answers = torch.stack([rep_in, ref_in.to(torch.int64)], dim=1).contiguous()
    back = torch.empty((rows.shape[0], 2), dtype=torch.int64, device=dev)
    dist.all_to_all_single(back, answers, output_split_sizes=send, input_split_sizes=recv,
                           group=group)
    mine = back.index_select(0, row_of)
    return mine[:, 0].contiguous(), mine[:, 1].to(torch.int32)
