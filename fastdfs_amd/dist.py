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
    to other ranks (32-byte rows out, 16-byte answers back; torch form only).
    """
    if comm is not None:
        return kernels.dedup_global(comm, sig, gidx)
    world = dist.get_world_size(group)
    dev = sig.device
    rows, counts, row_of = kernels.dedup_bucket(sig, gidx, world)
    recv_counts = torch.empty_like(counts)
    dist.all_to_all_single(recv_counts, counts, group=group)
    send = counts.cpu().tolist()
    recv = recv_counts.cpu().tolist()
    if stats is not None:
        me = dist.get_rank(group)
        stats["peer_bytes"] = stats.get("peer_bytes", 0) + 32 * (sum(send) - send[me]) + \
            16 * (sum(recv) - recv[me])
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
