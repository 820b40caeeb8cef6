"""Bulk / recovery ingest: the FastDHT state of a batch of stored files, in
bulk.

Today `storage_disk_recovery` (storage/storage_disk_recovery.c:512-761) and
the sync receiver (storage/storage_service.c:5468-5779) re-store files
without signatures, and a normal upload with `check_file_duplicate` pays one
FastDHT round trip per file plus two SETs on a miss and an INC per link
(storage/storage_service.c:2652,2714,2734,2984).  For a batch of files that
already have their file ids, `recovery_records` computes, on the GPU:

* the CRC32 and 24-byte signature of every file (fdfs_gpu_sig_batch);
* the dedup decision (fdfs_gpu_dedup): the class source is the first file
  of the batch with that signature, the class size is the "ref" count a
  sequential ingest leaves (A9);
* the three FastDHT record sets a sequential ingest writes, each routed to
  its FastDHT group and server and ordered group by group so that one
  `fdht_batch_set_ex` (storage/fdht_client/fdht_client.c:512) per group
  replaces the per-file RPCs:
    - "fid": key (ns, sig), value = the source's file id (:2714), sources only;
    - "ref": key (ns, source file id), value = class size (:2734, :2984);
    - "sig": key (ns, file id), value = sig, every file
      (storage_set_link_file_meta, :2996-3004).

The composition itself is C (fdfs_gpu_recovery_batch in libfdfs_gpu, the
daemon's language); this module only wraps it for torch tensors.  Every
byte of compute is a libfdfs_gpu kernel.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .api import Context


@dataclass
class Routed:
    """One FastDHT record set: records i = 0..m-1 with key hash, group,
    server; `order` lists them group by group, `group_start` the bounds."""
    index: torch.Tensor        # int64[m]: the file each record belongs to
    key_hash: torch.Tensor     # int32[m]
    group: torch.Tensor        # int32[m]
    server: torch.Tensor       # int32[m]
    order: torch.Tensor        # int64[m]
    group_start: torch.Tensor  # int64[group_count + 1]


@dataclass
class RecoveryBatch:
    crc: torch.Tensor   # int32[n] (uint32 bit pattern)
    sig: torch.Tensor   # uint8[n, 24]
    rep: torch.Tensor   # int64[n]: ingest index of the class source
    ref: torch.Tensor   # int32[n]: class size
    fid: Routed         # sources only; key = sig, value = file_ids[index]
    ref_rec: Routed     # sources only; key = file_ids[index], value = ref[index]
    sig_rec: Routed     # every file; key = file_ids[index], value = sig[index]


def recovery_records(ctx: Context, data: torch.Tensor, offsets: torch.Tensor, sizes: torch.Tensor,
                     file_ids: torch.Tensor, file_id_len: torch.Tensor, namespace: bytes,
                     group_count: int, servers_per_group: torch.Tensor | None = None,
                     method: int = 1, stream=None) -> RecoveryBatch:
    """file_ids: uint8[n, stride] (stride % 4 == 0, <= 128) holding each
    file's id "group/M00/00/00/<name><ext>" in its first file_id_len[i]
    (int32[n]) bytes; method: FDFS_SIG_HASH (1) or FDFS_SIG_MD5 (2).
    One call of fdfs_gpu_recovery_batch (the whole composition runs in the
    C library, stream-ordered); the fid / ref_rec sets are cut to the
    device-counted number of class sources here."""
    import ctypes

    from . import _lib
    from .api import _check_dev, _ptr, _stream_handle
    if method not in (1, 2):
        raise ValueError("method must be FDFS_SIG_HASH or FDFS_SIG_MD5 (dedup needs a signature)")
    for t, nm, dt in ((data, "data", torch.uint8), (offsets, "offsets", torch.int64),
                      (sizes, "sizes", torch.int64), (file_ids, "file_ids", torch.uint8),
                      (file_id_len, "file_id_len", torch.int32)):
        _check_dev(t, nm, dt)
    if servers_per_group is not None:
        _check_dev(servers_per_group, "servers_per_group", torch.int32)
    from .api import _check_batch
    n = _check_batch(data, offsets, sizes, True)
    if file_ids.dim() != 2 or file_ids.shape[0] != n or file_id_len.numel() != n:
        raise ValueError("one file id record per file")
    dev = data.device

    def e(dt, *shape):
        return torch.empty(shape, dtype=dt, device=dev)

    crc, sig, rep, ref, nsrc = e(torch.int32, n), e(torch.uint8, n, 24), e(torch.int64, n), \
        e(torch.int32, n), e(torch.int64, 1)
    sets = [[e(torch.int64, n), e(torch.int32, n), e(torch.int32, n), e(torch.int32, n),
             e(torch.int64, n), e(torch.int64, group_count + 1)] for _ in range(3)]
    out = _lib.FdfsGpuRecoveryOut(crc.data_ptr(), sig.data_ptr(), rep.data_ptr(), ref.data_ptr(),
                                  nsrc.data_ptr(),
                                  *[_lib.FdfsGpuRouted(*[t.data_ptr() for t in st]) for st in sets])
    b = _lib.FdfsGpuBatch(data.data_ptr(), offsets.data_ptr(), sizes.data_ptr(), n)
    ctx._rc(ctx._L.fdfs_gpu_recovery_batch(ctx._h, ctypes.byref(b), method, file_ids.data_ptr(),
                                           file_ids.shape[1], file_id_len.data_ptr(), namespace,
                                           len(namespace), group_count, _ptr(servers_per_group),
                                           ctypes.byref(out), _stream_handle(stream)),
            "fdfs_gpu_recovery_batch")
    # nsources was written on `stream`, which need not be torch's current one
    (stream if stream is not None else torch.cuda.current_stream()).synchronize()
    m = int(nsrc.item())

    def routed(st, k):
        return Routed(st[0][:k], st[1][:k], st[2][:k], st[3][:k], st[4][:k], st[5])

    return RecoveryBatch(crc=crc, sig=sig, rep=rep, ref=ref, fid=routed(sets[0], m),
                         ref_rec=routed(sets[1], m), sig_rec=routed(sets[2], n))
