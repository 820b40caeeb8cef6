"""Host-side API over libfdfs_gpu for torch-resident batches.

Mirrors the reference's call shape: one context per storage process /
device (storage_write_to_file initialises, dio_write_file computes,
storage_service_upload_file_done consumes), with the per-chunk CPU loops of
storage/storage_dio.c:465-515 replaced by one batched GPU call.
"""
from __future__ import annotations

import ctypes
import errno
import os

import torch

from . import _lib
from ._lib import SIG_CRC_ONLY, SIG_HASH, SIG_MD5, FLAG_UNSIGNED_HASH  # noqa: F401


class FdfsGpuError(RuntimeError):
    def __init__(self, rc: int, where: str, detail: str = ""):
        self.errno = rc
        msg = f"{where} failed: {errno.errorcode.get(rc, rc)} ({os.strerror(rc)})"
        if detail:
            msg += f": {detail}"
        super().__init__(msg)


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _stream_handle(stream) -> int | None:
    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream or None


def _check_dev(t: torch.Tensor, name: str, dtype=None):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor (got {t.device}); no CPU path exists")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")


_U32_MAX = 0xFFFFFFFF


def _check_batch(data: torch.Tensor, offsets: torch.Tensor, sizes: torch.Tensor, check_bounds: bool):
    """Batch shape checks before any device pointer reaches a kernel: n fits
    the C ABI's uint32 count, offsets/sizes pair up, and (check_bounds, one
    device reduction + sync) every file lies inside `data`."""
    _check_dev(data, "data", torch.uint8)
    _check_dev(offsets, "offsets", torch.int64)
    _check_dev(sizes, "sizes", torch.int64)
    n = offsets.numel()
    if sizes.numel() != n:
        raise ValueError("offsets and sizes differ in length")
    if n > _U32_MAX:
        raise ValueError(f"batch of {n} files exceeds the uint32 count of fdfs_gpu_batch")
    if check_bounds and n:
        lo = int(torch.minimum(offsets.min(), sizes.min()).item())
        hi = int((offsets + sizes).max().item())
        if lo < 0 or hi > data.numel():
            raise ValueError(f"file range [{lo}, {hi}) outside data of {data.numel()} bytes")
    return n


def _check_sig(sig: torch.Tensor, gidx: torch.Tensor | None, width: int = 24) -> int:
    _check_dev(sig, "sig", torch.uint8)
    if sig.dim() != 2 or sig.shape[1] != width:
        raise ValueError(f"sig must be uint8[n, {width}], got {tuple(sig.shape)}")
    n = sig.shape[0]
    if gidx is not None:
        _check_dev(gidx, "gidx", torch.int64)
        if gidx.numel() != n:
            raise ValueError(f"gidx has {gidx.numel()} entries for {n} records")
    return n


class Context:
    """A libfdfs_gpu context on one HIP device.

    unsigned_hash=False (default) is the signed-int CRC32_ex / ELFHash_ex
    state libfastcommon declares; True selects logical shifts (zlib CRC).
    """

    def __init__(self, device: int | None = None, unsigned_hash: bool = False, test_hooks: bool = False):
        # test_hooks: the context lives in the test-hooks build of the
        # library (fdfs_gpu_inject_error), for the error-path tests only
        self._L = _lib.load_test_hooks() if test_hooks else _lib.load()
        if device is None:
            device = torch.cuda.current_device()
        self.device = int(device)
        self.unsigned_hash = bool(unsigned_hash)
        h = ctypes.c_void_p()
        rc = self._L.fdfs_gpu_open(self.device, _lib.FLAG_UNSIGNED_HASH if unsigned_hash else 0,
                                   ctypes.byref(h))
        if rc:
            raise FdfsGpuError(rc, "fdfs_gpu_open")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.fdfs_gpu_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _rc(self, rc: int, where: str):
        if rc:
            raise FdfsGpuError(rc, where, (self._L.fdfs_gpu_last_error(self._h) or b"").decode())

    def set_timing(self, enable: bool = True):
        self._rc(self._L.fdfs_gpu_set_timing(self._h, 1 if enable else 0), "fdfs_gpu_set_timing")

    def read_timing(self, kernel: int) -> tuple[float, int]:
        """(summed ms, launches) of `kernel` (KERNEL_* in _lib) since the last read."""
        ms = ctypes.c_double()
        cnt = ctypes.c_uint64()
        self._rc(self._L.fdfs_gpu_read_timing(self._h, kernel, ctypes.byref(ms), ctypes.byref(cnt)),
                 "fdfs_gpu_read_timing")
        return ms.value, cnt.value

    def crc_lane_min_files(self) -> int:
        """fdfs_gpu_crc_lane_min_files: CRC-only batches of more files than
        this take the lane path (crc_lane_kernel)."""
        v = ctypes.c_uint64()
        self._rc(self._L.fdfs_gpu_crc_lane_min_files(self._h, ctypes.byref(v)), "fdfs_gpu_crc_lane_min_files")
        return v.value

    def inject_error(self, stream=None):
        """Test hook (fdfs_gpu_inject_error, contexts opened with
        test_hooks=True): queue a lane-path error on `stream`; a later call
        of this context fails with EIO once."""
        self._rc(self._L.fdfs_gpu_inject_error(self._h, _stream_handle(stream)), "fdfs_gpu_inject_error")

    def reserve(self, max_files: int, max_records: int = 0):
        self._rc(self._L.fdfs_gpu_reserve(self._h, max_files, max_records), "fdfs_gpu_reserve")

    # ------------------------------------------------------------- signature
    def sig_batch(self, data: torch.Tensor, offsets: torch.Tensor, sizes: torch.Tensor,
                  method: int = SIG_HASH, crc_out: torch.Tensor | None = None,
                  sig_out: torch.Tensor | None = None, codes_out: torch.Tensor | None = None,
                  want_sig: bool = True, want_codes: bool = False, stream=None,
                  check_bounds: bool = True):
        """CRC32 (+ 24-byte signature for SIG_HASH / SIG_MD5) of every file.

        data: uint8 device tensor; offsets/sizes: int64 device tensors [n].
        Returns (crc int32[n] holding the uint32 bit pattern, sig uint8[n,24]
        or None, codes int32[n,4] or None).  check_bounds verifies that every
        file lies inside `data` (one reduction + sync); callers that build
        the layout themselves (bench.py) turn it off.
        """
        n = _check_batch(data, offsets, sizes, check_bounds)
        dev = data.device
        if crc_out is None:
            crc_out = torch.empty(n, dtype=torch.int32, device=dev)
        if method != SIG_CRC_ONLY:
            if sig_out is None and want_sig:
                sig_out = torch.empty((n, 24), dtype=torch.uint8, device=dev)
            if codes_out is None and want_codes:
                codes_out = torch.empty((n, 4), dtype=torch.int32, device=dev)
        else:
            sig_out = codes_out = None
        b = _lib.FdfsGpuBatch(data.data_ptr(), offsets.data_ptr(), sizes.data_ptr(), n)
        self._rc(self._L.fdfs_gpu_sig_batch(self._h, ctypes.byref(b), method, crc_out.data_ptr(),
                                            _ptr(sig_out), _ptr(codes_out), _stream_handle(stream)),
                 "fdfs_gpu_sig_batch")
        return crc_out, sig_out, codes_out

    # ------------------------------------------- chunked (state-carrying) form
    def new_states(self, n: int, device=None, stream=None) -> torch.Tensor:
        """n fdfs_gpu_file_state records (uint8[n, 128] on the device),
        initialised as storage_write_to_file does (CRC32_XINIT,
        INIT_HASH_CODES4, my_md5_init)."""
        dev = torch.device("cuda", self.device) if device is None else device
        states = torch.empty((n, _lib.FILE_STATE_SIZE), dtype=torch.uint8, device=dev)
        if n > _U32_MAX:
            raise ValueError("too many states for a uint32 count")
        self._rc(self._L.fdfs_gpu_state_init(self._h, states.data_ptr(), n, _stream_handle(stream)),
                 "fdfs_gpu_state_init")
        return states

    @staticmethod
    def _check_states(states: torch.Tensor) -> int:
        _check_dev(states, "states", torch.uint8)
        if states.dim() != 2 or states.shape[1] != _lib.FILE_STATE_SIZE:
            raise ValueError(f"states must be uint8[n, {_lib.FILE_STATE_SIZE}]")
        return states.shape[0]

    def update_batch(self, states: torch.Tensor, data: torch.Tensor, offsets: torch.Tensor,
                     sizes: torch.Tensor, method: int = SIG_HASH,
                     state_idx: torch.Tensor | None = None, stream=None, check_bounds: bool = True):
        """dio_write_file's per-chunk update for a batch: chunk i (data
        [offsets[i], offsets[i] + sizes[i])) is hashed onto
        states[state_idx[i]] (state_idx int32[n], default i).  A state may
        appear at most once per call."""
        ns = self._check_states(states)
        n = _check_batch(data, offsets, sizes, check_bounds)
        if state_idx is not None:
            _check_dev(state_idx, "state_idx", torch.int32)
            if state_idx.numel() != n:
                raise ValueError("one state index per chunk")
            if check_bounds and n:
                lo, hi = int(state_idx.min().item()), int(state_idx.max().item())
                if lo < 0 or hi >= ns:
                    raise ValueError(f"state index range [{lo}, {hi}] outside {ns} states")
        elif n > ns:
            raise ValueError(f"{n} chunks for {ns} states")
        b = _lib.FdfsGpuBatch(data.data_ptr(), offsets.data_ptr(), sizes.data_ptr(), n)
        self._rc(self._L.fdfs_gpu_update_batch(self._h, ctypes.byref(b), _ptr(state_idx), method,
                                               states.data_ptr(), _stream_handle(stream)),
                 "fdfs_gpu_update_batch")

    def final_batch(self, states: torch.Tensor, method: int = SIG_HASH,
                    state_idx: torch.Tensor | None = None, want_sig: bool = True,
                    want_codes: bool = False, stream=None):
        """CRC32_FINAL + FINISH_HASH_CODES4 / my_md5_final + the 24-byte
        signature of each state (or of states[state_idx]): (crc int32[n],
        sig uint8[n,24] | None, codes int32[n,4] | None), as sig_batch."""
        ns = self._check_states(states)
        n = ns
        if state_idx is not None:
            _check_dev(state_idx, "state_idx", torch.int32)
            n = state_idx.numel()
        dev = states.device
        crc = torch.empty(n, dtype=torch.int32, device=dev)
        sig = torch.empty((n, 24), dtype=torch.uint8, device=dev) \
            if (want_sig and method != SIG_CRC_ONLY) else None
        codes = torch.empty((n, 4), dtype=torch.int32, device=dev) \
            if (want_codes and method != SIG_CRC_ONLY) else None
        self._rc(self._L.fdfs_gpu_final_batch(self._h, states.data_ptr(), _ptr(state_idx), n, method,
                                              crc.data_ptr(), _ptr(sig), _ptr(codes),
                                              _stream_handle(stream)), "fdfs_gpu_final_batch")
        return crc, sig, codes

    def crc_combine(self, crc_a: torch.Tensor, crc_b: torch.Tensor, len_b: torch.Tensor, stream=None):
        """crc32_combine over GF(2): the running CRC32_ex value of A||B from
        crc_a = CRC32_ex(A, init), crc_b = CRC32_ex(B, 0) and |B| (int64)."""
        _check_dev(crc_a, "crc_a", torch.int32)
        _check_dev(crc_b, "crc_b", torch.int32)
        _check_dev(len_b, "len_b", torch.int64)
        n = crc_a.numel()
        if crc_b.numel() != n or len_b.numel() != n:
            raise ValueError("crc_a, crc_b and len_b differ in length")
        out = torch.empty_like(crc_a)
        self._rc(self._L.fdfs_gpu_crc_combine(self._h, crc_a.data_ptr(), crc_b.data_ptr(),
                                              len_b.data_ptr(), n, out.data_ptr(),
                                              _stream_handle(stream)), "fdfs_gpu_crc_combine")
        return out

    # ----------------------------------------------------------------- dedup
    def sig_batch_host(self, data, offsets, sizes, method: int = SIG_HASH, want_sig: bool = True,
                       want_codes: bool = False, chunk_bytes: int = 0):
        """fdfs_gpu_sig_batch_host: the batch in HOST memory (numpy arrays or
        CPU tensors; a pinned tensor copies at the full PCIe rate), streamed
        to the device in double-buffered windows and hashed there.  Returns
        numpy (crc uint32[n], sig uint8[n,24] | None, codes int32[n,4] | None)."""
        import numpy as np

        def host(a, dt):
            if isinstance(a, torch.Tensor):
                if a.is_cuda:
                    raise ValueError("sig_batch_host takes host buffers; use sig_batch for device ones")
                a = a.numpy()
            return np.ascontiguousarray(a, dtype=dt)
        data_h = host(data, np.uint8)
        offs_h = host(offsets, np.uint64)
        sizes_h = host(sizes, np.uint64)
        n = offs_h.size
        if sizes_h.size != n:
            raise ValueError("offsets and sizes differ in length")
        crc = np.zeros(n, np.uint32)
        sig = np.zeros((n, 24), np.uint8) if (want_sig and method != SIG_CRC_ONLY) else None
        codes = np.zeros((n, 4), np.int32) if (want_codes and method != SIG_CRC_ONLY) else None
        b = _lib.FdfsGpuBatch(data_h.ctypes.data, offs_h.ctypes.data, sizes_h.ctypes.data, n)
        self._rc(self._L.fdfs_gpu_sig_batch_host(self._h, ctypes.byref(b), method, crc.ctypes.data,
                                                 None if sig is None else sig.ctypes.data,
                                                 None if codes is None else codes.ctypes.data,
                                                 chunk_bytes), "fdfs_gpu_sig_batch_host")
        return crc, sig, codes

    def dedup(self, sig: torch.Tensor, gidx: torch.Tensor | None = None, stream=None):
        """rep int64[n] (first ingest index of the class), ref int32[n] (class size)."""
        n = _check_sig(sig, gidx)
        rep = torch.empty(n, dtype=torch.int64, device=sig.device)
        ref = torch.empty(n, dtype=torch.int32, device=sig.device)
        self._rc(self._L.fdfs_gpu_dedup(self._h, sig.data_ptr(), _ptr(gidx), n, rep.data_ptr(),
                                        ref.data_ptr(), _stream_handle(stream)), "fdfs_gpu_dedup")
        return rep, ref

    def dedup_packed(self, sig: torch.Tensor, gidx: torch.Tensor | None = None, stream=None):
        """fdfs_gpu_dedup_packed: int64[n, 2] with [:, 0] = rep and [:, 1] =
        ref (the 16-byte fdfs_gpu_dedup_answer records; ref's reserved high
        word is 0)."""
        n = _check_sig(sig, gidx)
        out = torch.empty((n, 2), dtype=torch.int64, device=sig.device)
        self._rc(self._L.fdfs_gpu_dedup_packed(self._h, sig.data_ptr(), _ptr(gidx), n, out.data_ptr(),
                                               _stream_handle(stream)), "fdfs_gpu_dedup_packed")
        return out

    def dedup_global(self, comm: "Comm", sig: torch.Tensor, gidx: torch.Tensor | None, stream=None):
        """fdfs_gpu_dedup_global: this rank's share of a multi-GPU ingest
        grouped across every rank of `comm` over RCCL; (rep int64[n], ref
        int32[n]) for this rank's records (collective: all ranks call)."""
        n = _check_sig(sig, gidx)
        if gidx is None and comm.world > 1 and n:
            raise ValueError("dedup_global over more than one rank needs each record's global ingest index")
        rep = torch.empty(n, dtype=torch.int64, device=sig.device)
        ref = torch.empty(n, dtype=torch.int32, device=sig.device)
        self._rc(self._L.fdfs_gpu_dedup_global(self._h, comm.handle, sig.data_ptr(), _ptr(gidx), n,
                                               rep.data_ptr(), ref.data_ptr(), _stream_handle(stream)),
                 "fdfs_gpu_dedup_global")
        return rep, ref

    def dedup_global_local(self, sigs: list, gidxs: list, stream=None):
        """fdfs_gpu_dedup_global_local: len(sigs) VIRTUAL ranks on this
        device, rank p holding sigs[p] (uint8[n_p, 24]) with global ingest
        indices gidxs[p] (int64[n_p]); the RCCL form's bucket, exchange plan,
        group and answer routing with every segment moved by a device copy.
        Returns [(rep int64[n_p], ref int32[n_p])] per rank (synchronous)."""
        nr = len(sigs)
        if not 1 <= nr <= 64 or len(gidxs) != nr:
            raise ValueError("1..64 ranks, one gidx tensor per rank")
        outs = []
        for s, g in zip(sigs, gidxs):
            n = _check_sig(s, g)
            if g is None and nr > 1 and n:
                raise ValueError("more than one rank needs each record's global ingest index")
            outs.append((torch.empty(n, dtype=torch.int64, device=s.device),
                         torch.empty(n, dtype=torch.int32, device=s.device)))
        P = ctypes.c_void_p * nr
        U = ctypes.c_uint64 * nr
        self._rc(self._L.fdfs_gpu_dedup_global_local(
            self._h, nr, P(*[s.data_ptr() for s in sigs]),
            P(*[None if g is None else g.data_ptr() for g in gidxs]), U(*[s.shape[0] for s in sigs]),
            P(*[o[0].data_ptr() for o in outs]), P(*[o[1].data_ptr() for o in outs]),
            _stream_handle(stream)), "fdfs_gpu_dedup_global_local")
        return outs

    def dedup_global_stats(self) -> dict:
        """fdfs_gpu_dedup_global_stats: bytes the last dedup_global(_local)
        call moved between ranks (this rank's sends; every virtual rank's for
        _local): 32-byte rows to the other owners, 16-byte answer records
        back."""
        rb, ab = ctypes.c_uint64(), ctypes.c_uint64()
        self._rc(self._L.fdfs_gpu_dedup_global_stats(self._h, ctypes.byref(rb), ctypes.byref(ab)),
                 "fdfs_gpu_dedup_global_stats")
        return {"row_bytes": rb.value, "answer_bytes": ab.value}

    # ------------------------------------------------- split-file CRC (N GPUs)
    @staticmethod
    def _check_pieces(data, offsets, sizes, piece_file, piece_start):
        n = _check_batch(data, offsets, sizes, True)
        for t, name in ((piece_file, "piece_file"), (piece_start, "piece_start")):
            _check_dev(t, name, torch.int64)
            if t.numel() != n:
                raise ValueError(f"{name} must have one entry per piece")
        return n

    def crc_batch_global(self, comm: "Comm", data: torch.Tensor, offsets: torch.Tensor, sizes: torch.Tensor,
                         piece_file: torch.Tensor, piece_start: torch.Tensor, file_size: torch.Tensor,
                         stream=None) -> torch.Tensor:
        """fdfs_gpu_crc_batch_global: this rank holds pieces (bytes
        data[offsets[i] : + sizes[i]] = file piece_file[i] from byte
        piece_start[i]); file_size (int64[nfiles], equal on every rank).
        Returns the CRC32 of every file (int32 bit patterns) on every rank
        (collective: all ranks call)."""
        n = self._check_pieces(data, offsets, sizes, piece_file, piece_start)
        _check_dev(file_size, "file_size", torch.int64)
        nf = file_size.numel()
        crc = torch.empty(nf, dtype=torch.int32, device=file_size.device)
        b = _lib.FdfsGpuBatch(data.data_ptr(), offsets.data_ptr(), sizes.data_ptr(), n)
        self._rc(self._L.fdfs_gpu_crc_batch_global(self._h, comm.handle, ctypes.byref(b), piece_file.data_ptr(),
                                                   piece_start.data_ptr(), file_size.data_ptr(), nf,
                                                   crc.data_ptr(), _stream_handle(stream)),
                 "fdfs_gpu_crc_batch_global")
        return crc

    def crc_batch_global_local(self, ranks: list, file_size: torch.Tensor, stream=None) -> torch.Tensor:
        """fdfs_gpu_crc_batch_global_local: len(ranks) VIRTUAL ranks on this
        device, ranks[p] = (data, offsets, sizes, piece_file, piece_start) as
        crc_batch_global takes them.  Returns the files' CRC32s (synchronous)."""
        nr = len(ranks)
        if not 1 <= nr <= 64:
            raise ValueError("1..64 ranks")
        _check_dev(file_size, "file_size", torch.int64)
        nf = file_size.numel()
        B = _lib.FdfsGpuBatch * nr
        P = ctypes.c_void_p * nr
        bs = B(*[_lib.FdfsGpuBatch(d.data_ptr(), o.data_ptr(), s.data_ptr(), self._check_pieces(d, o, s, pf, ps))
                 for d, o, s, pf, ps in ranks])
        crc = torch.empty(nf, dtype=torch.int32, device=file_size.device)
        self._rc(self._L.fdfs_gpu_crc_batch_global_local(
            self._h, nr, bs, P(*[r[3].data_ptr() for r in ranks]), P(*[r[4].data_ptr() for r in ranks]),
            file_size.data_ptr(), nf, crc.data_ptr(), _stream_handle(stream)), "fdfs_gpu_crc_batch_global_local")
        return crc

    def dedup_bucket(self, sig: torch.Tensor, gidx: torch.Tensor | None, nranks: int, stream=None):
        """Pack {sig, gidx} rows by owner rank: (rows uint8[n,32], counts int64[nranks], row_of int64[n])."""
        n = _check_sig(sig, gidx)
        if not 1 <= nranks <= 64:
            raise ValueError("nranks must be in [1, 64]")
        rows = torch.empty((n, 32), dtype=torch.uint8, device=sig.device)
        counts = torch.empty(nranks, dtype=torch.int64, device=sig.device)
        row_of = torch.empty(n, dtype=torch.int64, device=sig.device)
        self._rc(self._L.fdfs_gpu_dedup_bucket(self._h, sig.data_ptr(), _ptr(gidx), n, nranks,
                                               rows.data_ptr(), counts.data_ptr(), row_of.data_ptr(),
                                               _stream_handle(stream)), "fdfs_gpu_dedup_bucket")
        return rows, counts, row_of

    def dedup_group(self, rows: torch.Tensor, stream=None):
        """Owner-side grouping of 32-byte rows: (rep int64[m], ref int32[m])."""
        m = _check_sig(rows, None, 32)
        rep = torch.empty(m, dtype=torch.int64, device=rows.device)
        ref = torch.empty(m, dtype=torch.int32, device=rows.device)
        self._rc(self._L.fdfs_gpu_dedup_group(self._h, rows.data_ptr(), m, rep.data_ptr(),
                                              ref.data_ptr(), _stream_handle(stream)),
                 "fdfs_gpu_dedup_group")
        return rep, ref

    # ------------------------------------------- formats, routing, scrub
    def file_ids(self, server_id: int, crc32: torch.Tensor, file_size: torch.Tensor,
                 timestamp: torch.Tensor, rnd: torch.Tensor, subdir_count: int = 256,
                 stream=None):
        """storage_gen_filename for a batch: (names uint8[n,27], sub_path uint8[n,2]).

        crc32 int32[n] (uint32 bit pattern), file_size int64[n], timestamp
        int32[n], rnd int32[n] (the rand() draws of COMBINE_RAND_FILE_SIZE)."""
        for t, nm, dt in ((crc32, "crc32", torch.int32), (file_size, "file_size", torch.int64),
                          (timestamp, "timestamp", torch.int32), (rnd, "rnd", torch.int32)):
            _check_dev(t, nm, dt)
        n = crc32.numel()
        names = torch.empty((n, 27), dtype=torch.uint8, device=crc32.device)
        sub = torch.empty((n, 2), dtype=torch.uint8, device=crc32.device)
        self._rc(self._L.fdfs_gpu_file_ids(self._h, server_id & 0xFFFFFFFF, crc32.data_ptr(),
                                           file_size.data_ptr(), timestamp.data_ptr(),
                                           rnd.data_ptr(), n, subdir_count, names.data_ptr(),
                                           sub.data_ptr(), _stream_handle(stream)),
                 "fdfs_gpu_file_ids")
        return names, sub

    def parse_file_ids(self, names: torch.Tensor, stream=None):
        """Decode 27-char names: (server_id int32, timestamp int32, file_size int64, crc32 int32)."""
        _check_dev(names, "names", torch.uint8)
        n = names.numel() // 27
        dev = names.device
        sid = torch.empty(n, dtype=torch.int32, device=dev)
        ts = torch.empty(n, dtype=torch.int32, device=dev)
        sz = torch.empty(n, dtype=torch.int64, device=dev)
        crc = torch.empty(n, dtype=torch.int32, device=dev)
        self._rc(self._L.fdfs_gpu_parse_file_ids(self._h, names.data_ptr(), n, sid.data_ptr(),
                                                 ts.data_ptr(), sz.data_ptr(), crc.data_ptr(),
                                                 _stream_handle(stream)),
                 "fdfs_gpu_parse_file_ids")
        return sid, ts, sz, crc

    def trunk_pack(self, file_type, alloc_size, file_size, crc32, mtime, ext, stream=None):
        """24-byte trunk headers uint8[n,24] (ext: uint8[n,7])."""
        for t, nm, dt in ((file_type, "file_type", torch.uint8), (alloc_size, "alloc_size", torch.int32),
                          (file_size, "file_size", torch.int32), (crc32, "crc32", torch.int32),
                          (mtime, "mtime", torch.int32), (ext, "ext", torch.uint8)):
            _check_dev(t, nm, dt)
        n = crc32.numel()
        hdr = torch.empty((n, 24), dtype=torch.uint8, device=crc32.device)
        self._rc(self._L.fdfs_gpu_trunk_pack(self._h, file_type.data_ptr(), alloc_size.data_ptr(),
                                             file_size.data_ptr(), crc32.data_ptr(), mtime.data_ptr(),
                                             ext.data_ptr(), n, hdr.data_ptr(),
                                             _stream_handle(stream)), "fdfs_gpu_trunk_pack")
        return hdr

    def trunk_unpack(self, hdr: torch.Tensor, stream=None):
        """(file_type u8, alloc_size i32, file_size i32, crc32 i32, mtime i32, ext u8[n,7])."""
        _check_dev(hdr, "hdr", torch.uint8)
        n = hdr.numel() // 24
        dev = hdr.device
        out = (torch.empty(n, dtype=torch.uint8, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
               torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
               torch.empty(n, dtype=torch.int32, device=dev), torch.empty((n, 7), dtype=torch.uint8, device=dev))
        self._rc(self._L.fdfs_gpu_trunk_unpack(self._h, hdr.data_ptr(), n, *[t.data_ptr() for t in out],
                                               _stream_handle(stream)), "fdfs_gpu_trunk_unpack")
        return out

    def fdht_route(self, sig: torch.Tensor, namespace: bytes, group_count: int,
                   servers_per_group: torch.Tensor | None = None, stream=None):
        """FastDHT routing of (namespace, sig, "fid") keys:
        (key_hash int32[n], group int32[n], server int32[n], order int64[n], group_start int64[G+1])."""
        _check_dev(sig, "sig", torch.uint8)
        if servers_per_group is not None:
            _check_dev(servers_per_group, "servers_per_group", torch.int32)
        n = sig.numel() // 24
        dev = sig.device
        kh = torch.empty(n, dtype=torch.int32, device=dev)
        grp = torch.empty(n, dtype=torch.int32, device=dev)
        srv = torch.empty(n, dtype=torch.int32, device=dev)
        order = torch.empty(n, dtype=torch.int64, device=dev)
        start = torch.empty(group_count + 1, dtype=torch.int64, device=dev)
        self._rc(self._L.fdfs_gpu_fdht_route(self._h, sig.data_ptr(), n, namespace, len(namespace),
                                             group_count, _ptr(servers_per_group), kh.data_ptr(),
                                             grp.data_ptr(), srv.data_ptr(), order.data_ptr(),
                                             start.data_ptr(), _stream_handle(stream)),
                 "fdfs_gpu_fdht_route")
        return kh, grp, srv, order, start

    def fdht_route_keys(self, keys: torch.Tensor, namespace: bytes, group_count: int,
                        key_len: torch.Tensor | None = None,
                        servers_per_group: torch.Tensor | None = None, stream=None):
        """FastDHT routing of (namespace, obj_id) keys given as records
        uint8[n, stride] (stride % 4 == 0, <= 128), the first key_len[i]
        (int32[n], default stride) bytes of each hashed.  Same outputs as
        fdht_route."""
        _check_dev(keys, "keys", torch.uint8)
        if keys.dim() != 2:
            raise ValueError("keys must be uint8[n, stride]")
        if key_len is not None:
            _check_dev(key_len, "key_len", torch.int32)
        if servers_per_group is not None:
            _check_dev(servers_per_group, "servers_per_group", torch.int32)
        n, stride = keys.shape
        dev = keys.device
        kh = torch.empty(n, dtype=torch.int32, device=dev)
        grp = torch.empty(n, dtype=torch.int32, device=dev)
        srv = torch.empty(n, dtype=torch.int32, device=dev)
        order = torch.empty(n, dtype=torch.int64, device=dev)
        start = torch.empty(group_count + 1, dtype=torch.int64, device=dev)
        self._rc(self._L.fdfs_gpu_fdht_route_keys(self._h, keys.data_ptr(), stride, _ptr(key_len), n,
                                                  namespace, len(namespace), group_count,
                                                  _ptr(servers_per_group), kh.data_ptr(),
                                                  grp.data_ptr(), srv.data_ptr(), order.data_ptr(),
                                                  start.data_ptr(), _stream_handle(stream)),
                 "fdfs_gpu_fdht_route_keys")
        return kh, grp, srv, order, start

    def scrub(self, data: torch.Tensor, offsets: torch.Tensor, sizes: torch.Tensor,
              expected_crc: torch.Tensor, stream=None):
        """Recompute every file's CRC32 and compare: (crc int32[n], bad uint8[n], nbad int32[1])."""
        n = _check_batch(data, offsets, sizes, True)
        _check_dev(expected_crc, "expected_crc", torch.int32)
        if expected_crc.numel() != n:
            raise ValueError("one expected CRC per file")
        dev = data.device
        crc = torch.empty(n, dtype=torch.int32, device=dev)
        bad = torch.empty(n, dtype=torch.uint8, device=dev)
        nbad = torch.zeros(1, dtype=torch.int32, device=dev)
        b = _lib.FdfsGpuBatch(data.data_ptr(), offsets.data_ptr(), sizes.data_ptr(), n)
        self._rc(self._L.fdfs_gpu_scrub(self._h, ctypes.byref(b), expected_crc.data_ptr(),
                                        crc.data_ptr(), bad.data_ptr(), nbad.data_ptr(),
                                        _stream_handle(stream)), "fdfs_gpu_scrub")
        return crc, bad, nbad


class Comm:
    """An RCCL communicator for fdfs_gpu_dedup_global, set up through
    torch.distributed (which carries rank 0's 128-byte id to the others).
    Collective: every rank of `group` constructs it together."""

    def __init__(self, ctx: Context, group=None):
        import torch.distributed as dist
        L = ctx._L
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        buf = ctypes.create_string_buffer(_lib.COMM_ID_BYTES)
        # the id travels with a status byte, so a failure on rank 0 is every
        # rank's error instead of leaving the others in the broadcast
        ok = not (rank == 0 and L.fdfs_gpu_comm_unique_id(buf))
        backend = dist.get_backend(group)
        dev = torch.device("cuda", ctx.device) if backend == "nccl" else torch.device("cpu")
        t = torch.frombuffer(bytearray(buf.raw + bytes([ok])), dtype=torch.uint8).to(dev)
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        raw = bytes(t.cpu().numpy().tobytes())
        if not raw[-1]:
            raise FdfsGpuError(errno.EIO, "fdfs_gpu_comm_unique_id (rank 0)")
        uid = raw[:-1]
        h = ctypes.c_void_p()
        ctx._rc(L.fdfs_gpu_comm_init(ctx._h, uid, world, rank, ctypes.byref(h)), "fdfs_gpu_comm_init")
        self._L, self.handle, self.rank, self.world = L, h, rank, world

    def close(self):
        if getattr(self, "handle", None):
            self._L.fdfs_gpu_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DedupIndex:
    """fdfs_gpu_index: the FastDHT "fid" / "ref" state of an ingest stream,
    kept in HBM across batches (include/fdfs_gpu.h)."""

    def __init__(self, ctx: Context, max_classes: int):
        h = ctypes.c_void_p()
        ctx._rc(ctx._L.fdfs_gpu_index_create(ctx._h, max_classes, ctypes.byref(h)), "fdfs_gpu_index_create")
        self.ctx, self._h = ctx, h

    def ingest(self, sig: torch.Tensor, gidx: torch.Tensor | None = None, stream=None):
        """Next batch of the stream: (rep int64[n], ref int32[n])."""
        n = _check_sig(sig, gidx)
        rep = torch.empty(n, dtype=torch.int64, device=sig.device)
        ref = torch.empty(n, dtype=torch.int32, device=sig.device)
        c = self.ctx
        c._rc(c._L.fdfs_gpu_index_ingest(c._h, self._h, sig.data_ptr(), _ptr(gidx), n, rep.data_ptr(),
                                         ref.data_ptr(), _stream_handle(stream)), "fdfs_gpu_index_ingest")
        return rep, ref

    def stats(self) -> dict:
        cl, rec, un = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        rc = self.ctx._L.fdfs_gpu_index_stats(self._h, ctypes.byref(cl), ctypes.byref(rec), ctypes.byref(un))
        if rc:
            raise FdfsGpuError(rc, "fdfs_gpu_index_stats")
        sl = ctypes.c_uint64()
        rc = self.ctx._L.fdfs_gpu_index_slots(self._h, ctypes.byref(sl))
        if rc:
            raise FdfsGpuError(rc, "fdfs_gpu_index_slots")
        return {"classes": cl.value, "records": rec.value, "unplaced": un.value, "slots": sl.value}

    def close(self):
        if getattr(self, "_h", None):
            self.ctx._L.fdfs_gpu_index_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
