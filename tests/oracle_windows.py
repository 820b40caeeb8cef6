"""The C oracle over a whole device-resident batch (test infrastructure).

VERDICT r05 item 3: the driver's own batches (config 2's 1M files, config
3's 100K photos, the seeds bench.py uses on rank 0) are compared with the
oracle file by file, not sampled.  The batch is copied to the host in
windows of at most `window` bytes of whole files and each window is hashed by
oracle.dio_batch (storage/storage_dio.c:465-515 restated, 256 KiB chunks) on
the host threads this process may use."""
from __future__ import annotations

import os

import numpy as np


def host_threads() -> int:
    """The host CPUs this process may use: the affinity set, capped by the
    share the pool box advertises (OMP_NUM_THREADS; its affinity mask shows
    every CPU of the host)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(omp))) if omp.isdigit() and int(omp) > 0 else n


def whole_batch(oracle, data, offs: np.ndarray, sizes: np.ndarray, method: int, variant: int = 0,
                window: int = 4 << 30):
    """(crc uint32[n], sig uint8[n, 24]) of every file of a device batch."""
    offs = np.asarray(offs, np.int64)
    sizes = np.asarray(sizes, np.int64)
    n = sizes.size
    crc = np.empty(n, np.uint32)
    sig = np.empty((n, 24), np.uint8)
    ends = offs + sizes
    threads = host_threads()
    i = 0
    while i < n:
        j = max(int(np.searchsorted(ends, offs[i] + window, side="right")), i + 1)
        lo, hi = int(offs[i]), int(ends[i:j].max())
        host = data[lo:hi].cpu().numpy()
        c, s = oracle.dio_batch(host, (offs[i:j] - lo).astype(np.uint64), sizes[i:j].astype(np.uint64),
                                method, variant, nthreads=threads)
        crc[i:j] = c
        sig[i:j] = s
        del host
        i = j
    return crc, sig
