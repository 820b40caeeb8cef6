"""Synthetic batch layouts for the BASELINE.json configs.

Sizes come from numpy with a fixed seed; contents are generated directly in
HBM (torch RNG on the device), so a 34.8 GB batch never crosses PCIe.
Files are packed back to back at `align`-byte boundaries; the gap bytes are
not part of any file.
"""
from __future__ import annotations

import numpy as np
import torch


def layout(sizes: np.ndarray, align: int = 16) -> tuple[np.ndarray, int]:
    """Offsets for files packed at `align` boundaries, and the buffer size."""
    sizes = np.asarray(sizes, dtype=np.int64)
    padded = (sizes + (align - 1)) // align * align if align > 1 else sizes
    offs = np.zeros(sizes.size, dtype=np.int64)
    if sizes.size > 1:
        offs[1:] = np.cumsum(padded)[:-1]
    total = int(padded.sum()) if sizes.size else 0
    return offs, total


def small_files_sizes(n: int, lo: int = 4096, hi: int = 65536, seed: int = 1) -> np.ndarray:
    """Config 2: n files of U[lo, hi] bytes (trunk_mgr-sized, 4-64 KB)."""
    return np.random.default_rng(seed).integers(lo, hi + 1, size=n, dtype=np.int64)


def photo_sizes(n: int, seed: int = 3) -> np.ndarray:
    """Config 3: n files of U[1 MiB, 4 MiB]."""
    return np.random.default_rng(seed).integers(1 << 20, (4 << 20) + 1, size=n, dtype=np.int64)


def fill_random(buf: torch.Tensor, seed: int) -> torch.Tensor:
    """Fill a uint8 device buffer with seeded random bytes, in place."""
    g = torch.Generator(device=buf.device)
    g.manual_seed(seed)
    words = buf.numel() // 8
    if words:
        buf[: words * 8].view(torch.int64).random_(generator=g)
    tail = buf.numel() - words * 8
    if tail:
        buf[words * 8:].random_(0, 256, generator=g)
    return buf


def device_batch(sizes: np.ndarray, seed: int, device, align: int = 16):
    """(data uint8, offsets int64, sizes int64) device tensors for a batch."""
    offs, total = layout(sizes, align)
    data = torch.empty(max(total, 1), dtype=torch.uint8, device=device)
    fill_random(data, seed)
    return (data, torch.from_numpy(offs).to(device),
            torch.from_numpy(np.asarray(sizes, dtype=np.int64)).to(device))


def dup_signatures(n: int, dup_frac: float = 0.1, seed: int = 5, device="cpu") -> torch.Tensor:
    """Config 5: n 24-byte signatures, (1-dup_frac)*n unique (random size field
    + 16 random bytes), the rest drawn uniformly from them, shuffled."""
    rng = np.random.default_rng(seed)
    nu = max(1, n - int(n * dup_frac))
    uniq = rng.integers(0, 256, size=(nu, 24), dtype=np.uint8)
    uniq[:, :5] = 0  # be64 file size < 2^24: a realistic size field
    pick = np.concatenate([np.arange(nu), rng.integers(0, nu, size=n - nu)])
    rng.shuffle(pick)
    return torch.from_numpy(uniq[pick]).to(device)


def c5_signatures(total: int, world: int = 1, rank: int = 0, dev="cuda"):
    """Config 5's signature set: `total` records, 10% duplicates drawn
    uniformly from the 90% unique ones (seed 5); every rank derives the same
    global set and takes its contiguous share.  Returns (sig, gidx)."""
    per = total // world
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    nu = total - total // 10
    uniq_idx = torch.randint(0, nu, (total - nu,), generator=g, device=dev)
    lo, hi = rank * per, (rank + 1) * per if rank < world - 1 else total
    idx = torch.arange(lo, hi, device=dev, dtype=torch.int64)
    src = torch.where(idx < nu, idx, uniq_idx[(idx - nu).clamp(min=0, max=max(total - nu - 1, 0))])
    # signature bytes = fixed mix of the unique id (deterministic, 16 random-looking bytes)
    sig = torch.zeros((hi - lo, 24), dtype=torch.uint8, device=dev)
    x = (src * (0x9E3779B97F4A7C15 - (1 << 64))) ^ 0x5DEECE66D
    for k in range(2):
        x = x ^ (x >> 31)
        x = x * 0x7FB5D329728EA185
        sig[:, 8 + 8 * k: 16 + 8 * k] = x.contiguous().view(torch.uint8).view(-1, 8)
    sig[:, 5:8] = (src % 251).to(torch.uint8).view(-1, 1)
    return sig, idx
