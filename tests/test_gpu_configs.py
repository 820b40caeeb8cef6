"""GPU parity at BASELINE.json's full configuration sizes:

* config 4: 1 GiB files and a file past 4 GiB (64-bit offsets, GF(2) powers
  up to 2^32), CRC only, both shift variants, 16-byte and byte alignment;
* config 3: the bench's 100K photo files (~262 GB resident), a sample from
  every size decile against the oracle and hashlib;
* config 5: the bench's own 100M-signature set on one GPU against the
  oracle's sequential-semantics dedup, and through the multi-GPU dedup's
  code at world 2, 3 and 8;
* signatures of the largest files: MD5 past 512 MiB (a 64-bit bit count)
  and of 1 GiB, one-shot and chunked; HASH of a file past 4 GiB.
"""
import hashlib

import numpy as np
import pytest
import torch

from fastdfs_amd import corpus as C

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctxs():
    import fastdfs_amd as F
    return {0: F.Context(0, unsigned_hash=False), 1: F.Context(0, unsigned_hash=True)}


def test_config4_gib_files(oracle, ctxs):
    """Two 1 GiB files and one of 4 GiB + 17 B (CRC only), at 16-byte and at
    odd byte alignment (the same bytes shifted), both variants."""
    torch.cuda.empty_cache()
    sizes = np.array([1 << 30, 1 << 30, (4 << 30) + 17], np.int64)
    offs16, total = C.layout(sizes, 16)
    data = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    C.fill_random(data, 44)
    host = data.cpu().numpy()
    want = {}
    for v in (0, 1):
        want[v], _ = oracle.dio_batch(host, offs16.astype(np.uint64), sizes.astype(np.uint64), 0, v,
                                      nthreads=3)
    del host
    shifted = torch.empty_like(data)
    shifted[7:] = data[:-7]  # every file at offset + 7: odd alignment, same bytes
    for v in (0, 1):
        for buf, offs in ((data, offs16), (shifted, offs16 + 7)):
            crc, _, _ = ctxs[v].sig_batch(buf, torch.from_numpy(offs).cuda(), torch.from_numpy(sizes).cuda(),
                                          method=0)
            torch.cuda.synchronize()
            assert np.array_equal(crc.cpu().numpy().view(np.uint32), want[v]), (v, offs[0] & 15)
    del data, shifted
    torch.cuda.empty_cache()


def test_config3_full_batch(oracle, ctxs):
    """Config 3 at its bench size, the batch bench.py hashes on rank 0: 100K
    files of U[1, 4] MiB (sizes seed 3, bytes seed 2: ~262 GB in HBM), CRC +
    MD5 signature.  Every file's CRC and 24-byte signature equal the oracle's
    (the whole batch in 4 GiB host windows on every host
    thread), the MD5 digests of 15 files from every size decile equal
    hashlib's, and every file's CRC equals the CRC-only path's."""
    from oracle_windows import whole_batch
    torch.cuda.empty_cache()
    n = 100_000
    sizes = C.photo_sizes(n, seed=3)
    data, offs_t, sizes_t = C.device_batch(sizes, seed=2, device="cuda:0")
    crc, sig, _ = ctxs[0].sig_batch(data, offs_t, sizes_t, method=2, check_bounds=False)
    torch.cuda.synchronize()
    crc_np, sig_np = crc.cpu().numpy().view(np.uint32), sig.cpu().numpy()
    offs = offs_t.cpu().numpy()
    ocrc, osig = whole_batch(oracle, data, offs, sizes, 2)
    bad = np.flatnonzero((crc_np != ocrc) | (sig_np != osig).any(axis=1))
    assert bad.size == 0, (bad.size, bad[:8], sizes[bad[:8]])
    order = np.argsort(sizes, kind="stable")
    rng = np.random.default_rng(33)
    picks = np.concatenate([rng.choice(d, 15, replace=False) for d in np.array_split(order, 10)]
                           + [order[:1], order[-1:]])
    for i in picks:
        d = data[int(offs[i]): int(offs[i] + sizes[i])].cpu().numpy()
        assert sig_np[i, 8:].tobytes() == hashlib.md5(d.tobytes()).digest(), i
        assert int.from_bytes(sig_np[i, :8].tobytes(), "big") == sizes[i]
    # every file's CRC (the pair kernel's loader lanes, or for the largest
    # files the CRC segment items its queue hands out after the MD5 chunks)
    # equals the segmented CRC-only path's
    crc0, _, _ = ctxs[0].sig_batch(data, offs_t, sizes_t, method=0, check_bounds=False)
    torch.cuda.synchronize()
    bad = np.flatnonzero(crc0.cpu().numpy().view(np.uint32) != crc_np)
    assert bad.size == 0, (bad.size, bad[:8], sizes[bad[:8]])
    del data, crc, sig, crc0
    torch.cuda.empty_cache()


def test_config1_upload_mix(oracle, ctxs):
    """Config 1 at its bench size, the batch bench.py's upload_mix line hashes
    on rank 0: test/test_upload.c:32-39's DEBUG mix of the gen_files sizes
    (65,560 files, 3.89 GB; sizes permuted with seed 1, bytes seed 2).  HASH:
    the ten 100 MB and fifty 10 MB files (>= kBigCrcMin) run their ELF chains
    on workgroups of their own, their CRC / simple / Time33 on the segmented
    kernels, the rest on the lanes; MD5: the wave pairs.  Every file's CRC and
    24-byte signature against the oracle (storage/storage_dio.c:465-515)."""
    from oracle_windows import whole_batch
    torch.cuda.empty_cache()
    mix = [(5 << 10, 50000), (50 << 10, 10000), (200 << 10, 5000), (1 << 20, 500), (10 << 20, 50),
           (100 << 20, 10)]
    sizes = np.concatenate([np.full(c, sz, np.int64) for sz, c in mix])
    sizes = sizes[np.random.default_rng(1).permutation(sizes.size)]
    data, offs_t, sizes_t = C.device_batch(sizes, seed=2, device="cuda:0")
    offs = offs_t.cpu().numpy()
    for method in (1, 2):
        crc, sig, _ = ctxs[0].sig_batch(data, offs_t, sizes_t, method=method, check_bounds=False)
        torch.cuda.synchronize()
        crc_np, sig_np = crc.cpu().numpy().view(np.uint32), sig.cpu().numpy()
        ocrc, osig = whole_batch(oracle, data, offs, sizes, method)
        bad = np.flatnonzero((crc_np != ocrc) | (sig_np != osig).any(axis=1))
        assert bad.size == 0, (method, bad.size, bad[:8], sizes[bad[:8]])
    del data, crc, sig
    torch.cuda.empty_cache()


C5_TOTAL = 100_000_000


@pytest.fixture(scope="module")
def c5_oracle(oracle):
    """The oracle's sequential-semantics answers for the bench's config-5
    set (computed once for the tests below)."""
    sig, _ = C.c5_signatures(C5_TOTAL, 1, 0, "cuda")
    sig_np = sig.cpu().numpy()
    del sig
    orep, oref = oracle.dedup(sig_np, nthreads=16)
    del sig_np
    return orep.astype(np.int64), oref.astype(np.int32)


def test_config5_bench_set(c5_oracle, ctxs):
    """The bench's config-5 set (100M signatures, 10 % duplicates) on one
    GPU: every record's class source and class size equal the oracle's, as
    rep/ref arrays and as packed records."""
    torch.cuda.empty_cache()
    orep, oref = c5_oracle
    sig, gidx = C.c5_signatures(C5_TOTAL, 1, 0, "cuda")
    rep, ref = ctxs[0].dedup(sig)
    torch.cuda.synchronize()
    assert np.array_equal(rep.cpu().numpy(), orep)
    assert np.array_equal(ref.cpu().numpy(), oref)
    del rep, ref
    out = ctxs[0].dedup_packed(sig).cpu().numpy()  # bench.py --answers packed
    del sig, gidx
    assert np.array_equal(out[:, 0], orep)
    assert np.array_equal(out[:, 1], oref.astype(np.int64))
    del out
    assert int(oref.max()) > 1 and (oref > 1).sum() > C5_TOTAL // 20
    torch.cuda.empty_cache()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_config5_dedup_global_ranks(c5_oracle, ctxs, world):
    """The multi-GPU dedup's own code (fdfs_gpu_dedup_global: bucket,
    announcement plan, exchange offsets, owner groups, answer routing) at
    world 2, 3 and 8 on the bench's 100M config-5 set, each rank's share
    exactly as bench.py --gpus N splits it (C.c5_signatures), the ranks
    virtual on this GPU with every (src, dst) segment a device copy where
    RCCL would send it: every rank's answers equal the oracle's over the
    concatenation."""
    torch.cuda.empty_cache()
    orep, oref = c5_oracle
    shares = [C.c5_signatures(C5_TOTAL, world, r, "cuda") for r in range(world)]
    outs = ctxs[0].dedup_global_local([s for s, _ in shares], [g for _, g in shares])
    for r, ((_, g), (rep, ref)) in enumerate(zip(shares, outs)):
        lo, hi = int(g[0]), int(g[-1]) + 1
        assert np.array_equal(rep.cpu().numpy(), orep[lo:hi]), (world, r)
        assert np.array_equal(ref.cpu().numpy(), oref[lo:hi]), (world, r)
    del shares, outs
    torch.cuda.empty_cache()


@pytest.mark.parametrize("size", [(512 << 20) + 13, 1 << 30])
def test_md5_big_files(oracle, ctxs, size):
    """MD5 signature (file_signature_method=md5, storage/storage_dio.c:480,
    512) of files whose bit count passes 2^32 (its high word non-zero,
    RFC 1321 3.2): one-shot, and through update_batch in 256 KiB (the
    daemon's buff_size) and 64 MiB chunks, against the oracle and hashlib."""
    torch.cuda.empty_cache()
    data = torch.empty(size + 64, dtype=torch.uint8, device="cuda")
    C.fill_random(data, size & 0xFFFF)
    host = data[:size].cpu().numpy()
    oc, osig, _ = oracle.dio_file(host, 2, 0)
    assert osig[8:] == hashlib.md5(host.tobytes()).digest()
    del host
    ctx = ctxs[0]
    offs = torch.tensor([0], dtype=torch.int64, device="cuda")
    crc, sig, _ = ctx.sig_batch(data, offs, torch.tensor([size], dtype=torch.int64, device="cuda"), method=2)
    torch.cuda.synchronize()
    assert int(crc.cpu().numpy().view(np.uint32)[0]) == oc
    assert sig.cpu().numpy()[0].tobytes() == osig
    for chunk in (256 << 10, 64 << 20):
        states = ctx.new_states(1)
        for p in range(0, size, chunk):
            c = min(chunk, size - p)
            ctx.update_batch(states, data, torch.tensor([p], dtype=torch.int64, device="cuda"),
                             torch.tensor([c], dtype=torch.int64, device="cuda"), method=2, check_bounds=False)
        crc, sig, _ = ctx.final_batch(states, method=2)
        torch.cuda.synchronize()
        assert int(crc.cpu().numpy().view(np.uint32)[0]) == oc, chunk
        assert sig.cpu().numpy()[0].tobytes() == osig, chunk
        bits = int(states.cpu().numpy()[0, 36:44].view(np.uint64)[0])
        assert bits == 8 * size
    del data
    torch.cuda.empty_cache()


def test_hash_file_past_4gib(oracle, ctxs):
    """HASH signature of a (4 GiB + 7 B) file: the ELF lane's 64-bit
    lengths, the big-file offload (segmented CRC + polynomial kernels) and
    the be64 size field, against the oracle (CRC32_ex + CALC_HASH_CODES4 in
    256 KiB chunks, storage/storage_dio.c:465-477)."""
    torch.cuda.empty_cache()
    size = (4 << 30) + 7
    data = torch.empty(size + 64, dtype=torch.uint8, device="cuda")
    C.fill_random(data, 4747)
    crc, sig, codes = ctxs[0].sig_batch(data, torch.tensor([0], dtype=torch.int64, device="cuda"),
                                        torch.tensor([size], dtype=torch.int64, device="cuda"), method=1,
                                        want_codes=True)
    torch.cuda.synchronize()
    host = data[:size].cpu().numpy()
    del data
    oc, osig, ocodes = oracle.dio_file(host, 1, 0)
    assert int(crc.cpu().numpy().view(np.uint32)[0]) == oc
    assert sig.cpu().numpy()[0].tobytes() == osig
    assert [int(x) for x in codes.cpu().numpy()[0]] == ocodes
    assert int.from_bytes(osig[:8], "big") == size
    torch.cuda.empty_cache()
