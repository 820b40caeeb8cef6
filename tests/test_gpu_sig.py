"""GPU parity: libfdfs_gpu's HIP kernels vs the CPU oracle, bit-exact.

Every comparison runs the product through the C ABI (fastdfs_amd.Context ->
libfdfs_gpu.so) and the checker through oracle/ (the C restatement of the
libfastcommon loops driven the way dio_write_file drives them).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

METHODS = (0, 1, 2)


@pytest.fixture(scope="module")
def ctxs():
    import fastdfs_amd as F
    if not torch.cuda.is_available():
        pytest.fail("gpu test collected without a GPU")
    return {0: F.Context(0, unsigned_hash=False), 1: F.Context(0, unsigned_hash=True)}


def _to_dev(buf, offs, sizes):
    dev = torch.device("cuda", 0)
    data = torch.from_numpy(np.ascontiguousarray(buf, dtype=np.uint8)).to(dev)
    if data.numel() == 0:
        data = torch.zeros(1, dtype=torch.uint8, device=dev)
    return (data, torch.from_numpy(np.asarray(offs, np.int64)).to(dev),
            torch.from_numpy(np.asarray(sizes, np.int64)).to(dev))


def _gpu(ctx, dev_batch, method):
    crc, sig, codes = ctx.sig_batch(*dev_batch, method=method, want_codes=True)
    torch.cuda.synchronize()
    crc = crc.cpu().numpy().view(np.uint32)
    if method == 0:
        return crc, None, None
    return crc, sig.cpu().numpy(), codes.cpu().numpy()


def _check(oracle, ctx, variant, buf, offs, sizes, methods=METHODS, dev_batch=None):
    dev_batch = dev_batch or _to_dev(buf, offs, sizes)
    for m in methods:
        crc, sig, _ = _gpu(ctx, dev_batch, m)
        ocrc, osig = oracle.dio_batch(buf, offs, sizes, m, variant, nthreads=8)
        bad = np.nonzero(crc != ocrc)[0]
        assert bad.size == 0, (m, variant, bad[:10], sizes[bad[:10]])
        if m:
            badsig = np.nonzero(np.any(sig != osig, axis=1))[0]
            # which 4-byte fields differ: size hi/lo, then crc/elf/simple/time33 (HASH)
            fields = [int(np.any(sig[:, 4 * k:4 * k + 4] != osig[:, 4 * k:4 * k + 4], axis=1).sum())
                      for k in range(6)]
            assert badsig.size == 0, (m, variant, badsig[:10], sizes[badsig[:10]], fields)


def _packed(sizes, align, rng, slack=0):
    sizes = np.asarray(sizes, np.int64)
    offs = np.zeros(sizes.size, np.int64)
    pos = 0
    for i, s in enumerate(sizes):
        if align > 1:
            pos = (pos + align - 1) // align * align
        else:
            pos += int(rng.integers(0, 16))  # random misalignment
        offs[i] = pos
        pos += int(s)
    buf = rng.integers(0, 256, size=pos + slack, dtype=np.uint8)
    return buf, offs, sizes


EDGE = [0, 1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 31, 32, 33, 55, 56, 57, 63, 64, 65, 127, 128, 255,
        256, 1023, 1024, 4031, 4032, 4095, 4096, 4097, 4111, 8191, 65535, 65536, 65537, 65552,
        131071, 131072, 131073, 200003, (1 << 20) - 1, 1 << 20, (1 << 20) + 5]


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("align", [16, 1])
def test_edge_sizes(oracle, ctxs, variant, align):
    rng = np.random.default_rng(100 + variant * 2 + (align == 1))
    buf, offs, sizes = _packed(EDGE, align, rng)
    _check(oracle, ctxs[variant], variant, buf, offs, sizes)


@pytest.mark.parametrize("variant", [0, 1])
def test_gen_files_corpus(oracle, ctxs, corpus, kat, variant):
    """Config 1: test/gen_files.c corpus (5K..100M), all methods."""
    buf, offs, sizes = corpus
    dev_batch = _to_dev(buf, offs, sizes)
    ctx = ctxs[variant]
    crc, _, _ = _gpu(ctx, dev_batch, 0)
    key = "crc_signed" if variant == 0 else "crc_unsigned"
    assert ["%08X" % c for c in crc] == kat["corpus"][key]
    crc1, sig1, codes1 = _gpu(ctx, dev_batch, 1)
    assert np.array_equal(crc1, crc)
    assert ["%08X" % (int(c) & 0xFFFFFFFF) for c in codes1[:, 2]] == kat["corpus"]["simple"]
    assert ["%08X" % (int(c) & 0xFFFFFFFF) for c in codes1[:, 3]] == kat["corpus"]["time33"]
    elf = kat["corpus"]["elf_signed" if variant == 0 else "elf_unsigned"]
    for i, v in elf.items():
        assert "%08X" % (int(codes1[int(i), 1]) & 0xFFFFFFFF) == v
    crc2, sig2, _ = _gpu(ctx, dev_batch, 2)
    assert np.array_equal(crc2, crc)
    assert [bytes(s[8:]).hex() for s in sig2] == kat["corpus"]["md5"]
    for i in range(6):
        assert int.from_bytes(bytes(sig1[i, :8]), "big") == int(sizes[i])
    _, osig1 = oracle.dio_batch(buf, offs, sizes, 1, variant, nthreads=6)
    assert np.array_equal(sig1, osig1)


@pytest.mark.parametrize("variant", [0, 1])
def test_small_files_random(oracle, ctxs, variant):
    """Config-2-shaped files (4-64 KiB) at 16-B and byte alignment."""
    rng = np.random.default_rng(7 + variant)
    sizes = rng.integers(4096, 65537, size=6000)
    for align in (16, 1):
        buf, offs, sz = _packed(sizes, align, rng)
        _check(oracle, ctxs[variant], variant, buf, offs, sz)


def test_tiny_and_mixed_batch(oracle, ctxs):
    """Mixed sizes in one batch (lane sort + multi-segment files together)."""
    rng = np.random.default_rng(11)
    sizes = np.concatenate([rng.integers(0, 64, 500), rng.integers(64, 70000, 500),
                            rng.integers(70000, 600000, 40)])
    rng.shuffle(sizes)
    buf, offs, sz = _packed(sizes, 1, rng)
    _check(oracle, ctxs[0], 0, buf, offs, sz)


@pytest.mark.parametrize("n", [1, 4095, 4096])
def test_crc_plan_small_boundary(oracle, ctxs, n):
    """CRC only: batches below 4,096 files are planned by one workgroup
    (plan_small_kernel), larger ones by the three-kernel scan; both sides of
    the boundary, and a batch of one file spanning many segments."""
    rng = np.random.default_rng(61 + n)
    sizes = rng.integers(0, 150_000, n) if n > 1 else np.array([(5 << 20) + 3])
    buf, offs, sz = _packed(sizes, 1, rng)
    _check(oracle, ctxs[0], 0, buf, offs, sz, methods=(0,))


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("n", [300, 4200])
def test_crc_fold_split(oracle, ctxs, variant, n):
    """CRC only, one batch across the kernel split (kFoldMinBytes = 96 KiB:
    smaller files take the table kernel, the others the sparse fold): sizes
    on both sides of and at the threshold, runs shorter and longer than the
    fold relation's degree (575 / 300 vectors) and than its ring (1024
    vectors), byte-aligned starts, both plans (one workgroup below 4,096
    files, the two scans above), both shift variants."""
    rng = np.random.default_rng(71 + variant + n)
    edge = [0, 1, 15, 16, 17, (96 << 10) - 1, 96 << 10, (96 << 10) + 1, (96 << 10) + 4000,
            16 * 575, 16 * 575 + 1, 16 * 1088 + 5, (1 << 20) + 7, (3 << 20) + 11]
    sizes = np.concatenate([edge, rng.integers(0, 300_000, n - len(edge) - 8),
                            rng.integers(96 << 10, 2 << 20, 8)])
    rng.shuffle(sizes)
    buf, offs, sz = _packed(sizes, 1, rng)
    _check(oracle, ctxs[variant], variant, buf, offs, sz, methods=(0,))


@pytest.mark.parametrize("variant", [0, 1])
def test_large_file_segmented(oracle, ctxs, variant):
    """Config 4 shape: large files split into 128 KiB segments + GF(2) combine."""
    rng = np.random.default_rng(21)
    sizes = np.array([(256 << 20) + 12345, 64 << 20, (3 << 16) + 1, 7 << 20], np.int64)
    buf, offs, sz = _packed(sizes, 1, rng)
    _check(oracle, ctxs[variant], variant, buf, offs, sz, methods=(0,))


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("align", [16, 1])
@pytest.mark.parametrize("pad", [False, True])
def test_big_file_crc_offload(oracle, ctxs, variant, align, pad):
    """HASH method with whole waves of files >= 4 MiB: their CRC, simple_hash
    and Time33 come from the segmented kernels and are patched into crc_out,
    the signature and the codes; files at and just below 4 MiB, a mixed wave
    and small files in the same batch.  pad=True adds 70,000 tiny files, so
    the batch has more files than one wave per SIMD and takes the fixed
    threshold kBigCrcMin = 4 MiB; without it big_plan_kernel chooses T."""
    rng = np.random.default_rng(31 + variant * 2 + (align == 1) + 4 * pad)
    big = rng.integers(4 << 20, (4 << 20) + 300_000, size=130)
    sizes = np.concatenate([big, [4 << 20, (4 << 20) - 1, (4 << 20) + 1, 9 << 20],
                            rng.integers(0, 70000, 200)])
    if pad:
        sizes = np.concatenate([sizes, rng.integers(0, 100, 70_000)])
    rng.shuffle(sizes)
    buf, offs, sz = _packed(sizes, align, rng)
    dev_batch = _to_dev(buf, offs, sz)
    _check(oracle, ctxs[variant], variant, buf, offs, sz, methods=(1,), dev_batch=dev_batch)
    crc, _, codes = _gpu(ctxs[variant], dev_batch, 1)
    assert np.array_equal(codes[:, 0].view(np.uint32), crc)
    crc0, _, _ = _gpu(ctxs[variant], dev_batch, 0)
    assert np.array_equal(crc0, crc)


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("top", [13, 17, 21, 23])
def test_adaptive_offload_threshold(oracle, ctxs, variant, top):
    """Small batches (one wave per SIMD or less) offload the CRC (HASH: and
    the polynomials) of the files >= T with T = 2^k chosen from the size
    histogram (big_plan_kernel): sizes 2^k - 1, 2^k, 2^k + 1 for every
    candidate k up to `top`, plus a few random files, put a file on each
    side of whichever T it picks.  HASH and MD5."""
    rng = np.random.default_rng(41 + variant + 2 * top)
    ks = range(12, top + 1)
    sizes = np.concatenate([[(1 << k) + d for k in ks for d in (-1, 0, 1)],
                            rng.integers(0, 1 << top, 20), [0, 1, 4095]])
    rng.shuffle(sizes)
    buf, offs, sz = _packed(sizes, 1, rng)
    _check(oracle, ctxs[variant], variant, buf, offs, sz, methods=(1, 2))


@pytest.mark.parametrize("variant", [0, 1])
def test_chain_workgroups(oracle, ctxs, variant):
    """The serial chain of a small batch's few big files on workgroups of
    their own: MD5 (md5_chain_wg: a helper wave makes each step's K + m sum
    in LDS, two slots of 32 blocks) and ELFHash_ex (elf_chain_wg: the bytes
    one per dword in LDS, two slots of 2 KiB), the CRC / simple / Time33 of
    those files from the segmented kernels: block counts odd, a slot boundary
    +- 1, byte-aligned starts, tails of 0-63 bytes, beside small files on the
    lanes.  Reference: storage/storage_dio.c:465-512 (CALC_HASH_CODES4,
    my_md5_update / my_md5_final)."""
    rng = np.random.default_rng(71 + variant)
    big = [(4 << 20) + 4095, (3 << 20) + 65, (2 << 20) - 1, 12_345_678, (2 << 20) + 2048 - 64,
           (2 << 20) + 2048 + 64, 6 << 20]
    sizes = np.concatenate([big, rng.integers(0, 5000, 60), [0, 63, 64, 65]]).astype(np.int64)
    rng.shuffle(sizes)
    buf, offs, sz = _packed(sizes, 1, rng)
    _check(oracle, ctxs[variant], variant, buf, offs, sz, methods=(1, 2))


@pytest.mark.parametrize("variant", [0, 1])
def test_chain_waves(oracle, ctxs, variant):
    """More big files than CUs, at most one per SIMD: each big file's MD5
    chain on a wave of its own that feeds its own LDS ring (md5_chain_wave,
    8-block slots loaded two slots ahead; HASH keeps these files' ELF chains
    on the lanes), byte-aligned starts, odd sizes, beside small files.
    Reference: storage/storage_dio.c:465-512."""
    rng = np.random.default_rng(81 + variant)
    sizes = np.concatenate([rng.integers(1 << 20, 2 << 20, 500), rng.integers(0, 5000, 300),
                            [(1 << 20) + 511, (1 << 20) + 512, (1 << 20) + 513]]).astype(np.int64)
    rng.shuffle(sizes)
    buf, offs, sz = _packed(sizes, 1, rng)
    _check(oracle, ctxs[variant], variant, buf, offs, sz, methods=(1, 2))


def test_crc_paths_agree_at_scale(oracle, ctxs):
    """Config 2 at full size, the batch bench.py hashes on rank 0 (1M files of
    U[4, 64] KiB, sizes seed 1, bytes seed 2, 16-byte aligned: ~34.8 GB in
    HBM): every file's CRC-only CRC (crc_lane_kernel + crc_seg_kernel) equals
    its HASH-path CRC, and every file's CRC and 24-byte HASH signature equal
    the oracle's (the whole batch, in 4 GiB host windows
    on every host thread, not a sample)."""
    from fastdfs_amd import corpus as C
    from oracle_windows import whole_batch
    n = 1_000_000
    sizes = C.small_files_sizes(n)
    data, offs_t, sizes_t = C.device_batch(sizes, seed=2, device="cuda:0")
    ctx = ctxs[0]
    crc0, _, _ = ctx.sig_batch(data, offs_t, sizes_t, method=0)
    crc1, sig1, _ = ctx.sig_batch(data, offs_t, sizes_t, method=1)
    torch.cuda.synchronize()
    assert torch.equal(crc0, crc1)
    ocrc, osig = whole_batch(oracle, data, offs_t.cpu().numpy(), sizes, 1)
    bad = np.flatnonzero(crc1.cpu().numpy().view(np.uint32) != ocrc)
    assert bad.size == 0, (bad.size, bad[:8])
    bad = np.flatnonzero((sig1.cpu().numpy() != osig).any(axis=1))
    assert bad.size == 0, (bad.size, bad[:8])
    del data
    torch.cuda.empty_cache()


@pytest.mark.parametrize("extra", [0, 1])
def test_offload_regime_boundary(oracle, ctxs, extra):
    """One wave per SIMD (lat_files = CUs x 4 x 64 files) is where the lane
    path switches from the threshold big_plan_kernel picks to the fixed one
    (HASH 4 MiB, MD5 no offload).  Batches of exactly lat_files and one more
    file, small files plus 4-6 MiB ones: the three methods' CRCs agree for
    every file, and a sample (every big file among it) matches the oracle."""
    from fastdfs_amd import corpus as C
    lat = torch.cuda.get_device_properties(0).multi_processor_count * 4 * 64
    n = lat + extra
    rng = np.random.default_rng(17 + extra)
    sizes = rng.integers(0, 65537, n)
    big = rng.choice(n, size=200, replace=False)
    sizes[big] = rng.integers(4 << 20, 6 << 20, 200)
    data, offs_t, sizes_t = C.device_batch(sizes, seed=9 + extra, device="cuda:0")
    ctx = ctxs[0]
    out = {m: ctx.sig_batch(data, offs_t, sizes_t, method=m) for m in (0, 1, 2)}
    torch.cuda.synchronize()
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][0], out[2][0])
    offs = offs_t.cpu().numpy()
    pick = np.concatenate([big[:12], rng.choice(n, size=400, replace=False)])
    for m in (1, 2):
        crc_np, sig_np = out[m][0].cpu().numpy().view(np.uint32), out[m][1].cpu().numpy()
        for i in pick:
            d = data[int(offs[i]): int(offs[i] + sizes[i])].cpu().numpy()
            c, s, _ = oracle.dio_file(d, m, 0)
            assert c == crc_np[i] and s == sig_np[i].tobytes(), (m, i, sizes[i])
    del data, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("variant", [0, 1])
def test_crc_lane_path(oracle, ctxs, variant):
    """CRC-only batches of more than 3 lat_files files take crc_lane_kernel
    (one lane per file, the lane fold) for files below kFoldMinBytes and the
    sparse fold for the rest (fdfs_gpu_sig_batch).  3 lat_files + 1 files of
    0 B .. 200 KiB packed at byte offsets, with sizes on both sides of 96 KiB
    and of the lane's 128-byte steps: every CRC equals the wave-per-file
    path's (the same files in sub-batches of lat_files), and a sample
    matches the oracle."""
    from fastdfs_amd import corpus as C
    lat = torch.cuda.get_device_properties(0).multi_processor_count * 4 * 64
    n = ctxs[variant].crc_lane_min_files() + 1
    assert n == 3 * lat + 1
    rng = np.random.default_rng(71 + variant)
    sizes = rng.integers(0, 100_000, n)
    edge = rng.choice(n, size=3000, replace=False)
    sizes[edge[:1000]] = (96 << 10) + rng.integers(-2, 3, 1000)
    sizes[edge[1000:2000]] = rng.integers(100_000, 200 << 10, 1000)
    sizes[edge[2000:2500]] = 128 * rng.integers(0, 8, 500) + rng.integers(0, 2, 500)
    sizes[edge[2500:]] = rng.integers(0, 20, 500)
    data, offs_t, sizes_t = C.device_batch(sizes, seed=13 + variant, device="cuda:0", align=1)
    ctx = ctxs[variant]
    crc, _, _ = ctx.sig_batch(data, offs_t, sizes_t, method=0)
    ref = torch.cat([ctx.sig_batch(data, offs_t[a:a + lat], sizes_t[a:a + lat], method=0)[0]
                     for a in range(0, n, lat)])
    torch.cuda.synchronize()
    assert torch.equal(crc, ref)
    crc_np = crc.cpu().numpy().view(np.uint32)
    offs = offs_t.cpu().numpy()
    for i in np.concatenate([edge[::25], rng.choice(n, size=200, replace=False)]):
        d = data[int(offs[i]): int(offs[i] + sizes[i])].cpu().numpy()
        assert oracle.dio_file(d, 0, variant)[0] == crc_np[i], (i, sizes[i])
    del data
    torch.cuda.empty_cache()


@pytest.mark.parametrize("variant", [0, 1])
def test_lane_fold_short_files(oracle, ctxs, variant):
    """The lane fold's edges: files of 0-700 B packed at every
    byte offset, so lanes run 0, 1, 2 or more 128-byte steps after a head of
    0-15 bytes and a lead of 0-7 vectors -- one step is exactly the fold's
    32-dword window, so nothing passes on before the window.  200K files
    (the CRC-only batch takes crc_lane_kernel): CRC-only and HASH CRCs agree
    for every file and a sample matches the oracle, with HASH signatures."""
    from fastdfs_amd import corpus as C
    rng = np.random.default_rng(83 + variant)
    ctx = ctxs[variant]
    # above the lane path's threshold on any CU count: the
    # library's own number, not a copy of its rule
    n = max(200_000, ctx.crc_lane_min_files() + 1)
    sizes = rng.integers(0, 701, n)
    sizes[:2000] = 128 * rng.integers(0, 6, 2000) + rng.integers(-1, 2, 2000).clip(0)
    data, offs_t, sizes_t = C.device_batch(sizes, seed=21 + variant, device="cuda:0", align=1)
    crc0, _, _ = ctx.sig_batch(data, offs_t, sizes_t, method=0)
    crc1, sig1, _ = ctx.sig_batch(data, offs_t, sizes_t, method=1)
    torch.cuda.synchronize()
    assert torch.equal(crc0, crc1)
    crc_np, sig_np = crc1.cpu().numpy().view(np.uint32), sig1.cpu().numpy()
    offs = offs_t.cpu().numpy()
    for i in np.concatenate([np.arange(0, 2000, 7), rng.choice(n, size=600, replace=False)]):
        d = data[int(offs[i]): int(offs[i] + sizes[i])].cpu().numpy()
        c, sg, _ = oracle.dio_file(d, 1, variant)
        assert c == crc_np[i] and sg == sig_np[i].tobytes(), (i, sizes[i], offs[i] % 16)
    del data
    torch.cuda.empty_cache()


def test_md5_staged_multiwave(oracle, ctxs):
    """MD5 method over several waves of the staged kernel: files of 0 B to
    1.2 MiB in one aligned batch (lanes finish at different rounds, partial
    last rounds, a ragged last wave), plus one byte-misaligned file: the
    staged cooperative loads read every file's stream at its own byte
    offset, so it takes the same path as the aligned ones."""
    rng = np.random.default_rng(31)
    sizes = np.concatenate([rng.integers(0, 300, 70), rng.integers(300, 70000, 150),
                            rng.integers(1 << 18, 1_200_000, 113)])
    rng.shuffle(sizes)
    buf, offs, sz = _packed(sizes, 16, rng, slack=64)
    _check(oracle, ctxs[0], 0, buf, offs, sz, methods=(2,))
    offs2 = offs.copy()
    offs2[len(offs2) // 2] += 3
    _check(oracle, ctxs[0], 0, buf, offs2, sz, methods=(2,))


def test_md5_many_chunks(oracle, ctxs):
    """Many more 64-file chunks than the MD5 kernel has queue waves (150K
    files = 2344 chunks > 4 waves x 256 CUs), so waves take chunk after chunk
    from the device queue counter; two misaligned files put byte-offset
    staged loads inside that sequence."""
    rng = np.random.default_rng(32)
    sizes = rng.integers(0, 2600, 150_000)
    buf, offs, sz = _packed(sizes, 16, rng, slack=64)
    offs2 = offs.copy()
    offs2[[5_000, 140_000]] += 5
    _check(oracle, ctxs[0], 0, buf, offs2, sz, methods=(2,))


@pytest.mark.parametrize("shape", ["packed", "packed_tiny", "queue"])
def test_md5_packed_lanes(oracle, ctxs, shape):
    """More files than the pair kernel has lanes (100K > 1,024 pairs x 64),
    so pairs take chunk after chunk from the queue: "packed" and
    "packed_tiny" are the batches round 5's lane-packed plan balanced
    (U[8, 32] KiB, the config-3 shape scaled down; the second with 3,000
    files of 0-299 bytes: files of no whole round, odd block counts) -- the
    plan ran them bit-exact on the GPU and measured slower on config 3, so it
    lives in the probe build (csrc/probes/md5_pack.patch) --;
    "queue" is a bimodal batch (8 and 32 KiB).  Every file's CRC and MD5
    signature against the oracle, plus two byte-misaligned files."""
    rng = np.random.default_rng({"packed": 41, "packed_tiny": 42, "queue": 43}[shape])
    n = 100_000
    if shape == "queue":
        sizes = np.where(rng.random(n) < 0.5, 32 << 10, 8 << 10) + rng.integers(0, 64, n)
    else:
        sizes = rng.integers(8 << 10, (32 << 10) + 1, n)
        if shape == "packed_tiny":
            tiny = rng.choice(n, 3000, replace=False)
            sizes[tiny] = rng.integers(0, 300, 3000)
    buf, offs, sz = _packed(sizes, 16, rng, slack=64)
    offs[[7, 70_000]] += np.array([3, 9])
    _check(oracle, ctxs[0], 0, buf, offs, sz, methods=(2,))


def test_md5_at_scale(oracle, ctxs):
    """Config 3 shape (24K photos of 1-4 MiB, ~63 GB in HBM): a random sample
    of files matches the oracle's CRC and MD5 signature bit for bit, and the
    MD5 digests of the sample equal hashlib's."""
    import hashlib
    from fastdfs_amd import corpus as C
    n = 24000
    sizes = C.photo_sizes(n)
    data, offs_t, sizes_t = C.device_batch(sizes, seed=4, device="cuda:0")
    crc, sig, _ = ctxs[0].sig_batch(data, offs_t, sizes_t, method=2)
    torch.cuda.synchronize()
    sig_np, crc_np = sig.cpu().numpy(), crc.cpu().numpy().view(np.uint32)
    offs = offs_t.cpu().numpy()
    for i in np.random.default_rng(6).choice(n, size=120, replace=False):
        d = data[int(offs[i]): int(offs[i] + sizes[i])].cpu().numpy()
        c, s, _ = oracle.dio_file(d, 2, 0)
        assert c == crc_np[i] and s == sig_np[i].tobytes(), i
        assert sig_np[i, 8:].tobytes() == hashlib.md5(d.tobytes()).digest(), i
    del data
    torch.cuda.empty_cache()


@pytest.mark.parametrize("method", [0, 1, 2])
def test_host_batch_streamed(oracle, ctxs, method):
    """fdfs_gpu_sig_batch_host: a host batch streamed in small windows (many
    chunks, a file larger than the window alone, unaligned starts, a gap)
    gives the device path's results."""
    rng = np.random.default_rng(90 + method)
    sizes = rng.integers(0, 40_000, size=600).astype(np.int64)
    sizes[[5, 300]] = [300_000, 1 << 20]  # larger than the 256 KiB window
    offs = np.zeros_like(sizes)
    offs[1:] = np.cumsum(sizes + rng.integers(0, 7, size=600))[:-1]
    offs[400:] += 12345  # a gap inside the batch
    buf = rng.integers(0, 256, size=int(offs[-1] + sizes[-1]) + 1, dtype=np.uint8)
    crc, sig, codes = ctxs[0].sig_batch_host(buf, offs, sizes, method=method, want_codes=True,
                                             chunk_bytes=256 << 10)
    ocrc, osig = oracle.dio_batch(buf, offs, sizes, method, 0, nthreads=8)
    assert np.array_equal(crc, ocrc)
    if method:
        assert np.array_equal(sig, osig)
    # pinned host memory: the same, one default-size window
    pinned = torch.from_numpy(buf).pin_memory()
    crc2, sig2, _ = ctxs[0].sig_batch_host(pinned, offs, sizes, method=method)
    assert np.array_equal(crc2, ocrc)
    if method:
        assert np.array_equal(sig2, osig)
