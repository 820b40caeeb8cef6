"""GPU parity for the bulk dedup (FastDHT replacement) vs the oracle."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import fastdfs_amd as F
    return F.Context(0)


def _sigs(n, nuniq, seed):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, size=(nuniq, 24), dtype=np.uint8)
    return base[rng.integers(0, nuniq, size=n)]


@pytest.mark.parametrize("n,nuniq", [(1, 1), (100, 7), (50_000, 45_000), (300_000, 1000)])
def test_dedup_vs_oracle(oracle, ctx, n, nuniq):
    sig = _sigs(n, nuniq, n)
    rep, ref = ctx.dedup(torch.from_numpy(sig).cuda())
    orep, oref = oracle.dedup(sig)
    assert np.array_equal(rep.cpu().numpy(), orep.astype(np.int64))
    assert np.array_equal(ref.cpu().numpy(), oref.astype(np.int32))


def test_dedup_with_gidx(oracle, ctx):
    sig = _sigs(20_000, 5000, 9)
    gidx = np.random.default_rng(9).permutation(10**9)[:20_000].astype(np.int64)
    rep, ref = ctx.dedup(torch.from_numpy(sig).cuda(), torch.from_numpy(gidx).cuda())
    orep, oref = oracle.dedup(sig)
    # the class representative is the smallest gidx in the class
    rep_np = rep.cpu().numpy()
    want = np.zeros(len(sig), np.int64)
    mins = {}
    for i, r in enumerate(sig):
        k = r.tobytes()
        mins[k] = min(mins.get(k, 1 << 62), gidx[i])
    for i, r in enumerate(sig):
        want[i] = mins[r.tobytes()]
    assert np.array_equal(rep_np, want)
    assert np.array_equal(ref.cpu().numpy(), oref.astype(np.int32))


@pytest.mark.parametrize("n", [1 << 20, 9_000_000])
def test_all_identical(ctx, n):
    """One class: one bucket, one partition over the LDS capacity (the HBM
    table); at 9M the bucket has more chunks than one gather batch holds."""
    sig = torch.zeros((n, 24), dtype=torch.uint8, device="cuda")
    rep, ref = ctx.dedup(sig)
    assert int(rep.max()) == 0 and int(ref.min()) == n


@pytest.mark.parametrize("nranks", [1, 2, 3, 8])
def test_bucket_exchange_in_process(oracle, ctx, nranks):
    """bucket -> (simulated all-to-all) -> group -> route back == dedup."""
    sig = _sigs(40_000, 30_000, nranks)
    n = len(sig)
    shards = np.array_split(np.arange(n), nranks)
    sig_t = torch.from_numpy(sig).cuda()
    sent = []
    for r in range(nranks):
        idx = torch.from_numpy(shards[r]).cuda()
        rows, counts, row_of = ctx.dedup_bucket(sig_t[idx].contiguous(), idx.to(torch.int64), nranks)
        sent.append((rows, counts.cpu().tolist(), row_of))
    # owners: concatenate the rows addressed to them, in source-rank order
    answers = {}
    for o in range(nranks):
        parts = []
        for r in range(nranks):
            rows, counts, _ = sent[r]
            st = sum(counts[:o])
            parts.append(rows[st: st + counts[o]])
        rows_in = torch.cat(parts).contiguous()
        rep, ref = ctx.dedup_group(rows_in)
        pos = 0
        for r in range(nranks):
            c = sent[r][1][o]
            answers[(o, r)] = (rep[pos: pos + c], ref[pos: pos + c])
            pos += c
    orep, oref = oracle.dedup(sig)
    for r in range(nranks):
        rows, counts, row_of = sent[r]
        back_rep = torch.cat([answers[(o, r)][0] for o in range(nranks)])
        back_ref = torch.cat([answers[(o, r)][1] for o in range(nranks)])
        got_rep = back_rep[row_of].cpu().numpy()
        got_ref = back_ref[row_of].cpu().numpy()
        assert np.array_equal(got_rep, orep[shards[r]].astype(np.int64))
        assert np.array_equal(got_ref, oref[shards[r]].astype(np.int32))


def test_c5_one_gpu_share(oracle, ctx):
    """Config 5 per-GPU share: 12.5M signatures with 10 % duplicates."""
    from fastdfs_amd import corpus as C
    n = 12_500_000
    sig = C.dup_signatures(n, 0.1, seed=5)
    rep, ref = ctx.dedup(sig.cuda())
    orep, oref = oracle.dedup(sig.numpy())
    assert np.array_equal(rep.cpu().numpy(), orep.astype(np.int64))
    assert np.array_equal(ref.cpu().numpy(), oref.astype(np.int32))


# ---- crafted hash collisions: distinct signatures with one 64-bit key ----

M64 = (1 << 64) - 1


def _fmix64(k):
    k ^= k >> 33
    k = (k * 0xff51afd7ed558ccd) & M64
    k ^= k >> 33
    k = (k * 0xc4ceb9fe1a85ec53) & M64
    k ^= k >> 33
    return k


def _colliding(count, seed):
    """`count` distinct signatures with identical 64-bit grouping hash
    (fmix64(a ^ fmix64(b ^ fmix64(c + K)))): pick b freely, solve for a."""
    rng = np.random.default_rng(seed)
    c = int(rng.integers(0, 1 << 62))
    inner = _fmix64((c + 0x9E3779B97F4A7C15) & M64)
    a0, b0 = int(rng.integers(0, 1 << 62)), int(rng.integers(0, 1 << 62))
    target = a0 ^ _fmix64(b0 ^ inner)
    out = np.zeros((count, 24), np.uint8)
    for i in range(count):
        b = (b0 + i * 0x1234567) & M64
        a = target ^ _fmix64(b ^ inner)
        out[i] = np.frombuffer(a.to_bytes(8, "little") + b.to_bytes(8, "little")
                               + c.to_bytes(8, "little"), np.uint8)
    return out


@pytest.mark.parametrize("ncoll,reps", [(40, 3), (700, 2), (3500, 1)])
def test_dedup_full_hash_collisions(oracle, ctx, ncoll, reps):
    """Distinct signatures sharing the whole 64-bit key (one partition, one
    probe chain) stay distinct classes; with 3500 of them the partition is
    over the LDS capacity and takes the HBM-table path."""
    coll = _colliding(ncoll, ncoll)
    bg = _sigs(30_000, 20_000, 77)
    sig = np.concatenate([np.tile(coll, (reps, 1)), bg])
    sig = sig[np.random.default_rng(ncoll).permutation(len(sig))]
    rep, ref = ctx.dedup(torch.from_numpy(np.ascontiguousarray(sig)).cuda())
    orep, oref = oracle.dedup(sig)
    assert np.array_equal(rep.cpu().numpy(), orep.astype(np.int64))
    assert np.array_equal(ref.cpu().numpy(), oref.astype(np.int32))


@pytest.mark.parametrize("n", [2, 1023, 1025, 3000, 2_100_000])
def test_dedup_partition_plans(oracle, ctx, n):
    """Sizes around the partition-plan steps (one, two and three levels)."""
    sig = _sigs(n, max(1, n * 9 // 10), n + 3)
    rep, ref = ctx.dedup(torch.from_numpy(sig).cuda())
    orep, oref = oracle.dedup(sig)
    assert np.array_equal(rep.cpu().numpy(), orep.astype(np.int64))
    assert np.array_equal(ref.cpu().numpy(), oref.astype(np.int32))


def _packed_case(name):
    if name == "uniform":
        return _sigs(300_000, 250_000, 5), None
    if name == "gidx":
        sig = _sigs(20_000, 5000, 9)
        return sig, np.random.default_rng(9).permutation(10**9)[:20_000].astype(np.int64)
    if name == "heavy":  # one class over the LDS table: the HBM-table path
        sig = _sigs(200_000, 50_000, 11)
        sig[::3] = sig[0]
        return sig, None
    coll = _colliding(3500, 3500)  # "collisions": one probe chain past the LDS table
    sig = np.concatenate([np.tile(coll, (2, 1)), _sigs(30_000, 20_000, 78)])
    return np.ascontiguousarray(sig[np.random.default_rng(5).permutation(len(sig))]), None


@pytest.mark.parametrize("case", ["uniform", "gidx", "heavy", "collisions"])
def test_dedup_packed_equals_arrays(oracle, ctx, case):
    """fdfs_gpu_dedup_packed: the same rep / ref as fdfs_gpu_dedup in 16-byte
    records (reserved word 0), through the LDS and the HBM-table groups and
    with ingest indices (the class minimum read back from the packed
    records); the arrays form against the oracle as well."""
    sig, gidx = _packed_case(case)
    st = torch.from_numpy(sig).cuda()
    gt = None if gidx is None else torch.from_numpy(gidx).cuda()
    rep, ref = ctx.dedup(st, gt)
    out = ctx.dedup_packed(st, gt).cpu().numpy()
    assert np.array_equal(out[:, 0], rep.cpu().numpy())
    assert np.array_equal(out[:, 1], ref.cpu().numpy().astype(np.int64))
    if gidx is None:
        orep, oref = oracle.dedup(sig)
        assert np.array_equal(out[:, 0], orep.astype(np.int64))
        assert np.array_equal(out[:, 1], oref.astype(np.int64))


def test_misaligned_records_rejected(ctx):
    """Records are read as u64 words: a signature buffer off an 8-byte
    boundary is EINVAL (0-or-errno convention), never a misaligned read."""
    import errno
    from fastdfs_amd import FdfsGpuError
    buf = torch.zeros(24 * 100 + 8, dtype=torch.uint8, device="cuda")
    with pytest.raises(FdfsGpuError) as ei:
        ctx.dedup(buf[1:1 + 24 * 100].view(100, 24))
    assert ei.value.errno == errno.EINVAL
    with pytest.raises(FdfsGpuError) as ei:
        ctx.dedup_bucket(buf[4:4 + 24 * 100].view(100, 24), None, 2)
    assert ei.value.errno == errno.EINVAL


def test_dedup_global_rccl_one_rank(oracle, ctx):
    """dedup_global over a real RCCL group (one rank on this box): the three
    all-to-alls run on the HIP kernels' device tensors, with the exact dtypes
    and split sizes the multi-GPU bench uses, and the answer equals the
    single-GPU dedup.  Ranks > 1 are covered by the gloo tests."""
    import socket
    import torch.distributed as dist
    from fastdfs_amd.dist import dedup_global

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        sig = torch.from_numpy(_sigs(100_000, 60_000, 11)).cuda()
        gidx = torch.arange(sig.shape[0], dtype=torch.int64, device="cuda")
        stats = {}
        rep, ref = dedup_global(ctx, sig, gidx, stats=stats)
        torch.cuda.synchronize()
        orep, oref = oracle.dedup(sig.cpu().numpy())
        assert np.array_equal(rep.cpu().numpy(), orep.astype(np.int64))
        assert np.array_equal(ref.cpu().numpy(), oref.astype(np.int32))
        assert stats["peer_bytes"] == 0
    finally:
        dist.destroy_process_group()


def test_empty_batch(ctx):
    """A rank with no files: dedup, bucket and group all return empty results
    (bucket counts zeroed) without launching a zero-size grid."""
    sig = torch.empty((0, 24), dtype=torch.uint8, device="cuda")
    rep, ref = ctx.dedup(sig)
    assert rep.numel() == 0 and ref.numel() == 0
    rows, counts, row_of = ctx.dedup_bucket(sig, torch.empty(0, dtype=torch.int64, device="cuda"), 4)
    assert rows.shape == (0, 32) and row_of.numel() == 0
    assert counts.cpu().tolist() == [0, 0, 0, 0]
    rep, ref = ctx.dedup_group(rows)
    torch.cuda.synchronize()
    assert rep.numel() == 0 and ref.numel() == 0


def test_dedup_global_c_abi_one_rank(oracle, ctx):
    """fdfs_gpu_dedup_global (the C daemon's multi-GPU entry) over its own
    RCCL communicator, set up with fdfs_gpu_comm_unique_id / comm_init (the
    id carried by torch.distributed): one rank on this box, so every RCCL
    call runs (count all-to-all, grouped exchanges) with one peer.  The
    answer equals the single-GPU dedup; an empty share works too.  Ranks > 1
    are not measurable on a one-GPU box."""
    import socket
    import torch.distributed as dist
    from fastdfs_amd.api import Comm
    from fastdfs_amd.dist import dedup_global

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    comm = None
    try:
        comm = Comm(ctx)
        assert comm.world == 1 and comm.rank == 0
        for n, nu in [(120_000, 70_000), (0, 1), (5, 2)]:
            sig = torch.from_numpy(_sigs(n, nu, 13 + n)).cuda().view(n, 24)
            gidx = torch.arange(n, dtype=torch.int64, device="cuda") + 1000
            rep, ref = dedup_global(ctx, sig, gidx, comm=comm)
            torch.cuda.synchronize()
            orep, oref = oracle.dedup(sig.cpu().numpy())
            assert np.array_equal(rep.cpu().numpy(), orep.astype(np.int64) + 1000)
            assert np.array_equal(ref.cpu().numpy(), oref.astype(np.int32))
    finally:
        if comm is not None:
            comm.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("nranks", [1, 2, 3, 8, 64])
def test_dedup_global_local_vs_oracle(oracle, ctx, nranks):
    """fdfs_gpu_dedup_global's own code path (bucket, announcement plan,
    per-(src, dst) offsets, owner groups, answer routing) for nranks virtual
    ranks on this GPU, segments moved by device copies where RCCL would send
    them.  Shares of uneven size (one empty), duplicates across ranks,
    ingest indices with gaps: every rank's answers equal the oracle's over
    the concatenation."""
    n = 60_000
    sig = _sigs(n, 35_000, 100 + nranks)
    gidx = np.cumsum(np.random.default_rng(nranks).integers(1, 5, n)).astype(np.int64)
    cuts = np.sort(np.random.default_rng(7 * nranks).choice(np.arange(1, n), nranks - 1, replace=False)) \
        if nranks > 1 else np.array([], np.int64)
    bounds = [0] + list(cuts) + [n]
    if nranks > 2:
        bounds[2] = bounds[1]  # rank 1 holds nothing
    sig_t, g_t = torch.from_numpy(sig).cuda(), torch.from_numpy(gidx).cuda()
    shares = [(sig_t[bounds[p]:bounds[p + 1]].contiguous(), g_t[bounds[p]:bounds[p + 1]].contiguous())
              for p in range(nranks)]
    outs = ctx.dedup_global_local([s for s, _ in shares], [g for _, g in shares])
    orep, oref = oracle.dedup(sig)
    for p in range(nranks):
        lo, hi = bounds[p], bounds[p + 1]
        rep, ref = outs[p]
        assert np.array_equal(rep.cpu().numpy(), gidx[orep[lo:hi].astype(np.int64)]), p
        assert np.array_equal(ref.cpu().numpy(), oref[lo:hi].astype(np.int32)), p


def _owners(ctx, sig_t, nranks):
    """Each record's owner rank, from the public bucket (rows grouped by owner)."""
    _, counts, row_of = ctx.dedup_bucket(sig_t, None, nranks)
    ends = np.cumsum(counts.cpu().numpy())
    return np.searchsorted(ends, row_of.cpu().numpy(), side="right")


@pytest.mark.parametrize("nranks,hot", [(4, 0.0), (4, 0.6), (8, 0.3)])
def test_dedup_global_local_sink_bytes_and_skew(oracle, ctx, nranks, hot):
    """Round 6's exchange: the owners return only the records of
    multi-member classes (16-byte sink records), the rows of a rank's own
    owner never cross, and a share whose owners are skewed far past the
    one-pass bucket's fixed capacity (`hot` of all records one signature:
    one owner gets them all) falls back to the exact layout on every rank.
    Answers equal the oracle's; the bytes the library reports equal what the
    owner of every record implies."""
    n = 80_000
    sig = _sigs(n, 50_000, 7 + nranks)
    nh = int(hot * n)
    if nh:
        sig[np.random.default_rng(3).choice(n, nh, replace=False)] = sig[0]
    gidx = np.arange(n, dtype=np.int64) * 3 + 11
    bounds = np.linspace(0, n, nranks + 1).astype(np.int64)
    sig_t, g_t = torch.from_numpy(sig).cuda(), torch.from_numpy(gidx).cuda()
    shares = [(sig_t[bounds[p]:bounds[p + 1]].contiguous(), g_t[bounds[p]:bounds[p + 1]].contiguous())
              for p in range(nranks)]
    outs = ctx.dedup_global_local([s for s, _ in shares], [g for _, g in shares])
    st = ctx.dedup_global_stats()
    orep, oref = oracle.dedup(sig)
    rows = ans = 0
    for p in range(nranks):
        lo, hi = bounds[p], bounds[p + 1]
        rep, ref = outs[p]
        assert np.array_equal(rep.cpu().numpy(), gidx[orep[lo:hi].astype(np.int64)]), p
        assert np.array_equal(ref.cpu().numpy(), oref[lo:hi].astype(np.int32)), p
        own = _owners(ctx, shares[p][0], nranks)
        away = own != p
        rows += int(away.sum())
        ans += int((away & (oref[lo:hi] > 1)).sum())
    assert st == {"row_bytes": 32 * rows, "answer_bytes": 16 * ans}
    assert st["answer_bytes"] < st["row_bytes"] / 2  # the round-5 protocol's answers: 16 B per row


def test_dedup_global_needs_gidx_over_ranks(ctx):
    """without ingest indices, records of different ranks share
    numbers and the class minimum would pick another rank's record.  More
    than one rank without gidx is EINVAL (C) / ValueError (Python)."""
    import ctypes
    import errno
    sig = torch.zeros((10, 24), dtype=torch.uint8, device="cuda")
    with pytest.raises(ValueError):
        ctx.dedup_global_local([sig, sig], [None, None])
    L = ctx._L
    rep = torch.empty(10, dtype=torch.int64, device="cuda")
    ref = torch.empty(10, dtype=torch.int32, device="cuda")
    P, U = ctypes.c_void_p * 2, ctypes.c_uint64 * 2
    rc = L.fdfs_gpu_dedup_global_local(ctx._h, 2, P(sig.data_ptr(), sig.data_ptr()), P(None, None), U(10, 10),
                                       P(rep.data_ptr(), rep.data_ptr()), P(ref.data_ptr(), ref.data_ptr()), None)
    assert rc == errno.EINVAL


@pytest.mark.parametrize("nbatch", [1, 2, 5])
def test_incremental_index_matches_sequential_ingest(oracle, ctx, nbatch):
    """fdfs_gpu_index: a stream ingested in k batches.  After batch j every
    record's source is the first file ever ingested with its signature and
    its ref the class size so far: the oracle's sequential dedup over the
    prefix of batches 0..j, restricted to batch j."""
    from fastdfs_amd.api import DedupIndex
    n = 300_000
    sig = _sigs(n, 200_000, 40 + nbatch)
    cuts = np.sort(np.random.default_rng(nbatch).choice(np.arange(1, n), nbatch - 1, replace=False))
    bounds = [0] + list(cuts) + [n]
    ix = DedupIndex(ctx, 250_000)
    try:
        for j in range(nbatch):
            lo, hi = bounds[j], bounds[j + 1]
            part = torch.from_numpy(sig[lo:hi]).cuda()
            rep, ref = ix.ingest(part)
            torch.cuda.synchronize()
            orep, oref = oracle.dedup(sig[:hi], nthreads=8)
            assert np.array_equal(rep.cpu().numpy(), orep[lo:hi].astype(np.int64)), j
            assert np.array_equal(ref.cpu().numpy(), oref[lo:hi].astype(np.int32)), j
        st = ix.stats()
        assert st["records"] == n and st["unplaced"] == 0
        assert st["classes"] == np.unique(sig, axis=0).shape[0]
    finally:
        ix.close()


def test_incremental_index_gidx_and_collisions(oracle, ctx):
    """Explicit increasing ingest indices, crafted signatures sharing a whole
    64-bit dedup key across batches, and an index created far too small: it
    grows (rehashing every class) before a batch that might not fit, so every
    class is placed and every answer is the stream's, never "within its
    batch only" (VERDICT r02)."""
    from fastdfs_amd.api import DedupIndex
    coll = _colliding(300, 5)
    sig = np.concatenate([coll, coll[:100], _sigs(5000, 3000, 6), coll[50:250]])
    gidx = np.cumsum(np.random.default_rng(2).integers(1, 9, len(sig))).astype(np.int64)
    ix = DedupIndex(ctx, 20_000)
    try:
        for lo, hi in [(0, 350), (350, 3000), (3000, len(sig))]:
            rep, ref = ix.ingest(torch.from_numpy(sig[lo:hi]).cuda(), torch.from_numpy(gidx[lo:hi]).cuda())
            orep, oref = oracle.dedup(sig[:hi])
            assert np.array_equal(rep.cpu().numpy(), gidx[orep[lo:hi].astype(np.int64)])
            assert np.array_equal(ref.cpu().numpy(), oref[lo:hi].astype(np.int32))
    finally:
        ix.close()
    small = DedupIndex(ctx, 10)  # 1024 slots (768 classes) for ~3,300 classes
    try:
        assert small.stats()["slots"] == 1024
        for lo, hi in [(0, 700), (700, 900), (900, len(sig))]:
            rep, ref = small.ingest(torch.from_numpy(sig[lo:hi]).cuda())
            orep, oref = oracle.dedup(sig[:hi])
            assert np.array_equal(rep.cpu().numpy(), orep[lo:hi].astype(np.int64)), lo
            assert np.array_equal(ref.cpu().numpy(), oref[lo:hi].astype(np.int32)), lo
        st = small.stats()
        assert st["unplaced"] == 0 and st["classes"] == np.unique(sig, axis=0).shape[0]
        assert st["slots"] >= 4096 and st["classes"] <= st["slots"] * 3 // 4
    finally:
        small.close()


def test_dedup_600m_known_classes(ctx):
    """600M records (the split kernel's 4096-bin form: d2 = 11), checked by
    construction instead of the oracle: 300M distinct signatures, record i
    and i + 300M carry the same one, so rep = i mod 300M and ref = 2."""
    half = 300_000_000
    n = 2 * half
    free, _ = torch.cuda.mem_get_info()
    if free < 80 << 30:
        pytest.skip("needs ~60 GB of device memory")
    cls = torch.arange(half, dtype=torch.int64, device="cuda")
    words = torch.stack([cls, cls * 0x9E3779B97F4A7C15 + 12345, cls ^ 0x5555AAAA5555AAAA], dim=1)
    one = words.contiguous().view(torch.uint8).view(half, 24)
    sig = torch.cat([one, one])
    del words, one
    rep, ref = ctx.dedup(sig)
    torch.cuda.synchronize()
    del sig
    idx = torch.arange(n, dtype=torch.int64, device="cuda")
    assert torch.equal(rep, idx % half)
    assert int(ref.min()) == 2 and int(ref.max()) == 2
