"""GPU parity of the chunked (state-carrying) path: fdfs_gpu_state_init /
update_batch / final_batch, i.e. the per-chunk loop of dio_write_file
(storage/storage_dio.c:465-515) on the GPU, against the oracle's one-shot
result (chunking never changes the reference's values: every primitive is a
streaming recurrence) and against the GPU one-shot path.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctxs():
    import fastdfs_amd as F
    if not torch.cuda.is_available():
        pytest.fail("gpu test collected without a GPU")
    return {0: F.Context(0, unsigned_hash=False), 1: F.Context(0, unsigned_hash=True)}


def _splits(rng, size, small_frac=0.3, max_chunk=70_000):
    """Random cut points of one file: chunk sizes mix tiny (<= 63, MD5 tail
    fills), zero-length and 1..max_chunk byte chunks."""
    cuts, pos = [], 0
    while pos < size:
        u = rng.random()
        if u < small_frac:
            step = int(rng.integers(0, 64))
        else:
            step = int(rng.integers(1, max_chunk))
        step = min(step, size - pos)
        cuts.append(step)
        pos += step
    if not cuts or rng.random() < 0.2:
        cuts.append(0)  # an empty chunk (a zero-length update)
    return cuts


def _stream(ctx, method, files, rng, order_shuffle=True, dev="cuda:0"):
    """Feed every file chunk by chunk: call k carries chunk k of each file
    that has one, the chunks placed at random byte alignment in a fresh
    device buffer, in a random order, addressed by state_idx."""
    n = len(files)
    cuts = [_splits(rng, len(f)) for f in files]
    states = ctx.new_states(n)
    starts = [0] * n
    k = 0
    while True:
        live = [i for i in range(n) if k < len(cuts[i])]
        if not live:
            break
        if order_shuffle:
            rng.shuffle(live)
        offs, sizes, parts, pos = [], [], [], 0
        for i in live:
            pos += int(rng.integers(0, 16))
            c = cuts[i][k]
            offs.append(pos)
            sizes.append(c)
            parts.append((pos, files[i][starts[i]: starts[i] + c]))
            starts[i] += c
            pos += c
        buf = np.zeros(pos + 16, np.uint8)
        for p0, b in parts:
            buf[p0: p0 + len(b)] = b
        ctx.update_batch(states, torch.from_numpy(buf).to(dev),
                         torch.tensor(offs, dtype=torch.int64, device=dev),
                         torch.tensor(sizes, dtype=torch.int64, device=dev), method=method,
                         state_idx=torch.tensor(live, dtype=torch.int32, device=dev))
        k += 1
    assert all(starts[i] == len(files[i]) for i in range(n))
    return states, k


def _final(ctx, states, method):
    crc, sig, codes = ctx.final_batch(states, method=method, want_codes=True)
    torch.cuda.synchronize()
    crc = crc.cpu().numpy().view(np.uint32)
    if method == 0:
        return crc, None, None
    return crc, sig.cpu().numpy(), codes.cpu().numpy()


def _files(rng, sizes):
    return [rng.integers(0, 256, size=int(s), dtype=np.uint8) for s in sizes]


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("method", [0, 1, 2])
def test_random_chunking_vs_oracle(oracle, ctxs, variant, method):
    """Random files cut at random chunk boundaries (tiny, empty and large
    chunks, any alignment), fed over many calls: the final CRC / signature /
    codes equal the oracle's one-shot values and the GPU one-shot path's."""
    rng = np.random.default_rng(500 + 10 * method + variant)
    sizes = np.concatenate([[0, 1, 63, 64, 65, 127, 128, 129], rng.integers(0, 300_000, 150)])
    files = _files(rng, sizes)
    states, calls = _stream(ctxs[variant], method, files, rng)
    assert calls > 5
    crc, sig, codes = _final(ctxs[variant], states, method)
    for i, f in enumerate(files):
        oc, os_, ocodes = oracle.dio_file(f, method, variant)
        assert crc[i] == oc, (i, len(f))
        if method:
            assert sig[i].tobytes() == os_, (i, len(f))
            assert [int(x) for x in codes[i]] == ocodes, (i, len(f))
    # the one-shot GPU path over the same files agrees
    offs = np.zeros(len(files), np.int64)
    offs[1:] = np.cumsum([len(f) for f in files])[:-1]
    data = torch.from_numpy(np.concatenate(files + [np.zeros(16, np.uint8)])).cuda()
    c1, s1, _ = ctxs[variant].sig_batch(data, torch.from_numpy(offs).cuda(),
                                        torch.from_numpy(sizes.astype(np.int64)).cuda(), method=method)
    assert np.array_equal(c1.cpu().numpy().view(np.uint32), crc)
    if method:
        assert np.array_equal(s1.cpu().numpy(), sig)


@pytest.mark.parametrize("method", [1, 2])
def test_state_matches_oracle_mid_stream(oracle, ctxs, method):
    """The state after each chunk is the reference's running state: crc32 =
    CRC32_ex(prefix, XINIT), hash codes = CALC_HASH_CODES4 over the prefix,
    MD5 count and pending-buffer bytes as my_md5_update leaves them."""
    rng = np.random.default_rng(77 + method)
    f = rng.integers(0, 256, size=200_003, dtype=np.uint8)
    ctx = ctxs[0]
    states = ctx.new_states(1)
    pos = 0
    for c in [5, 59, 0, 64, 1000, 63, 70_000, 1, 128_811]:
        d = torch.from_numpy(f[pos: pos + c].copy() if c else np.zeros(1, np.uint8)).cuda()
        ctx.update_batch(states, d, torch.zeros(1, dtype=torch.int64, device="cuda"),
                         torch.tensor([c], dtype=torch.int64, device="cuda"), method=method)
        pos += c
        st = states.cpu().numpy()[0]
        crc32 = int(st[0:4].view(np.int32)[0])
        assert crc32 == oracle.crc32_ex(f[:pos], -1, 0), pos
        bits = int(st[36:44].view(np.uint64)[0])
        assert bits == 8 * pos
        if method == 1:
            h = st[4:20].view(np.int32)
            assert int(h[0]) == crc32
            assert int(h[1]) == oracle.elf_ex(f[:pos], 0, 0)
            assert int(h[2]) == oracle.simple_ex(f[:pos], 0)
            assert int(h[3]) == oracle.time33_ex(f[:pos], 0)
        else:
            r = pos % 64
            assert st[44: 44 + r].tobytes() == f[pos - r: pos].tobytes()
    assert pos == f.size


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("method", [1, 2])
def test_big_chunks_hash(oracle, ctxs, variant, method):
    """Updates with big chunks take the segment-parallel CRC (HASH: and
    polynomial) kernels; the state they start from is carried over them
    (GF(2) advance for the CRC, M^len for simple_hash / Time33).  With at
    most one big chunk per CU each chunk's ELF / MD5 chain runs on a
    workgroup of its own, starting from the state: MD5 first completes the
    bytes my_md5_update left pending (chunk sizes not multiples of 64) and
    leaves the chunk's tail pending."""
    rng = np.random.default_rng(91 + variant)
    files = _files(rng, [(9 << 20) + 12345, (5 << 20) + 7, 300_000])
    cuts = [[1234, (4 << 20) + 5, (9 << 20) + 12345 - 1234 - (4 << 20) - 5],
            [17, (5 << 20) - 10],
            [150_000, 150_000]]
    cuts[1].append(len(files[1]) - sum(cuts[1]))
    ctx = ctxs[variant]
    states = ctx.new_states(3)
    pos = [0, 0, 0]
    for k in range(3):
        live = [i for i in range(3) if k < len(cuts[i])]
        offs, sizes, chunks, p = [], [], [], 0
        for i in live:
            c = cuts[i][k]
            offs.append(p + 3)
            sizes.append(c)
            chunks.append(np.zeros(3, np.uint8))
            chunks.append(files[i][pos[i]: pos[i] + c])
            pos[i] += c
            p += 3 + c
        ctx.update_batch(states, torch.from_numpy(np.concatenate(chunks)).cuda(),
                         torch.tensor(offs, dtype=torch.int64, device="cuda"),
                         torch.tensor(sizes, dtype=torch.int64, device="cuda"), method=method,
                         state_idx=torch.tensor(live, dtype=torch.int32, device="cuda"))
    assert pos == [len(f) for f in files]
    crc, sig, codes = _final(ctx, states, method)
    for i, f in enumerate(files):
        oc, os_, ocodes = oracle.dio_file(f, method, variant)
        assert crc[i] == oc and sig[i].tobytes() == os_, i
        if method == 1:
            assert [int(x) for x in codes[i]] == ocodes, i


@pytest.mark.parametrize("variant", [0, 1])
def test_crc_combine(oracle, ctxs, variant):
    """crc32_combine: CRC32_ex(A||B, X) from CRC32_ex(A, X), CRC32_ex(B, 0), |B|."""
    rng = np.random.default_rng(3 + variant)
    a_list, b_list, want = [], [], []
    for la, lb in [(0, 0), (0, 5), (7, 0), (100, 1), (4096, 65536), (12345, 1 << 20), (3, (1 << 22) + 9)]:
        a = rng.integers(0, 256, la, dtype=np.uint8)
        b = rng.integers(0, 256, lb, dtype=np.uint8)
        a_list.append(oracle.crc32_ex(a, -1, variant))
        b_list.append(oracle.crc32_ex(b, 0, variant))
        want.append((oracle.crc32_ex(np.concatenate([a, b]), -1, variant) & 0xFFFFFFFF, lb))
    out = ctxs[variant].crc_combine(torch.tensor(a_list, dtype=torch.int32).cuda(),
                                    torch.tensor(b_list, dtype=torch.int32).cuda(),
                                    torch.tensor([w[1] for w in want], dtype=torch.int64).cuda())
    got = out.cpu().numpy().view(np.uint32)
    assert [int(x) for x in got] == [w[0] for w in want]


@pytest.mark.parametrize("method", [1, 2])
def test_many_uploads_one_chunk_each(oracle, ctxs, method):
    """The daemon's shape: 2,000 concurrent uploads, each call advances every
    one by one 256 KiB-or-less chunk (the first shorter by a header).  For
    HASH such a batch is latency-bound and offloads the CRC and polynomials
    of its chunks at the threshold big_plan_kernel picks."""
    rng = np.random.default_rng(12 + method)
    sizes = rng.integers(0, 1_200_000, 2000)
    files = _files(rng, sizes)
    ctx = ctxs[0]
    n = len(files)
    states = ctx.new_states(n)
    pos = np.zeros(n, np.int64)
    first = rng.integers(200_000, 262_144, n)
    k = 0
    while True:
        live = [i for i in range(n) if pos[i] < len(files[i]) or (k == 0)]
        if not live:
            break
        offs, szs, parts, p = [], [], [], 0
        for i in live:
            c = int(min(first[i] if k == 0 else 262_144, len(files[i]) - pos[i]))
            offs.append(p)
            szs.append(c)
            parts.append(files[i][pos[i]: pos[i] + c])
            pos[i] += c
            p += c
        ctx.update_batch(states, torch.from_numpy(np.concatenate(parts + [np.zeros(1, np.uint8)])).cuda(),
                         torch.tensor(offs, dtype=torch.int64, device="cuda"),
                         torch.tensor(szs, dtype=torch.int64, device="cuda"), method=method,
                         state_idx=torch.tensor(live, dtype=torch.int32, device="cuda"))
        k += 1
    crc, sig, _ = _final(ctx, states, method)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(sizes)[:-1]
    ocrc, osig = oracle.dio_batch(np.concatenate(files), offs, sizes.astype(np.uint64), method, 0, nthreads=8)
    assert np.array_equal(crc, ocrc)
    assert np.array_equal(sig, osig)


def test_crc_batch_global_one_rank(oracle, ctxs):
    """dist.crc_batch_global on the HIP kernels over a real RCCL group (one
    rank): every file cut into several pieces (zero-state updates, the
    all-gather, crc32_combine folds in byte order) gives the oracle's CRC.
    The multi-rank exchange is covered by the gloo tests."""
    import socket
    import torch.distributed as dist
    from fastdfs_amd.dist import crc_batch_global

    rng = np.random.default_rng(61)
    sizes = np.array([0, 5, (3 << 20) + 11, 70_001, 1 << 20], np.int64)
    files = _files(rng, sizes)
    plan = [[]]
    for f, n in enumerate(sizes):
        cuts = np.sort(rng.choice(np.arange(1, max(int(n), 2)), size=min(3, max(int(n) - 1, 0)), replace=False))
        edges = [0] + [int(c) for c in cuts] + [int(n)]
        for a, b in zip(edges[:-1], edges[1:]):
            plan[0].append((f, a, b - a))
    offs, parts, pos = [], [], 0
    for f, a, ln in plan[0]:
        pos += int(rng.integers(0, 5))
        offs.append(pos)
        parts.append((pos, files[f][a:a + ln]))
        pos += ln
    buf = np.zeros(pos + 1, np.uint8)
    for p0, b in parts:
        buf[p0:p0 + len(b)] = b
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    from fastdfs_amd.api import Comm
    try:
        for v in (0, 1):
            want = [oracle.crc32(f, v) for f in files]
            comm = Comm(ctxs[v])
            try:
                # torch.distributed steps, then the same plan through
                # fdfs_gpu_crc_batch_global on libfdfs_gpu's communicator
                for c in (None, comm):
                    crc = crc_batch_global(ctxs[v], sizes, plan, torch.from_numpy(buf).cuda(),
                                           torch.tensor(offs, dtype=torch.int64, device="cuda"), comm=c)
                    got = crc.cpu().numpy().view(np.uint32)
                    assert [int(x) for x in got] == want, (v, c is None)
            finally:
                comm.close()
    finally:
        dist.destroy_process_group()


def _rank_pieces(files, pieces, rng, dev="cuda"):
    """One rank's share as crc_batch_global takes it: its pieces' bytes
    packed at random gaps (any alignment) in one device buffer."""
    offs, pos, chunks = [], 0, []
    for f, a, ln in pieces:
        pos += int(rng.integers(0, 9))
        offs.append(pos)
        chunks.append((pos, files[f][a:a + ln]))
        pos += ln
    buf = np.zeros(pos + 1, np.uint8)
    for p0, b in chunks:
        buf[p0:p0 + len(b)] = b
    t = lambda x: torch.tensor(x, dtype=torch.int64, device=dev)  # noqa: E731
    return (torch.from_numpy(buf).to(dev), t(offs), t([p[2] for p in pieces]), t([p[0] for p in pieces]),
            t([p[1] for p in pieces]))


@pytest.mark.parametrize("world", [2, 3, 8])
def test_crc_batch_global_ranks(oracle, ctxs, world):
    """fdfs_gpu_crc_batch_global's blocks and fold at world 2, 3 and 8
    (virtual ranks on this GPU, each block where the all-gather puts it):
    (a) plan_crc_pieces' equal byte shares of 300 files incl. two of 48 MiB
    that span several ranks, (b) every file cut at random points into pieces
    dealt to random ranks in random order.  Both variants equal the oracle's
    CRC32 of every file."""
    from fastdfs_amd.dist import plan_crc_pieces

    rng = np.random.default_rng(700 + world)
    sizes = np.concatenate([[0, 1, 48 << 20], rng.integers(0, 400_000, 296), [(48 << 20) + 5]]).astype(np.int64)
    files = _files(rng, sizes)
    offs = np.zeros(sizes.size, np.uint64)
    offs[1:] = np.cumsum(sizes)[:-1]
    allb = np.concatenate(files)
    fs = torch.from_numpy(sizes).cuda()
    rnd: list[list[tuple[int, int, int]]] = [[] for _ in range(world)]
    for f, n in enumerate(sizes.tolist()):
        k = int(rng.integers(1, 6))
        edges = np.unique(np.concatenate([[0, n], rng.integers(0, n + 1, k)])) if n else np.array([0, 0])
        for a, b in zip(edges[:-1], edges[1:]):
            rnd[int(rng.integers(0, world))].append((f, int(a), int(b - a)))
    for pcs in rnd:
        rng.shuffle(pcs)
    for v in (0, 1):
        want, _ = oracle.dio_batch(allb, offs, sizes.astype(np.uint64), 0, v, nthreads=8)
        for plan in (plan_crc_pieces(sizes, world), rnd):
            ranks = [_rank_pieces(files, plan[r], rng) for r in range(world)]
            crc = ctxs[v].crc_batch_global_local(ranks, fs)
            assert np.array_equal(crc.cpu().numpy().view(np.uint32), want), (world, v, plan is rnd)


def test_crc_batch_global_rejects_bad_tilings(ctxs):
    """Pieces that do not tile their files make the call fail (EINVAL), not
    return a wrong CRC: a piece past its file's end, a file index past
    nfiles, a gap, an overlap, and an overlap whose lengths still add up to
    the file size (a matching gap)."""
    import fastdfs_amd as F
    rng = np.random.default_rng(77)
    sizes = np.array([1000, 5000, 0], np.int64)
    files = _files(rng, sizes)
    fs = torch.from_numpy(sizes).cuda()
    good = [[(0, 0, 600), (1, 0, 5000)], [(0, 600, 400)]]
    crc = ctxs[0].crc_batch_global_local([_rank_pieces(files, p, rng) for p in good], fs)
    assert crc.numel() == 3
    bad = {"past end": [[(0, 0, 600), (1, 0, 5000)], [(0, 600, 401)]],
           "file index": [[(0, 0, 600), (1, 0, 5000)], [(0, 600, 400), (3, 0, 0)]],
           "gap": [[(0, 0, 600), (1, 0, 5000)], [(0, 601, 399)]],
           "overlap": [[(0, 0, 600), (1, 0, 5000)], [(0, 500, 500)]],
           # lengths add up (600 + 400) but [500, 600) is covered twice and
           # [900, 1000) not at all: caught by the boundary sum
           "overlap+gap": [[(0, 0, 600), (1, 0, 5000)], [(0, 500, 400)]]}
    for name, plan in bad.items():
        pieces = [[(f, a, n) for f, a, n in p if f < 3] for p in plan]
        ranks = [_rank_pieces(files, pieces[r], rng) for r in range(2)]
        if name == "file index":  # a piece naming file 3 of 3
            d, o, s, pf, ps = ranks[1]
            ranks[1] = (d, torch.cat([o, o[:1]]), torch.cat([s, torch.zeros_like(s[:1])]),
                        torch.cat([pf, torch.full_like(pf[:1], 3)]), torch.cat([ps, torch.zeros_like(ps[:1])]))
        with pytest.raises(F.FdfsGpuError) as ei:
            ctxs[0].crc_batch_global_local(ranks, fs)
        assert ei.value.errno == 22, name


def test_two_streams_one_context(oracle):
    """The context contract (include/fdfs_gpu.h): one context used from two
    host threads on two streams at once, with batches that grow (the
    workspace is regrown while the other stream's kernels may still run):
    HASH signatures on one, dedup on the other, every result exact."""
    import threading

    import fastdfs_amd as F
    ctx = F.Context(0)
    dev = torch.device("cuda", 0)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    errors = []

    def sigs():
        try:
            rng = np.random.default_rng(41)
            for n in (200, 3000, 20_000, 60_000):
                sizes = rng.integers(0, 9000, n)
                offs = np.zeros(n, np.int64)
                offs[1:] = np.cumsum(sizes)[:-1]
                buf = rng.integers(0, 256, int(sizes.sum()) + 1, dtype=np.uint8)
                with torch.cuda.stream(s1):
                    d = torch.from_numpy(buf).to(dev, non_blocking=False)
                    o = torch.from_numpy(offs).to(dev)
                    z = torch.from_numpy(sizes.astype(np.int64)).to(dev)
                    crc, sig, _ = ctx.sig_batch(d, o, z, method=F.SIG_HASH, stream=s1)
                s1.synchronize()
                ocrc, osig = oracle.dio_batch(buf, offs, sizes, 1, 0, nthreads=4)
                assert np.array_equal(crc.cpu().numpy().view(np.uint32), ocrc), ("crc", n)
                assert np.array_equal(sig.cpu().numpy(), osig), ("sig", n)
        except Exception as e:  # noqa: BLE001 - reported by the main thread
            errors.append(e)

    def dedups():
        try:
            rng = np.random.default_rng(43)
            for n in (1000, 50_000, 400_000, 1_500_000):
                base = rng.integers(0, 256, size=(max(1, n // 2), 24), dtype=np.uint8)
                sig = base[rng.integers(0, len(base), size=n)]
                with torch.cuda.stream(s2):
                    st = torch.from_numpy(sig).to(dev)
                    rep, ref = ctx.dedup(st, stream=s2)
                s2.synchronize()
                orep, oref = oracle.dedup(sig)
                assert np.array_equal(rep.cpu().numpy(), orep.astype(np.int64)), ("rep", n)
                assert np.array_equal(ref.cpu().numpy(), oref.astype(np.int32)), ("ref", n)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=sigs), threading.Thread(target=dedups)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    ctx.close()
    assert not errors, errors


@pytest.mark.parametrize("method", [0, 1, 2])
def test_update_rejects_repeated_state(ctxs, method):
    """include/fdfs_gpu.h: a state may appear at most once per update call
    (storage/storage_nio.h:96 -- one chunk of an upload in flight at a time).
    A repeated index, or the reserved 0xFFFFFFFF, is EINVAL before any state
    is touched; a permutation passes."""
    import errno
    from fastdfs_amd import FdfsGpuError
    ctx = ctxs[0]
    n = 5000
    states = ctx.new_states(n)
    before = states.clone()
    data = torch.randint(0, 256, (n * 100,), dtype=torch.uint8, device="cuda")
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * 100
    sizes = torch.full((n,), 100, dtype=torch.int64, device="cuda")
    for bad in ([3, 4], [0, 4999], None):
        idx = torch.randperm(n, device="cuda").to(torch.int32)
        if bad is None:
            idx[77] = -1  # 0xFFFFFFFF
        else:
            idx[bad[1]] = idx[bad[0]]
        with pytest.raises(FdfsGpuError) as ei:
            ctx.update_batch(states, data, offs, sizes, method=method, state_idx=idx, check_bounds=False)
        assert ei.value.errno == errno.EINVAL
        assert torch.equal(states, before)
    ctx.update_batch(states, data, offs, sizes, method=method,
                     state_idx=torch.randperm(n, device="cuda").to(torch.int32))
    torch.cuda.synchronize()
    assert not torch.equal(states, before)


def test_lane_error_is_sticky(oracle):
    """a lane-path error must reach the caller even when another
    call is queued behind it before anything synchronises.  The fault is
    injected on a stream (fdfs_gpu_inject_error: what a corrupt size binning
    leaves), a HASH batch is queued right behind it, and further calls follow:
    exactly one of them fails with EIO (the first whose entry check sees the
    error), the ones after it succeed, and their results are exact."""
    import errno
    import fastdfs_amd as F
    ctx = F.Context(0, test_hooks=True)  # the shipped library has no fault injection
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    rng = np.random.default_rng(5)
    sizes = rng.integers(0, 20_000, 3000)
    offs = np.zeros(len(sizes), np.int64)
    offs[1:] = np.cumsum(sizes)[:-1]
    buf = rng.integers(0, 256, int(sizes.sum()) + 1, dtype=np.uint8)
    d = torch.from_numpy(buf).to(dev)
    o = torch.from_numpy(offs).to(dev)
    z = torch.from_numpy(sizes.astype(np.int64)).to(dev)
    torch.cuda.synchronize()
    ocrc, osig = oracle.dio_batch(buf, offs, sizes, 1, 0, nthreads=4)
    rcs = []
    ctx.inject_error(stream=s)
    for k in range(4):
        try:
            crc, sig, _ = ctx.sig_batch(d, o, z, method=F.SIG_HASH, stream=s, check_bounds=False)
            rcs.append(0)
        except F.FdfsGpuError as e:
            rcs.append(e.errno)
        if k:  # the first batch is queued behind the fault with no synchronisation
            s.synchronize()
    assert rcs.count(errno.EIO) == 1 and rcs[-1] == 0, rcs
    s.synchronize()
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), ocrc)
    assert np.array_equal(sig.cpu().numpy(), osig)
    ctx.close()
