"""CPU: the multi-rank paths over gloo (world_size 2 and 3).

The exchange logic of fastdfs_amd.dist.dedup_global (counts all-to-all, row
all-to-all, answers back, routing by row_of) runs for real over gloo; the two
device kernels it calls are replaced by a CPU test double that follows the
same contract (bucket rows by owner; group rows by 24-byte key).  The double
lives here, in tests/, and is never reachable from the product.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fastdfs_amd.dist import crc_batch_global, dedup_global, plan_crc_pieces, shard_lpt


class CpuKernelsDouble:
    """Test double of Context.dedup_bucket / dedup_group (owner = first byte mod n)."""

    def dedup_bucket(self, sig, gidx, nranks):
        sig_np = sig.numpy()
        own = sig_np[:, 8].astype(np.int64) % nranks
        order = np.argsort(own, kind="stable")
        rows = np.zeros((len(sig_np), 32), np.uint8)
        rows[:, :24] = sig_np[order]
        rows[:, 24:] = gidx.numpy()[order].astype("<i8").view(np.uint8).reshape(-1, 8)
        row_of = np.empty(len(sig_np), np.int64)
        row_of[order] = np.arange(len(sig_np))
        counts = np.bincount(own, minlength=nranks).astype(np.int64)
        return torch.from_numpy(rows), torch.from_numpy(counts), torch.from_numpy(row_of)

    def dedup_group(self, rows):
        r = rows.numpy()
        g = r[:, 24:].copy().view("<i8").reshape(-1)
        keys = [bytes(x) for x in r[:, :24]]
        mins, cnt = {}, {}
        for k, gi in zip(keys, g):
            mins[k] = min(mins.get(k, 1 << 62), int(gi))
            cnt[k] = cnt.get(k, 0) + 1
        return (torch.tensor([mins[k] for k in keys], dtype=torch.int64),
                torch.tensor([cnt[k] for k in keys], dtype=torch.int32))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, sig_all, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shards = np.array_split(np.arange(len(sig_all)), world)
        mine = shards[rank]
        sig = torch.from_numpy(sig_all[mine].copy())
        gidx = torch.from_numpy(mine.astype(np.int64))
        kern = CpuKernelsDouble()
        stats = {}
        rep, ref = dedup_global(kern, sig, gidx, stats=stats)
        # bytes to peers: this rank's rows owned elsewhere out, answers for
        # rows it owns from elsewhere back
        _, counts, _ = kern.dedup_bucket(sig, gidx, world)
        out_rows = int(counts.sum()) - int(counts[rank])
        assert stats["peer_bytes"] >= 32 * out_rows
        out_q.put((rank, rep.numpy(), ref.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_dedup_global_gloo(oracle, world):
    rng = np.random.default_rng(world)
    base = rng.integers(0, 256, size=(300, 24), dtype=np.uint8)
    sig_all = base[rng.integers(0, 300, size=2000)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sig_all, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (rep, ref)) for r, rep, ref in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    orep, oref = oracle.dedup(sig_all)
    shards = np.array_split(np.arange(len(sig_all)), world)
    for r in range(world):
        assert np.array_equal(got[r][0], orep[shards[r]].astype(np.int64))
        assert np.array_equal(got[r][1], oref[shards[r]].astype(np.int32))


def test_shard_lpt_balances_and_covers():
    rng = np.random.default_rng(0)
    sizes = rng.integers(4096, 1 << 20, size=5000)
    parts = shard_lpt(sizes, 8)
    allidx = np.concatenate(parts)
    assert np.array_equal(np.sort(allidx), np.arange(5000))
    loads = [sizes[p].sum() for p in parts]
    assert max(loads) / min(loads) < 1.01
    for p in parts:
        assert np.all(np.diff(p) > 0)


def test_shard_lpt_huge_file_alone():
    parts = shard_lpt(np.array([1 << 30, 10, 10, 10]), 2)
    assert [len(p) for p in parts] in ([1, 3], [3, 1])


@pytest.mark.parametrize("world", [2, 3, 8])
def test_c5_signature_shares(world):
    """bench.py's config-5 set (corpus.c5_signatures): the ranks' contiguous
    shares concatenate to the one-rank set (what the strong-scaled dedup line
    relies on), with 10% of the records duplicating earlier unique ones."""
    from fastdfs_amd import corpus as C
    total = 10_000
    one, gidx1 = C.c5_signatures(total, 1, 0, torch.device("cpu"))
    parts = [C.c5_signatures(total, world, r, torch.device("cpu")) for r in range(world)]
    assert torch.equal(torch.cat([p[0] for p in parts]), one)
    assert torch.equal(torch.cat([p[1] for p in parts]), gidx1)
    assert torch.equal(gidx1, torch.arange(total))
    uniq = np.unique(one.numpy(), axis=0).shape[0]
    assert uniq <= total - total // 10 and uniq > total * 0.85


class CpuCrcDouble:
    """Test double of Context.update_batch (CRC only) and crc_combine, from
    the oracle's CRC32_ex restatement: update = CRC32_ex(chunk, state),
    combine(a, b, n) = CRC32_ex(n zero bytes, a) ^ b."""

    def __init__(self, variant=0):
        from oracle import oracle as O
        self.O, self.v = O, variant

    def update_batch(self, states, data, offsets, sizes, method=0):
        assert method == 0
        d = data.numpy()
        crc = states[:, :4].contiguous().view(torch.int32).view(-1)
        for i, (o, n) in enumerate(zip(offsets.tolist(), sizes.tolist())):
            c = self.O.crc32_ex(d[o:o + n], int(crc[i]), self.v)
            states[i, :4] = torch.tensor([c], dtype=torch.int32).view(torch.uint8)

    def crc_combine(self, a, b, n):
        out = [self.O.crc32_ex(np.zeros(int(ln), np.uint8), int(x), self.v) ^ int(y)
               for x, y, ln in zip(a.tolist(), b.tolist(), n.tolist())]
        return torch.tensor(np.array(out, np.int64).astype(np.uint32).view(np.int32))


def _crc_worker(rank, world, port, sizes, blob, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        starts = np.concatenate([[0], np.cumsum(sizes)[:-1]])
        plan = plan_crc_pieces(sizes, world)
        parts, offs, pos = [], [], 0
        for f, a, ln in plan[rank]:
            offs.append(pos)
            parts.append(blob[starts[f] + a: starts[f] + a + ln])
            pos += ln
        data = torch.from_numpy(np.concatenate(parts + [np.zeros(1, np.uint8)]))
        crc = crc_batch_global(CpuCrcDouble(), sizes, plan, data, torch.tensor(offs, dtype=torch.int64))
        out_q.put((rank, crc.numpy().view(np.uint32)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_crc_batch_global_gloo(oracle, world):
    """Files split across ranks by bytes: one file much larger
    than a share is cut over every rank, small ones straddle cuts; the
    partial CRC32_ex states travel by all-gather and fold by crc32_combine
    to the oracle's CRC on every rank."""
    rng = np.random.default_rng(10 + world)
    sizes = np.array([3, 70_000, 0, 11, 5_000, 1234, 1], np.int64)
    blob = rng.integers(0, 256, int(sizes.sum()), dtype=np.uint8)
    plan = plan_crc_pieces(sizes, world)
    assert sum(1 for p in plan for _ in p) > len(sizes) - 1  # something was split
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_crc_worker, args=(r, world, port, sizes, blob, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    want = np.array([oracle.crc32(blob[s:s + n]) for s, n in zip(starts, sizes)], np.uint32)
    for r in range(world):
        assert np.array_equal(got[r], want)


def test_plan_crc_pieces_balance():
    sizes = np.array([1 << 30] * 4, np.int64)  # 4 x 1 GiB on 8 GPUs: every file on 2 ranks
    plan = plan_crc_pieces(sizes, 8)
    loads = [sum(p[2] for p in pr) for pr in plan]
    assert loads == [1 << 29] * 8
    for f in range(4):
        pcs = sorted((a, ln) for pr in plan for g, a, ln in pr if g == f)
        assert pcs[0][0] == 0 and sum(ln for _, ln in pcs) == 1 << 30
    assert plan_crc_pieces(np.array([], np.int64), 3) == [[], [], []]


class _CommLibDouble:
    """Test double of the two communicator calls Comm makes:
    the unique id fails on rank 0 when `fail`, else is 128 known bytes;
    comm_init records the id it was given."""

    def __init__(self, rank, fail):
        self.rank, self.fail, self.init_ids = rank, fail, []

    def fdfs_gpu_comm_unique_id(self, buf):
        import errno
        if self.fail:
            return errno.EIO
        for k in range(len(buf)):
            buf[k] = (7 * k + 1) & 0xFF
        return 0

    def fdfs_gpu_comm_init(self, h, uid, world, rank, out):
        self.init_ids.append(bytes(uid))
        return 0

    def fdfs_gpu_comm_destroy(self, h):
        return 0


class _CtxDouble:
    def __init__(self, L):
        self._L, self._h, self.device = L, None, 0

    def _rc(self, rc, where):
        assert rc == 0, where


def _comm_worker(rank, world, port, fail, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fastdfs_amd.api import Comm, FdfsGpuError
        L = _CommLibDouble(rank, fail and rank == 0)
        try:
            Comm(_CtxDouble(L))
            out_q.put((rank, "ok", L.init_ids))
        except FdfsGpuError as e:
            out_q.put((rank, f"FdfsGpuError {e.errno}", L.init_ids))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fail", [True, False])
def test_comm_rank0_failure_reaches_every_rank(fail):
    """api.Comm broadcasts rank 0's communicator id with a status byte: when
    fdfs_gpu_comm_unique_id fails on rank 0, every rank raises FdfsGpuError
    (EIO) and none calls fdfs_gpu_comm_init (none waits in it for a rank that
    will not come); otherwise every rank initialises with rank 0's id.
    gloo, world 3, the two library calls replaced by a test double."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, world, port, fail, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {r: (what, ids) for r, what, ids in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = bytes((7 * k + 1) & 0xFF for k in range(128))
    for r in range(world):
        what, ids = got[r]
        if fail:
            assert what == "FdfsGpuError 5" and ids == [], (r, what)
        else:
            assert what == "ok" and ids == [want], (r, what)
