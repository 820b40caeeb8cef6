"""Formats that consume the file CRC, FastDHT routing and scrub (SURVEY.md 8(f)
rows 2-4): the oracle pinned against the reference's own file ids and an
independent Python restatement (CPU), then the HIP kernels through the C ABI
against the oracle (GPU, bit-exact).

Pinned: the file-id byte layout and base64 alphabet, by the three real file
ids in the reference's PHP client tests (tests/golden/kat.json "file_ids") and
Python's urlsafe base64.  Unpinned: PJWHash's sign handling (libfastcommon is
absent; the classic `(h ^ (g >> 24)) & ~HIGH_BITS` form with the signed-int
shift is used, the same choice as CRC32_ex/ELFHash_ex),
so the store sub path and the FastDHT group/server are checked only against
the restatement.
"""
import base64

import numpy as np
import pytest
import torch


def _pjw_py(data: bytes, signed: bool = True) -> int:
    h = 0
    for b in data:
        h = ((h << 4) + b) & 0xFFFFFFFF
        x = h & 0xF0000000
        if x:
            s = ((x - (1 << 32)) >> 24) & 0xFFFFFFFF if (signed and x >> 31) else x >> 24
            h = (h ^ s) & 0x0FFFFFFF
    return h


# ------------------------------------------------------------------ CPU: oracle

def test_base64_alphabet_vs_python(oracle, kat):
    for v in kat["base64"]:
        raw = bytes.fromhex(v["hex"])
        assert oracle.base64_encode(raw).decode() == v["enc"]
        assert oracle.base64_decode(v["enc"].encode()) == raw


def test_parse_reference_file_ids(oracle, kat):
    """The reference's own file ids decode to the independently restated values."""
    names = np.frombuffer("".join(v["core"] for v in kat["file_ids"]).encode(),
                          np.uint8).reshape(-1, 27)
    sid, ts, sz, crc = oracle.parse_file_ids(names)
    for i, v in enumerate(kat["file_ids"]):
        assert int(sid[i]) == v["server_id"], v["source"]
        assert int(ts[i]) == v["timestamp"]
        assert int(sz[i]) == v["file_size"]
        assert "%08X" % int(crc[i]) == v["crc32"]


def test_file_id_roundtrip_and_layout(oracle):
    rng = np.random.default_rng(7)
    n = 300
    sizes = rng.integers(0, 1 << 33, size=n).astype(np.int64)
    sizes[:5] = [0, 1, 0xFFFFFFFF, 1 << 32, (1 << 59) | 77]  # edges + a trunk-marked size
    crc = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    ts = rng.integers(0, 1 << 31, size=n).astype(np.int32)
    rnd = rng.integers(0, 1 << 31, size=n).astype(np.uint32)
    names, sub = oracle.file_ids(0x0A0B0C0D, crc, sizes, ts, rnd, subdir_count=256)
    for i in range(n):
        raw = base64.urlsafe_b64decode(bytes(names[i]) + b"=")
        assert raw[0:4] == bytes([0x0D, 0x0C, 0x0B, 0x0A])
        assert int.from_bytes(raw[4:8], "big") == int(ts[i])
        size_field = int.from_bytes(raw[8:16], "big")
        if int(sizes[i]) >> 32 == 0:
            assert size_field == ((((int(rnd[i]) & 0x007FFFFF) | 0x80000000) << 32) | int(sizes[i]))
        else:
            assert size_field == int(sizes[i])
        assert int.from_bytes(raw[16:20], "big") == int(crc[i])
        h = _pjw_py(bytes(names[i])) % (1 << 16)
        assert (sub[i, 0], sub[i, 1]) == ((h >> 8) & 0xFF, h & 0xFF)
    sid, ts2, sz2, crc2 = oracle.parse_file_ids(names)
    assert np.all(sid == 0x0A0B0C0D) and np.array_equal(ts2, ts) and np.array_equal(crc2, crc)
    want = sizes.copy()
    want[4] = 77  # trunk mark -> FDFS_TRUNK_FILE_TRUE_SIZE
    assert np.array_equal(sz2, want)


def test_appender_and_masked_decode(oracle):
    """Appender ids (COMBINE_RAND_FILE_SIZE(0) | INFINITE_FILE_SIZE,
    storage/storage_service.c:2457-2460) decode to size -1, crc 0."""
    app = ((0x80000000 | 0x1234) << 32) | (1 << 58)
    sizes = np.array([app - (1 << 64), (1 << 58) | 5], np.int64)
    crc = np.array([0xDEADBEEF, 0x12345678], np.uint32)
    names, _ = oracle.file_ids(1, crc, sizes, np.zeros(2, np.int32), np.zeros(2, np.uint32))
    _, _, sz, c = oracle.parse_file_ids(names)
    assert list(sz) == [-1, -1] and list(c) == [0, 0]


def test_subdir_count_modulo(oracle):
    crc = np.arange(64, dtype=np.uint32)
    z = np.zeros(64, np.int32)
    for sc in (1, 3, 100, 256):
        _, sub = oracle.file_ids(5, crc, np.full(64, 1000, np.int64), z, crc, subdir_count=sc)
        assert sub.max() < sc


def test_pjw_oracle_vs_python(oracle):
    rng = np.random.default_rng(3)
    for n in (0, 1, 7, 8, 9, 27, 89, 200):
        buf = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        for signed, variant in ((True, 0), (False, 1)):
            assert oracle.pjw_hash(buf, variant) & 0xFFFFFFFF == _pjw_py(buf, signed)


def test_fdht_route_oracle(oracle):
    rng = np.random.default_rng(11)
    sig = rng.integers(0, 256, size=(500, 24), dtype=np.uint8)
    servers = np.array([1, 2, 3, 5, 8], np.uint32)
    kh, grp, srv = oracle.fdht_route(b"fdfs", sig, 5, servers)
    for i in range(len(sig)):
        h = _pjw_py(b"fdfs\x01" + sig[i].tobytes())
        h &= 0x7FFFFFFF
        assert int(kh[i]) == h and int(grp[i]) == h % 5
        nh = ((h << 16) | (h >> 16)) & 0xFFFFFFFF
        nh &= 0x7FFFFFFF
        assert int(srv[i]) == nh % int(servers[grp[i]])


def test_trunk_pack_layout(oracle):
    hdr = oracle.trunk_pack([1], [0x01020304], [-2], [0xA0B0C0D0], [0x11223344],
                            np.frombuffer(b"jpg\0\0\0\0", np.uint8))
    assert hdr[0].tobytes() == (b"\x01" + bytes.fromhex("01020304") + bytes.fromhex("FFFFFFFE")
                                + bytes.fromhex("A0B0C0D0") + bytes.fromhex("11223344") + b"jpg\0\0\0\0")


# ------------------------------------------------------------------ GPU: kernels

@pytest.fixture(scope="module")
def ctxs():
    import fastdfs_amd as F
    if not torch.cuda.is_available():
        pytest.fail("gpu test collected without a GPU")
    return {0: F.Context(0, unsigned_hash=False), 1: F.Context(0, unsigned_hash=True)}


def _cuda(a):
    return torch.from_numpy(np.array(a, copy=True, order="C")).cuda()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("n", [1, 1000, 70_001])
def test_gpu_file_ids(oracle, ctxs, variant, n):
    rng = np.random.default_rng(n + variant)
    sizes = rng.integers(0, 1 << 34, size=n).astype(np.int64)
    sizes[rng.random(n) < 0.5] >>= 3
    crc = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    ts = rng.integers(0, 1 << 31, size=n).astype(np.int32)
    rnd = rng.integers(0, 1 << 31, size=n).astype(np.uint32)
    sc = 256 if n != 1000 else 37
    names, sub = ctxs[variant].file_ids(0xC0A8D16C, _cuda(crc.view(np.int32)), _cuda(sizes),
                                        _cuda(ts), _cuda(rnd.view(np.int32)), subdir_count=sc)
    torch.cuda.synchronize()
    m = min(n, 5000)  # the oracle loops per record in Python; check a prefix + the tail
    idx = np.unique(np.r_[np.arange(m), np.arange(max(0, n - 100), n)])
    onames, osub = oracle.file_ids(0xC0A8D16C, crc[idx], sizes[idx], ts[idx], rnd[idx], sc, variant)
    assert np.array_equal(names.cpu().numpy()[idx], onames)
    assert np.array_equal(sub.cpu().numpy()[idx], osub)
    # full-size property: decode(encode(x)) on the GPU returns the inputs
    sid, ts2, sz2, crc2 = ctxs[variant].parse_file_ids(names)
    assert np.all(sid.cpu().numpy().view(np.uint32) == 0xC0A8D16C)
    assert np.array_equal(ts2.cpu().numpy(), ts)
    assert np.array_equal(crc2.cpu().numpy().view(np.uint32), crc)
    assert np.array_equal(sz2.cpu().numpy(), sizes)


@pytest.mark.gpu
def test_gpu_parse_reference_ids(oracle, ctxs, kat):
    core = "".join(v["core"] for v in kat["file_ids"]).encode()
    names = _cuda(np.frombuffer(core, np.uint8).copy())
    sid, ts, sz, crc = ctxs[0].parse_file_ids(names)
    for i, v in enumerate(kat["file_ids"]):
        assert int(sid[i].item()) & 0xFFFFFFFF == v["server_id"]
        assert int(ts[i].item()) == v["timestamp"]
        assert int(sz[i].item()) == v["file_size"]
        assert "%08X" % (int(crc[i].item()) & 0xFFFFFFFF) == v["crc32"]
    # appender / trunk / masked decode vs the oracle
    rng = np.random.default_rng(5)
    raw = rng.integers(0, 256, size=(4000, 20), dtype=np.uint8)
    raw[:1000, 8] = 0x84          # bit 63 + appender (2^58)
    raw[1000:2000, 8] = 0x08      # trunk mark only
    raw[2000:3000, 8] = 0x04      # appender only
    nm = np.frombuffer(b"".join(base64.urlsafe_b64encode(r.tobytes()).rstrip(b"=") for r in raw),
                       np.uint8).reshape(-1, 27)
    g = ctxs[0].parse_file_ids(_cuda(nm))
    o = oracle.parse_file_ids(nm)
    for a, b in zip(g, o):
        assert np.array_equal(a.cpu().numpy().view(b.dtype) if a.dtype != torch.int64 else a.cpu().numpy(), b)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 777, 100_000])
def test_gpu_trunk_roundtrip(oracle, ctxs, n):
    rng = np.random.default_rng(n)
    ft = rng.integers(0, 256, size=n, dtype=np.uint8)
    al = rng.integers(-(1 << 31), 1 << 31, size=n).astype(np.int32)
    fs = rng.integers(-(1 << 31), 1 << 31, size=n).astype(np.int32)
    crc = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    mt = rng.integers(0, 1 << 31, size=n).astype(np.int32)
    ext = rng.integers(0, 256, size=(n, 7), dtype=np.uint8)
    hdr = ctxs[0].trunk_pack(_cuda(ft), _cuda(al), _cuda(fs), _cuda(crc.view(np.int32)), _cuda(mt),
                             _cuda(ext))
    m = min(n, 3000)
    ohdr = oracle.trunk_pack(ft[:m], al[:m], fs[:m], crc[:m], mt[:m], ext[:m])
    assert np.array_equal(hdr.cpu().numpy()[:m], ohdr)
    back = ctxs[0].trunk_unpack(hdr)
    for a, b in zip(back, (ft, al, fs, crc.view(np.int32), mt, ext)):
        assert np.array_equal(a.cpu().numpy(), b)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("n,groups", [(1, 1), (5000, 7), (200_000, 64)])
def test_gpu_fdht_route(oracle, ctxs, variant, n, groups):
    rng = np.random.default_rng(n * 3 + variant)
    sig = rng.integers(0, 256, size=(n, 24), dtype=np.uint8)
    servers = rng.integers(1, 6, size=groups).astype(np.uint32)
    ns = b"FastDFS"
    kh, grp, srv, order, start = ctxs[variant].fdht_route(_cuda(sig), ns, groups,
                                                         _cuda(servers.view(np.int32)))
    torch.cuda.synchronize()
    m = min(n, 5000)
    okh, ogrp, osrv = oracle.fdht_route(ns, sig[:m], groups, servers, variant)
    assert np.array_equal(kh.cpu().numpy()[:m], okh)
    assert np.array_equal(grp.cpu().numpy()[:m].view(np.uint32), ogrp)
    assert np.array_equal(srv.cpu().numpy()[:m].view(np.uint32), osrv)
    # order lists every record once, grouped; group_start are the boundaries
    g = grp.cpu().numpy()
    o = order.cpu().numpy()
    st = start.cpu().numpy()
    assert st[0] == 0 and st[-1] == n and np.all(np.diff(st) == np.bincount(g, minlength=groups))
    assert np.array_equal(np.sort(o), np.arange(n))
    assert np.array_equal(g[o], np.repeat(np.arange(groups), np.diff(st)))


@pytest.mark.gpu
def test_gpu_scrub(oracle, ctxs):
    rng = np.random.default_rng(21)
    sizes = rng.integers(0, 200_000, size=3000).astype(np.int64)
    offs = np.zeros_like(sizes)
    offs[1:] = np.cumsum((sizes + 15) // 16 * 16)[:-1]
    buf = rng.integers(0, 256, size=int(offs[-1] + sizes[-1]) + 1, dtype=np.uint8)
    ocrc, _ = oracle.dio_batch(buf, offs, sizes, 0, 0, nthreads=8)
    expect = ocrc.copy()
    flip = rng.choice(len(sizes), size=37, replace=False)
    expect[flip] ^= 1
    crc, bad, nbad = ctxs[0].scrub(_cuda(buf), _cuda(offs), _cuda(sizes), _cuda(expect.view(np.int32)))
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), ocrc)
    assert set(np.nonzero(bad.cpu().numpy())[0]) == set(flip)
    assert int(nbad.item()) == 37


# ---- FastDHT routing of file-id keys, recovery batch ----

def _file_id_table(n, rng, stride=64):
    """n file ids "group1/M00/XX/YY/<27 chars>.<ext>" as uint8[n, stride] + lengths."""
    import base64 as b64
    ids = np.zeros((n, stride), np.uint8)
    lens = np.zeros(n, np.int32)
    for i in range(n):
        core = b64.urlsafe_b64encode(rng.integers(0, 256, 20, dtype=np.uint8).tobytes())[:27]
        ext = [b"", b".jpg", b".c", b".part2.c"][i % 4]
        s = b"group1/M%02X/%02X/%02X/" % (i % 3, rng.integers(0, 256), rng.integers(0, 256)) + core + ext
        ids[i, :len(s)] = np.frombuffer(s, np.uint8)
        lens[i] = len(s)
    return ids, lens


def test_fdht_route_keys_oracle_matches_sig_route(oracle):
    rng = np.random.default_rng(12)
    sig = rng.integers(0, 256, size=(50, 24), dtype=np.uint8)
    servers = np.array([2, 3, 1], np.uint32)
    a = oracle.fdht_route(b"ns", sig, 3, servers)
    b = oracle.fdht_route_keys(b"ns", sig, np.full(50, 24), 3, servers)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    ids, lens = _file_id_table(20, rng)
    kh, _, _ = oracle.fdht_route_keys(b"ns", ids, lens, 3, servers)
    for i in range(20):
        want = _pjw_py(b"ns\x01" + ids[i, :lens[i]].tobytes()) & 0x7FFFFFFF
        assert int(kh[i]) == want


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1])
def test_gpu_fdht_route_keys(oracle, ctxs, variant):
    rng = np.random.default_rng(31 + variant)
    ids, lens = _file_id_table(3000, rng)
    servers = np.array([1, 2, 3, 4, 5], np.uint32)
    kh, grp, srv, order, start = ctxs[variant].fdht_route_keys(
        _cuda(ids), b"FastDFS", 5, _cuda(lens), _cuda(servers.view(np.int32)))
    okh, ogrp, osrv = oracle.fdht_route_keys(b"FastDFS", ids, lens, 5, servers, variant)
    assert np.array_equal(kh.cpu().numpy(), okh)
    assert np.array_equal(grp.cpu().numpy().view(np.uint32), ogrp)
    assert np.array_equal(srv.cpu().numpy().view(np.uint32), osrv)
    g, o, st = grp.cpu().numpy(), order.cpu().numpy(), start.cpu().numpy()
    assert np.array_equal(np.sort(o), np.arange(3000))
    assert np.array_equal(g[o], np.repeat(np.arange(5), np.diff(st)))


@pytest.mark.gpu
@pytest.mark.parametrize("method", [1, 2])
def test_gpu_recovery_records(oracle, ctxs, method):
    from fastdfs_amd.ingest import recovery_records
    rng = np.random.default_rng(40 + method)
    # 400 distinct contents, 1000 files: duplicates across the batch
    uniq = [rng.integers(0, 256, size=int(rng.integers(0, 20_000)), dtype=np.uint8) for _ in range(400)]
    pick = rng.integers(0, 400, size=1000)
    sizes = np.array([len(uniq[p]) for p in pick], np.int64)
    offs = np.zeros_like(sizes)
    offs[1:] = np.cumsum((sizes + 15) // 16 * 16)[:-1]
    buf = np.zeros(int(offs[-1] + sizes[-1]) + 16, np.uint8)
    for i, p in enumerate(pick):
        buf[offs[i]:offs[i] + sizes[i]] = uniq[p]
    ids, lens = _file_id_table(1000, rng)
    servers = np.array([2, 1, 3, 2], np.uint32)
    rb = recovery_records(ctxs[0], _cuda(buf), _cuda(offs), _cuda(sizes), _cuda(ids), _cuda(lens),
                          b"FastDFS", 4, _cuda(servers.view(np.int32)), method=method)
    ocrc, osig = oracle.dio_batch(buf, offs, sizes, method, 0, nthreads=4)
    orep, oref = oracle.dedup(osig)
    assert np.array_equal(rb.crc.cpu().numpy().view(np.uint32), ocrc)
    assert np.array_equal(rb.sig.cpu().numpy(), osig)
    assert np.array_equal(rb.rep.cpu().numpy(), orep.astype(np.int64))
    assert np.array_equal(rb.ref.cpu().numpy(), oref.astype(np.int32))
    src = np.nonzero(orep == np.arange(1000))[0]
    assert np.array_equal(rb.fid.index.cpu().numpy(), src)
    assert len(src) == len(np.unique(pick))
    for rec, keys, klen in ((rb.fid, osig[src], np.full(len(src), 24)),
                            (rb.ref_rec, ids[src], lens[src]),
                            (rb.sig_rec, ids, lens)):
        okh, ogrp, osrv = oracle.fdht_route_keys(b"FastDFS", keys, klen, 4, servers)
        assert np.array_equal(rec.key_hash.cpu().numpy(), okh)
        assert np.array_equal(rec.group.cpu().numpy().view(np.uint32), ogrp)
        assert np.array_equal(rec.server.cpu().numpy().view(np.uint32), osrv)
        o, st = rec.order.cpu().numpy(), rec.group_start.cpu().numpy()
        assert np.array_equal(ogrp[o], np.repeat(np.arange(4), np.diff(st)).astype(np.uint32))
