"""fdfs_crc32_gpu, the C drop-in for client/fdfs_crc32.c built on the C ABI:
same usage line, "%u\\n" output and errno exit status
(client/fdfs_crc32.c:29-33,37-45,97-101).  CPU: the error paths (and the
loud ENODEV without a GPU); GPU: the gen_files corpus written to disk and
hashed by the tool, against the pinned corpus CRCs (both shift variants)."""
import errno
import os
import subprocess
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "fastdfs_amd", "lib", "fdfs_crc32_gpu")


def _run(args, env=None):
    if not os.path.exists(TOOL):
        pytest.fail("fdfs_crc32_gpu not built (python -c 'import __graft_entry__ as g; g.build()')")
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run([TOOL] + args, capture_output=True, text=True, timeout=300, env=e)


def _has_gpu():
    import torch
    return torch.cuda.is_available()


def test_usage():
    r = _run([])
    assert r.returncode == 1
    assert r.stdout.startswith("Usage: ") and "<filename>" in r.stdout


def test_missing_file_errno():
    r = _run(["/nonexistent/fdfs_crc32_test"])
    assert r.returncode == errno.ENOENT
    assert "open file /nonexistent/fdfs_crc32_test fail" in r.stdout


def test_no_gpu_fails_loudly(tmp_path):
    if _has_gpu():
        pytest.skip("a GPU is present")
    f = tmp_path / "x"
    f.write_bytes(b"123456789")
    r = _run([str(f)])
    assert r.returncode == errno.ENODEV and "fdfs_gpu_open fail" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("unsigned", [False, True])
def test_corpus_files(tmp_path, corpus, kat, unsigned):
    buf, offs, sizes = corpus
    paths = []
    for i, (o, s) in enumerate(zip(offs, sizes)):
        p = tmp_path / f"gen_{i}"
        p.write_bytes(buf[o:o + s].tobytes())
        paths.append(str(p))
    empty = tmp_path / "empty"
    empty.write_bytes(b"")
    check = tmp_path / "check"
    check.write_bytes(b"123456789")
    r = _run((["-u"] if unsigned else []) + paths + [str(empty), str(check)])
    assert r.returncode == 0, r.stdout
    got = [int(x) for x in r.stdout.split()]
    key = "crc_unsigned" if unsigned else "crc_signed"
    want = [int(h, 16) for h in kat["corpus"][key]] + [0, int(kat["check"][key], 16)]
    assert got == want
    if unsigned:
        assert got[-1] == zlib.crc32(b"123456789")


@pytest.mark.gpu
def test_many_small_files(tmp_path, oracle):
    rng = np.random.default_rng(4)
    paths, bufs = [], []
    for i, n in enumerate([1, 2, 15, 16, 17, 4095, 4096, 65537, 300_000]):
        b = rng.integers(0, 256, size=n, dtype=np.uint8)
        p = tmp_path / f"f{i}"
        p.write_bytes(b.tobytes())
        paths.append(str(p))
        bufs.append(b)
    r = _run(paths)
    assert r.returncode == 0, r.stdout
    got = np.array([int(x) for x in r.stdout.split()], np.uint32)
    sizes = np.array([len(b) for b in bufs], np.int64)
    offs = np.zeros_like(sizes)
    offs[1:] = np.cumsum(sizes)[:-1]
    ocrc, _ = oracle.dio_batch(np.concatenate(bufs), offs, sizes, 0, 0, nthreads=4)
    assert np.array_equal(got, ocrc)


@pytest.mark.gpu
def test_streamed_windows(tmp_path, oracle):
    """Files larger than the tool's 64 MiB window continue in the next ones
    (their CRC32_ex state carried on the device), small files around them."""
    rng = np.random.default_rng(8)
    sizes = [3, (130 << 20) + 17, 0, 70_000, (64 << 20), 5]
    paths, bufs = [], []
    for i, n in enumerate(sizes):
        b = rng.integers(0, 256, size=n, dtype=np.uint8)
        p = tmp_path / f"w{i}"
        p.write_bytes(b.tobytes())
        paths.append(str(p))
        bufs.append(b)
    r = _run(paths)
    assert r.returncode == 0, r.stdout
    got = [int(x) for x in r.stdout.split()]
    assert got == [oracle.crc32(b) for b in bufs]
