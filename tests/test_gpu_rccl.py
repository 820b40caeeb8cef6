"""Multi-process RCCL tests of libfdfs_gpu's multi-GPU C entry points
(fdfs_gpu_dedup_global, fdfs_gpu_crc_batch_global): one fresh process per
visible GPU (tests/rccl_child.py), each started before it makes any GPU call
(the pytest process never re-execs itself), joined over RCCL / xGMI, each
checking its own answers against the oracle over the concatenated input.

On a box with one visible GPU the multi-rank case skips with its reason; the
world-1 case still runs the same child end to end (its communicator setup,
the announcement all-gather, the grouped send/recv self segments).
"""
import os
import signal
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = os.path.join(ROOT, "tests", "rccl_child.py")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run_world(world: int, timeout: float = 240.0):
    port = _free_port()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["MASTER_ADDR"] = "127.0.0.1"
    procs = [subprocess.Popen([sys.executable, "-u", CHILD, "--rank", str(r), "--world", str(world),
                               "--port", str(port)], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True, start_new_session=True)
             for r in range(world)]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append(out)
    except subprocess.TimeoutExpired:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
        for p in procs:
            p.wait()
        pytest.fail(f"world {world}: a rank did not finish in {timeout:.0f} s")
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{out[-4000:]}"
        assert f"RANK {r} OK" in out, out[-4000:]
    return outs


def test_rccl_child_world1():
    """The multi-process harness itself at world 1 (runs on a one-GPU box)."""
    _run_world(1)


def test_rccl_multi_gpu():
    """dedup_global and the split-file CRC over RCCL between real GPUs, one
    process per visible GPU (up to 8)."""
    ngpu = torch.cuda.device_count()
    if ngpu < 2:
        pytest.skip(f"{ngpu} GPU visible: the multi-process RCCL exchange needs at least 2")
    _run_world(min(ngpu, 8))
