"""bench.py -- FastDFS upload-path CRC32 + dedup-signature throughput on MI355X.

Default workload (BASELINE.json configs[1], "config 2"): per GPU, a batch of
1,000,000 files of U[4 KiB, 64 KiB] bytes (~34.8 GB) resident in HBM.  One
step = the whole upload-path signature work for the batch
(fdfs_gpu_sig_batch, FDFS_SIG_HASH: CRC32 + INIT/CALC/FINISH_HASH_CODES4 +
STORAGE_GEN_FILE_SIGNATURE for every file) followed by the bulk dedup of the
step's signatures across all ranks (bucket -> RCCL all-to-all -> group ->
all-to-all back).  Weak scaling: every rank owns its own batch.  The same
line carries "dedup_100m": config 5's 100M-signature dedup split over the
run's ranks (strong scaling), so the 1/2/4/8-GPU runs of the default bench
give the dedup scaling curve too, and "large_file": config 4 (8 x 1 GiB per
GPU, CRC32 only, the segmented crc_seg_kernel) -- the north star's
large-file corpus -- with its own roofline and CPU baseline.

Other workloads: --config c3 (MD5 method, 1-4 MiB files), c4 (1 GiB files,
CRC-only segmented path), c5 (dedup only, 100M signatures, strong scaling).

Prints ONE JSON line on rank 0 (contract in the task statement), with a
"roofline" object for the dominant kernel (its duration measured by HIP
events recorded inside libfdfs_gpu on the launch stream) and a
"cpu_baseline" object (the C oracle of the reference loops on host cores,
over a bounded sample: at most 4 GiB copied to the host, repeated to ~10 s).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import fastdfs_amd as F  # noqa: E402
from fastdfs_amd import _lib, corpus as C  # noqa: E402
from fastdfs_amd.dist import dedup_global  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
VALU_PEAK_TOPS = 78.6  # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz int32 lane-ops/s (1 op/lane/clk)

METRIC = "GB/s CRC32+signature per node; dedup files/sec at 1/2/4/8 MI355X"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c4", "c5"])
    p.add_argument("--files", type=int, default=0, help="override files per GPU")
    p.add_argument("--method", default="", choices=["", "crc", "hash", "md5"],
                   help="override the config's signature method (crc = check_file_duplicate=0)")
    p.add_argument("--align", type=int, default=16,
                   help="file start alignment in the batch buffer (1 = packed back to back)")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="CPU baseline threads (0 = every core this process may run on)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--unsigned-hash", action="store_true")
    p.add_argument("--answers", default="arrays", choices=["arrays", "packed"],
                   help="one-GPU dedup output: rep/ref arrays (fdfs_gpu_dedup) or packed 16-byte "
                        "records (fdfs_gpu_dedup_packed)")
    p.add_argument("--exchange", default="rccl", choices=["rccl", "torch"],
                   help="N>1 dedup exchange: libfdfs_gpu's fdfs_gpu_dedup_global over its own RCCL "
                        "communicator, or the same steps over torch.distributed")
    return p.parse_args()


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    return world, rank, local


def barrier(world):
    if world > 1:
        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def timed(fn, steps, warmup, world):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    return max_over_ranks(time.perf_counter() - t0, world)


COMM = None  # fastdfs_amd.api.Comm of the run (N > 1, --exchange rccl)
PACKED = False  # --answers packed


def dedup_step(ctx, sig, gidx, world, stats=None):
    if world > 1:
        return dedup_global(ctx, sig, gidx, stats=stats, comm=COMM)
    # one GPU holds the whole ingest in order: the ingest index is the
    # position (gidx NULL in fdfs_gpu_dedup, the same answers as arange)
    return ctx.dedup_packed(sig) if PACKED else ctx.dedup(sig)


def cgroup_cpus() -> float | None:
    """CPUs granted by the cgroup v2 quota (cpu.max), or None if unlimited."""
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            return int(quota) / int(period)
    except (OSError, ValueError):
        pass
    return None


def host_threads(args) -> int:
    """Every CPU this process may run on: the affinity set, capped by the
    cgroup quota (a GPU box's share of a larger host shows the whole host in
    its affinity mask)."""
    if args.cpu_threads:
        return args.cpu_threads
    n = len(os.sched_getaffinity(0))
    q = cgroup_cpus()
    if q is None and os.environ.get("OMP_NUM_THREADS", "").isdigit():
        q = int(os.environ["OMP_NUM_THREADS"])  # the share a pool box advertises
    return max(1, min(n, int(q))) if q else n


HOST_SAMPLE_CAP = 4 << 30  # bytes copied to the host for a CPU baseline sample


def host_sample(data, offs_np, sizes_np, budget, threads):
    """The first files of the batch as a host buffer of about `budget` bytes:
    at least min(n, threads) files (one per thread), each file cut to its
    first `cap` bytes when whole files would not fit the budget (1 GiB files:
    the per-byte loop rate does not depend on where a file is cut).  Returns
    (host bytes, offsets, sizes, k files, cap or None)."""
    n = len(sizes_np)
    m = max(1, min(n, threads))
    cap = max(64 << 10, int(budget // m))
    cut = sizes_np[:max(m, 1)].max() > cap
    sz = np.minimum(sizes_np, cap) if cut else sizes_np
    cum = np.cumsum(sz)
    k = int(min(n, max(m, np.searchsorted(cum, budget) + 1)))
    sz = np.asarray(sz[:k], dtype=np.int64)
    if not cut:
        end = int(offs_np[k - 1] + sizes_np[k - 1])
        return data[:end].cpu().numpy(), offs_np[:k], sz, k, None
    parts = [data[int(o):int(o) + int(s)] for o, s in zip(offs_np[:k], sz)]
    host = torch.cat(parts).cpu().numpy()
    offs = np.zeros(k, np.int64)
    offs[1:] = np.cumsum(sz)[:-1]
    return host, offs, sz, k, cap


def cpu_baseline(data, offs_np, sizes_np, method, variant, seconds, threads):
    """The C oracle (restated reference loops, 256 KiB chunks as dio_write_file
    gets them) on a bounded sample of the same batch, `threads` host threads,
    one file per thread at a time.  At most HOST_SAMPLE_CAP
    bytes are copied to the host; a sample shorter than ~`seconds` of work is
    hashed again (`passes`), so the timing covers ~`seconds` either way."""
    from oracle import oracle as O
    O.lib()

    def run(smp, reps):
        host, offs, sz = smp[0], smp[1], smp[2]
        t0 = time.perf_counter()
        for _ in range(reps):
            O.dio_batch(host, offs, sz, method, variant, 256 * 1024, threads)
        return time.perf_counter() - t0, int(sz.sum()) * reps

    n = len(sizes_np)
    budget = 64 << 20
    while True:  # probe until the timing is meaningful
        smp = host_sample(data, offs_np, sizes_np, budget, threads)
        dt, nb = run(smp, 1)
        whole = smp[3] == n and smp[4] is None
        if dt >= 0.5 or whole or budget >= HOST_SAMPLE_CAP:
            break
        budget = min(HOST_SAMPLE_CAP, budget * 4)
    want = nb / dt * seconds  # bytes of ~`seconds` of CPU work
    if want > nb and not whole and budget < HOST_SAMPLE_CAP:
        smp = host_sample(data, offs_np, sizes_np, min(want, HOST_SAMPLE_CAP), threads)
    reps = max(1, int(round(want / max(int(smp[2].sum()), 1))))
    dt, nb = run(smp, reps)
    k, cap = smp[3], smp[4]
    busy = min(threads, k)
    what = f"first {k} files of the rank-0 batch" + (f", each cut to its first {cap >> 20} MiB" if cap else "")
    return {"value": round(nb / dt / 1e9, 4), "unit": "GB/s", "cores": busy, "kind": "port",
            "threads": threads, "host_cpus": len(os.sched_getaffinity(0)), "cgroup_cpus": cgroup_cpus(),
            "sample": f"{what} ({int(smp[2].sum()) / 1e9:.2f} GB host copy) x {reps} pass(es), "
                      f"oracle/fdfs_oracle.c orc_dio_batch, 256 KiB chunks, {threads} threads "
                      f"({busy} with a file), {dt:.1f} s", "cpu_model": cpu_model()}


# The reference's own dedup decision costs at least one synchronous FastDHT
# GET per uploaded file (storage/storage_service.c:2652, fdht_get_ex1), plus
# two SETs on a miss (:2714, :2734) and an INC per link (:2984): MODELLED
# here, not measured (no FastDHT server exists in this pipeline), at a
# same-rack TCP round trip.
FDHT_RTT_US = 100.0


def fdht_model():
    return {"kind": "modelled", "rtt_us": FDHT_RTT_US,
            "files_per_s_per_connection": round(1e6 / FDHT_RTT_US, 1),
            "note": "one synchronous FastDHT GET per file (storage/storage_service.c:2652) per "
                    "dio thread; a miss adds 2 SETs, a link 1 INC (:2714,:2734,:2984)"}


def cpu_dedup_baseline(sig: torch.Tensor, seconds: float, threads: int):
    """The oracle's grouping (hash partition, sort by signature + run
    detection per partition: the CPU form of the FastDHT semantics,
    oracle/fdfs_oracle.c orc_dedup_mt) on `threads` host cores and on one,
    over prefixes of the bench's signatures that double until ~`seconds` of
    CPU work."""
    from oracle import oracle as O

    def rate(nt, budget):
        n, spent, m = 1 << 20, 0.0, 0
        while True:
            m = min(n, sig.shape[0])
            host = sig[:m].cpu().numpy()
            t0 = time.perf_counter()
            O.dedup(host, nt, partitioned=True)
            spent = time.perf_counter() - t0
            if spent * 2.5 > budget or m == sig.shape[0]:
                break
            n *= 2
        return m / spent, m
    r_all, m_all = rate(threads, seconds / 2)
    r_one, m_one = rate(1, seconds / 2)
    return {"value": round(r_all, 1), "unit": "files/s", "cores": threads, "kind": "port",
            "sample": f"first {m_all} of the bench's signatures, oracle/fdfs_oracle.c orc_dedup_mt, "
                      f"{threads} threads ({cpu_model()})",
            "single_thread": {"value": round(r_one, 1), "unit": "files/s",
                              "sample": f"first {m_one} signatures, orc_dedup_mt, 1 thread"},
            "reference_fdht_model": fdht_model()}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_traffic(config: str, kernel: str):
    """HBM bytes per launch from a committed rocprofv3 --pmc pass (see
    profiles/README.md), or None."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    try:
        d = json.load(open(path))
        if d.get("kernel") == kernel:
            return d.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)
    except (OSError, ValueError):
        pass
    return None, None


# name prefixes of the dominant kernels in the pmc_sq files (round 5 dropped
# the probe-mode template parameters: sig_hash_kernel<true, false>)
SQ_KERNEL = {"c2": ("sig_hash_kernel<true, false>", "sig_hash_kernel<true, 0, 0"), "c3": ("md5_pair_kernel<true",)}


def load_valu(config: str, avg_ms: float):
    """VALU issue of the dominant kernel: SQ_INSTS_VALU per launch from the
    newest committed rocprofv3 --pmc pass (profiles/r06, else r05, r04, r03, r02,
    r01, pmc_sq_<config>.txt; the count does not depend on timing) over the
    live kernel time, in int32 lane-ops/s against VALU_PEAK_TOPS."""
    for rnd in ("r06", "r05", "r04", "r03", "r02", "r01"):
        path = os.path.join(ROOT, "profiles", rnd, f"pmc_sq_{config}.txt")
        try:
            for line in open(path):
                name, _, js = line.partition(" {")
                if config in SQ_KERNEL and name.strip().startswith(SQ_KERNEL[config]):
                    insts = json.loads("{" + js)["SQ_INSTS_VALU"]
                    tops = insts * 64 / (avg_ms * 1e-3) / 1e12
                    return {"insts_per_launch": round(insts), "achieved_tops": round(tops, 2),
                            "peak_tops": VALU_PEAK_TOPS, "frac": round(tops / VALU_PEAK_TOPS, 4),
                            "source": os.path.relpath(path, ROOT)}
        except (OSError, ValueError, KeyError):
            pass
    return None


def peer_bytes(ctx, sig, gidx, world):
    """Bytes this rank sends to other ranks in one global dedup (one untimed
    call): (rows, answers).  libfdfs_gpu's exchange reports them itself
    (fdfs_gpu_dedup_global_stats: the 32-byte rows for other owners, and the
    16-byte answer records of multi-member classes it returns to their
    senders); the torch form sends 32 B per row out and 16 B per row back."""
    if world == 1:
        return 0.0, 0.0
    stats = {}
    dedup_step(ctx, sig, gidx, world, stats=stats)
    torch.cuda.synchronize()
    return float(stats.get("row_bytes", 0)), float(stats.get("answer_bytes", 0))


def dedup_strong(ctx, sig, gidx, world, steps, warmup):
    """Timed dedup steps over one signature set (all ranks): (seconds for
    `steps`, mean ms of the rank's dedup_group kernels, bytes all ranks sent
    to peers per step over xGMI)."""
    ctx.reserve(0, 2 * sig.shape[0])
    ctx.set_timing(True)
    ctx.read_timing(_lib.KERNEL_DEDUP)
    dt = timed(lambda: dedup_step(ctx, sig, gidx, world), steps, warmup, world)
    kms, launches = ctx.read_timing(_lib.KERNEL_DEDUP)
    ctx.set_timing(False)
    rows, answers = peer_bytes(ctx, sig, gidx, world)
    peer = {"rows": sum_over_ranks(rows, world), "answers": sum_over_ranks(answers, world)}
    return dt, kms / max(launches, 1), peer


METHODS = {"crc": F.SIG_CRC_ONLY, "hash": F.SIG_HASH, "md5": F.SIG_MD5}
KERNEL_OF = {F.SIG_CRC_ONLY: (_lib.KERNEL_CRC_SEG, "crc_seg_kernel<SAR>"),
             F.SIG_HASH: (_lib.KERNEL_SIG_LANE, "sig_hash_kernel<SAR>"),
             F.SIG_MD5: (_lib.KERNEL_SIG_LANE, "md5_pair_kernel<SAR>")}


def chain_floor_ms(ctx, data, offs_t, sizes_t, sizes, method, kernel, alone=False):
    """The lane-serial floor of a lane-per-file batch: the same kernel over
    a batch holding the batch's largest file (one lane, one dependent chain:
    MD5 / ELFHash have no intra-file parallel form), timed by the library's
    HIP events on the launch stream.  The largest file goes in with as many
    empty files as keep the batch above the library's small-batch threshold
    (one wave per SIMD, CUs x 256 files) when the real batch is above it, so
    the file takes the path it takes in the batch (config 3: CRC fused into
    its MD5 lane); alone=True times it as a one-file batch (config 3: the
    small-batch path moves its CRC to the segmented kernel, the MD5 chain
    alone)."""
    k = int(np.argmax(sizes))
    lat = torch.cuda.get_device_properties(data.device).multi_processor_count * 256
    pad = lat if (len(sizes) > lat and not alone) else 0
    o1 = torch.cat([offs_t[k:k + 1], offs_t[k:k + 1].expand(pad)]).contiguous()
    s1 = torch.cat([sizes_t[k:k + 1], torch.zeros(pad, dtype=sizes_t.dtype, device=sizes_t.device)]).contiguous()
    ctx.sig_batch(data, o1, s1, method=method, check_bounds=False)
    torch.cuda.synchronize()
    ctx.set_timing(True)
    ctx.read_timing(kernel)
    for _ in range(2):
        ctx.sig_batch(data, o1, s1, method=method, check_bounds=False)
    ms, cnt = ctx.read_timing(kernel)
    ctx.set_timing(False)
    return ms / max(cnt, 1), int(sizes[k])


CLOCK_MAX_GHZ = 2.4  # MI355X_MICROARCH.md: peak engine clock
SIMDS_PER_CU = 4


def load_chain_ubench():
    """Per-lane dependent-chain cost and per-SIMD throughput of the two
    byte-serial recurrences (scripts/ubench/chain_ubench.hip, data in
    registers, the library's own device code), from the newest committed
    run (profiles/r06/chain_ubench.json), or None."""
    path = os.path.join(ROOT, "profiles", "r06", "chain_ubench.json")
    try:
        runs = json.load(open(path))["runs"]
    except (OSError, ValueError, KeyError):
        return None
    out = {"source": os.path.relpath(path, ROOT)}
    for k in ("md5", "elf4", "elfc"):
        rs = [r for r in runs if r["kernel"] == k]
        if not rs:
            return None
        lat = min(rs, key=lambda r: r["waves_per_simd"])
        out[k] = {"cycles_per_byte_lane": lat["cycles_per_byte_lane"],
                  "simd_bytes_per_cycle": max(r["simd_bytes_per_cycle"] for r in rs),
                  "clock_ghz_measured": lat["clock_ghz"]}
    # One chain alone with its operands made by another wave
    # (scripts/ubench/chain_lds_ubench.hip: md5k = the K + m sums given,
    # elfb = the bytes one per dword): the fastest single chain the hardware
    # shows, so the largest file's term is priced with it
    lds = os.path.join(ROOT, "profiles", "r06", "chain_lds_ubench.json")
    try:
        lruns = {r["kernel"]: r for r in json.load(open(lds))["runs"]}
        for k, alt in (("md5", "md5k"), ("elf4", "elfb"), ("elfc", "elfb")):
            if alt in lruns and lruns[alt]["cycles_per_byte_lane"] < out[k]["cycles_per_byte_lane"]:
                out[k].update(cycles_per_byte_lane=lruns[alt]["cycles_per_byte_lane"],
                              clock_ghz_measured=lruns[alt]["clock_ghz"], lat_form=alt)
        out["source"] += " + " + os.path.relpath(lds, ROOT)
    except (OSError, ValueError, KeyError):
        pass
    return out


def chain_roof(method, sizes, ncu, kernel_ms):
    """The hardware roof of a lane-per-file batch whose signature is a
    byte-serial chain (MD5 / ELFHash: no intra-file parallel form): the
    batch cannot end before its largest file's chain (that file's bytes x
    the chain's cycles per byte on one lane) nor before every SIMD has
    issued its share of the chain work (total bytes / the SIMD's best
    bytes per cycle), both at the peak engine clock, with the cycle counts
    measured by the chain microbenchmark.  Upper bounds: the data sits in
    registers there and the CRC and the other hashes are not counted.  The
    per-lane term takes the fastest single chain measured, operands prepared
    by another wave included (load_chain_ubench)."""
    ub = load_chain_ubench()
    if ub is None:
        return None
    # sig_hash_kernel's big-file lanes (>= 4 MiB) run ELF in the 3-op chain
    # form, its other lanes the asm 4-VALU form; md5_pair_kernel: MD5
    big = method == F.SIG_HASH and int(sizes.max()) >= (4 << 20)
    c = ub["md5"] if method == F.SIG_MD5 else ub["elfc" if big else "elf4"]
    f = CLOCK_MAX_GHZ * 1e9
    t_lat = float(sizes.max()) * c["cycles_per_byte_lane"] / f
    t_thr = float(sizes.sum()) / (ncu * SIMDS_PER_CU * c["simd_bytes_per_cycle"] * f)
    t = max(t_lat, t_thr)
    return {"bound": "md5_chain" if method == F.SIG_MD5 else "elf_chain",
            "peak": round(float(sizes.sum()) / t / 1e9, 3), "frac": round(t * 1e3 / kernel_ms, 4),
            "roof_ms": round(t * 1e3, 3), "roof_term": "largest file's chain" if t_lat >= t_thr else "SIMD issue",
            "chain_cycles_per_byte_lane": c["cycles_per_byte_lane"], "chain_form": c.get("lat_form", "in-lane"),
            "simd_bytes_per_cycle": c["simd_bytes_per_cycle"], "clock_ghz": CLOCK_MAX_GHZ,
            "ubench_clock_ghz": c["clock_ghz_measured"], "ubench_source": ub["source"]}


def c1_sizes(rank):
    """test/test_upload.c:32-39 (DEBUG): 65,560 files / 3,889,152,000 B of
    the six gen_files sizes, in a seeded random order."""
    mix = [(5 << 10, 50000), (50 << 10, 10000), (200 << 10, 5000), (1 << 20, 500),
           (10 << 20, 50), (100 << 20, 10)]
    sizes = np.concatenate([np.full(c, sz, np.int64) for sz, c in mix])
    return sizes[np.random.default_rng(1 + 1000 * rank).permutation(sizes.size)]


C1_WORKLOAD = "config 1: test_upload DEBUG mix (gen_files sizes 5K..100M, 65,560 files)"


def c4_sizes(n):
    return np.full(n, 1 << 30, dtype=np.int64)


def c4_workload(n):
    return f"config 4: {n} x 1 GiB files/GPU, segmented CRC32 (128 KiB segments) + GF(2) combine"


def batch_line(args, ctx, world, rank, dev, config, sizes, method, workload, steps, warmup, threads,
               variant, traffic_ok):
    """One signature workload (configs 1-4): a batch per rank resident in
    HBM, `steps` timed steps of fdfs_gpu_sig_batch (+ the global dedup of the
    step's signatures when the method makes them); the dominant kernel's
    mean duration from the library's HIP events on its launch stream; the
    CPU baseline on rank 0 at N = 1.  The batch is freed on return."""
    n = len(sizes)
    kernel, kname = KERNEL_OF[method]
    if method == F.SIG_CRC_ONLY and n > ctx.crc_lane_min_files():
        # fdfs_gpu_sig_batch's lane path (more than 3 waves per SIMD of files)
        kname = "crc_lane_kernel<SAR> (+ crc_seg_kernel<SAR> for files >= 96 KiB)"
    workload += {F.SIG_CRC_ONLY: ", CRC32 only (check_file_duplicate=0)",
                 F.SIG_HASH: ", CRC32 + HASH_CODES4 signature + bulk dedup per step",
                 F.SIG_MD5: ", CRC32 + MD5 signature + bulk dedup per step"}[method]
    if config == "c4" and method == F.SIG_CRC_ONLY:
        workload = workload.split(", CRC32 only")[0] + ", CRC32 only (check_file_duplicate=0, the default)"
    data, offs_t, sizes_t = C.device_batch(sizes, seed=2 + 1000 * rank, device=dev, align=args.align)
    nbytes = int(sizes.sum())
    gidx = (torch.arange(n, device=dev, dtype=torch.int64) + rank * n)
    ctx.reserve(n, n)

    def step():
        crc, sig, _ = ctx.sig_batch(data, offs_t, sizes_t, method=method, check_bounds=False)
        if sig is not None:
            dedup_step(ctx, sig, gidx, world)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    ctx.set_timing(True)
    ctx.read_timing(kernel)
    dt = timed(step, steps, 0, world)
    kms, launches = ctx.read_timing(kernel)
    ctx.set_timing(False)
    total_bytes = sum_over_ranks(float(nbytes), world) * steps
    out = {"value": round(total_bytes / dt / 1e9, 3), "unit": "GB/s",
           "ms_per_step": round(dt / steps * 1e3, 3), "scaling": "weak",
           "files_per_s": round(sum_over_ranks(float(n), world) * steps / dt, 1)}
    avg_ms = kms / max(launches, 1)
    per_launch = float(nbytes)  # each file byte read once; 28 B/file of outputs on top
    achieved = per_launch / (avg_ms * 1e-3) / 1e9
    traffic, tsrc = load_traffic(config, kname) if traffic_ok else (None, None)
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic, "kernel": kname,
            "kernel_ms_avg": round(avg_ms, 4), "launches": launches,
            "algorithmic_bytes_per_launch": nbytes}
    if tsrc:
        roof["traffic_source"] = tsrc
    if config == "c2" and method == F.SIG_HASH:
        roof["note"] = ("below the HBM roof: the hash step is bound by VALU issue (ELF 4 VALU per byte, "
                        "the CRC's lane fold 1.5) at the ~1.6-1.75 of 2.4 GHz the chip holds under this "
                        "load; DESIGN.md 4.2, profiles/r05/issue_clock_c2.txt, profiles/r05/lane_fold_ab.txt")
    if config in ("c1", "c3", "c4") and method != F.SIG_CRC_ONLY:
        # lane-per-file batches whose dependent chains (MD5 / ELFHash)
        # outlast the HBM stream: the roof is the chain's hardware cost
        # (chain_roof); the largest file timed alone on
        # the batch's own path stays beside it as a second figure
        fms, fbytes = chain_floor_ms(ctx, data, offs_t, sizes_t, sizes, method, kernel)
        hw = chain_roof(method, sizes, torch.cuda.get_device_properties(dev).multi_processor_count, avg_ms)
        roof.update({"hbm_frac": round(achieved / HBM_PEAK_GBS, 4),
                     "chain_floor_ms": round(fms, 3), "chain_floor_file_bytes": fbytes,
                     "chain_floor_frac": round(fms / avg_ms, 4),
                     "chain_floor_note": "the same kernel over a batch holding the largest file "
                                         "alone on the path it takes in the batch (one lane's serial "
                                         "chain; the other files of that timing batch are empty)"})
        if hw:
            roof.update(hw)
        else:  # no committed microbenchmark run: the round-5 self-referential roof
            roof.update({"bound": "md5_chain" if method == F.SIG_MD5 else "elf_chain",
                         "peak": round(per_launch / (fms * 1e-3) / 1e9, 1), "frac": round(fms / avg_ms, 4)})
        if method == F.SIG_MD5 and config != "c4":
            ams, _ = chain_floor_ms(ctx, data, offs_t, sizes_t, sizes, method, kernel, alone=True)
            roof["md5_alone_floor_ms"] = round(ams, 3)
            roof["md5_alone_note"] = ("the largest file as a one-file batch: its CRC moves to the "
                                      "segmented kernel and the lane runs MD5 alone")
    out["roofline"] = roof
    valu = load_valu(config, avg_ms) if not args.method else None
    if valu:
        out["valu"] = valu
    if method != F.SIG_CRC_ONLY:
        # dedup-only throughput of the same signatures (files/s, all ranks)
        _, sig, _ = ctx.sig_batch(data, offs_t, sizes_t, method=method, check_bounds=False)
        ddt = timed(lambda: dedup_step(ctx, sig, gidx, world), steps, 1, world)
        out["dedup_files_per_s"] = round(sum_over_ranks(float(n), world) * steps / ddt, 1)
        del sig
    out["config"] = {"workload": workload, "files_per_gpu": n, "bytes_per_gpu": nbytes,
                     "method": {0: "crc_only", 1: "hash", 2: "md5"}[method],
                     "crc_variant": "unsigned" if variant else "signed", "align": args.align,
                     "parallelism": f"dp{world} (files sharded, dedup all-to-all)"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        offs_np = C.layout(sizes, args.align)[0]
        cb = cpu_baseline(data, offs_np, sizes, method, variant, args.cpu_seconds, threads)
        one = cpu_baseline(data, offs_np, sizes, method, variant, args.cpu_seconds / 2, 1)
        cb["single_thread"] = {k: one[k] for k in ("value", "unit", "sample")}
        # the GPU line over the CPU line, so a reader sees at once where the
        # host's cores would win (ratio < 1)
        cb["gpu_over_cpu"] = round(out["value"] / cb["value"], 2) if cb["value"] else None
        out["cpu_baseline"] = cb
    else:
        out["cpu_baseline"] = None
    del data, offs_t, sizes_t, gidx
    torch.cuda.empty_cache()
    return out


def rccl_exchange_check(ctx, world, rank, dev):
    """N > 1: set up libfdfs_gpu's RCCL communicator and check that
    fdfs_gpu_dedup_global gives every rank the same answers as the
    torch.distributed form of the exchange on a seeded 200K-record set with
    duplicates across ranks.  All ranks share their outcome (mismatching
    records per rank, all-gathered) before the timed run.  A failure or a
    mismatch anywhere is printed on stderr by rank 0 with the ranks and
    record counts, and every rank then exits non-zero: a multi-GPU line is
    fdfs_gpu_dedup_global's or none (no silent fallback to another
    transport).  Returns (Comm, the check's record for the JSON line)."""
    from fastdfs_amd.api import Comm
    comm, why, bad, mine = None, "ok", 0, 0
    try:
        comm = Comm(ctx)
        g = torch.Generator(device="cpu").manual_seed(97)
        base = torch.randint(0, 256, (150_000, 24), dtype=torch.uint8, generator=g)
        pick = torch.randint(0, base.shape[0], (200_000,), generator=g)
        per = (200_000 + world - 1) // world
        lo, hi = rank * per, min(200_000, (rank + 1) * per)
        mine = hi - lo
        sig = base[pick[lo:hi]].contiguous().to(dev)
        gidx = torch.arange(lo, hi, dtype=torch.int64, device=dev)
        rep_a, ref_a = dedup_global(ctx, sig, gidx, comm=comm)
        rep_b, ref_b = dedup_global(ctx, sig, gidx, comm=None)
        torch.cuda.synchronize()
        bad = int(((rep_a != rep_b) | (ref_a != ref_b)).sum().item())
        if bad:
            why = "mismatch"
    except Exception as e:  # noqa: BLE001 - reported in the JSON line
        why = f"error: {e}"[:200]
        bad = -1
    # every rank's outcome: (mismatching records or -1 on an error, records)
    out = torch.tensor([bad, mine], dtype=torch.int64, device=dev)
    allv = [torch.empty_like(out) for _ in range(world)]
    dist.all_gather(allv, out)
    per_rank = [tuple(int(x) for x in v.cpu().tolist()) for v in allv]
    if all(b == 0 for b, _ in per_rank):
        return comm, {"records": 200_000, "vs_torch_exchange": "equal"}
    if comm is not None:
        comm.close()
    failed = {r: ("error" if b < 0 else f"{b} of {m} records differ") for r, (b, m) in enumerate(per_rank) if b}
    if rank == 0:
        print("=" * 72 + "\nERROR: fdfs_gpu_dedup_global (RCCL) disagrees with the torch.distributed "
              f"exchange: {failed} (rank 0: {why}).\nNo line is printed: the multi-GPU dedup must be "
              "libfdfs_gpu's.\n" + "=" * 72, file=sys.stderr, flush=True)
    ctx.close()
    dist.destroy_process_group()
    sys.exit(3)


def main():
    args = parse()
    world, rank, local = setup_dist(args)
    dev = torch.device("cuda", local)
    ctx = F.Context(local, unsigned_hash=args.unsigned_hash)
    global COMM, PACKED
    PACKED = args.answers == "packed"
    rccl_check = None
    if world > 1 and args.exchange == "rccl":
        COMM, rccl_check = rccl_exchange_check(ctx, world, rank, dev)
    variant = 1 if args.unsigned_hash else 0
    threads = host_threads(args)
    res = {"metric": METRIC, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "higher_is_better": True, "vs_baseline": None, "dtype": "u8",
           "data": "synthetic (seeded sizes, random bytes generated in HBM)"}

    if args.config in ("c1", "c2", "c3", "c4"):
        if args.config == "c1":
            sizes = c1_sizes(rank)
            method = F.SIG_HASH
            workload = C1_WORKLOAD
        elif args.config == "c2":
            sizes = C.small_files_sizes(args.files or 1_000_000, seed=1 + 1000 * rank)
            method = F.SIG_HASH
            workload = "config 2: 1M files/GPU of U[4,64] KiB"
        elif args.config == "c3":
            n = args.files or 100_000  # the full config (~262 GB resident in HBM)
            sizes = C.photo_sizes(n, seed=3 + 1000 * rank)
            method = F.SIG_MD5
            workload = f"config 3: {n} files/GPU of U[1,4] MiB"
        else:
            sizes = c4_sizes(args.files or 8)
            method = F.SIG_CRC_ONLY
            workload = c4_workload(len(sizes))
        if args.method:
            method = METHODS[args.method]
        res.update(batch_line(args, ctx, world, rank, dev, args.config, sizes, method, workload,
                              args.steps, args.warmup, threads, variant,
                              traffic_ok=args.align == 16 and not args.method))
        if args.config == "c2" and not args.files and not args.method and args.align == 16:
            # configs 3 and 1 ride along, each with its
            # own steps, roofline (the chain roof, hbm_frac beside it) and CPU
            # baseline; config 3's 262 GB batch runs first, before the 100M
            # dedup below reserves its workspace
            keys = ("value", "unit", "ms_per_step", "scaling", "files_per_s", "roofline", "cpu_baseline",
                    "dedup_files_per_s", "config")
            ph = batch_line(args, ctx, world, rank, dev, "c3", C.photo_sizes(100_000, seed=3 + 1000 * rank),
                            F.SIG_MD5, "config 3: 100000 files/GPU of U[1,4] MiB", min(args.steps, 3), 1,
                            threads, variant, traffic_ok=True)
            res["photos"] = {k: ph[k] for k in keys if k in ph}
            um = batch_line(args, ctx, world, rank, dev, "c1", c1_sizes(rank), F.SIG_HASH, C1_WORKLOAD,
                            min(args.steps, 3), 1, threads, variant, traffic_ok=True)
            res["upload_mix"] = {k: um[k] for k in keys if k in um}
            # config 5's 100M-record dedup, strong-scaled over the ranks of
            # this run: the driver's 1/2/4/8-GPU runs of the default bench
            # give its scaling curve
            total = 100_000_000
            sig5, gidx5 = C.c5_signatures(total, world, rank, dev)
            st5 = min(args.steps, 5)
            ddt, dms, peer = dedup_strong(ctx, sig5, gidx5, world, st5, 1)
            res["dedup_100m"] = {"files_per_s": round(total * st5 / ddt, 1),
                                 "ms_per_step": round(ddt / st5 * 1e3, 3), "records_total": total,
                                 "scaling": "strong", "group_kernel_ms_avg": round(dms, 4),
                                 "workload": "config 5 (10% duplicates), bucket + RCCL all-to-all + group"}
            if world > 1:
                tot = peer["rows"] + peer["answers"]
                res["dedup_100m"]["xgmi_bytes_per_step"] = round(tot)
                res["dedup_100m"]["xgmi_row_bytes_per_step"] = round(peer["rows"])
                res["dedup_100m"]["xgmi_answer_bytes_per_step"] = round(peer["answers"])
                res["dedup_100m"]["xgmi_gbs"] = round(tot / (ddt / st5) / 1e9, 1)
            del sig5, gidx5
            torch.cuda.empty_cache()
            # the north star's large-file corpus (config 4: 8 x 1 GiB per
            # GPU, CRC32 only -- the upload path's default with
            # check_file_duplicate=0 -- crc_seg_kernel), weak-scaled like the
            # main line, with its own roofline and CPU baseline
            lf = batch_line(args, ctx, world, rank, dev, "c4", c4_sizes(8), F.SIG_CRC_ONLY,
                            c4_workload(8), min(args.steps, 10), 2, threads, variant, traffic_ok=True)
            res["large_file"] = {k: lf[k] for k in ("value", "unit", "ms_per_step", "scaling", "files_per_s",
                                                    "roofline", "cpu_baseline", "config")}
    else:  # c5: dedup only, strong scaling over a fixed 100M-signature set
        total = args.files or 100_000_000
        sig, gidx = C.c5_signatures(total, world, rank, dev)
        dt, avg_ms, peer = dedup_strong(ctx, sig, gidx, world, args.steps, args.warmup)
        res.update({"metric": METRIC, "value": round(total * args.steps / dt, 1),
                    "unit": "files/s", "ms_per_step": round(dt / args.steps * 1e3, 3),
                    "scaling": "strong",
                    "config": {"workload": "config 5: 100M-file dedup, 10% duplicates, "
                                           "bucket + RCCL all-to-all + hash grouping",
                               "records_total": total, "parallelism": f"dp{world}",
                               "answers": ("fdfs_gpu_dedup_packed (16-byte {rep, ref} records)" if PACKED
                                           else "fdfs_gpu_dedup (rep u64[n] + ref u32[n])") if world == 1
                               else "fdfs_gpu_dedup_global (rep u64[n] + ref u32[n])"}})
        if world > 1:  # all ranks' bytes to peers per step, over the step time
            tot = peer["rows"] + peer["answers"]
            res["xgmi"] = {"bytes_per_step": round(tot), "row_bytes_per_step": round(peer["rows"]),
                           "answer_bytes_per_step": round(peer["answers"]),
                           "gbs": round(tot / (dt / args.steps) / 1e9, 1),
                           "links_peak_gbs": 7 * 153.0 * world}
        # algorithmic bytes per record: one GPU reads the 24-byte signature
        # and writes rep (8 B) + ref (4 B); N GPUs group the 32-byte exchange
        # rows {sig, gidx} instead
        m = float(total) / world
        per_rec = 36.0 if world == 1 else 44.0
        nb = m * per_rec
        res["roofline"] = {"bound": "hbm", "achieved": round(nb / (avg_ms * 1e-3) / 1e9, 1),
                           "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": round(nb / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                           "traffic": None,
                           "kernel": "dedup_group (dp_tile + scan + chunks + dp_split + dp_group)",
                           "kernel_ms_avg": round(avg_ms, 4), "algorithmic_bytes_per_launch": nb,
                           "algorithmic_bytes_per_record": per_rec}
        if world == 1:
            traffic, tsrc = load_traffic("c5", res["roofline"]["kernel"])
            if traffic:
                res["roofline"]["traffic"] = traffic
                res["roofline"]["traffic_source"] = tsrc
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_dedup_baseline(sig, args.cpu_seconds, threads)
        else:
            res["cpu_baseline"] = None
    if rccl_check is not None:
        res.setdefault("config", {})["rccl_check"] = rccl_check
    if world > 1:
        res.setdefault("config", {})["dedup_exchange"] = (
            "fdfs_gpu_dedup_global (libfdfs_gpu, RCCL send/recv)" if COMM is not None
            else "torch.distributed all_to_all_single")
    if rank == 0:
        print(json.dumps(res), flush=True)
    if COMM is not None:
        COMM.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
