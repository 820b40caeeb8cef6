#!/bin/bash
# Chunked-path sweep: production library (offload threshold chosen by
# big_plan_kernel for small batches, also captured in a hipGraph) against the
# probe build held at the fixed thresholds (FDFS_GPU_LAT_FILES=0), plus the
# lane-path parity tests and the config-3 (MD5) bench line.
# Usage: bash scripts/gpu_chunk_ab.sh [sweep args]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_sig.py tests/test_gpu_stream.py > gpurun_out/chunk_tests.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/chunk_sweep.py "$@" > gpurun_out/chunk_adaptive.txt 2>&1 || exit 1
FDFS_GPU_PROBE_LIB=1 FDFS_GPU_LAT_FILES=0 timeout -k 10 200 python -u scripts/chunk_sweep.py --graph 0 "$@" \
    > gpurun_out/chunk_fixed.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config c3 --steps 5 --no-cpu-baseline > gpurun_out/chunk_bench_c3.txt 2>&1 || exit 1
