#!/bin/bash
# CRC-only small-batch latency: the sweep (CRC method) on the production
# library, the CRC/stream parity tests first.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_sig.py tests/test_gpu_stream.py > gpurun_out/crc_small_tests.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/chunk_sweep.py --methods 0 "$@" > gpurun_out/crc_small.txt 2>&1 || exit 1
