# Small-kernel changes check: lane-path, dedup and format parity tests, then kernel stats of the c2 bench.
export TMPDIR=/tmp
O=gpurun_out/${OUT:-bin}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_sig.py tests/test_gpu_graph.py tests/test_gpu_stream.py tests/test_gpu_dedup.py tests/test_formats.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/stats_c2.log 2>&1 || exit $?
tail -1 $O/stats_c2.log | cut -c1-400
f=$(find $O/stats_c2 -name '*kernel_stats.csv' | head -1); head -30 "$f" | cut -d, -f1-4
