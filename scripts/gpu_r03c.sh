# Round 3: repeated-state test, graph node dumps (kernel zeroing vs memset
# zeroing), the default bench line, then hash CRC table A/B (probe build:
# TM 0 = slice-by-16 byte tables, TM 3 = rotated conflict-free rep8 + quad loads), c5.
export TMPDIR=/tmp
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stream.py -m gpu -v -k repeated --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
FDFS_GPU_PROBE_LIB=1 timeout -k 10 120 python3 scripts/graph_memset_probe.py $O/graph_kernel_zero > $O/graph.log 2>&1
FDFS_GPU_PROBE_LIB=1 FDFS_GPU_MEMSET=1 timeout -k 10 120 python3 scripts/graph_memset_probe.py $O/graph_memset >> $O/graph.log 2>&1
tail -2 $O/graph.log | cut -c1-600
timeout -k 10 600 python3 bench.py > $O/bench_c2.log 2>&1 || exit $?
tail -1 $O/bench_c2.log | cut -c1-300
for r in 1 2; do
  for tm in 0 3; do
    FDFS_GPU_PROBE_LIB=1 FDFS_GPU_HASH_TM=$tm timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 > $O/ab_tm${tm}_$r.log 2>&1 || exit $?
    echo "tm=$tm r=$r $(tail -1 $O/ab_tm${tm}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms_avg"], d["roofline"]["frac"])')"
  done
done | tee $O/ab.txt
timeout -k 10 600 python3 bench.py --config c5 --steps 5 --warmup 1 > $O/bench_c5.log 2>&1 || exit $?
tail -1 $O/bench_c5.log | cut -c1-300
exit $rc
