# Round 3 (session 2): dedup group with 32-bit LDS words, four entries per
# thread and a joined-entry list -- dedup parity first, then config 5 new
# (production) vs HEAD (`make ab`), alternating, and a kernel trace.
export TMPDIR=/tmp
O=gpurun_out/r03o; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_dedup.py tests/test_gpu_configs.py tests/test_gpu_graph.py -k "dedup or config5 or graph or index" -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do for lib in new ab; do
  L=; [ $lib = ab ] && L=ab
  for a in arrays packed; do
    FDFS_GPU_PROBE_LIB=$L timeout -k 10 300 python3 bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline --answers $a > $O/c5_${lib}_${a}_$r.log 2>&1 || exit $?
    python3 -c "import json;d=json.loads(open('$O/c5_${lib}_${a}_$r.log').read().strip().split('\n')[-1]);print('$lib $a r=$r', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
  done
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/stats_c5.log 2>&1 || exit $?
find $O -name "*kernel_stats.csv" | xargs -I{} sh -c 'head -12 {}'
# config 3 probes: the pair kernel with no CRC arithmetic (pmode 2) and with no MD5 arithmetic (pmode 3)
for m in 1 3 4; do
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_MD5_PAIR=$m timeout -k 10 300 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_m${m}.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('$O/c3_m${m}.log').read().strip().split('\n')[-1]);print('pair=$m', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline'].get('chain_floor_ms'))"
done
