# Round 3: every GPU test, the graph dumps (production zeroing kernels and
# round 2's memset zeroing, probe build), the default bench line and c5.
export TMPDIR=/tmp
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -le 1 ] || exit $rc
FDFS_GPU_PROBE_LIB=1 timeout -k 10 120 python3 scripts/graph_memset_probe.py $O/graph_kernel_zero.dot > $O/graph.log 2>&1 || exit $?
FDFS_GPU_PROBE_LIB=1 FDFS_GPU_MEMSET=1 timeout -k 10 120 python3 scripts/graph_memset_probe.py $O/graph_memset.dot >> $O/graph.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py > $O/bench_c2.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py --config c5 --steps 5 --warmup 1 > $O/bench_c5.log 2>&1 || exit $?
for c in c2 c5; do tail -1 $O/bench_$c.log | cut -c1-400; done
exit $rc
