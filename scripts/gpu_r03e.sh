# Round 3: per-kernel dedup timing, new group form vs round 2's (`make ab`),
# and the graph node listings (kernel zeroing vs memset zeroing).  CSV only.
export TMPDIR=/tmp
O=gpurun_out/r03e; mkdir -p $O
FDFS_GPU_PROBE_LIB=1 timeout -k 10 120 python3 scripts/graph_memset_probe.py $O/graph_kernel_zero > $O/graph.log 2>&1 || exit $?
FDFS_GPU_PROBE_LIB=1 FDFS_GPU_MEMSET=1 timeout -k 10 120 python3 scripts/graph_memset_probe.py $O/graph_memset >> $O/graph.log 2>&1 || exit $?
rm -f $O/*.dot
for lib in new ab; do
  if [ $lib = ab ]; then export FDFS_GPU_PROBE_LIB=ab; else unset FDFS_GPU_PROBE_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_$lib -o run --output-format csv -- python3 bench.py --config c5 --steps 6 --warmup 2 --no-cpu-baseline > $O/stats_$lib.log 2>&1 || exit $?
done
unset FDFS_GPU_PROBE_LIB
find $O -name "*kernel_trace.csv" -delete
for f in $(find $O -name "*kernel_stats.csv"); do echo "== $f"; grep -E "dp_|scan|bucket" $f | cut -d, -f1-4; done
