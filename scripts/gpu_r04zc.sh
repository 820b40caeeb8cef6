# Round 4: config-2 evidence of the final hash kernel (pair-cooperative loads):
# the default bench line, rocprofv3 kernel stats, FETCH/WRITE and SQ passes,
# and the loads-alone / compute-alone probes, as gpu_round.sh does for c2.
export TMPDIR=/tmp
O=gpurun_out/round_r04zc
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
B="python3 bench.py --no-cpu-baseline"
step bench_c2 600 python3 bench.py || exit $?
tail -1 $O/bench_c2.log | cut -c1-300
step stats_c2 600 rocprofv3 --kernel-trace --stats -d $O/stats_c2 -o run --output-format csv -- $B --steps 10 --warmup 3 || exit $?
find $O -name "*kernel_trace.csv" -size +8M -delete
step fetch_c2 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_c2 -o run --output-format csv -- $B --config c2 --steps 1 --warmup 1 || exit $?
step write_c2 300 rocprofv3 --pmc WRITE_SIZE -d $O/write_c2 -o run --output-format csv -- $B --config c2 --steps 1 --warmup 1 || exit $?
step sq_c2 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $O/sq_c2 -o run --output-format csv -- $B --steps 1 --warmup 1 || exit $?
for m in 1 2; do
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_HASH_MODE=$m step probe_c2_mode$m 300 $B || exit $?
done
echo done
