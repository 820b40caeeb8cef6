# Round 4: config 2 loads-alone / compute-alone probes of the pair-load kernel
# (the compute-only mode skips the pair loads since this round's last fix).
export TMPDIR=/tmp
O=gpurun_out/round_r04ze
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
B="python3 bench.py --no-cpu-baseline"
for m in 1 2; do
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_HASH_MODE=$m step probe_c2_mode$m 300 $B || exit $?
  grep -o '"kernel_ms_avg": [0-9.]*' $O/probe_c2_mode$m.log
done
step bench_c2 300 $B || exit $?
grep -o '"kernel_ms_avg": [0-9.]*' $O/bench_c2.log
