# Round 4 (probe build): config 2 power ablations.  The production kernel
# runs at ~2.0 GHz while its loads alone or its compute alone hold 2.4 GHz
# (r04n): which part of the compute costs the clock?  HASH_MODE 9 = no MFMA
# planes, 10 = no ELF, 11 = no CRC (all wrong results), 0 = production:
# shader clock beside back-to-back batches, then the kernel time.
export TMPDIR=/tmp
O=gpurun_out/r04o
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
export FDFS_GPU_PROBE_LIB=1
for m in 0 9 10 11; do
  FDFS_GPU_HASH_MODE=$m step clock_m$m 200 python3 scripts/clock_under_load.py c2 8 || exit $?
  FDFS_GPU_HASH_MODE=$m step bench_m$m 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 || exit $?
  echo "m$m $(grep -o '"kernel_ms_avg": [0-9.]*' $O/bench_m$m.log) $(grep sample $O/clock_m$m.log | awk '{print $3}' | sort -n | awk '{a[NR]=$1} END {print "clock n", NR, "min", a[1], "median", a[int(NR/2)+1], "max", a[NR]}')"
done
