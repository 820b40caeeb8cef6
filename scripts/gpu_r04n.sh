# Round 4 (probe build): is config 2's "overlap loss" a clock effect?
#  1. shader clock beside back-to-back config-2 batches in production form
#     (HASH_MODE 0), loads only (1) and compute only (2);
#  2. SQ counters (waits, VALU issue, busy) and GRBM_GUI_ACTIVE for the
#     same three modes, one --pmc pass each.
export TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
export FDFS_GPU_PROBE_LIB=1
step idle 60 scripts/probes/clock_probe 5 200 20 || exit $?
for m in 0 1 2; do
  FDFS_GPU_HASH_MODE=$m step clock_m$m 200 python3 scripts/clock_under_load.py c2 10 || exit $?
  echo "m$m $(grep -v sample $O/clock_m$m.log | tr '\n' ' ') $(grep sample $O/clock_m$m.log | awk '{print $3}' | sort -n | awk '{a[NR]=$1} END {print "n", NR, "min", a[1], "median", a[int(NR/2)+1], "max", a[NR]}')"
done
B2="python3 bench.py --no-cpu-baseline --steps 1 --warmup 1"
SQ="GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS"
for m in 0 1 2; do
  FDFS_GPU_HASH_MODE=$m step sq_m$m 300 timeout -s KILL 240 rocprofv3 --pmc $SQ -d $O/sq_m$m -o run --output-format csv -- $B2 || exit $?
done
for m in 0 1 2; do
  FDFS_GPU_HASH_MODE=$m step bench_m$m 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 || exit $?
  echo "m$m $(grep -o '"kernel_ms_avg": [0-9.]*' $O/bench_m$m.log)"
done
