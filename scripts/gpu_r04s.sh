# Round 4 (probe build): what the per-step Horner multiply of the MFMA
# accumulators costs config 2 (HASH_MODE 13 skips it: wrong results),
# alternating against production, with the shader clock.
export TMPDIR=/tmp
O=gpurun_out/r04s
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
show() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
clk() { echo "$1 $(grep sample $O/$1.log | awk '{print $3}' | sort -n | awk '{a[NR]=$1} END {print "clock n", NR, "min", a[1], "median", a[int(NR/2)+1], "max", a[NR]}')"; }
export FDFS_GPU_PROBE_LIB=1
B2="python3 bench.py --no-cpu-baseline --steps 10 --warmup 3"
for k in 1 2 3; do
  for m in 0 13; do
    FDFS_GPU_HASH_MODE=$m step c2_m${m}_$k 300 $B2 || exit $?; show c2_m${m}_$k
  done
done
FDFS_GPU_HASH_MODE=13 step clock_m13 200 python3 scripts/clock_under_load.py c2 8 || exit $?; clk clock_m13
