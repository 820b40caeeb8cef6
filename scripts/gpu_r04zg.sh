# Round 4 (probe build): is config 3 power-limited too?  Shader clock beside
# back-to-back config-3 batches and the kernel time, for the production pair
# kernel (FDFS_GPU_MD5_PAIR=1) and without its CRC arithmetic (=3, PM 2:
# wrong CRCs), alternating.
export TMPDIR=/tmp
O=gpurun_out/r04zg
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
clk() { echo "$1 $(grep sample $O/$1.log | awk '{print $3}' | sort -n | awk '{a[NR]=$1} END {print "clock n", NR, "min", a[1], "median", a[int(NR/2)+1], "max", a[NR]}')"; }
show() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log | head -1)"; }
export FDFS_GPU_PROBE_LIB=1
B3="python3 bench.py --config c3 --no-cpu-baseline --steps 3 --warmup 1"
for p in 1 3; do
  FDFS_GPU_MD5_PAIR=$p step clock_p$p 200 python3 scripts/clock_under_load.py c3 12 || exit $?; clk clock_p$p
  FDFS_GPU_MD5_PAIR=$p step c3_p$p 300 $B3 || exit $?; show c3_p$p
done
