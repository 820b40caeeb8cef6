# Round 4 (probe build): config 2 is co-bound by VALU issue and the LDS
# (bank conflicts), at a power-limited ~2.0 GHz (r04n, r04o).  The rotated
# conflict-free CRC tables (TM 3: 64 KiB, quad loads) now fit two 512-thread
# workgroups per CU with the compact B: alternating against production (TM 0,
# 256 threads) and TM 3 in 1024-thread workgroups (round 3's form), then the
# clock and LDS counters of TM 3 at 512 against production.
export TMPDIR=/tmp
O=gpurun_out/r04p
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
for k in 1 2; do
  step prod_$k 300 $B2 || exit $?; show prod_$k
  FDFS_GPU_HASH_TM=3 FDFS_GPU_HASH_BLOCK=512 step tm3b512_$k 300 $B2 || exit $?; show tm3b512_$k
  FDFS_GPU_HASH_TM=3 step tm3b1024_$k 300 $B2 || exit $?; show tm3b1024_$k
done
step clock_prod 200 python3 scripts/clock_under_load.py c2 8 || exit $?; clk clock_prod
FDFS_GPU_HASH_TM=3 FDFS_GPU_HASH_BLOCK=512 step clock_tm3 200 python3 scripts/clock_under_load.py c2 8 || exit $?; clk clock_tm3
SQ="GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
step sq_prod 300 timeout -s KILL 240 rocprofv3 --pmc $SQ -d $O/sq_prod -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 || exit $?
FDFS_GPU_HASH_TM=3 FDFS_GPU_HASH_BLOCK=512 step sq_tm3 300 timeout -s KILL 240 rocprofv3 --pmc $SQ -d $O/sq_tm3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 || exit $?
