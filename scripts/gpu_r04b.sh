# Round 4: config 3 CRC offload of the largest files (probe build knobs):
# sequential, side stream first, side stream after the pair kernel (low prio).
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
B="python3 bench.py --config c3 --no-cpu-baseline --steps 5 --warmup 2"
show() { echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $O/$1.log) $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
export FDFS_GPU_PROBE_LIB=1
FDFS_GPU_MD5_PAIR=6 step pair_timeline 600 python3 -u scripts/pair_timeline.py --reps 2 --out $O/pairs.npz || exit $?
for cfg in "0 0" "688 0" "688 1" "688 2" "0 0" "696 2" "680 2" "672 2" "0 0"; do
  set -- $cfg
  FDFS_GPU_MD5_T_BIN=$1 FDFS_GPU_SIDE=$2 step c3_t$1_s$2 400 $B || exit $?
  show c3_t$1_s$2
done
