# Round 4, fifth box:
#  1. md5_pair_kernel PM 8 (probe FDFS_GPU_MD5_PAIR=9: static boustrophedon
#     chunk pairing, priority over the pair's remaining rounds): MD5 parity,
#     then config 3 alternating against production (PAIR=1);
#  2. round-end evidence of the current production library
#     (scripts/gpu_round.sh PART 1: smoke, GPU suite, bench lines, kernel stats).
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
show() { echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $O/$1.log) $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
PT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
FDFS_GPU_PROBE_LIB=1 FDFS_GPU_MD5_PAIR=9 step pm8_parity 600 $PT tests/test_gpu_sig.py tests/test_gpu_configs.py -k "md5 or config3"; rc=$?
tail -2 $O/pm8_parity.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ $rc -eq 0 ]; then
  B3="python3 bench.py --config c3 --no-cpu-baseline --steps 5 --warmup 2"
  for k in 1 2 3; do
    for p in 1 9; do
      FDFS_GPU_PROBE_LIB=1 FDFS_GPU_MD5_PAIR=$p step c3_p${p}_$k 300 $B3 || exit $?
      show c3_p${p}_$k
    done
  done
fi
TAG=r04 PART=1 bash scripts/gpu_round.sh
