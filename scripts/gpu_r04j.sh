# Round 4 (probe build): the pair kernel's priority granularity on config 3,
# alternating: PAIR 1 = production (1 MiB units, every 256 rounds), 10 = 512
# KiB units, 11 = 2 MiB units, 12 = 1 MiB units every 64 rounds.
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
show() { echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $O/$1.log) $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
export FDFS_GPU_PROBE_LIB=1
FDFS_GPU_MD5_PAIR=10 step prio_parity 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_configs.py -k config3; rc=$?
tail -2 $O/prio_parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
B3="python3 bench.py --config c3 --no-cpu-baseline --steps 5 --warmup 2"
for k in 1 2; do
  for p in 1 10 11 12; do
    FDFS_GPU_MD5_PAIR=$p step c3_p${p}_$k 300 $B3 || exit $?
    show c3_p${p}_$k
  done
done
