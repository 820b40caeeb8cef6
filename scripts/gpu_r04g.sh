# Round 4, seventh box (probe build): config 3 with the CRC of the tail
# chunks (those taken after the pair kernel's first G) as CRC segment items
# of its own queue (FDFS_GPU_SIDE=4), the loaders of those chunks staging
# rows for MD5 only.  Parity (every CRC against the CRC-only path), then
# alternating against production (SIDE=0).
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
show() { echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $O/$1.log) $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
PT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
export FDFS_GPU_PROBE_LIB=1
FDFS_GPU_SIDE=4 step tail_parity 600 $PT tests/test_gpu_configs.py tests/test_gpu_sig.py -k "config3 or md5"; rc=$?
tail -2 $O/tail_parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
B3="python3 bench.py --config c3 --no-cpu-baseline --steps 5 --warmup 2"
for k in 1 2 3; do
  for sd in 0 4; do
    FDFS_GPU_SIDE=$sd step c3_s${sd}_$k 300 $B3 || exit $?
    show c3_s${sd}_$k
  done
done
