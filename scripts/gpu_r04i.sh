# Round 4 (probe build): config 2 with coarser size bins (FDFS_GPU_BIN_SHIFT
# s: 2^s of the 1/32-octave bins merged, so a wave's 64 files come from a
# narrower index range of the batch, at a wider size spread per wave).
# HASH parity under s = 2, then alternating s = 0 / 2 / 3.
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
show() { echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $O/$1.log) $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
export FDFS_GPU_PROBE_LIB=1
FDFS_GPU_BIN_SHIFT=2 step bin_parity 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_sig.py -k "not md5 and not host_batch"; rc=$?
tail -2 $O/bin_parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
B2="python3 bench.py --no-cpu-baseline --steps 10 --warmup 3"
for k in 1 2; do
  for b in 0 2 3 5; do
    FDFS_GPU_BIN_SHIFT=$b step c2_b${b}_$k 300 $B2 || exit $?
    show c2_b${b}_$k
  done
done
