# Round 4 (probe build): crc_seg_kernel with two 4 KiB blocks in flight per
# wave (FDFS_GPU_SEG_PF=2; the first two blocks' loads issued before block 0
# is folded) against one: CRC parity under PF 2, then config 4 alternating.
export TMPDIR=/tmp
O=gpurun_out/r04x
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
show() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
PT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
export FDFS_GPU_PROBE_LIB=1
FDFS_GPU_SEG_PF=2 step pf_parity 600 $PT tests/test_gpu_configs.py tests/test_gpu_sig.py -k "config4 or crc or big or offload or md5_big"; rc=$?
tail -2 $O/pf_parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
B4="python3 bench.py --config c4 --no-cpu-baseline --steps 20 --warmup 5"
for k in 1 2 3; do
  for v in 1 2; do
    FDFS_GPU_SEG_PF=$v step c4_pf${v}_$k 300 $B4 || exit $?; show c4_pf${v}_$k
  done
done
