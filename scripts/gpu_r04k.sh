# Round 4 (probe build): crc_seg_kernel with quad-cooperative segment loads
# (FDFS_GPU_SEG_QUAD=1): the CRC parity tests, then config 4 and config 2
# CRC-only alternating against the production load pattern.
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
show() { echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $O/$1.log) $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
export FDFS_GPU_PROBE_LIB=1
FDFS_GPU_SEG_QUAD=1 step segq_parity 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_sig.py tests/test_gpu_configs.py tests/test_gpu_stream.py -k "not md5_big and not config5 and not config3"; rc=$?
tail -2 $O/segq_parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
B4="python3 bench.py --config c4 --no-cpu-baseline --steps 10 --warmup 3"
B2="python3 bench.py --method crc --no-cpu-baseline --steps 10 --warmup 3"
for k in 1 2 3; do
  for q in 0 1; do
    FDFS_GPU_SEG_QUAD=$q step c4_q${q}_$k 300 $B4 || exit $?
    show c4_q${q}_$k
  done
done
for k in 1 2; do
  for q in 0 1; do
    FDFS_GPU_SEG_QUAD=$q step c2crc_q${q}_$k 300 $B2 || exit $?
    show c2crc_q${q}_$k
  done
done
