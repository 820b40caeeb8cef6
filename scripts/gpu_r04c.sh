# Round 4, third box:
#  1. the role-split hash kernel (probe build, FDFS_GPU_HASH_SPLIT=1): the
#     HASH-method parity tests, then config 2 alternating against the
#     production sig_hash_kernel;
#  2. the production library with the pair kernel's issue priority: the
#     MD5 parity tests and config 3.
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
show() { echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $O/$1.log) $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
PT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
FDFS_GPU_PROBE_LIB=1 FDFS_GPU_HASH_SPLIT=1 step split_parity 600 $PT tests/test_gpu_sig.py \
  -k "not md5 and not host_batch"; rc=$?
tail -3 $O/split_parity.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ $rc -eq 0 ]; then
  B2="python3 bench.py --no-cpu-baseline --steps 10 --warmup 3"
  for k in 1 2 3; do
  for sp in 0 1; do
    FDFS_GPU_PROBE_LIB=1 FDFS_GPU_HASH_SPLIT=$sp step c2_split${sp}_$k 300 $B2 || exit $?
    show c2_split${sp}_$k
  done
  done
fi
step md5_parity 900 $PT tests/test_gpu_configs.py tests/test_gpu_sig.py tests/test_isa.py -k "md5 or config3 or isa or checker or hazard or probe"; rc=$?
tail -3 $O/md5_parity.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B3="python3 bench.py --config c3 --no-cpu-baseline --steps 5 --warmup 2"
step c3_prod 300 $B3 || exit $?
show c3_prod
