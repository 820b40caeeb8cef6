# Round 4: sig_hash_kernel with the compacted MFMA B table (1.25 KB of LDS
# instead of 16 KB; production library, uncommitted at the time) -- the
# HASH parity tests, then config 2 alternating against the previous
# library (`make ab`, FDFS_GPU_PROBE_LIB=ab: the full B table) and the probe
# build at 128-thread workgroups (FDFS_GPU_HASH_BLOCK=128: eight per CU).
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
show() { echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $O/$1.log) $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
step cb_parity 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sig.py \
  tests/test_gpu_stream.py tests/test_gpu_configs.py tests/test_isa.py -k "not md5 and not config3 and not config5"; rc=$?
tail -2 $O/cb_parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
FDFS_GPU_PROBE_LIB=1 FDFS_GPU_HASH_BLOCK=128 step b128_parity 600 python3 -u -m pytest -x -v --timeout 300 \
  --timeout-method thread tests/test_gpu_sig.py -k "not md5 and not host_batch"; rc=$?
tail -2 $O/b128_parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
B2="python3 bench.py --no-cpu-baseline --steps 10 --warmup 3"
for k in 1 2 3; do
  step c2_new_$k 300 $B2 || exit $?
  show c2_new_$k
  FDFS_GPU_PROBE_LIB=ab step c2_old_$k 300 $B2 || exit $?
  show c2_old_$k
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_HASH_BLOCK=128 step c2_b128_$k 300 $B2 || exit $?
  show c2_b128_$k
done
