# Round 4 (probe build): pair-cooperative loads in sig_hash_kernel (HASH_MODE
# 14: 32 contiguous bytes per lane pair per instruction, one transpose stage,
# 4 VALU per vector instead of 8) against the quad form: HASH parity under
# MODE 14, then config 2 alternating, and loads alone for both forms.
export TMPDIR=/tmp
O=gpurun_out/r04za
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
show() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
export FDFS_GPU_PROBE_LIB=1
FDFS_GPU_HASH_MODE=14 step pair_parity 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sig.py -k "not md5 and not host_batch"; rc=$?
tail -2 $O/pair_parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
B2="python3 bench.py --no-cpu-baseline --steps 10 --warmup 3"
for k in 1 2 3; do
  for m in 0 14; do
    FDFS_GPU_HASH_MODE=$m step c2_m${m}_$k 300 $B2 || exit $?; show c2_m${m}_$k
  done
done
