# Round 4 (probe build): the rotated conflict-free CRC tables (TM 3, 512-thread
# workgroups) against production again, now that the hash step carries less
# VALU (grouped Horner, ELF exact fold once per file): HASH parity under TM 3,
# then config 2 alternating.
export TMPDIR=/tmp
O=gpurun_out/r04y
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
show() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
export FDFS_GPU_PROBE_LIB=1
FDFS_GPU_HASH_TM=3 FDFS_GPU_HASH_BLOCK=512 step tm3_parity 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sig.py -k "not md5 and not host_batch"; rc=$?
tail -2 $O/tm3_parity.log
B2="python3 bench.py --no-cpu-baseline --steps 10 --warmup 3"
for k in 1 2 3; do
  step prod_$k 300 $B2 || exit $?; show prod_$k
  FDFS_GPU_HASH_TM=3 FDFS_GPU_HASH_BLOCK=512 step tm3_$k 300 $B2 || exit $?; show tm3_$k
done
