# Round 4: md5_pair_kernel loader addressing -- each load slot clamps its
# round to its last round inside the file (v_min_u32 + 64-bit add) instead of
# a 64-bit compare and a 64-bit select to `safe`.  GPU suite, then config 3
# alternating against the previous library (make ab).
export TMPDIR=/tmp
O=gpurun_out/r04w
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
show() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
step pytest 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread; rc=$?
tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
B3="python3 bench.py --config c3 --no-cpu-baseline --steps 3 --warmup 1"
for k in 1 2 3; do
  step c3new_$k 300 $B3 || exit $?; show c3new_$k
  FDFS_GPU_PROBE_LIB=ab step c3old_$k 300 $B3 || exit $?; show c3old_$k
done
