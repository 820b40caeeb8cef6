# Round 4: pair-cooperative loads promoted to production in sig_hash_kernel.
# The whole GPU suite on the new library, then config 2 alternating against
# the previous library (make ab: the quad form).
export TMPDIR=/tmp
O=gpurun_out/r04zb
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
show() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
step pytest 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread; rc=$?
tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
B2="python3 bench.py --no-cpu-baseline --steps 10 --warmup 3"
for k in 1 2 3; do
  step new_$k 300 $B2 || exit $?; show new_$k
  FDFS_GPU_PROBE_LIB=ab step old_$k 300 $B2 || exit $?; show old_$k
done
step c1new 900 python3 bench.py --no-cpu-baseline --config c1 --steps 2 --warmup 1 || exit $?; show c1new
FDFS_GPU_PROBE_LIB=ab step c1old 900 python3 bench.py --no-cpu-baseline --config c1 --steps 2 --warmup 1 || exit $?; show c1old
# lane-per-file loads, no transposes (probe FDFS_GPU_HASH_QUAD=0) against the pair form
for k in 1 2; do
  FDFS_GPU_PROBE_LIB=1 step pair_$k 300 $B2 || exit $?; show pair_$k
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_HASH_QUAD=0 step lane_$k 300 $B2 || exit $?; show lane_$k
done
