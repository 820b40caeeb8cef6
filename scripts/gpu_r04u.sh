# Round 4: ELF top nibble left dirty across vectors, made exact once from the last t sign.
export TMPDIR=/tmp
O=gpurun_out/r04u
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
B2="python3 bench.py --no-cpu-baseline --steps 10 --warmup 3"
for k in 1 2 3; do
  step new_$k 300 $B2 || exit $?; show new_$k
  FDFS_GPU_PROBE_LIB=ab step old_$k 300 $B2 || exit $?; show old_$k
done
