# Round 4, first box: smoke, the whole GPU suite (sticky lane-error count,
# the tiling check, the RCCL child harness), the default bench line, c3/c5.
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
step() {  # name timeout cmd...   (every GPU step under its own time limit)
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
step pytest 1000 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread; rc=$?
tail -3 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step bench_c2 600 python3 bench.py || exit $?
tail -1 $O/bench_c2.log | cut -c1-700
B="python3 bench.py --no-cpu-baseline --steps 5 --warmup 2"
step bench_c3 400 $B --config c3 || exit $?
tail -1 $O/bench_c3.log | cut -c1-500
step bench_c5 400 $B --config c5 || exit $?
tail -1 $O/bench_c5.log | cut -c1-500
