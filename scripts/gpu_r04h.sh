# Round 4: the final library (after the probe-only plumbing of r04e-g) on a
# fresh box: smoke, the whole GPU suite, the default bench line, config 3.
export TMPDIR=/tmp
O=gpurun_out/r04h
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
step pytest 1000 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread; rc=$?
tail -3 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step bench_c2 600 python3 bench.py || exit $?
tail -1 $O/bench_c2.log | cut -c1-400
step bench_c3 400 python3 bench.py --no-cpu-baseline --config c3 --steps 5 --warmup 2 || exit $?
tail -1 $O/bench_c3.log | cut -c1-400
