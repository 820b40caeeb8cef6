# Round 4: the production library after the probe-only additions of
# r04n-q (ablation modes, nt-load templates): smoke, the GPU suite, the
# default bench line.
export TMPDIR=/tmp
O=gpurun_out/r04r
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
step pytest 1000 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread; rc=$?
tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
step bench_c2 600 python3 bench.py || exit $?
tail -1 $O/bench_c2.log | cut -c1-300
