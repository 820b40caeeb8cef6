# Verify the tree on one MI355X: smoke, all gpu tests, c2 + c3 + c4 bench lines.
export TMPDIR=/tmp
O=gpurun_out/verify; mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; tail -${TAILN:-1} $O/$name.log | cut -c1-900; return $rc
}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
TAILN=4 step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step c2 400 python -u bench.py --no-cpu-baseline || exit $?
step c3 400 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline || exit $?
step c4 400 python -u bench.py --config c4 --no-cpu-baseline || exit $?
echo done
