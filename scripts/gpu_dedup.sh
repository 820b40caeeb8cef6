# Dedup path: parity tests, then c5 and c2 bench lines.
export TMPDIR=/tmp
O=gpurun_out/dd; mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-1} | cut -c1-400; return $rc
}
TAILN=6 step pytest 600 python3 -u -m pytest tests/test_gpu_dedup.py -x -v --timeout 200 --timeout-method thread || exit $?
step c5 300 python3 -u bench.py --config c5 --no-cpu-baseline --steps 5 --warmup 1 || exit $?
step c2 300 python3 -u bench.py --config c2 --no-cpu-baseline --steps 5 --warmup 2 || exit $?
echo done
