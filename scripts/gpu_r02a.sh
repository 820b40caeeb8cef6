# Round 2: full-size config tests + bench lines for the new shapes.
export TMPDIR=/tmp
O=gpurun_out/r02a
mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; tail -2 $O/$name.log | cut -c1-400; return $rc
}
step cfgtests 600 python3 -u -m pytest tests/test_gpu_configs.py -x -v --timeout 400 --timeout-method thread || exit $?
step c3 600 python3 bench.py --config c3 --steps 3 --warmup 1 || exit $?
step c3_a1 600 python3 bench.py --config c3 --steps 3 --warmup 1 --align 1 --no-cpu-baseline || exit $?
step c2_crc 300 python3 bench.py --method crc --no-cpu-baseline || exit $?
step c2_a1 300 python3 bench.py --align 1 --no-cpu-baseline || exit $?
step c2 400 python3 bench.py || exit $?
echo done
