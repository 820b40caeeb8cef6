# HASH-method big-file CRC offload: parity tests, c1 and c2 bench lines.
export TMPDIR=/tmp
O=gpurun_out/big; mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-1} | cut -c1-400; return $rc
}
TAILN=4 step pytest 900 python3 -u -m pytest tests/test_gpu_sig.py tests/test_tool.py -x -v --timeout 300 --timeout-method thread || exit $?
step c1 600 python3 -u bench.py --config c1 --no-cpu-baseline --steps 2 --warmup 1 || exit $?
step c2 300 python3 -u bench.py --config c2 --no-cpu-baseline --steps 10 --warmup 3 || exit $?
step stats_c1 600 rocprofv3 --kernel-trace --stats -d $O/stats_c1 -o run --output-format csv -- python3 bench.py --config c1 --no-cpu-baseline --steps 2 --warmup 1 || exit $?
find $O/stats_c1 -name "*kernel_stats.csv" -exec cut -d, -f1-4 {} \; | head -8
echo done
