# Dedup path: parity tests, then c5 and c2 bench lines and c5 kernel stats.
# Usage: O=gpurun_out/dd bash scripts/gpu_dedup.sh
export TMPDIR=/tmp
O=${O:-gpurun_out/dd}; mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-1} | cut -c1-400; return $rc
}
TAILN=6 step pytest 600 python3 -u -m pytest tests/test_gpu_dedup.py tests/test_formats.py tests/test_gpu_configs.py::test_config5_bench_set -x -v --timeout 200 --timeout-method thread || exit $?
step c5 300 python3 -u bench.py --config c5 --no-cpu-baseline --steps 5 --warmup 1 || exit $?
step stats_c5 300 rocprofv3 --kernel-trace --stats -d $O/stats_c5 -o run --output-format csv -- python3 bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 || exit $?
find $O/stats_c5 -name "*kernel_stats.csv" -exec cut -d, -f1-4 {} \; | grep -v at::native | head -14
echo done
