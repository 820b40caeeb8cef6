# Dedup group change check: parity (dedup tests + the bench's 100M set),
# config-5 lines and kernel stats.
export TMPDIR=/tmp
O=gpurun_out/dd2; mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-1} | cut -c1-400; return $rc
}
TAILN=3 step pytest 900 python3 -u -m pytest tests/test_gpu_dedup.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "not config4 and not config3" || exit $?
for r in 1 2; do
  step c5_$r 300 python3 -u bench.py --config c5 --no-cpu-baseline --steps 5 --warmup 1 || exit $?
done
step stats_c5 300 rocprofv3 --kernel-trace --stats -d $O/stats_c5 -o run --output-format csv -- python3 bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 || exit $?
echo done
