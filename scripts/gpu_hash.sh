# HASH path: parity tests, then c2 (and optionally c1) bench lines.
# Usage: O=gpurun_out/h1 [C1=1] bash scripts/gpu_hash.sh
export TMPDIR=/tmp
O=${O:-gpurun_out/h}; mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-1} | cut -c1-300; return $rc
}
TAILN=3 step pytest 900 python3 -u -m pytest tests/test_gpu_sig.py tests/test_gpu_stream.py tests/test_tool.py -x -v --timeout 300 --timeout-method thread || exit $?
step c2 300 python3 -u bench.py --no-cpu-baseline --steps 10 --warmup 3 || exit $?
python3 -c "import json; d=json.loads(open('$O/c2.log').read().strip().splitlines()[-1]); print('c2', d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline']['frac'])"
step c2b 300 python3 -u bench.py --no-cpu-baseline --steps 10 --warmup 3 || exit $?
python3 -c "import json; d=json.loads(open('$O/c2b.log').read().strip().splitlines()[-1]); print('c2b', d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline']['frac'])"
if [ -n "$C1" ]; then
step c1 600 python3 -u bench.py --config c1 --no-cpu-baseline --steps 3 --warmup 1 || exit $?
fi
echo done
