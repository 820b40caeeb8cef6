# Quick check on one MI355X: smoke, signature parity tests, c2/c3/c4 bench lines.
export TMPDIR=/tmp
O=gpurun_out/verify; mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-1} | cut -c1-300; return $rc
}
bl() { python3 -c "import json,sys;d=json.loads(open('$O/$1.log').read().strip().split('\n')[-1]);r=d['roofline'];print('   $1', d['value'], d['unit'], 'ms/step', d['ms_per_step'], 'kernel_ms', r['kernel_ms_avg'], 'frac', r['frac'])"; }
step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
TAILN=3 step pytest 900 python3 -u -m pytest tests/test_gpu_sig.py -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} || exit $?
for c in ${CONFIGS:-c2 c3 c4}; do
  step $c 400 python3 -u bench.py --config $c --no-cpu-baseline --steps ${STEPS:-5} --warmup 2 > /dev/null || exit $?; bl $c
done
echo done
