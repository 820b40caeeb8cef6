# Conflict-free rotated slice-by-8 CRC tables: parity (seg kernel default, lane VAR 7), A/B benches.
export TMPDIR=/tmp
O=gpurun_out/exp3; mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-1} | cut -c1-400; return $rc
}
bl() { python3 -c "import json,sys;d=json.loads(open('$O/$1.log').read().strip().split('\n')[-1]);r=d['roofline'];print('   $1', d['value'], d['unit'], 'kernel_ms', r['kernel_ms_avg'], 'frac', r['frac'])"; }
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
TAILN=2 step pytest_seg 600 python -u -m pytest tests/test_gpu_sig.py -x -q --timeout 300 --timeout-method thread || exit $?
FDFS_GPU_LANE_VARIANT=7 TAILN=2 step pytest_v7 600 python -u -m pytest tests/test_gpu_sig.py -x -q --timeout 300 --timeout-method thread -k "edge or small or corpus or mixed or scale" || exit $?
for v in 5 7 5 7; do
  FDFS_GPU_LANE_VARIANT=$v step c2_v$v 300 python -u bench.py --no-cpu-baseline --steps 10 || exit $?; bl c2_v$v
done
for t in rep8 byte rep8 byte; do
  FDFS_GPU_CRC_TABLES=$t step c4_$t 300 python -u bench.py --config c4 --no-cpu-baseline --steps 10 || exit $?; bl c4_$t
done
step c3 400 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline || exit $?; bl c3
echo done
