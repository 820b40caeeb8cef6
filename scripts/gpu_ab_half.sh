# A/B of the config-2 hash loop: 128-byte steps vs 64-byte half steps (FDFS_GPU_HASH_HALF).
export TMPDIR=/tmp
O=gpurun_out/abhf; mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-1} | cut -c1-300; return $rc
}
bl() { python3 -c "import json,sys;d=json.loads(open('$O/$1.log').read().strip().split('\n')[-1]);r=d['roofline'];print('   $1', d['value'], d['unit'], 'ms/step', d['ms_per_step'], 'kernel_ms', r['kernel_ms_avg'], 'frac', r['frac'])"; }
FDFS_GPU_HASH_HALF=1 TAILN=3 step pytest 600 python3 -u -m pytest tests/test_gpu_sig.py -x -q --timeout 200 --timeout-method thread -k "edge or small or tiny or corpus" || exit $?
for v in 1 0; do
  FDFS_GPU_HASH_HALF=$v step c2_h$v 300 python3 -u bench.py --config c2 --no-cpu-baseline --steps 5 --warmup 2 || exit $?; bl c2_h$v
done
echo done
