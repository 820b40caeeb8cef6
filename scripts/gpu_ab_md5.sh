# A/B of the config-3 MD5 kernel schedule: chunk queue over one wave per SIMD
# (default) vs one chunk per wave, all waves resident (FDFS_GPU_MD5_QUEUE=0).
export TMPDIR=/tmp
O=gpurun_out/abm; mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-1} | cut -c1-300; return $rc
}
bl() { python3 -c "import json,sys;d=json.loads(open('$O/$1.log').read().strip().split('\n')[-1]);r=d['roofline'];print('   $1', d['value'], d['unit'], 'ms/step', d['ms_per_step'], 'kernel_ms', r['kernel_ms_avg'], 'frac', r['frac'])"; }
TAILN=3 step pytest 600 python3 -u -m pytest tests/test_gpu_sig.py tests/test_formats.py -x -q --timeout 300 --timeout-method thread -k "md5 or corpus or edge or small or host or recovery" || exit $?
for v in ${VARIANTS:-1 0 1 0}; do
  FDFS_GPU_MD5_QUEUE=$v step c3_q$v 400 python3 -u bench.py --config c3 --no-cpu-baseline --steps 3 --warmup 1 || exit $?; bl c3_q$v
done
echo done
