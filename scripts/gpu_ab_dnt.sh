# A/B of non-temporal accesses in dp_group (probe build, GM_INDEX only):
# FDFS_GPU_DEDUP_PROBE 4 = answer stores, 8 = confirmation row loads, 12 = both.
# Parity of variant 12 first, then config-5 lines, twice.
export TMPDIR=/tmp
O=gpurun_out/dnt; mkdir -p $O
export FDFS_GPU_PROBE_LIB=1
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-1} | cut -c1-300; return $rc
}
bl() { python3 -c "import json;d=json.loads(open('$O/$1.log').read().strip().split('\n')[-1]);r=d['roofline'];print('   $1', d['value'], d['unit'], 'ms/step', d['ms_per_step'], 'kernel_ms', r['kernel_ms_avg'])"; }
FDFS_GPU_DEDUP_PROBE=${PP:-12} TAILN=3 step pytest 600 python3 -u -m pytest tests/test_gpu_dedup.py -x -q --timeout 300 --timeout-method thread || exit $?
for r in 1 2; do
  for v in ${VARIANTS:-0 4 8 12}; do
    FDFS_GPU_DEDUP_PROBE=$v step c5_p${v}_$r 300 python3 -u bench.py --config c5 --no-cpu-baseline --steps 10 --warmup 2 || exit $?; bl c5_p${v}_$r
  done
done
echo done
