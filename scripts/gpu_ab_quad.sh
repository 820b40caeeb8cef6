# A/B of sig_hash_kernel's quad-cooperative loads (probe build knob
# FDFS_GPU_HASH_QUAD): parity of the quad path first, then config-2 lines
# for quad 0/1, full kernel and loads only (FDFS_GPU_HASH_MODE=1), twice.
export TMPDIR=/tmp
O=gpurun_out/abq; mkdir -p $O
export FDFS_GPU_PROBE_LIB=1
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-1} | cut -c1-300; return $rc
}
bl() { python3 -c "import json,sys;d=json.loads(open('$O/$1.log').read().strip().split('\n')[-1]);r=d['roofline'];print('   $1', d['value'], d['unit'], 'ms/step', d['ms_per_step'], 'kernel_ms', r['kernel_ms_avg'], 'frac', r['frac'])"; }
FDFS_GPU_HASH_QUAD=${PQ:-1} TAILN=3 step pytest 600 python3 -u -m pytest tests/test_gpu_sig.py -x -q --timeout 200 --timeout-method thread -k "${PYTEST_K:-edge or small or tiny or corpus or scale}" || exit $?
for r in 1 2; do
for v in ${VARIANTS:-0 1}; do
  for m in ${MODES:-0 1}; do
    FDFS_GPU_HASH_QUAD=$v FDFS_GPU_HASH_MODE=$m step c2_q${v}_m${m}_$r 300 python3 -u bench.py --config c2 --no-cpu-baseline --steps 5 --warmup 2 || exit $?; bl c2_q${v}_m${m}_$r
  done
done
done
echo done
if [ -n "$PMC_Q" ]; then  # HBM fetch of one variant (separate pass)
  FDFS_GPU_HASH_QUAD=$PMC_Q step fetch_q$PMC_Q 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_q$PMC_Q -o run --output-format csv -- python3 bench.py --config c2 --no-cpu-baseline --steps 1 --warmup 1 || exit $?
  python3 scripts/pmc_summary.py $O/fetch_q$PMC_Q 2>/dev/null | grep sig_hash | cut -c1-200
fi
