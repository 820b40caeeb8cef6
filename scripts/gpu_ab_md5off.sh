# Config-3 A/B: CRC of the largest files offloaded to crc_seg_kernel
# (FDFS_GPU_MD5_T_BIN = the size bin of T), sequential (FDFS_GPU_SIDE=0) or
# on a side stream beside md5_stage_kernel (FDFS_GPU_SIDE=1).  Parity first.
export TMPDIR=/tmp
O=gpurun_out/abm; mkdir -p $O
export FDFS_GPU_PROBE_LIB=1
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-1} | cut -c1-300; return $rc
}
bl() { python3 -c "import json,sys;d=json.loads(open('$O/$1.log').read().strip().split('\n')[-1]);r=d['roofline'];print('   $1', d['value'], d['unit'], 'ms/step', d['ms_per_step'], 'kernel_ms', r['kernel_ms_avg'])"; }
FDFS_GPU_LAT_FILES=0 FDFS_GPU_MD5_T_BIN=680 FDFS_GPU_SIDE=1 TAILN=3 step pytest 600 python3 -u -m pytest tests/test_gpu_sig.py -x -q --timeout 200 --timeout-method thread -k "md5 or edge or tiny or big or offload or scale or corpus" || exit $?
for r in 1 2; do
for v in ${VARIANTS:-0:0 688:0 688:1 680:1 696:1 672:1}; do
  b=${v%%:*}; s=${v##*:}
  FDFS_GPU_MD5_T_BIN=$b FDFS_GPU_SIDE=$s step c3_${b}_${s}_$r 300 python3 -u bench.py --config c3 --no-cpu-baseline --steps 3 --warmup 1 || exit $?; bl c3_${b}_${s}_$r
done
done
echo done
