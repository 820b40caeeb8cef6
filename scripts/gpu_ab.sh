# A/B of kernel variants in one box session (smoke each variant, bench each).
mkdir -p gpurun_out
for v in 0 1 2; do
  FDFS_GPU_LANE_VARIANT=$v timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ab_smoke_$v.log 2>&1; rc=$?; echo smoke_v$v=$rc
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/ab_smoke_$v.log; exit $rc; fi
done
FDFS_GPU_CRC_TABLES=byte timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ab_smoke_byte.log 2>&1; rc=$?; echo smoke_byte=$rc
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -m pytest tests/test_gpu_sig.py -q -x -k "edge or large or corpus" > gpurun_out/ab_pytest.log 2>&1; rc=$?; echo pytest=$rc; tail -3 gpurun_out/ab_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in 0 1 2; do
  FDFS_GPU_LANE_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/ab_c2_v$v.log 2>&1; rc=$?; echo c2_v$v=$rc
  if [ $rc -ne 0 ]; then exit $rc; fi
  python -c "import json,sys;d=json.loads(open('gpurun_out/ab_c2_v$v.log').read().strip().split('\n')[-1]);print('  c2 v$v', d['value'], d['roofline']['kernel_ms_avg'])"
done
for t in byte nib; do
  FDFS_GPU_CRC_TABLES=$t timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 5 > gpurun_out/ab_c4_$t.log 2>&1; rc=$?; echo c4_$t=$rc
  if [ $rc -ne 0 ]; then exit $rc; fi
  python -c "import json,sys;d=json.loads(open('gpurun_out/ab_c4_$t.log').read().strip().split('\n')[-1]);print('  c4 $t', d['value'], d['roofline']['kernel_ms_avg'])"
done
