mkdir -p gpurun_out
FDFS_GPU_CRC_TABLES=nib timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ab2_smoke.log 2>&1; rc=$?; echo smoke_nib=$rc
if [ $rc -ne 0 ]; then tail -20 gpurun_out/ab2_smoke.log; exit $rc; fi
FDFS_GPU_CRC_TABLES=nib timeout -k 10 900 python -m pytest tests/test_gpu_sig.py -q -x -k "edge or large or corpus or mixed" > gpurun_out/ab2_pytest.log 2>&1; rc=$?; echo pytest_nib=$rc; tail -3 gpurun_out/ab2_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for t in byte nib byte nib; do
  FDFS_GPU_CRC_TABLES=$t timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 10 > gpurun_out/ab2_c4_$t.log 2>&1; rc=$?; echo c4_$t=$rc
  if [ $rc -ne 0 ]; then exit $rc; fi
  python -c "import json,sys;d=json.loads(open('gpurun_out/ab2_c4_$t.log').read().strip().split('\n')[-1]);print('  c4 $t', d['value'], d['roofline']['kernel_ms_avg'])"
done
