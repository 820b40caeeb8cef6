mkdir -p gpurun_out
for v in 2 5; do
  FDFS_GPU_LANE_VARIANT=$v timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ab4_smoke_$v.log 2>&1; rc=$?; echo smoke_v$v=$rc
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/ab4_smoke_$v.log; exit $rc; fi
done
FDFS_GPU_LANE_VARIANT=5 timeout -k 10 900 python -m pytest tests/test_gpu_sig.py -q -x -k "edge or small or corpus or large" > gpurun_out/ab4_pytest.log 2>&1; rc=$?; echo pytest_v5=$rc; tail -3 gpurun_out/ab4_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in 2 5 2 5; do
  FDFS_GPU_LANE_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/ab4_c2_v$v.log 2>&1; rc=$?; echo c2_v$v=$rc
  if [ $rc -ne 0 ]; then exit $rc; fi
  python -c "import json,sys;d=json.loads(open('gpurun_out/ab4_c2_v$v.log').read().strip().split('\n')[-1]);print('  c2 v$v', d['value'], d['roofline']['kernel_ms_avg'])"
done
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 10 > gpurun_out/ab4_c4.log 2>&1; rc=$?; echo c4=$rc
python -c "import json,sys;d=json.loads(open('gpurun_out/ab4_c4.log').read().strip().split('\n')[-1]);print('  c4', d['value'], d['roofline']['kernel_ms_avg'])"
