mkdir -p gpurun_out
for v in 6; do
  FDFS_GPU_LANE_VARIANT=$v timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ab5_smoke_$v.log 2>&1; rc=$?; echo smoke_v$v=$rc
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/ab5_smoke_$v.log; exit $rc; fi
done
for v in 5 6 5 6; do
  FDFS_GPU_LANE_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/ab5_c2_v$v.log 2>&1; rc=$?; echo c2_v$v=$rc
  if [ $rc -ne 0 ]; then exit $rc; fi
  python -c "import json,sys;d=json.loads(open('gpurun_out/ab5_c2_v$v.log').read().strip().split('\n')[-1]);print('  c2 v$v', d['value'], d['roofline']['kernel_ms_avg'])"
done
