# Round 3 (session 2): md5_pair_kernel with both waves of a workgroup at
# s_setprio 2 while their chunk is among the largest quarter (probe pmode 4,
# FDFS_GPU_MD5_PAIR=5) vs production (FDFS_GPU_MD5_PAIR=1), probe library,
# config 3, alternating.
export TMPDIR=/tmp
O=gpurun_out/r03zg; mkdir -p $O
for r in 1 2 3; do for m in 1 5; do
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_MD5_PAIR=$m timeout -k 10 300 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_m${m}_$r.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('$O/c3_m${m}_$r.log').read().strip().split('\n')[-1]);print('pair=$m r=$r', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline'].get('chain_floor_ms'))"
done; done
