# Round 3 (session 2): config 2 hash kernel with the step's loads issued at
# s_setprio 2 (probe MODE 8) vs production (probe MODE 0), alternating.
export TMPDIR=/tmp
O=gpurun_out/r03z; mkdir -p $O
for r in 1 2 3; do for m in 0 8; do
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_HASH_MODE=$m timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/c2_m${m}_$r.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('$O/c2_m${m}_$r.log').read().strip().split('\n')[-1]);print('c2 mode=$m r=$r', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline']['frac'])"
done; done
