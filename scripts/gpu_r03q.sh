# Round 3 (session 2): hash kernel load pipeline with four 64-byte load sets
# (probe MODE 7: 192 bytes of lookahead in the same 64 VGPRs) vs production
# (two 128-byte sets), config 2 and config 1, alternating; signed-variant
# parity of MODE 7 on the hash tests.
export TMPDIR=/tmp
O=gpurun_out/r03q; mkdir -p $O
for r in 1 2; do for m in 0 7; do
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_HASH_MODE=$m timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/c2_m${m}_$r.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('$O/c2_m${m}_$r.log').read().strip().split('\n')[-1]);print('c2 mode=$m r=$r', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline']['frac'])"
done; done
for m in 0 7; do
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_HASH_MODE=$m timeout -k 10 400 python3 bench.py --config c1 --steps 2 --warmup 1 --no-cpu-baseline > $O/c1_m${m}.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('$O/c1_m${m}.log').read().strip().split('\n')[-1]);print('c1 mode=$m', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline'].get('chain_floor_ms'))"
done
FDFS_GPU_PROBE_LIB=1 FDFS_GPU_HASH_MODE=7 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_sig.py tests/test_gpu_configs.py -k "hash or corpus or offload or big" -v --timeout 300 --timeout-method thread > $O/pytest_m7.log 2>&1
tail -3 $O/pytest_m7.log; grep -E "FAILED" $O/pytest_m7.log | head -20
exit 0
