# Round 3 (session 2): md5_pair_kernel as 4 pairs per CU with conflict-free
# rotated slice-by-8 CRC tables and LDS-counter pair sync -- MD5 parity, then
# config 3: fused (pair=0) vs pair (1), no-CRC (3) and no-MD5 (4) probes.
export TMPDIR=/tmp
O=gpurun_out/r03p; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -k "md5 or config3 or offload or smoke or corpus or stream" -v --timeout 300 --timeout-method thread > $O/pytest_md5.log 2>&1; rc=$?
tail -3 $O/pytest_md5.log; grep -E "FAILED|ERROR" $O/pytest_md5.log | head
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do for m in 0 1 3 4; do
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_MD5_PAIR=$m timeout -k 10 300 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_m${m}_$r.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('$O/c3_m${m}_$r.log').read().strip().split('\n')[-1]);print('pair=$m r=$r', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline'].get('chain_floor_ms'))"
done; done
