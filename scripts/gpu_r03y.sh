# Round 3 (session 2): md5_pair_kernel with LDS-counter sync and the loader's
# CRC a round behind its staging (CTR, production) vs one barrier per round
# (probe FDFS_GPU_MD5_CTR=0) -- MD5 parity first, then config 3 alternating,
# then the aliased-buffer probe of both.
export TMPDIR=/tmp
O=gpurun_out/r03y; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -k "md5 or config3 or offload or smoke or corpus or stream or graph" -v --timeout 300 --timeout-method thread > $O/pytest_md5.log 2>&1; rc=$?
tail -3 $O/pytest_md5.log; grep -E "FAILED|ERROR" $O/pytest_md5.log | head
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do for c in 1 0; do
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_MD5_CTR=$c timeout -k 10 300 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_ctr${c}_$r.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('$O/c3_ctr${c}_$r.log').read().strip().split('\n')[-1]);print('ctr=$c r=$r', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline'].get('chain_floor_ms'))"
done; done
for c in 1 0; do
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_MD5_CTR=$c timeout -k 10 200 python3 scripts/md5_alias_probe.py > $O/alias_ctr$c.txt 2>&1 || exit $?
  echo "ctr=$c $(grep aliased $O/alias_ctr$c.txt)"
done
