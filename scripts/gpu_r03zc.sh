# Round 3 (session 2): md5_pair_kernel loader reading its rows for both
# blocks of a round in one LDS round trip before the CRC lookups -- MD5 parity,
# then config 3 vs HEAD (ab), alternating.
export TMPDIR=/tmp
O=gpurun_out/r03zc; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -k "md5 or config3 or offload or smoke or corpus or stream or graph" -v --timeout 300 --timeout-method thread > $O/pytest_md5.log 2>&1; rc=$?
tail -3 $O/pytest_md5.log; grep -E "FAILED|ERROR" $O/pytest_md5.log | head
[ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do for v in new ab; do
  case $v in new) E="FDFS_GPU_PROBE_LIB=";; ab) E="FDFS_GPU_PROBE_LIB=ab";; esac
  env $E timeout -k 10 300 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_${v}_$r.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('$O/c3_${v}_$r.log').read().strip().split('\n')[-1]);print('$v r=$r', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline'].get('chain_floor_ms'))"
done; done
