# Round 3 (session 2): paired MD5 waves (md5_pair_kernel) -- MD5 parity
# first, then config 3 fused vs paired vs paired+setprio (probe library,
# alternating), then every gpu test and the config 5 / config 2 lines.
export TMPDIR=/tmp
O=gpurun_out/r03n; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -k "md5 or config3 or offload or smoke or corpus" -v --timeout 300 --timeout-method thread > $O/pytest_md5.log 2>&1; rc=$?
tail -3 $O/pytest_md5.log; grep -E "FAILED|ERROR" $O/pytest_md5.log | head
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do for m in 0 1 2; do
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_MD5_PAIR=$m timeout -k 10 300 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_m${m}_$r.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('$O/c3_m${m}_$r.log').read().strip().split('\n')[-1]);print('pair=$m r=$r', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline'].get('chain_floor_ms'))"
done; done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do for a in arrays packed; do
  timeout -k 10 300 python3 bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline --answers $a > $O/c5_${a}_$r.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('$O/c5_${a}_$r.log').read().strip().split('\n')[-1]);print('$a r=$r', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
done; done
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/c2.log 2>&1 || exit $?
tail -1 $O/c2.log | cut -c1-600
