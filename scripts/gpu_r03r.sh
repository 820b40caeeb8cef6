# Round 3 (session 2): big-file ELF chain steps with four 64-byte load sets
# in flight (production) -- hash parity (both CRC variants), then config 1
# and config 2 against HEAD (`make ab`), alternating.
export TMPDIR=/tmp
O=gpurun_out/r03r; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -k "hash or corpus or offload or big or stream or graph or tool or c1 or config" -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do for lib in new ab; do
  L=; [ $lib = ab ] && L=ab
  FDFS_GPU_PROBE_LIB=$L timeout -k 10 400 python3 bench.py --config c1 --steps 2 --warmup 1 --no-cpu-baseline > $O/c1_${lib}_$r.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('$O/c1_${lib}_$r.log').read().strip().split('\n')[-1]);print('c1 $lib r=$r', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline'].get('chain_floor_ms'))"
done; done
for lib in new ab; do
  L=; [ $lib = ab ] && L=ab
  FDFS_GPU_PROBE_LIB=$L timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/c2_${lib}.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('$O/c2_${lib}.log').read().strip().split('\n')[-1]);print('c2 $lib', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
done
