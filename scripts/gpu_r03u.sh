# Round 3 (session 2): md5_pair_kernel variants on config 3 -- HEAD (`make
# ab`), the loader's next loads issued right after staging + the MD5 wave's
# row read in one burst (probe library), and that plus the round's CRC as two
# independent 64-byte chains joined by one 64-byte advance (production).
# MD5 parity of the production form first.
export TMPDIR=/tmp
O=gpurun_out/r03u; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -k "md5 or config3 or offload or smoke or corpus or stream or graph" -v --timeout 300 --timeout-method thread > $O/pytest_md5.log 2>&1; rc=$?
tail -3 $O/pytest_md5.log; grep -E "FAILED|ERROR" $O/pytest_md5.log | head
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do for v in two reorder ab; do
  case $v in two) L=;; reorder) L=1;; ab) L=ab;; esac
  FDFS_GPU_PROBE_LIB=$L timeout -k 10 300 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_${v}_$r.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('$O/c3_${v}_$r.log').read().strip().split('\n')[-1]);print('$v r=$r', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline'].get('chain_floor_ms'))"
done; done
