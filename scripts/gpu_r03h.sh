# Round 3: hash kernel with 64-byte steps (probe MODE 6: two 16-VGPR load
# sets, 96 registers, 25 KB LDS -> five waves per SIMD): parity under the
# probe build, then A/B against the production form (MODE 0).
export TMPDIR=/tmp
O=gpurun_out/r03h; mkdir -p $O
export FDFS_GPU_PROBE_LIB=1 FDFS_GPU_HASH_MODE=6
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_sig.py tests/test_gpu_stream.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_m6.log 2>&1; rc=$?
tail -3 $O/pytest_m6.log
[ $rc -le 1 ] || exit $rc
B="python3 bench.py --files 1000000 --no-cpu-baseline --steps 10 --warmup 3"
for r in 1 2; do
  for v in 0 6; do
    export FDFS_GPU_HASH_MODE=$v
    timeout -k 10 300 $B > $O/c2_m${v}_$r.log 2>&1 || exit $?
    echo "m$v r=$r $(tail -1 $O/c2_m${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_avg"], d["roofline"]["frac"])')"
  done
done | tee $O/ab.txt
