# Round 3: hash-kernel tests on the new production build, the hash A/B
# (production = explicit 4-wave occupancy; ab = round-2 form; probe MODE 4 =
# ELF in the 3-op chain form), then the memset-zeroing graph replay (last).
export TMPDIR=/tmp
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_sig.py tests/test_gpu_graph.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="python3 bench.py --files 1000000 --no-cpu-baseline --steps 10 --warmup 3"
for r in 1 2; do
  for v in new ab m4; do
    case $v in new) unset FDFS_GPU_PROBE_LIB FDFS_GPU_HASH_MODE;; ab) export FDFS_GPU_PROBE_LIB=ab; unset FDFS_GPU_HASH_MODE;; m4) export FDFS_GPU_PROBE_LIB=1 FDFS_GPU_HASH_MODE=4;; esac
    timeout -k 10 300 $B > $O/c2_${v}_$r.log 2>&1 || exit $?
    echo "$v r=$r $(tail -1 $O/c2_${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_avg"], d["roofline"]["frac"])')"
  done
done | tee $O/ab.txt
unset FDFS_GPU_PROBE_LIB FDFS_GPU_HASH_MODE
FDFS_GPU_PROBE_LIB=1 FDFS_GPU_MEMSET=1 timeout -k 10 180 python3 -u scripts/graph_memset_replay.py > $O/replay.log 2>&1; echo "replay rc=$?"
grep replay $O/replay.log
