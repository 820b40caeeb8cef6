# Round 3: does the conflict-free rotated-table CRC (TM 3) lose because of
# its 1024-thread workgroups?  Probe build: production code at 256 threads
# (mode 0), at 1024 threads (mode 5), rotated tables at 1024 (TM 3).
export TMPDIR=/tmp
O=gpurun_out/r03g; mkdir -p $O
export FDFS_GPU_PROBE_LIB=1
B="python3 bench.py --files 1000000 --no-cpu-baseline --steps 10 --warmup 3"
for r in 1 2; do
  for v in m0 m5 tm3; do
    case $v in m0) export FDFS_GPU_HASH_MODE=0 FDFS_GPU_HASH_TM=0;; m5) export FDFS_GPU_HASH_MODE=5 FDFS_GPU_HASH_TM=0;; tm3) export FDFS_GPU_HASH_MODE=0 FDFS_GPU_HASH_TM=3;; esac
    timeout -k 10 300 $B > $O/c2_${v}_$r.log 2>&1 || exit $?
    echo "$v r=$r $(tail -1 $O/c2_${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_avg"], d["roofline"]["frac"])')"
  done
done | tee $O/ab.txt
