# Round 4, first box: smoke, the whole GPU suite (the sticky lane-error
# count, the tiling check, the RCCL child harness), the default bench line.
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
step() {  # name timeout cmd...   (every GPU step under its own time limit)
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
step pytest 1000 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread; rc=$?
tail -3 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step bench_c2 600 python3 bench.py || exit $?
tail -1 $O/bench_c2.log | cut -c1-600
FDFS_GPU_PROBE_LIB=1 FDFS_GPU_MD5_PAIR=6 step pair_timeline 600 python3 -u scripts/pair_timeline.py --out $O/pairs.npz || exit $?
cat $O/pair_timeline.log | cut -c1-900
# role-split bound: compute-only hash kernel at 4 and 3 waves/SIMD,
# with and without the quad transposes (FDFS_GPU_HASH_LDSPAD caps occupancy)
B="python3 bench.py --no-cpu-baseline --steps 5 --warmup 2"
for cfg in "2 1 0" "2 0 0" "2 0 12288" "2 1 12288" "0 1 12288" "0 1 0"; do
  set -- $cfg
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_HASH_MODE=$1 FDFS_GPU_HASH_QUAD=$2 FDFS_GPU_HASH_LDSPAD=$3 step split_m$1_q$2_p$3 300 $B || exit $?
  echo "mode=$1 quad=$2 pad=$3 $(grep -o '"kernel_ms_avg": [0-9.]*' $O/split_m$1_q$2_p$3.log)"
done
