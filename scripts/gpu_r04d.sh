# Round 4, fourth box (probe build unless noted):
#  1. md5_multi_kernel (FDFS_GPU_MD5_PAIR 9 = 3 pairs x 2 workgroups per CU,
#     10 = 7 pairs x 1): the MD5 parity tests, then config 3 alternating
#     against the production pair kernel (PAIR 1);
#  2. SQ / LDS counters of the config-2 hash kernels: production
#     sig_hash_kernel and the role-split sig_split_kernel;
#  3. the pair kernel's per-workgroup timeline (PM 5).
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
show() { echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $O/$1.log) $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
PT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
export FDFS_GPU_PROBE_LIB=1
ok9=0
FDFS_GPU_MD5_PAIR=9 step multi9_parity 600 $PT tests/test_gpu_sig.py tests/test_gpu_configs.py -k "md5 or config3"; rc=$?
tail -2 $O/multi9_parity.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ $rc -eq 0 ] && ok9=1
ok10=0
FDFS_GPU_MD5_PAIR=10 step multi10_parity 600 $PT tests/test_gpu_configs.py -k "config3"; rc=$?
tail -2 $O/multi10_parity.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ $rc -eq 0 ] && ok10=1
B3="python3 bench.py --config c3 --no-cpu-baseline --steps 5 --warmup 2"
for k in 1 2; do
  for p in 1 9 10; do
    [ $p = 9 ] && [ $ok9 = 0 ] && continue
    [ $p = 10 ] && [ $ok10 = 0 ] && continue
    FDFS_GPU_MD5_PAIR=$p step c3_p${p}_$k 300 $B3 || exit $?
    show c3_p${p}_$k
  done
done
B2="python3 bench.py --no-cpu-baseline --steps 1 --warmup 1"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for sp in 0 1; do
  FDFS_GPU_HASH_SPLIT=$sp step sq_c2_split$sp 300 timeout -s KILL 240 rocprofv3 --pmc $SQ -d $O/sq_c2_split$sp -o run --output-format csv -- $B2 || exit $?
done
FDFS_GPU_MD5_PAIR=6 step pair_timeline 300 python3 -u scripts/pair_timeline.py --reps 2 --out $O/pairs.npz || exit $?
cat $O/pair_timeline.log | cut -c1-1200
