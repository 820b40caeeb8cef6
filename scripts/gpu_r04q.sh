# Round 4 (probe build): non-temporal loads.  Config 4 (crc_seg_kernel,
# HBM-bound, FDFS_GPU_SEG_NT=1) and config 2 (sig_hash_kernel quad loads,
# FDFS_GPU_HASH_MODE=12): parity under the nt form, then alternating against
# the default cache policy; shader clock for config 2.
export TMPDIR=/tmp
O=gpurun_out/r04q
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
show() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
clk() { echo "$1 $(grep sample $O/$1.log | awk '{print $3}' | sort -n | awk '{a[NR]=$1} END {print "clock n", NR, "min", a[1], "median", a[int(NR/2)+1], "max", a[NR]}')"; }
PT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
export FDFS_GPU_PROBE_LIB=1
FDFS_GPU_SEG_NT=1 step nt_parity 600 $PT tests/test_gpu_configs.py tests/test_gpu_sig.py -k "config4 or crc" ; rc=$?
tail -2 $O/nt_parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
FDFS_GPU_HASH_MODE=12 step nt_hash_parity 600 $PT tests/test_gpu_sig.py -k "not md5 and not host_batch"; rc=$?
tail -2 $O/nt_hash_parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
B4="python3 bench.py --config c4 --no-cpu-baseline --steps 20 --warmup 5"
B2="python3 bench.py --no-cpu-baseline --steps 10 --warmup 3"
for k in 1 2 3; do
  for v in 0 1; do
    FDFS_GPU_SEG_NT=$v step c4_nt${v}_$k 300 $B4 || exit $?; show c4_nt${v}_$k
  done
done
for k in 1 2; do
  for m in 0 12; do
    FDFS_GPU_HASH_MODE=$m step c2_m${m}_$k 300 $B2 || exit $?; show c2_m${m}_$k
  done
done
FDFS_GPU_HASH_MODE=12 step clock_m12 200 python3 scripts/clock_under_load.py c2 8 || exit $?; clk clock_m12
