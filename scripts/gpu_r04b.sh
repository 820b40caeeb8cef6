# Round 4, second box (probe build unless noted):
#  1. config 3 CRC offload of the largest files: FDFS_GPU_MD5_T_BIN = first
#     offloaded size bin (1/32 octave: 680 = 2.5 MiB, 688 = 3 MiB, 696 =
#     3.5 MiB, 700 = 3.75 MiB); FDFS_GPU_SIDE 0 = segmented CRC before the
#     pair kernel, 1 = beside it, 2 = enqueued after it on a lowest-priority
#     stream.  Controls ("0 0") alternate with the variants.
#  2. config 3 issue-priority policies (FDFS_GPU_MD5_PAIR 7 = by remaining
#     rounds, 8 = young chunks first; 1 = production).
#  3. config 2 role-split bound: the compute-only hash kernel (MODE 2) at four
#     and three waves per SIMD (LDSPAD caps occupancy), with and without the
#     quad transposes.
#  4. config 5: singleton answers written by dp_split instead of dp_tile.
#  5. config 4 with the signature on (production library): --method hash/md5.
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
show() { echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $O/$1.log) $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
B3="python3 bench.py --config c3 --no-cpu-baseline --steps 5 --warmup 2"
# FDFS_GPU_SIDE 3 = the CRC segments as md5_pair_kernel queue items: parity
# first (every file's CRC against the CRC-only path, MD5 samples vs hashlib)
FDFS_GPU_PROBE_LIB=1 FDFS_GPU_MD5_T_BIN=688 FDFS_GPU_SIDE=3 step inline_parity 400 python3 -u -m pytest -x -v \
  --timeout 300 --timeout-method thread tests/test_gpu_configs.py -k config3_full_batch; rc=$?
tail -2 $O/inline_parity.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
INL='"0 0" "688 3" "696 3" "680 3" "0 0" "700 3" "672 3" "688 3"'
[ $rc -eq 0 ] || INL=""
i=0
eval "set -- $INL \"0 0\" \"688 0\" \"688 1\" \"688 2\" \"0 0\" \"696 2\" \"680 2\" \"700 2\" \"0 0\""
for cfg in "$@"; do
  set -- $cfg
  i=$((i+1))
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_MD5_T_BIN=$1 FDFS_GPU_SIDE=$2 step c3_${i}_t$1_s$2 300 $B3 || exit $?
  show c3_${i}_t$1_s$2
done
for k in 1 2; do
for p in 1 7 8; do
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_MD5_PAIR=$p step c3_p${p}_$k 300 $B3 || exit $?
  show c3_p${p}_$k
done
done
B2="python3 bench.py --no-cpu-baseline --steps 5 --warmup 2"
for cfg in "0 1 0" "2 1 0" "2 0 0" "2 0 12288" "2 1 12288" "0 1 12288" "0 1 0"; do
  set -- $cfg
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_HASH_MODE=$1 FDFS_GPU_HASH_QUAD=$2 FDFS_GPU_HASH_LDSPAD=$3 step c2_m$1_q$2_p$3 300 $B2 || exit $?
  show c2_m$1_q$2_p$3
done
B5="python3 bench.py --config c5 --no-cpu-baseline --steps 10 --warmup 3"
for k in 1 2 3; do
for d in 0 1; do
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_DEDUP_DEF=$d step c5_def${d}_$k 300 $B5 || exit $?
  show c5_def${d}_$k
done
done
B4="python3 bench.py --config c4 --no-cpu-baseline --steps 2 --warmup 1"
step c4_crc 300 $B4 || exit $?
show c4_crc
step c4_hash 400 $B4 --method hash || exit $?
show c4_hash
step c4_md5 500 $B4 --method md5 || exit $?
show c4_md5
