# Config-2 PMC passes for the quad-load hash kernel (separate FETCH / WRITE /
# SQ passes) and the loads-only / compute-only probes, into round_$TAG.
export TMPDIR=/tmp
TAG=${TAG:-r02q}
O=gpurun_out/round_$TAG
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
B="python3 bench.py --no-cpu-baseline"
step fetch_c2 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_c2 -o run --output-format csv -- $B --config c2 --steps 1 --warmup 1 || exit $?
step write_c2 300 rocprofv3 --pmc WRITE_SIZE -d $O/write_c2 -o run --output-format csv -- $B --config c2 --steps 1 --warmup 1 || exit $?
step sq_c2 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $O/sq_c2 -o run --output-format csv -- $B --steps 1 --warmup 1 || exit $?
for m in 1 2; do
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_HASH_MODE=$m step probe_c2_mode$m 300 $B || exit $?
done
echo done
