# rocprofv3: kernel-trace stats + separate PMC passes (HBM bytes, SQ) for c2 and c4.
# Usage: PROF_TAG=r01 bash scripts/gpu_prof.sh
export TMPDIR=/tmp
TAG=${PROF_TAG:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
run() {  # name, timeout, rocprof args..., -- cmd
  local name=$1; local to=$2; shift 2
  timeout -k 10 $to rocprofv3 "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name=$rc"
  return $rc
}
for cfg in c2 c4; do
  run stats_$cfg 600 --kernel-trace --stats -d $OUT/stats_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --no-cpu-baseline --steps 5 --warmup 2 || exit $?
  run fetch_$cfg 600 --pmc FETCH_SIZE -d $OUT/fetch_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --no-cpu-baseline --steps 2 --warmup 1 || exit $?
  run write_$cfg 600 --pmc WRITE_SIZE -d $OUT/write_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --no-cpu-baseline --steps 2 --warmup 1 || exit $?
  run sq_$cfg 600 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --no-cpu-baseline --steps 2 --warmup 1 || exit $?
done
find $OUT -name "*.csv" | head -50
