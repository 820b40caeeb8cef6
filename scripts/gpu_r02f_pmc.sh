# Config-5 PMC passes for the final dedup chain (separate FETCH / WRITE / SQ
# passes) into round_$TAG.
export TMPDIR=/tmp
TAG=${TAG:-r02f}
O=gpurun_out/round_$TAG
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
B="python3 bench.py --no-cpu-baseline"
step fetch_c5 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_c5 -o run --output-format csv -- $B --config c5 --steps 1 --warmup 1 || exit $?
step write_c5 300 rocprofv3 --pmc WRITE_SIZE -d $O/write_c5 -o run --output-format csv -- $B --config c5 --steps 1 --warmup 1 || exit $?
step sq_c5 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $O/sq_c5 -o run --output-format csv -- $B --config c5 --steps 1 --warmup 1 || exit $?
echo done
