# Round-2 refresh: full round-end evidence (PART=1 of gpu_round.sh) plus the
# config-5 HBM PMC passes for the new dedup kernels.
export TMPDIR=/tmp
TAG=${TAG:-r02c}
O=gpurun_out/round_$TAG
mkdir -p $O
TAG=$TAG PART=1 bash scripts/gpu_round.sh || exit $?
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
B="python3 bench.py --no-cpu-baseline"
step fetch_c5 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_c5 -o run --output-format csv -- $B --config c5 --steps 1 --warmup 1 || exit $?
step write_c5 300 rocprofv3 --pmc WRITE_SIZE -d $O/write_c5 -o run --output-format csv -- $B --config c5 --steps 1 --warmup 1 || exit $?
echo done
