# Full round-end evidence on one MI355X, in parts that each fit one gpurun
# call: smoke + every gpu test, bench lines for all configs (CPU baselines
# beside them), rocprofv3 kernel stats, and separate PMC passes.
# Usage: TAG=r05 PART=tests|bench|stats|pmc bash scripts/gpu_round.sh
#        (results under gpurun_out/round_$TAG; PART=all runs every part)
export TMPDIR=/tmp
TAG=${TAG:-r06}
PART=${PART:-all}
O=gpurun_out/round_$TAG
mkdir -p $O
step() {  # name timeout cmd...   (every GPU step under its own time limit)
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
part() { [ "$PART" = all ] || [ "$PART" = "$1" ]; }
B="python3 bench.py --no-cpu-baseline"
S="--steps 3 --warmup 1"
if part tests; then
  step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
  step pytest 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread; rc=$?
  tail -3 $O/pytest.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if part bench; then
  step bench_c2 600 python3 bench.py || exit $?
  step bench_c3 600 python3 bench.py --config c3 --steps 3 --warmup 1 || exit $?
  step bench_c4 600 python3 bench.py --config c4 || exit $?
  step bench_c5 600 python3 bench.py --config c5 --steps 5 --warmup 1 || exit $?
  step bench_c1 900 python3 bench.py --config c1 --steps 3 --warmup 1 || exit $?
  step bench_c4_hash 600 python3 bench.py --config c4 --method hash --steps 2 --warmup 1 || exit $?
  step bench_c4_md5 600 python3 bench.py --config c4 --method md5 --steps 2 --warmup 1 || exit $?
  step bench_c2_crc 600 python3 bench.py --config c2 --method crc || exit $?
  for c in c1 c2 c3 c4 c5 c4_hash c4_md5 c2_crc; do tail -1 $O/bench_$c.log | cut -c1-300; done
fi
if part stats; then
  # config 2 alone (--files: without the default line's sub-lines, whose
  # sig_hash_kernel / md5_pair_kernel dispatches would mix into its figures)
  step stats_c2 600 rocprofv3 --kernel-trace --stats -d $O/stats_c2 -o run --output-format csv -- $B --config c2 --files 1000000 --steps 10 --warmup 3 || exit $?
  step stats_c3 600 rocprofv3 --kernel-trace --stats -d $O/stats_c3 -o run --output-format csv -- $B --config c3 --steps 2 --warmup 1 || exit $?
  step stats_c4 600 rocprofv3 --kernel-trace --stats -d $O/stats_c4 -o run --output-format csv -- $B --config c4 $S || exit $?
  step stats_c5 600 rocprofv3 --kernel-trace --stats -d $O/stats_c5 -o run --output-format csv -- $B --config c5 $S || exit $?
  step stats_c1 900 rocprofv3 --kernel-trace --stats -d $O/stats_c1 -o run --output-format csv -- $B --config c1 --steps 2 --warmup 1 || exit $?
  find $O -name "*kernel_trace.csv" -size +8M -delete  # keep the small traces (steady-state means)
fi
if part pmc; then
  for c in c2 c3 c4 c5; do
    F=""; [ $c = c2 ] && F="--files 1000000"  # config 2 alone (no sub-lines)
    step fetch_$c 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$c -o run --output-format csv -- $B --config $c $F --steps 1 --warmup 1 || exit $?
    step write_$c 300 rocprofv3 --pmc WRITE_SIZE -d $O/write_$c -o run --output-format csv -- $B --config $c $F --steps 1 --warmup 1 || exit $?
  done
  # issue picture (scripts/pmc_clock.py: clock, SIMD issue occupancy)
  SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
  step sq_c2 300 rocprofv3 --pmc $SQ -d $O/sq_c2 -o run --output-format csv -- $B --config c2 --files 1000000 --steps 2 --warmup 1 || exit $?
  step sq_c3 600 rocprofv3 --pmc $SQ -d $O/sq_c3 -o run --output-format csv -- $B --config c3 --steps 1 --warmup 1 || exit $?
  step sq_c4 300 rocprofv3 --pmc $SQ -d $O/sq_c4 -o run --output-format csv -- $B --config c4 --steps 2 --warmup 1 || exit $?
fi
echo done
