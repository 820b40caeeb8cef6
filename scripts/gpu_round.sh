# Full round-end check on one MI355X: smoke, every gpu test, bench lines for
# all configs, rocprofv3 kernel stats + HBM PMC passes for the headline config.
# Usage: TAG=r01 bash scripts/gpu_round.sh
export TMPDIR=/tmp
TAG=${TAG:-r01}
O=gpurun_out/round_$TAG
mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step pytest 1500 python -m pytest tests -m gpu -q; rc=$?
tail -3 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step bench_c2 600 python bench.py || exit $?
tail -1 $O/bench_c2.log
step bench_c3 600 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline || exit $?
tail -1 $O/bench_c3.log
step bench_c4 600 python bench.py --config c4 || exit $?
tail -1 $O/bench_c4.log
step bench_c5 600 python bench.py --config c5 --steps 5 --warmup 1 || exit $?
tail -1 $O/bench_c5.log
rocprofv3 -L > $O/counters_list.txt 2>&1
step prof_stats_c2 600 rocprofv3 --kernel-trace --stats -d $O/stats_c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 || exit $?
step prof_fetch_c2 600 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 || exit $?
step prof_write_c2 600 rocprofv3 --pmc WRITE_SIZE -d $O/write_c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 || exit $?
step prof_sq_c2 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/sq_c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 || exit $?
step prof_stats_c4 600 rocprofv3 --kernel-trace --stats -d $O/stats_c4 -o run --output-format csv -- python3 bench.py --config c4 --no-cpu-baseline --steps 5 --warmup 2 || exit $?
step prof_fetch_c4 600 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_c4 -o run --output-format csv -- python3 bench.py --config c4 --no-cpu-baseline --steps 2 --warmup 1 || exit $?
step prof_write_c4 600 rocprofv3 --pmc WRITE_SIZE -d $O/write_c4 -o run --output-format csv -- python3 bench.py --config c4 --no-cpu-baseline --steps 2 --warmup 1 || exit $?
echo done
