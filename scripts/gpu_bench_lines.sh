# Bench lines only (all configs), e.g. after refreshing profiles/pmc_*.json.
# Usage: TAG=r01g bash scripts/gpu_bench_lines.sh   (results under gpurun_out/round_$TAG)
export TMPDIR=/tmp
O=gpurun_out/round_${TAG:-r01g}
mkdir -p $O
step() { local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name=$rc"; return $rc; }
step bench_c2 600 python3 bench.py || exit $?
step bench_c3 600 python3 bench.py --no-cpu-baseline --config c3 --steps 3 --warmup 1 || exit $?
step bench_c4 600 python3 bench.py --config c4 || exit $?
step bench_c5 600 python3 bench.py --config c5 --steps 5 --warmup 1 || exit $?
for c in c2 c3 c4 c5; do tail -1 $O/bench_$c.log | cut -c1-200; done
