# Last check of the committed library: smoke, every GPU test, the default
# bench line and the config-5 line.
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python3 bench.py > $O/bench_c2.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py --config c5 --steps 5 --warmup 1 > $O/bench_c5.log 2>&1 || exit $?
for c in c2 c5; do tail -1 $O/bench_$c.log | cut -c1-300; done
