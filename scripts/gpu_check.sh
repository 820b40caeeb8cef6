# GPU round-trip: smoke, parity tests, bench (c2 default, c4), rocprof stats.
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo smoke=$rc
if [ $rc -ne 0 ]; then tail -30 gpurun_out/smoke.log; exit $rc; fi
timeout -k 10 1200 python -m pytest tests -m gpu -q -x ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest.log 2>&1; rc=$?; echo pytest=$rc
tail -15 gpurun_out/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/bench_c2.log 2>&1; rc=$?; echo bench_c2=$rc
tail -2 gpurun_out/bench_c2.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --config c4 --steps 5 > gpurun_out/bench_c4.log 2>&1; rc=$?; echo bench_c4=$rc
tail -2 gpurun_out/bench_c4.log
