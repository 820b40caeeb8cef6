export TMPDIR=/tmp
O=gpurun_out/s3a; mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python3 bench.py > $O/bench_c2.log 2>&1 || exit $?
tail -1 $O/bench_c2.log | cut -c1-600
