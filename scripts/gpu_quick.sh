# smoke + sig parity subset + c2 bench + FETCH_SIZE pass for the lane kernel
export TMPDIR=/tmp
O=gpurun_out/quick; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo smoke=$rc; [ $rc -ne 0 ] && { tail $O/smoke.log; exit $rc; }
timeout -k 10 900 python -m pytest tests/test_gpu_sig.py -q -x > $O/pytest.log 2>&1; rc=$?; echo pytest=$rc; tail -2 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2.log 2>&1; rc=$?; echo c2=$rc; tail -1 $O/c2.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/fetch.log 2>&1; echo fetch=$?
python3 scripts/pmc_summary.py $O/fetch sig_lane
