export TMPDIR=/tmp
O=gpurun_out/md5; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo smoke=$rc; [ $rc -ne 0 ] && { tail $O/smoke.log; exit $rc; }
timeout -k 10 900 python -m pytest tests/test_gpu_sig.py -q -x -k "edge or small or corpus or mixed" > $O/pytest.log 2>&1; rc=$?; echo pytest=$rc; tail -2 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config c3 --files 24000 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_24k.log 2>&1; rc=$?; echo c3_24k=$rc; tail -1 $O/c3_24k.log | cut -c1-420; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --config c3 --steps 3 --warmup 1 > $O/c3_100k.log 2>&1; rc=$?; echo c3_100k=$rc; tail -3 $O/c3_100k.log | cut -c1-900
