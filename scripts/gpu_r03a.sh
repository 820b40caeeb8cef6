# Round 3: the virtual-rank dedup_global tests (small + the 100M config-5 set at world 2/3/8)
export TMPDIR=/tmp
O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dedup.py tests/test_gpu_configs.py -m gpu -v -k "global or config5" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
exit $rc
