# Round 3 (session 2): the shipped library after the last source change (inert
# probe branch in md5_pair_kernel): smoke and the MD5 / config-3 / stream GPU tests.
export TMPDIR=/tmp
O=gpurun_out/r03zh; mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python3 -u -m pytest tests -m gpu -k "md5 or config3 or offload or smoke or corpus or stream or graph" -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head
exit $rc
