# Round 3: full GPU suite + smoke on the production library after the hash
# kernel's step generalisation and the dp_split swizzle; config-5 kernel
# stats and the split's LDS counters afterwards.
export TMPDIR=/tmp
O=gpurun_out/r03j; mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo smoke=$? || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 6 --warmup 2 --no-cpu-baseline > $O/stats_c5.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $O/lds -o run --output-format csv -- python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/lds.log 2>&1 || exit $?
find $O -name "*kernel_trace.csv" -delete
for f in $(find $O/stats_c5 -name "*kernel_stats.csv"); do grep -E "dp_|scan" $f | cut -d, -f1-4; done
python3 scripts/pmc_summary.py $O/lds | grep -E "dp_split|dp_tile" | cut -c1-300
find $O -name "*.csv" -size +4M -delete
tail -1 $O/stats_c5.log | cut -c1-400
