# dp_split descriptor change: dedup/format/graph parity, then config-5 lines and kernel stats.
export TMPDIR=/tmp
O=gpurun_out/split; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dedup.py tests/test_formats.py tests/test_gpu_graph.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --steps 10 --warmup 2 > $O/c5_$r.log 2>&1 || exit $?
python3 -c "import json;d=json.loads(open('$O/c5_$r.log').read().strip().split('\n')[-1]);print('c5', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_c5 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --config c5 --steps 3 --warmup 1 > $O/stats_c5.log 2>&1 || exit $?
