# Config-3 bench line with its CPU baseline (orc_dio_batch MD5 on the box's
# CPU share), which the round script skips for time.
export TMPDIR=/tmp
O=${O:-gpurun_out/c3cpu}; mkdir -p $O
timeout -k 10 600 python3 -u bench.py --config c3 --steps 3 --warmup 1 > $O/bench_c3.log 2>&1; rc=$?
tail -1 $O/bench_c3.log | cut -c1-200; exit $rc
