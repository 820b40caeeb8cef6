export TMPDIR=/tmp
O=gpurun_out/md5probe; mkdir -p $O
timeout -k 10 300 python scripts/md5_probe.py > $O/probe.log 2>&1; rc=$?; echo probe=$rc; cat $O/probe.log | grep -v amdgpu.ids
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU -d $O/sq -o run --output-format csv -- python3 bench.py --config c3 --files 24000 --steps 1 --warmup 1 --no-cpu-baseline > $O/sq.log 2>&1; echo sq=$?
python3 scripts/pmc_summary.py $O/sq sig_lane
