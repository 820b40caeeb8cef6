# MD5 staged kernel: parity, A/B vs the lane-load path, c3 bench; SQ/TCP counters for c2.
export TMPDIR=/tmp
O=gpurun_out/exp2; mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-1} | cut -c1-700; return $rc
}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
TAILN=3 step pytest 600 python -u -m pytest tests/test_gpu_sig.py -x -q --timeout 300 --timeout-method thread -k "md5 or edge or corpus or mixed" || exit $?
TAILN=4 step probe_staged 300 python -u scripts/lane_probe.py 1000 || exit $?
FDFS_GPU_MD5_LANE=1 TAILN=4 step probe_lane 300 python -u scripts/lane_probe.py 1000 || exit $?
step c3 400 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline || exit $?
step pmc_sq_c2 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $O/sq_c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 || exit $?
python3 scripts/pmc_summary.py $O/sq_c2 sig_lane
step pmc_tcp_c2 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_REQUEST TCP_TCP_LATENCY -d $O/tcp_c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 || exit $?
python3 scripts/pmc_summary.py $O/tcp_c2 sig_lane
echo done
