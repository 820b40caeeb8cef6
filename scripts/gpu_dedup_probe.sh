# Dedup group A/B: production timing, then the probe build's variants
# (FDFS_GPU_DEDUP_PROBE 1 = no confirmation reads, 2 = no final stores, 3 = both).
export TMPDIR=/tmp
O=${O:-gpurun_out/ddp}; mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; grep -v amdgpu.ids $O/$name.log | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline'].get('kernel_ms_avg'))" ; return $rc
}
step c5 300 python3 -u bench.py --config c5 --no-cpu-baseline --steps 10 --warmup 2 || exit $?
for m in 0 1 2 3; do
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_DEDUP_PROBE=$m step probe$m 300 python3 -u bench.py --config c5 --no-cpu-baseline --steps 10 --warmup 2 || exit $?
done
step stats_c5 300 rocprofv3 --kernel-trace --stats -d $O/stats_c5 -o run --output-format csv -- python3 bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 || exit $?
echo done
