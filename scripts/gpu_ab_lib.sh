# Same-box A/B: production lib (FDFS_GPU_PROBE_LIB=0) vs lib/probes (=1),
# alternating.  Usage: O=... ARGS="--config c4" bash scripts/gpu_ab_lib.sh
export TMPDIR=/tmp
O=${O:-gpurun_out/ab}; mkdir -p $O
for r in 1 2 3; do
  for L in 0 1; do
    FDFS_GPU_PROBE_LIB=$L timeout -k 10 300 python3 -u bench.py $ARGS --no-cpu-baseline --steps 10 --warmup 3 > $O/r${r}_L$L.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$O/r${r}_L$L.log').read().strip().splitlines()[-1]); print('lib$L', d['value'], d['roofline']['kernel_ms_avg'])"
  done
done
