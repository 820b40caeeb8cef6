# CRC path: parity tests (incl. config 4's GiB files), c4 and c2 CRC-only lines.
export TMPDIR=/tmp
O=${O:-gpurun_out/crc}; mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-1} | cut -c1-200; return $rc
}
TAILN=2 step pytest 900 python3 -u -m pytest tests/test_gpu_sig.py tests/test_gpu_configs.py::test_config4_gib_files tests/test_gpu_stream.py tests/test_formats.py -x -v --timeout 400 --timeout-method thread || exit $?
for r in 1 2; do
step c4_$r 300 python3 -u bench.py --config c4 --no-cpu-baseline --steps 10 --warmup 3 || exit $?
python3 -c "import json; d=json.loads(open('$O/c4_$r.log').read().strip().splitlines()[-1]); print('c4', d['value'], d['roofline']['kernel_ms_avg'], d['roofline']['frac'])"
step c2crc_$r 300 python3 -u bench.py --method crc --no-cpu-baseline --steps 10 --warmup 3 || exit $?
python3 -c "import json; d=json.loads(open('$O/c2crc_$r.log').read().strip().splitlines()[-1]); print('c2crc', d['value'], d['roofline']['kernel_ms_avg'], d['roofline']['frac'])"
done
echo done
