# Upload-shape bench lines on the final library: config 2 CRC only
# (check_file_duplicate=0), config 2 and 3 byte-packed (--align 1).
export TMPDIR=/tmp
O=gpurun_out/shapes; mkdir -p $O
step() { local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name=$rc"; return $rc; }
step bench_c2_crc 600 python3 bench.py --method crc || exit $?
step bench_c2_a1 600 python3 bench.py --align 1 --no-cpu-baseline || exit $?
step bench_c3_a1 600 python3 bench.py --config c3 --align 1 --no-cpu-baseline --steps 3 --warmup 1 || exit $?
for c in bench_c2_crc bench_c2_a1 bench_c3_a1; do tail -1 $O/$c.log | cut -c1-200; done
