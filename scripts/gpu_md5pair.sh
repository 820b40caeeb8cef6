# MD5 wave-pair kernel: parity (MD5 tests) then c3 bench A/B against the single-wave kernel.
export TMPDIR=/tmp
O=gpurun_out/md5pair; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sig.py -x -q --timeout 200 --timeout-method thread \
  -k "md5 or host_batch" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 1 0; do
  FDFS_GPU_MD5_PAIR=$v timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --steps 5 --warmup 2 \
    > $O/c3_pair$v.log 2>&1 || { tail -5 $O/c3_pair$v.log; exit 1; }
  echo "pair=$v"; tail -1 $O/c3_pair$v.log | cut -c1-400
done
