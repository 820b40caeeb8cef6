# Round 3 (session 2): md5_stage_kernel (the chunked update_batch path) reading
# a round's row once, outside the lane branches, so block 1's words arrive
# while block 0 is hashed -- stream/MD5 parity, then the chunked path at
# daemon batch sizes (scripts/chunk_sweep.py, MD5 method, 256 KiB chunks):
# this library vs HEAD (ab), alternating.
export TMPDIR=/tmp
O=gpurun_out/r03ze; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -k "md5 or stream or dio or chunk" -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do for v in new ab; do
  case $v in new) E="FDFS_GPU_PROBE_LIB=";; ab) E="FDFS_GPU_PROBE_LIB=ab";; esac
  env $E timeout -k 10 300 python3 scripts/chunk_sweep.py --methods 2 --ns 1024,4096,16384 --calls 30 --graph 0 > $O/sweep_${v}_$r.log 2>&1 || exit $?
  sed "s/^/$v r=$r /" $O/sweep_${v}_$r.log
done; done
