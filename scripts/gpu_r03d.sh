# Round 3: dedup group with 2048-slot tables / 512-thread workgroups (four
# partitions in flight per CU) vs round 2's form (`make ab`): dedup GPU tests
# on the new library, then c5 lines alternating, then the config-5 PMC passes.
export TMPDIR=/tmp
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dedup.py tests/test_gpu_configs.py -m gpu -v -k "dedup or config5" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for lib in new ab; do
    if [ $lib = ab ]; then export FDFS_GPU_PROBE_LIB=ab; else unset FDFS_GPU_PROBE_LIB; fi
    timeout -k 10 300 python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/c5_${lib}_$r.log 2>&1 || exit $?
    echo "$lib r=$r $(tail -1 $O/c5_${lib}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_avg"])')"
  done
done | tee $O/ab.txt
unset FDFS_GPU_PROBE_LIB
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o c5 -- python3 $R/bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > $R/$O/prof.log 2>&1 || exit $?
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES"; do
  tag=$(echo $pmc | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d $R/$O/pmc_$tag -o c5 -- python3 $R/bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/pmc_$tag.log 2>&1 || exit $?
done
ls -R $R/$O | head -40
