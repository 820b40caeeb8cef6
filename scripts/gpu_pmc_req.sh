# L2 -> fabric request sizes for the dedup kernels (config 5) and the hash
# kernel (config 2): 32-B / 64-B / 128-B (bubble) read requests, DRAM reads,
# and 64-B write requests, each pass on its own run.
export TMPDIR=/tmp
O=${O:-gpurun_out/pmcreq}; mkdir -p $O
B="python3 bench.py --no-cpu-baseline --steps 1 --warmup 1"
for c in c5 c2; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum -d $O/rd_$c -o run --output-format csv -- $B --config $c > $O/rd_$c.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $O/wr_$c -o run --output-format csv -- $B --config $c > $O/wr_$c.log 2>&1 || exit $?
done
echo done
