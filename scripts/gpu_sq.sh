# SQ stall breakdown for the lane kernel (config 2) in separate PMC passes.
export TMPDIR=/tmp
O=gpurun_out/sq_$(date +%H%M); mkdir -p $O
B="python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 ${BENCH_EXTRA}"
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d $O/p1 -o run --output-format csv -- $B > $O/p1.log 2>&1; echo p1=$?
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE -d $O/p2 -o run --output-format csv -- $B > $O/p2.log 2>&1; echo p2=$?
timeout -k 10 400 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_CYCLES SQ_BUSY_CU_CYCLES -d $O/p3 -o run --output-format csv -- $B > $O/p3.log 2>&1; echo p3=$?
python3 scripts/pmc_summary.py $O sig_lane
