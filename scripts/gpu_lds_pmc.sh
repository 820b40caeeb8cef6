# LDS pipe counters of the final hash kernel on config 2 (one pass, 8 SQ counters).
export TMPDIR=/tmp
O=gpurun_out/lds; mkdir -p $O
timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/lds_c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 > $O/lds_c2.log 2>&1 || exit $?
python3 scripts/pmc_summary.py $O/lds_c2 sig_hash | cut -c1-600
