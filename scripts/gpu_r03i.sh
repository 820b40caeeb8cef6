# Round 3: per-kernel counters of the config-5 dedup chain (production library):
# SQ occupancy / waits / instruction mix, LDS bank conflicts, HBM fetch / write.
export TMPDIR=/tmp
O=gpurun_out/r03i; mkdir -p $O
B="python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline"
step() { local name=$1; shift; timeout -s KILL 180 rocprofv3 --pmc "$@" -d $O/$name -o run --output-format csv -- $B > $O/$name.log 2>&1; echo "$name=$?"; }
step sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU || exit 1
step lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE || exit 1
step fetch FETCH_SIZE || exit 1
step write WRITE_SIZE || exit 1
for d in sq lds fetch write; do echo "== $d"; python3 scripts/pmc_summary.py $O/$d | grep -E "dp_|scan" | cut -c1-400; done | tee $O/summary.txt
find $O -name "*.csv" -size +4M -delete
