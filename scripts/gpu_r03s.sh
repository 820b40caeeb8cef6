# Round 3 (session 2): config 3 LDS pipe counters of the pair kernel --
# production, and the probe modes without CRC (3) and without MD5 (4) --
# to tell an LDS bound from an issue bound.
export TMPDIR=/tmp
O=gpurun_out/r03s; mkdir -p $O
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for m in 1 3 4; do
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_MD5_PAIR=$m timeout -k 10 300 rocprofv3 --pmc $C -d $O/lds_m$m -o run --output-format csv -- python3 bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline > $O/lds_m$m.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob, collections
for m in (1, 3, 4):
    f = glob.glob(f"gpurun_out/r03s/lds_m{m}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "md5_pair_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(m, {k: round(v / max(n[k], 1)) for k, v in sorted(acc.items())})
PY
