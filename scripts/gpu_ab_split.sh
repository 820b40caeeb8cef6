# A/B of the dedup split chunk (FDFS_GPU_DEDUP_SPLIT=4 -> 4096-entry chunks, default 8192).
export TMPDIR=/tmp
O=gpurun_out/abs; mkdir -p $O
for v in 8 4 8 4; do
  FDFS_GPU_DEDUP_SPLIT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s$v -o run --output-format csv -- python3 bench.py --config c5 --no-cpu-baseline --steps 5 --warmup 1 > $O/c5_$v.log 2>&1 || exit 1
  python3 -c "
import csv,glob
f=glob.glob('$O/s$v/**/*kernel_stats.csv',recursive=True)[0]
print('split=$v', ' '.join(r['Name'].split('(')[0].replace('fdfs::','')+'='+str(round(float(r['AverageNs'])/1e6,3)) for r in csv.DictReader(open(f)) if 'dp_' in r['Name']))"
  rm -rf $O/s$v
done
echo done
