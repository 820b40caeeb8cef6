# Round 3 (session 2): config 3's sizes with every file aliasing one
# cache-resident 4 MiB buffer (no HBM streaming, one small page set) --
# production pair kernel, its no-CRC / no-MD5 probes, and the fused kernel.
export TMPDIR=/tmp
O=gpurun_out/r03x; mkdir -p $O
timeout -k 10 200 python3 scripts/md5_alias_probe.py > $O/alias_pair.txt 2>&1 || exit $?
for m in 0 3 4; do
  FDFS_GPU_PROBE_LIB=1 FDFS_GPU_MD5_PAIR=$m timeout -k 10 200 python3 scripts/md5_alias_probe.py > $O/alias_m$m.txt 2>&1 || exit $?
done
grep -h "aliased" $O/*.txt
