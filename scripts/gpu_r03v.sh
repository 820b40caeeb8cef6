# Round 3 (session 2): shader clock idle and under the config 2 / config 3
# signature batches (scripts/clock_under_load.py, scripts/probes/clock_probe).
export TMPDIR=/tmp
O=gpurun_out/r03v; mkdir -p $O
timeout -k 10 60 scripts/probes/clock_probe 5 200 20 > $O/idle.txt 2>&1 || exit $?
cat $O/idle.txt
timeout -k 10 200 python3 scripts/clock_under_load.py c3 20 > $O/c3.txt 2>&1 || exit $?
timeout -k 10 200 python3 scripts/clock_under_load.py c2 12 > $O/c2.txt 2>&1 || exit $?
for f in c3 c2; do echo "== $f"; grep -v sample $O/$f.txt; grep sample $O/$f.txt | awk '{print $3}' | sort -n | awk '{a[NR]=$1} END {print "n", NR, "min", a[1], "median", a[int(NR/2)+1], "max", a[NR]}'; done
