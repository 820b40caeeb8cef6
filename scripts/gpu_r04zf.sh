# Round 4: the final tree's smoke and default bench line.
export TMPDIR=/tmp
O=gpurun_out/r04zf
mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-1500
