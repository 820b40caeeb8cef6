# Round 4: config 1 (ELF chain bound) alternating between the pair-load
# library and the previous one (make ab): the chain loop's instruction order is
# identical in both, the registers differ.
export TMPDIR=/tmp
O=gpurun_out/r04zd
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
show() { tail -1 $O/$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$1', d['ms_per_step'], r.get('kernel_ms_avg'), r.get('chain_floor_ms'))"; }
B1="python3 bench.py --no-cpu-baseline --config c1 --steps 2 --warmup 1"
for k in 1 2 3; do
  step old_$k 600 env FDFS_GPU_PROBE_LIB=ab $B1 || exit $?; show old_$k
  step new_$k 600 $B1 || exit $?; show new_$k
done
