# Round 4: config 3 issue-priority policies against the oldest-wave-first
# default (probe build): PM 6 = by remaining rounds, PM 7 = young first chunks
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
B="python3 bench.py --config c3 --no-cpu-baseline --steps 5 --warmup 2"
show() { echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $O/$1.log) $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
export FDFS_GPU_PROBE_LIB=1
for k in 1 2; do
for p in 1 7 8; do
  FDFS_GPU_MD5_PAIR=$p step c3_p${p}_$k 400 $B || exit $?
  show c3_p${p}_$k
done
done
