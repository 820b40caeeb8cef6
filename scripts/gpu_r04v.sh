# Round 4: ELF as one asm statement per 16-byte vector (one hipcc asm-boundary
# s_nop per vector instead of four) and the slice-by-16 CRC XORs as v_bitop3
# builtins (no asm statements around the lookups; also the MD5 loader's CRC).
# GPU suite, then configs 2 and 3 alternating against the previous library.
export TMPDIR=/tmp
O=gpurun_out/r04v
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name=$rc"; return $rc
}
show() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' $O/$1.log)"; }
step pytest 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread; rc=$?
tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
B2="python3 bench.py --no-cpu-baseline --steps 10 --warmup 3"
B3="python3 bench.py --config c3 --no-cpu-baseline --steps 3 --warmup 1"
for k in 1 2 3; do
  step new_$k 300 $B2 || exit $?; show new_$k
  FDFS_GPU_PROBE_LIB=ab step old_$k 300 $B2 || exit $?; show old_$k
done
for k in 1 2; do
  step c3new_$k 300 $B3 || exit $?; show c3new_$k
  FDFS_GPU_PROBE_LIB=ab step c3old_$k 300 $B3 || exit $?; show c3old_$k
done
