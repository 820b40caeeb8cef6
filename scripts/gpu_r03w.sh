# Round 3 (session 2) final evidence on the final library: smoke, every gpu
# test, bench lines and kernel stats (gpu_round.sh PART=1, TAG=r03c), then
# the shader-clock probe idle / beside config 3 / beside config 2.
export TMPDIR=/tmp
TAG=r03c PART=1 bash scripts/gpu_round.sh || exit $?
bash scripts/gpu_r03v.sh
