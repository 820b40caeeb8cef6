# Round 3 (session 2): the end-of-round evidence set again on another box
# (r03d's box clocked the issue-bound kernels low): PART=1 of gpu_round.sh,
# TAG=r03e, then the shader-clock probe beside config 2 and 3 (gpu_r03v.sh).
export TMPDIR=/tmp
TAG=r03e PART=1 bash scripts/gpu_round.sh || exit $?
bash scripts/gpu_r03v.sh
