# Round 3 (session 2) final evidence on the final library (MD5 wave read-ahead
# kept): smoke, every gpu test, bench lines and kernel stats (gpu_round.sh
# PART=1, TAG=r03d).
export TMPDIR=/tmp
TAG=r03d PART=1 bash scripts/gpu_round.sh
