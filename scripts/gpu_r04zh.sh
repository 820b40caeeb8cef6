# Round 4, final library (pair-cooperative loads): round-end evidence, PART 1
# of scripts/gpu_round.sh (smoke, GPU suite, bench lines, kernel stats).
TAG=r04zh PART=1 bash scripts/gpu_round.sh
