# Round 4, sixth box: the PMC passes of the round-end production library
# (scripts/gpu_round.sh PART 2: FETCH_SIZE / WRITE_SIZE per config, SQ
# passes of configs 2 and 3, the loads-only / compute-only probes of config 2).
TAG=r04 PART=2 bash scripts/gpu_round.sh
