# Round 4, final library (compact MFMA B table): round-end evidence, both
# parts of scripts/gpu_round.sh (tests, bench lines, kernel stats; PMC
# passes and the config-2 probes) under TAG r04m.
TAG=r04m PART=1 bash scripts/gpu_round.sh || exit $?
TAG=r04m PART=2 bash scripts/gpu_round.sh
