# Round 4, final library (grouped Horner, ELF exact fold once per file):
# round-end evidence, both parts of scripts/gpu_round.sh under TAG r04z.
TAG=r04z PART=1 bash scripts/gpu_round.sh || exit $?
TAG=r04z PART=2 bash scripts/gpu_round.sh
