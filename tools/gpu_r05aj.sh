# round-5 final check: GPU tests, smoke, bench line
set -u
PROFILE=0 STEPS=5 bash tools/gpu_round.sh r05aj || exit $?
