# round-5 measurement session 1: tests, smoke, bench (default line), headline + f32 mode profiles
set -u
OUT=gpurun_out; mkdir -p $OUT
PROFILE=0 STEPS=5 bash tools/gpu_round.sh r05u || exit $?
bash tools/profile.sh r05u --steps 2 --warmup 2 --no-cpu-baseline --no-modes --configs none || exit $?
bash tools/profile.sh r05u_f32 --precision f32 --steps 2 --warmup 2 --no-cpu-baseline --no-modes --configs none || exit $?
bash tools/profile.sh r05u_f32plain --precision f32 --tuning hit64=0 --steps 2 --warmup 2 --no-cpu-baseline --no-modes --configs none || exit $?
