# round-5 final: GPU tests, smoke, bench; PMC of the changed f64 light-grid kernel (C3 / C5)
set -u
OUT=gpurun_out; mkdir -p $OUT
PROFILE=0 STEPS=5 bash tools/gpu_round.sh r05ad || exit $?
bash tools/gpu_prof_c3.sh r05ad_C3_f64 C3 f64 || exit $?
bash tools/gpu_prof_c3.sh r05ad_C5_f64 C5 f64 || exit $?
