#!/bin/bash
# round-3 GPU session: f64 stealing A/B, C3 / C5 full size (tree), the cold
# pilot breakdown, and the C5 cost of the closest-hit query (RTW_EXP=9) and
# of the light pdf (RTW_EXP=2) by repetition.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
CONFIGS=C3,C5 SPP_SCALE=1 bash tools/gpu_ab.sh r03_ab9 "tree,nosteal64" "f64" || exit $?
RTW_DEBUG_LPT=1 timeout -k 10 200 python -u tools/rank_split_time.py --ns 1,8 --reps 2 --tuning lpt_pilot_depth=12 2>&1 | cut -c1-250 || exit 1
for v in exp9 exp2; do
  echo "== $v C5 (spp x0.5)"
  RTW_LIB_OVERRIDE=$PWD/build/variants/$v/librtw.so timeout -k 10 300 python -u tools/bench_configs.py --configs C5 --spp-scale 0.5 2>&1 | cut -c1-260 | grep config || exit 1
done
echo "== tree C5 (spp x0.5)"
timeout -k 10 300 python -u tools/bench_configs.py --configs C5 --spp-scale 0.5 2>&1 | cut -c1-260 | grep config || exit 1
