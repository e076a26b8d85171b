#!/bin/bash
# Light grid vs light BVH: parity tests, then C3 / C5 at several grid resolutions.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "light_bvh_equals or c3_scene or c5_scene" > $OUT/grid_tests.log 2>&1 || { tail -30 $OUT/grid_tests.log; exit 1; }
tail -12 $OUT/grid_tests.log
for g in ${GRIDS:-0 4 8 16 32}; do
  echo "== light_grid=$g"
  timeout -k 10 300 python tools/bench_configs.py --configs ${CONFIGS:-C5,C3} --spp-scale 0.5 --steps 2 \
    --tuning light_grid=$g || exit $?
done
