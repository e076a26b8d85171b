#!/bin/bash
# C5 (1M spheres, 50k lights, 1920x1080, spp x0.25): a fresh kernel-trace +
# PMC profile of the render kernel, then a sweep of the runtime knobs that
# shape its traversal (leaf size, tree kind, light grid, item order).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
PROG=tools/bench_configs.py WORKLOAD=c5_1920x1080_64spp_depth50 \
  bash tools/profile.sh r03_c5 --configs C5 --spp-scale 0.25 || exit $?
for t in "" bvh_leaf=4 bvh_leaf=12 bvh_kind=2 light_grid=16 light_grid=1 item_order=0 bvh_leaf=4,bvh_kind=2; do
  echo "== $t"
  timeout -k 10 200 python -u tools/bench_configs.py --configs C5 --spp-scale 0.25 --tuning "$t" 2>&1 | grep config | cut -c1-420 || exit 1
done > $OUT/r03_c5_sweep.log
cat $OUT/r03_c5_sweep.log
