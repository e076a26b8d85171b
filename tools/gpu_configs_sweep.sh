#!/bin/bash
# C3 / C5 at a quarter of their spp under BVH traversal variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for t in "bvh_kind=1" "bvh_kind=2" "bvh_kind=0" "bvh_kind=1,bvh_leaf=2" "bvh_kind=1,bvh_leaf=8"; do
  echo "== $t"
  timeout -k 10 300 python tools/bench_configs.py --configs C3,C5 --spp-scale ${SPP_SCALE:-0.25} --tuning "$t" || exit $?
done
