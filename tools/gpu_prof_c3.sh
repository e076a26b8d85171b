#!/bin/bash
# PMC traffic + attribution passes (profile.sh's default sets) of C3 / C5 (tools/bench_configs.py) in one precision:
#   tools/gpu_prof_c3.sh TAG CONFIG PRECISION
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; CFG=$2; PREC=$3
case $CFG in
  C3) WL=C3_simple_grid100_1920x1080_1024spp_depth50;;
  C5) WL=C5_simple_grid1000_1920x1080_256spp_depth50;;
esac
PROG=tools/bench_configs.py WORKLOAD=$WL \
  bash "$ROOT/tools/profile.sh" "$TAG" --configs $CFG --precision $PREC --steps 1
