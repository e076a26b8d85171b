#!/bin/bash
# Round-3 v7 check: GPU tests, C3 / C5 at their configured spp, and a
# kernel-trace + PMC profile of C5 (light grid at 1/2 cell per light).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu_r03_v7.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu_r03_v7.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_configs.py --configs C3,C5 > $OUT/r03_v7_configs_C3_C5.jsonl 2>/dev/null || exit $?
cut -c1-250 $OUT/r03_v7_configs_C3_C5.jsonl
PROG=tools/bench_configs.py WORKLOAD=c5_1920x1080_256spp_depth50 \
  bash tools/profile.sh r03_v7_c5 --configs C5 || exit $?
