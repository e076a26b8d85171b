#!/bin/bash
# Round-3 v8 session: tests + smoke + bench + PMC of the headline and f64
# kernels (tools/gpu_round.sh), a kernel-trace + PMC profile of C5 at its
# configured 256 spp, and the rank-split projection.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out
bash tools/gpu_round.sh r03_v8 || exit $?
PROG=tools/bench_configs.py WORKLOAD=c5_1920x1080_256spp_depth50 \
  bash tools/profile.sh r03_v8_c5 --configs C5 || exit $?
RTW_DEBUG_LPT=1 timeout -k 10 300 python -u tools/rank_split_time.py > $OUT/r03_v8_rank_split.jsonl 2>&1
rc=$?; grep nranks $OUT/r03_v8_rank_split.jsonl | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_configs.py --configs C3,C5 > $OUT/r03_v8_configs_C3_C5.jsonl 2>/dev/null
rc=$?; cut -c1-250 $OUT/r03_v8_configs_C3_C5.jsonl; exit $rc
