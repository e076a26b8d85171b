#!/bin/bash
# Round-3 v3 session: tests + smoke + bench + PMC of both kernels
# (tools/gpu_round.sh), then the A/B against the HEAD build
# (build/variants/head) and the rank-split projection.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out
bash tools/gpu_round.sh r03_v3 || exit $?
timeout -k 10 600 python -u tools/ab_bench.py --variants tree,head,h64w5,plainw4 --modes f32,plain --rounds 2 > $OUT/r03_v3_ab_head.jsonl 2>&1
rc=$?; cat $OUT/r03_v3_ab_head.jsonl; [ $rc -eq 0 ] || exit $rc
RTW_DEBUG_LPT=1 timeout -k 10 300 python -u tools/rank_split_time.py > $OUT/r03_v3_rank_split.jsonl 2>&1
rc=$?; grep nranks $OUT/r03_v3_rank_split.jsonl | cut -c1-400; exit $rc
