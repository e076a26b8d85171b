#!/bin/bash
# C2 rank splits: the counting (first) render's task size, and the steady task count.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
for t in "" lpt_cold_group=1 lpt_cold_group=2 lpt_cold_group=4 target_tasks=262144 target_tasks=524288; do
  timeout -k 10 200 python -u tools/rank_split_time.py --ns 1,4,8 --tuning "$t" 2>&1 | grep nranks | cut -c1-520 || exit 1
done | tee $OUT/r03_share2.jsonl
