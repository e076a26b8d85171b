#!/bin/bash
# 8-rank share of C2: per-wave timeline and the task-count knob.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u tools/share_timeline.py run --ns 1,8 2>&1 | grep nranks | tee $OUT/r03_share_timeline.jsonl || exit 1
for tt in 16384 32768 65536 131072 262144; do
  timeout -k 10 200 python -u tools/rank_split_time.py --ns 1,8 --tuning target_tasks=$tt 2>&1 | grep nranks | cut -c1-700 || exit 1
done | tee $OUT/r03_share_tasks.jsonl
