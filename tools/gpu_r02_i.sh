#!/bin/bash
# r02 step I: per-rank split timing (hit64 default) vs task size (group), N = 1, 8
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT
for g in 0 4 8 14; do
  t=""; [ $g -gt 0 ] && t="group=$g"
  echo "== group $g"
  timeout -k 10 200 python -u tools/rank_split_time.py --ns 1,8 --reps 3 --tuning "$t" 2>&1 | grep nranks || exit 1
done
echo "== N=8 ranks in reverse order (order effect)"
timeout -k 10 200 python -u tools/rank_split_time.py --ns 8 --reps 3 2>&1 | grep nranks || exit 1
