#!/bin/bash
# r02 step O: with longest-tiles-first, the wave timeline of C2 and an 8-way
# share, and the task size (target_tasks / group) at N = 1 and N = 8
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT
T=${TAG:-r02_o}
timeout -k 10 200 python -u tools/share_timeline.py run --ns 1,8 > $OUT/${T}_timeline.txt 2>&1 || { tail -5 $OUT/${T}_timeline.txt; exit 1; }
cat $OUT/${T}_timeline.txt
for tu in target_tasks=131072 target_tasks=262144 target_tasks=1048576 group=2 group=8 group=16; do
  timeout -k 10 200 python -u tools/rank_split_time.py --ns 1,8 --reps 3 --tuning $tu > $OUT/${T}_split_$tu.jsonl 2>&1 || { tail -5 $OUT/${T}_split_$tu.jsonl; exit 1; }
  cut -c1-200 $OUT/${T}_split_$tu.jsonl | grep nranks
done
