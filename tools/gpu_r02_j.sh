#!/bin/bash
# r02 step J: N=8 share time (ranks 0, 3) vs persistent grid size and task size
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
for t in "persist=1024" "persist=1024,group=2" "persist=2048,group=2" "persist=4096" "persist=1024,group=4" "persist=768" "persist=0"; do
  echo "== $t"
  timeout -k 10 200 python -u tools/rank_split_time.py --ns 8 --ranks 0,3 --reps 3 --tuning "$t" 2>&1 | grep nranks || exit 1
done
