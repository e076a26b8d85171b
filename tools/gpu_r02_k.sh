#!/bin/bash
# r02 step K: the guided tail + resident grid vs task size at N = 1 and 8
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT
for t in "item_order=0" "item_order=0,group=14" "group=14,persist=4096" "group=14,persist=512" "target_tasks=1048576" "group=2" "persist=0"; do
  echo "== $t"
  timeout -k 10 200 python -u tools/rank_split_time.py --ns 1 --reps 2 --tuning "$t" > $OUT/k1.log 2>&1 || { tail -5 $OUT/k1.log; exit 1; }
  timeout -k 10 200 python -u tools/rank_split_time.py --ns 8 --ranks 0,3 --reps 3 --tuning "$t" > $OUT/k8.log 2>&1 || { tail -5 $OUT/k8.log; exit 1; }
  python3 -c "import json; a=json.loads(open('$OUT/k1.log').read().strip().splitlines()[-1]); b=json.loads(open('$OUT/k8.log').read().strip().splitlines()[-1]); print('N1 %.2f ms  N8 share %s ms  ratio %.2f' % (a['max_rank_ms'], b['per_rank_ms'], a['max_rank_ms']/b['max_rank_ms']))"
done
