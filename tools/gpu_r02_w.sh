#!/bin/bash
# r02 step W: cost-sized task list -- parity subset, rank split, C4 share,
# C3 / C5, one 8-way share's wave timeline
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT
T=${TAG:-r02_w}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/${T}_pytest.log 2>&1
rc=$?; tail -2 $OUT/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/${T}_pytest.log | head -30; exit $rc; }
timeout -k 10 300 python -u tools/rank_split_time.py --ns 1,2,4,8 --reps 3 > $OUT/${T}_rank_split.jsonl 2>&1 || { tail -5 $OUT/${T}_rank_split.jsonl; exit 1; }
python3 -c "
import json,sys
for l in open('$OUT/${T}_rank_split.jsonl'):
    if 'nranks' in l: d=json.loads(l); print(d['nranks'], d['max_rank_ms'], d['per_rank_ms'])"
timeout -k 10 300 python -u tools/rank_split_time.py --ns 2,8 --reps 2 --size 3840x2160 --spp 500 --ranks 0 > $OUT/${T}_split_c4.jsonl 2>&1 || { tail -5 $OUT/${T}_split_c4.jsonl; exit 1; }
cut -c1-200 $OUT/${T}_split_c4.jsonl | grep nranks
timeout -k 10 300 python -u tools/bench_configs.py --configs C3,C5 > $OUT/${T}_configs_C3_C5.jsonl 2>&1 || { tail -5 $OUT/${T}_configs_C3_C5.jsonl; exit 1; }
grep -o "\"config\": \"C[35]\"\|\"kernel_ms\": [0-9.]*" $OUT/${T}_configs_C3_C5.jsonl | paste - -
for k in 4 6; do timeout -k 10 120 python -u tools/share_timeline.py run --ns 8 --rank $k > $OUT/${T}_tl_$k.txt 2>&1 || exit 1; grep -o '{"nranks.*' $OUT/${T}_tl_$k.txt | cut -c1-330; done
