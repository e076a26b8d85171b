#!/bin/bash
# r02 step N: longest-tiles-first task order -- parity (knobs, rank split),
# rank-split timing with lpt on / off, the default bench
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT
T=${TAG:-r02_n}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "scheduling or rank_split" > $OUT/${T}_pytest.log 2>&1
rc=$?; tail -2 $OUT/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/${T}_pytest.log | head -30; exit $rc; }
timeout -k 10 300 python -u tools/rank_split_time.py --ns 1,2,4,8 --reps 3 > $OUT/${T}_split_lpt1.jsonl 2>&1 || { tail -5 $OUT/${T}_split_lpt1.jsonl; exit 1; }
cut -c1-230 $OUT/${T}_split_lpt1.jsonl
timeout -k 10 300 python -u tools/rank_split_time.py --ns 1,8 --reps 3 --tuning lpt=0 > $OUT/${T}_split_lpt0.jsonl 2>&1 || { tail -5 $OUT/${T}_split_lpt0.jsonl; exit 1; }
cut -c1-230 $OUT/${T}_split_lpt0.jsonl
timeout -k 10 300 python -u tools/rank_split_time.py --ns 2,4 --reps 2 --size 3840x2160 --spp 500 --ranks 0 > $OUT/${T}_split_c4.jsonl 2>&1 || { tail -5 $OUT/${T}_split_c4.jsonl; exit 1; }
cut -c1-230 $OUT/${T}_split_c4.jsonl
timeout -k 10 400 python -u bench.py --no-modes --no-cpu-baseline > $OUT/${T}_bench.json 2> $OUT/${T}_bench.err || { tail -20 $OUT/${T}_bench.err; exit 1; }
cut -c1-400 $OUT/${T}_bench.json
