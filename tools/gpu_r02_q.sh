#!/bin/bash
# r02 step Q: the whole GPU suite, rank split, C3/C5 and the default bench
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT
T=${TAG:-r02_q}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/${T}_pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/${T}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/${T}_pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 300 python -u tools/rank_split_time.py --ns 1,2,4,8 --reps 3 > $OUT/${T}_rank_split.jsonl 2>&1 || { tail -5 $OUT/${T}_rank_split.jsonl; exit 1; }
cut -c1-230 $OUT/${T}_rank_split.jsonl | grep nranks
timeout -k 10 300 python -u tools/rank_split_time.py --ns 2,4,8 --reps 2 --size 3840x2160 --spp 500 --ranks 0 > $OUT/${T}_split_c4.jsonl 2>&1 || { tail -5 $OUT/${T}_split_c4.jsonl; exit 1; }
cut -c1-230 $OUT/${T}_split_c4.jsonl | grep nranks
timeout -k 10 300 python -u tools/bench_configs.py --configs C3,C5 > $OUT/${T}_configs_C3_C5.jsonl 2>&1 || { tail -5 $OUT/${T}_configs_C3_C5.jsonl; exit 1; }
cut -c1-300 $OUT/${T}_configs_C3_C5.jsonl
timeout -k 10 400 python -u bench.py > $OUT/${T}_bench.json 2> $OUT/${T}_bench.err || { tail -20 $OUT/${T}_bench.err; exit 1; }
cut -c1-400 $OUT/${T}_bench.json
