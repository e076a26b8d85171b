#!/bin/bash
# C3 / C5 at their configured size (GPU tests + full-spp timings) and the
# C2 / C4 rank-split projection with pilots and the gather estimate.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT; T=${1:-r03}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/${T}_pytest_c3c5.log 2>&1
rc=$?; tail -3 $OUT/${T}_pytest_c3c5.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/${T}_pytest_c3c5.log | head -30; exit $rc; }
timeout -k 10 400 python -u tools/bench_configs.py --configs C3,C5 > $OUT/${T}_configs_C3_C5.jsonl 2>&1 || { tail -5 $OUT/${T}_configs_C3_C5.jsonl; exit 1; }
cut -c1-300 $OUT/${T}_configs_C3_C5.jsonl
timeout -k 10 300 python -u tools/rank_split_time.py --ns 1,2,4,8 --reps 3 > $OUT/${T}_rank_split.jsonl 2>&1 || { tail -5 $OUT/${T}_rank_split.jsonl; exit 1; }
cut -c1-420 $OUT/${T}_rank_split.jsonl
timeout -k 10 300 python -u tools/rank_split_time.py --ns 8 --reps 1 --size 3840x2160 --spp 4096 --ranks 0 > $OUT/${T}_rank_split_c4_share.jsonl 2>&1 || { tail -5 $OUT/${T}_rank_split_c4_share.jsonl; exit 1; }
cut -c1-420 $OUT/${T}_rank_split_c4_share.jsonl
