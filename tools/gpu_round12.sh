#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
STEPS=5 bash tools/gpu_round.sh r01_v12 || exit $?
timeout -k 10 400 python tools/bench_configs.py --configs C3,C5 > $OUT/configs_r01_v12.jsonl 2> $OUT/configs_r01_v12.err; rc=$?
echo "configs rc=$rc"; cat $OUT/configs_r01_v12.jsonl
exit $rc
