#!/bin/bash
# v13 (light grid): tests, smoke, bench + rocprof, the C3 / C5 configurations
# and their kernel-trace summary.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
STEPS=5 bash tools/gpu_round.sh r01_v13 || exit $?
timeout -k 10 400 python tools/bench_configs.py --configs C3,C5 > $OUT/configs_r01_v13.jsonl 2> $OUT/configs_r01_v13.err; rc=$?
echo "configs rc=$rc"; cat $OUT/configs_r01_v13.jsonl
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_configs_r01_v13" -o run \
    --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" --configs C3,C5 --spp-scale 0.25 \
    > "$GRAFT_REPO_ROOT/$OUT/prof_configs_r01_v13.log" 2>&1 )
rc=$?; echo "rocprof configs rc=$rc"
exit $rc
