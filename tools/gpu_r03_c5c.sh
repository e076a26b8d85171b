#!/bin/bash
# Tile costs from node visits + sphere tests + segments (was: segments):
# C5 at full spp without / with longest-tiles-first (timeline + bench_configs),
# C3, and the C2 A/B against the HEAD build.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
T=${TAG:-r03_c5c}
for t in "" "lpt=2"; do
  timeout -k 10 300 python -u tools/share_timeline.py run --ns 1 --config C5 --tuning "$t" 2>&1 | grep nranks || exit 1
done | tee $OUT/${T}_timeline.jsonl
for t in "" "lpt=2"; do
  for v in tree head; do
    if [ $v = tree ]; then unset RTW_LIB_OVERRIDE; else export RTW_LIB_OVERRIDE=$PWD/build/variants/$v/librtw.so; fi
    echo "== $v $t"
    timeout -k 10 300 python -u tools/bench_configs.py --configs C3,C5 --tuning "$t" 2>&1 | grep config | cut -c1-300 || exit 1
  done
done | tee $OUT/${T}_configs.log
unset RTW_LIB_OVERRIDE
timeout -k 10 600 python -u tools/ab_bench.py --variants tree,head --modes f32 --rounds 2 2>&1 | grep -v amdgpu | tee $OUT/${T}_ab.jsonl
