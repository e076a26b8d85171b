#!/bin/bash
# C5: per-wave timeline of one 64-spp render (RTW_TIMELINE build) and the
# render time against spp (is there a fixed cost per render?).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u tools/share_timeline.py run --ns 1 --config C5 --spp 64 > $OUT/r03_c5_timeline.jsonl 2>&1
rc=$?; grep nranks $OUT/r03_c5_timeline.jsonl; [ $rc -eq 0 ] || { tail -5 $OUT/r03_c5_timeline.jsonl; exit $rc; }
for s in 0.015625 0.0625 0.125; do
  timeout -k 10 200 python -u tools/bench_configs.py --configs C5 --spp-scale $s 2>&1 | grep config | cut -c1-300 || exit 1
done | tee $OUT/r03_c5_spp.log
