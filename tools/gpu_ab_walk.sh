#!/bin/bash
# A/B of light-grid walk variants on C3 / C5 (both precisions), alternating.
set -u
OUT=gpurun_out; mkdir -p $OUT
for round in 1 2; do
  for v in "$@"; do
    for p in f32 f64; do
      RTW_LIB_OVERRIDE=build/variants/$v/librtw.so timeout -k 10 200 python tools/bench_configs.py --configs C3,C5 \
        --precision $p --spp-scale 0.5 --steps 2 >> $OUT/ab_walk.jsonl 2>> $OUT/ab_walk.err || exit $?
    done
    echo "round $round $v done"
  done
done
