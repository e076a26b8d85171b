#!/bin/bash
# r02 step B: f32/f64 images for the bias map; N=8 share scheduling sweep
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT
T=${TAG:-r02_b}
timeout -k 10 300 python -u tools/f32_tolerance.py --save $OUT/f32_imgs_$T.npz > $OUT/f32_tol_$T.json 2> $OUT/f32_tol_$T.err
rc=$?; echo "f32_tol rc=$rc"; [ $rc -eq 0 ] || exit $rc
for tn in "group=4" "group=8" "group=16" "group=2" "group=4,persist=1280" "group=4,persist=4096" "group=4,item_order=0"; do
  timeout -k 10 120 python -u tools/rank_split_time.py --ns 8 --ranks 0,3 --reps 3 --tuning $tn >> $OUT/split8_$T.jsonl 2>> $OUT/split8_$T.err || exit $?
done
timeout -k 10 120 python -u tools/rank_split_time.py --ns 1 --reps 2 --tuning group=4 >> $OUT/split8_$T.jsonl 2>> $OUT/split8_$T.err || exit $?
timeout -k 10 120 python -u tools/rank_split_time.py --ns 8 --ranks 0,3 --reps 2 --spp 4000 >> $OUT/split8_$T.jsonl 2>> $OUT/split8_$T.err || exit $?
cat $OUT/split8_$T.jsonl
