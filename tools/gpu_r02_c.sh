#!/bin/bash
# r02 step C: f64 hit points in the f32 kernel (tuning hit64): statistics and time
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT
T=${TAG:-r02_c}
timeout -k 10 300 python -u tools/f32_tolerance.py --tuning hit64=1 --save $OUT/f32_imgs_$T.npz > $OUT/f32_tol_$T.json 2> $OUT/f32_tol_$T.err
rc=$?; echo "f32_tol rc=$rc"; cat $OUT/f32_tol_$T.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --tuning hit64=1 > $OUT/bench_$T.json 2> $OUT/bench_$T.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench_$T.json
