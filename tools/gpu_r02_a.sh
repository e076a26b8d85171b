#!/bin/bash
# r02 step A: GPU tests (tile interleave, ABI 6), the f32-vs-f64 statistics at
# C2, bench lines (f32 headline, f64 parity mode), rank-split timing (C2 and
# one C4 share).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT
T=${TAG:-r02_a}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rA --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$T.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_gpu_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/f32_tolerance.py > $OUT/f32_tol_$T.json 2> $OUT/f32_tol_$T.err
rc=$?; echo "f32_tol rc=$rc"; cat $OUT/f32_tol_$T.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_$T.json 2> $OUT/bench_$T.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench_$T.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --precision f64 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_f64_$T.json 2> $OUT/bench_f64_$T.err
rc=$?; echo "bench f64 rc=$rc"; cat $OUT/bench_f64_$T.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/rank_split_time.py --ns 1,2,4,8 --reps 2 > $OUT/rank_split_$T.jsonl 2> $OUT/rank_split_$T.err
rc=$?; echo "split rc=$rc"; cat $OUT/rank_split_$T.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/rank_split_time.py --size 3840x2160 --spp 4096 --ns 8 --ranks 0,7 --reps 1 > $OUT/rank_split_c4_$T.jsonl 2> $OUT/rank_split_c4_$T.err
rc=$?; echo "split c4 rc=$rc"; cat $OUT/rank_split_c4_$T.jsonl
exit $rc
