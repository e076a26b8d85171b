#!/bin/bash
# r02 step D: GPU tests (hit64 default), f32 statistics, bench + kernel trace
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT
T=${TAG:-r02_d}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread > $OUT/pytest_gpu_$T.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest_gpu_$T.log | tail -12
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u tools/f32_tolerance.py > $OUT/f32_tol_$T.json 2> $OUT/f32_tol_$T.err
rc=$?; echo "f32_tol rc=$rc"; cat $OUT/f32_tol_$T.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_$T.json 2> $OUT/bench_$T.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench_$T.json; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof_$T" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$ROOT/$OUT/prof_$T.log" 2>&1 )
rc=$?; echo "rocprof rc=$rc"; cat $OUT/prof_$T/run_kernel_stats.csv | cut -c1-200
exit $rc
