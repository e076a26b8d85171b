#!/bin/bash
# Quick GPU session: parity tests, then an optional tuning sweep, then bench.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
TAG="${1:-q}"
timeout -k 10 600 python -m pytest tests -m gpu -q -rfE -x > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest_gpu_$TAG.log"
# any failure ends the GPU session here (a failing kernel may have faulted)
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "${SWEEP:-}" ]; then
  timeout -k 10 600 python tools/sweep.py $SWEEP > "$OUT/sweep_$TAG.log" 2>&1
  rc=$?; echo "sweep rc=$rc"; cat "$OUT/sweep_$TAG.log" | tail -30
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 600 python bench.py $BENCH > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
  rc=$?; echo "bench rc=$rc"; cat "$OUT/bench_$TAG.json"; tail -2 "$OUT/bench_$TAG.err"
fi
exit $rc
