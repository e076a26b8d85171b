#!/bin/bash
# One GPU session: parity tests, smoke, bench, then rocprofv3 kernel-trace +
# PMC passes of the headline (f64 parity, round 4 on) and the f32 hit64
# kernels, each summarised on the box against the library that ran
# (ISA-hash stamped).
# Stops at the first fault-type exit (abort/segfault/timeout); a plain test
# failure (pytest rc 1) still lets the measurement steps run.
#   tools/gpu_round.sh TAG          (PROFILE=0: no rocprofv3 steps)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
TAG="${1:-r03}"
STEPS="${STEPS:-5}"

fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }

timeout -k 10 600 python -u -m pytest tests -m gpu -v -rA --timeout 120 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu_$TAG.log"
if fatal $rc; then exit $rc; fi

timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke_$TAG.log"
if fatal $rc; then exit $rc; fi

timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 2 > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; echo "bench rc=$rc"; cut -c1-1500 "$OUT/bench_$TAG.json"; tail -3 "$OUT/bench_$TAG.err"
if [ $rc -ne 0 ]; then exit $rc; fi

if [ "${PROFILE:-1}" = "1" ]; then
  bash "$ROOT/tools/profile.sh" "$TAG" --steps 2 --warmup 2 --no-cpu-baseline --no-modes --configs none || exit $?
  bash "$ROOT/tools/profile.sh" "${TAG}_f32" --precision f32 --steps 2 --warmup 2 --no-cpu-baseline --no-modes \
    --configs none || exit $?
fi
exit 0
