#!/bin/bash
# GPU tests, then the PMC profiles of the f32 kernels (C2 hit64, C3 f32, C5 f32)
#   tools/gpu_f32_prof.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; TAG=$1
timeout -k 10 400 python -u -m pytest tests -m gpu -v -rA --timeout 120 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu_$TAG.log"; [ $rc -eq 0 ] || exit $rc
bash tools/profile.sh "${TAG}_f32" --precision f32 --steps 2 --warmup 2 --no-cpu-baseline --no-modes --configs none > "$OUT/${TAG}_f32_prof.log" 2>&1 || exit $?
echo "profiled C2 f32"
for cfg in C3 C5; do
  bash tools/gpu_prof_c3.sh "${TAG}_${cfg}_f32" $cfg f32 > "$OUT/${TAG}_${cfg}_f32_prof.log" 2>&1 || exit $?
  echo "profiled $cfg f32"
done
