#!/bin/bash
# Price parts of the per-segment work: build librtw.so variants that repeat
# one part (RTW_EXP, see render_kernel.hpp) and time the
# C2 render with each (tools/sweep.py, default tuning).  Profiling only.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
CS="$ROOT/ray_tracing_weekend_amd/csrc"
for e in ${EXPS:-1 2 3 4 5}; do
  D=/tmp/rtw_exp$e; mkdir -p $D
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fno-slp-vectorize --offload-arch=gfx950 -I$CS -I$ROOT/include \
    -ffp-contract=on -DRTW_EXP=$e -c $CS/render_f32.hip -o $D/render_f32.o || exit 1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/librtw.so $D/render_f32.o \
    $ROOT/ray_tracing_weekend_amd/build/render_f64.o $ROOT/ray_tracing_weekend_amd/build/render_f64_lgrid.o $ROOT/ray_tracing_weekend_amd/build/capi.o \
    $ROOT/ray_tracing_weekend_amd/build/rtw_host.o $ROOT/ray_tracing_weekend_amd/build/bvh.o || exit 1
done
echo "base"; timeout -k 10 300 python tools/sweep.py --grid bvh_kind=3 --rounds 2 || exit $?
for e in ${EXPS:-1 2 3 4 5}; do
  echo "exp $e"
  RTW_LIB_OVERRIDE=/tmp/rtw_exp$e/librtw.so timeout -k 10 300 python tools/sweep.py --grid bvh_kind=3 --rounds 2 || exit $?
done
