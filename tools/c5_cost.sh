#!/bin/bash
# Price parts of the C5 per-segment work (1M spheres, 50k lights): librtw.so
# variants that repeat one part (RTW_EXP, rtw_probes.hpp: 7 = the light pdf
# along the same direction, 9 = the f32 closest-hit traversal along a
# permuted direction) timed by tools/bench_configs.py on C5 at reduced spp.
# Profiling only.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
CS="$ROOT/ray_tracing_weekend_amd/csrc"
B="$ROOT/ray_tracing_weekend_amd/build"
EXPS="${EXPS:-7 9}"
SCALE="${SCALE:-0.25}"
for e in $EXPS; do
  D=$ROOT/build/exp$e; mkdir -p $D; [ -f $D/librtw.so ] && [ "${REBUILD:-0}" = 0 ] && continue
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fno-slp-vectorize --offload-arch=gfx950 -I$CS -I$ROOT/include \
    -ffp-contract=on -DRTW_EXP=$e -c $CS/render_f32.hip -o $D/render_f32.o || exit 1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/librtw.so $D/render_f32.o \
    $B/render_f64.o $B/render_f64_lgrid.o $B/capi.o $B/rtw_host.o $B/bvh.o || exit 1
done
for rd in 1 2; do
  echo "base"; timeout -k 10 300 python -u tools/bench_configs.py --configs C5 --spp-scale "$SCALE" || exit $?
  for e in $EXPS; do
    echo "exp $e"
    RTW_LIB_OVERRIDE=$ROOT/build/exp$e/librtw.so timeout -k 10 300 python -u tools/bench_configs.py --configs C5 \
      --spp-scale "$SCALE" || exit $?
  done
done
