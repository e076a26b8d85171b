#!/bin/bash
# Price parts of the f64 parity kernel's per-segment work:
# librtw.so variants whose render_f64.o repeats one part (RTW_EXP, see
# rtw_probes.hpp: 1 closest-hit query, 2 light pdf sum, 3 stream seeding,
# 4 Lambertian direction sampling, 5 plane tests, 6 closest hit along another
# direction), built HERE (`build` step, CPU) into build_exp/, timed on the box
# (`run` step) by tools/sweep.py --precision f64.  Profiling only.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
CS="$ROOT/ray_tracing_weekend_amd/csrc"
B="$ROOT/ray_tracing_weekend_amd/build"
EXPS="${EXPS:-1 2 3 4 5 6}"
if [ "${1:-run}" = build ]; then
  for e in $EXPS; do
    D="$ROOT/build_exp/f64_exp$e"; mkdir -p "$D"
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fno-slp-vectorize --offload-arch=gfx950 -I$CS -I$ROOT/include \
      -ffp-contract=off -DRTW_EXP=$e -c $CS/render_f64.hip -o $D/render_f64.o || exit 1
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/librtw.so $B/render_f32.o $D/render_f64.o $B/render_f64_lgrid.o \
      $B/capi.o $B/rtw_host.o $B/bvh.o -ldl || exit 1
  done
  exit 0
fi
echo "base"; timeout -k 10 300 python tools/sweep.py --precision f64 --grid bvh_kind=3 --rounds 2 || exit $?
for e in $EXPS; do
  echo "exp $e"
  RTW_LIB_OVERRIDE="$ROOT/build_exp/f64_exp$e/librtw.so" timeout -k 10 300 \
    python tools/sweep.py --precision f64 --grid bvh_kind=3 --rounds 2 || exit $?
done
