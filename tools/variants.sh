#!/bin/bash
# A/B timing of compile-time kernel variants (profiling only).
#   tools/variants.sh build "base:" "exp1:-DRTW_EXP=1" ...   (here, CPU: hipcc cross-compiles)
#   tools/variants.sh run base exp1 ...                        (on the GPU box)
# build puts each variant's librtw.so under build/variants/<name>/ (git-ignored,
# shipped to the box with the tree); run times the C2 render with each through
# RTW_LIB_OVERRIDE (tools/sweep.py, default tuning), twice in alternation.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
CS="$ROOT/ray_tracing_weekend_amd/csrc"
B="$ROOT/ray_tracing_weekend_amd/build"
mode="$1"; shift
if [ "$mode" = build ]; then
  for spec in "$@"; do
    name="${spec%%:*}"; defs="${spec#*:}"
    D="$ROOT/build/variants/$name"; mkdir -p "$D"
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fno-slp-vectorize --offload-arch=gfx950 -I$CS -I$ROOT/include \
      -ffp-contract=on $defs -c $CS/render_f32.hip -o $D/render_f32.o || exit 1
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/librtw.so $D/render_f32.o \
      $B/render_f64.o $B/render_f64_lgrid.o $B/capi.o $B/rtw_host.o $B/bvh.o || exit 1
    echo "built $name ($defs)"
  done
else
  OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
  for round in 1 2; do
    for name in "$@"; do
      echo "== $name (round $round)"
      RTW_LIB_OVERRIDE="$ROOT/build/variants/$name/librtw.so" timeout -k 10 300 \
        python tools/sweep.py --grid "${GRID:-bvh_kind=3}" --rounds 2 || exit $?
    done
  done
fi
