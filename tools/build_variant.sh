#!/bin/bash
# Build the current sources into build/variants/NAME/librtw.so (A/B timing with
# tools/ab_bench.py --variants ...); extra args go to every hipcc compile
# (e.g. -DRTW_WAVES_F64=3).  CPU only.
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME="$1"; shift
CS="$ROOT/ray_tracing_weekend_amd/csrc"; B="$ROOT/ray_tracing_weekend_amd/build"
D="$ROOT/build/variants/$NAME"; mkdir -p "$D"
C="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fno-slp-vectorize --offload-arch=gfx950 -I$CS -I$ROOT/include $*"
$C -ffp-contract=off -c "$CS/render_f64.hip" -o "$D/render_f64.o" &
$C -ffp-contract=on -c "$CS/render_f32.hip" -o "$D/render_f32.o" &
$C -ffp-contract=off -c "$CS/capi.cpp" -o "$D/capi.o" &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$D/librtw.so" "$D/render_f32.o" "$D/render_f64.o" \
  "$D/capi.o" "$B/rtw_host.o" "$B/bvh.o" -ldl
rm -f "$D"/*.o
echo "built $D/librtw.so"
