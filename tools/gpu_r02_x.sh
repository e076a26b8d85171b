#!/bin/bash
# Round-2 session x: GPU tests with the in-tree library and with a variant
# (LIBV, default lp), then C2 render times of the variants listed in VARIANTS
# in f64 and f32 (tools/sweep.py through RTW_LIB_OVERRIDE).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
LIBV="${LIBV:-lp}"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu_x.log" 2>&1
rc=$?; echo "pytest (in-tree) rc=$rc"; tail -2 "$OUT/pytest_gpu_x.log"
[ $rc -ne 0 ] && exit $rc
RTW_LIB_OVERRIDE="$ROOT/build/variants/$LIBV/librtw.so" timeout -k 10 300 python -u -m pytest tests -m gpu -x -q \
  --timeout 120 --timeout-method thread > "$OUT/pytest_gpu_x_$LIBV.log" 2>&1
rc=$?; echo "pytest ($LIBV) rc=$rc"; tail -2 "$OUT/pytest_gpu_x_$LIBV.log"
[ $rc -ne 0 ] && exit $rc
for prec in ${PRECS:-f64 f32}; do
  for v in ${VARIANTS:-base lp}; do
    echo "== $v $prec"
    RTW_LIB_OVERRIDE="$ROOT/build/variants/$v/librtw.so" timeout -k 10 300 \
      python tools/sweep.py --precision $prec --grid "bvh_kind=3" --rounds 3 || exit $?
  done
done
