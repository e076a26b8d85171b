#!/bin/bash
# r02 step G: GPU tests of the wave-level counters + f64 plane t, then A/B of
# kernel variants (C2, hit64 on/off) and the f32-vs-f64 tolerance of two of them
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_g.log 2>&1
rc=$?; tail -4 $OUT/pytest_g.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest_g.log | head -30; exit $rc; }
GRID="hit64=1,0" timeout -k 10 600 bash tools/variants.sh run base cnt h5 dir0 > $OUT/variants_g.log 2>&1 || { tail -20 $OUT/variants_g.log; exit 1; }
grep -E "==|cfg" $OUT/variants_g.log
for v in cnt dir0; do
  RTW_LIB_OVERRIDE=$ROOT/build/variants/$v/librtw.so timeout -k 10 200 python -u tools/f32_tolerance.py > $OUT/tol_g_$v.json 2>&1 || { tail -5 $OUT/tol_g_$v.json; exit 1; }
  echo "tol $v: $(cat $OUT/tol_g_$v.json)"
done
