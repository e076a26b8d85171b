#!/bin/bash
# r02 step H: GPU tests with the f64 Book-1 kernels without prims (3 waves) and
# the f64 tree in LDS, then f64 and f32 C2 timings (new vs base library)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_h.log 2>&1
rc=$?; tail -3 $OUT/pytest_h.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest_h.log | head -30; exit $rc; }
for v in base f64np; do
  echo "== $v f64"
  RTW_LIB_OVERRIDE=$ROOT/build/variants/$v/librtw.so timeout -k 10 300 python -u tools/sweep.py --precision f64 --rounds 1 --grid "bvh_kind=3,1" 2>&1 | grep -E "cfg|segments" || exit 1
done
echo "== f64np f32"
RTW_LIB_OVERRIDE=$ROOT/build/variants/f64np/librtw.so timeout -k 10 300 python -u tools/sweep.py --rounds 2 --grid "hit64=1,0" 2>&1 | grep -E "cfg" || exit 1
