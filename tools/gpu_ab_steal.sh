#!/bin/bash
# A/B of prebuilt render-kernel variants (build/variants/<name>/librtw.so):
# GPU tests with the in-tree library, then C2 times per variant over a tuning
# grid (GRID, default hit64 x bvh_kind), alternating; F64=1 adds the f64 C2
# time of the in-tree library; CONFIGS=C3,C5 the other configs per variant.
#   tools/gpu_ab_steal.sh TAG v1 v2 ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
T=$1; shift
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/${T}_pytest.log 2>&1
rc=$?; tail -3 $OUT/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/${T}_pytest.log | head -30; exit $rc; }
for r in 1 2; do for v in "$@"; do
  echo "== $v C2 (round $r)"
  RTW_LIB_OVERRIDE=$PWD/build/variants/$v/librtw.so timeout -k 10 300 python -u tools/sweep.py --grid "${GRID:-hit64=1,0;bvh_kind=3,1}" --rounds 2 2>&1 | grep -E "cfg|segments" || exit 1
done; done
if [ "${F64:-0}" = 1 ]; then
  echo "== in-tree f64 C2"
  timeout -k 10 300 python -u tools/sweep.py --precision f64 --grid "bvh_kind=3,1" --rounds 2 2>&1 | grep -E "cfg|segments" || exit 1
fi
if [ -n "${CONFIGS:-}" ]; then for v in "$@"; do
  echo "== $v $CONFIGS"
  RTW_LIB_OVERRIDE=$PWD/build/variants/$v/librtw.so timeout -k 10 300 python -u tools/bench_configs.py --configs $CONFIGS --spp-scale 0.25 2>&1 | cut -c1-330 | grep config || exit 1
done; fi
