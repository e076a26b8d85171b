#!/bin/bash
# A/B of two prebuilt librtw.so (build/variants/<a>, <b>): C2 sweep, then C3/C5, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A=${1:-prev}; B=${2:-cur}
for r in 1 2; do for v in $A $B; do
  echo "== $v C2"
  RTW_LIB_OVERRIDE=$PWD/build/variants/$v/librtw.so timeout -k 10 300 python tools/sweep.py --grid "item_order=1" --rounds 2 || exit $?
done; done
if [ -n "${CONFIGS:-}" ]; then for v in $A $B; do
  echo "== $v $CONFIGS"
  RTW_LIB_OVERRIDE=$PWD/build/variants/$v/librtw.so timeout -k 10 300 python tools/bench_configs.py --configs $CONFIGS --spp-scale 0.5 || exit $?
done; fi
