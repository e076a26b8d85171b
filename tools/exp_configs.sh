#!/bin/bash
# Price parts of the C3 / C5 work with RTW_EXP variants (tools/variants.sh build ...).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${VARIANTS:-cur exp1 exp6}; do
  echo "== $v"
  RTW_LIB_OVERRIDE=$PWD/build/variants/$v/librtw.so timeout -k 10 300 python tools/bench_configs.py --configs ${CONFIGS:-C5,C3} --spp-scale 0.5 --steps 2 ${TUNING:+--tuning $TUNING} || exit $?
done
