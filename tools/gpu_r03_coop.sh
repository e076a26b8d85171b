#!/bin/bash
# Wave-cooperative light-grid walk: GPU tests, then C5 / C3 A/B against the
# HEAD build (build/head) and over grid_piece.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/coop_pytest.log 2>&1
rc=$?; tail -3 $OUT/coop_pytest.log; [ $rc -le 1 ] || exit $rc
for rd in 1 2; do
  echo "head"; RTW_LIB_OVERRIDE=$PWD/build/variants/head/librtw.so timeout -k 10 300 python -u tools/bench_configs.py --configs C5,C3 --spp-scale 0.25 || exit $?
  for gp in 8 0 4 16; do
    echo "grid_piece=$gp"; timeout -k 10 300 python -u tools/bench_configs.py --configs C5,C3 --spp-scale 0.25 --tuning grid_piece=$gp || exit $?
  done
done
