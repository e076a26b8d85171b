#!/bin/bash
# NaN-ray traversal skip + cooperative light-grid walk: GPU tests, C2 bench
# against the HEAD build, C3 / C5 at their configured spp over grid_piece.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/coop2_pytest.log 2>&1
rc=$?; tail -3 $OUT/coop2_pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u tools/ab_bench.py --variants tree,head --modes f32,f64 --rounds 2 || exit $?
for gp in 8 4 6; do
  echo "grid_piece=$gp"; timeout -k 10 300 python -u tools/bench_configs.py --configs C5,C3 --tuning grid_piece=$gp || exit $?
done
echo "head"; RTW_LIB_OVERRIDE=$PWD/build/variants/head/librtw.so timeout -k 10 300 python -u tools/bench_configs.py --configs C5,C3 || exit $?
