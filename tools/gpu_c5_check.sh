#!/bin/bash
# GPU tests, then C3 / C5 at their configured spp (tools/bench_configs.py), twice.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/c5check_pytest.log 2>&1
rc=$?; tail -3 $OUT/c5check_pytest.log; [ $rc -eq 0 ] || exit $rc
for rd in 1 2; do
  timeout -k 10 400 python -u tools/bench_configs.py --configs C3,C5 2>/dev/null | cut -c1-250 || exit $?
done
