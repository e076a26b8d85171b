#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "scheduling or rank_sharding or rank_split" --timeout 300 --timeout-method thread || exit $?
timeout -k 10 300 python tools/sweep.py --grid "xcd=0,2" --rounds 2 || exit $?
for t in xcd=0 xcd=2 xcd=2,target_tasks=65536 xcd=0,target_tasks=65536; do
  echo "== $t"
  timeout -k 10 300 python tools/bench_configs.py --configs C3,C5 --spp-scale 0.5 --tuning "$t" || exit $?
done
