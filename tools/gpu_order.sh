#!/bin/bash
# item_order (pixel- vs sample-major wave item pool) x group size on C2; then C3/C5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python tools/sweep.py --grid "item_order=0,1;target_tasks=262144,65536" --rounds 2 || exit $?
for x in 0 1; do
  echo "== item_order=$x"
  timeout -k 10 300 python tools/bench_configs.py --configs C3,C5 --spp-scale 0.5 --tuning "item_order=$x" || exit $?
done
