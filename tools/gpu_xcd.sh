#!/bin/bash
# XCD-aware task mapping on/off: C2 (tools/sweep.py) and C3/C5 (bench_configs, half spp).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python tools/sweep.py --grid "xcd=1,0" --rounds 3 || exit $?
for x in 1 0 1 0; do
  echo "== xcd=$x"
  timeout -k 10 300 python tools/bench_configs.py --configs C3,C5 --spp-scale 0.5 --tuning "xcd=$x" || exit $?
done
