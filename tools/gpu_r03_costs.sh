#!/bin/bash
# C2 cost of each part of the per-segment work by repetition (RTW_EXP builds,
# csrc/rtw_probes.hpp): the in-tree kernel vs the variants that repeat one part.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TESTS=0 ROUNDS=1 bash tools/gpu_ab.sh r03_costs "tree,exp2,exp3,exp4,exp8,exp10,exp11" "f32"
