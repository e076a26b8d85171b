#!/bin/bash
# PMC traffic passes of C3 / C5 (tools/bench_configs.py) in one precision:
#   tools/gpu_prof_c3.sh TAG CONFIG PRECISION
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; CFG=$2; PREC=$3
case $CFG in
  C3) WL=C3_simple_grid100_1920x1080_1024spp_depth50;;
  C5) WL=C5_simple_grid1000_1920x1080_256spp_depth50;;
esac
PROG=tools/bench_configs.py WORKLOAD=$WL PMC_SETS="${PMC_SETS:-FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY;SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE}" \
  bash "$ROOT/tools/profile.sh" "$TAG" --configs $CFG --precision $PREC --steps 1
