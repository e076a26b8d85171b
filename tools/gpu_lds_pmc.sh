#!/bin/bash
# One PMC pass of the headline bench for the LDS counters (bank / address
# conflicts, LDS-active and LDS-wait cycles).   tools/gpu_lds_pmc.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
PMC_SETS="SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_LDS_UNALIGNED_STALL SQ_WAVES" \
  bash tools/profile.sh "${1:-lds}" --steps 2 --warmup 2 --no-cpu-baseline --no-modes --configs none
