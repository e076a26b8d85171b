#!/bin/bash
# v16 (persistent waves): tests, smoke, bench + rocprof kernel
# trace, PMC passes (FETCH_SIZE / WRITE_SIZE / SQ set, one pass each), and
# the C3 / C5 configurations.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT
STEPS=5 bash tools/gpu_round.sh r01_v16 || exit $?
PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
  bash tools/profile.sh r01_v16 || exit $?
cd "$ROOT"
python3 tools/pmc_summary.py $OUT/prof_r01_v16 --traffic $OUT/r01_v16_traffic.json > $OUT/r01_v16_pmc_summary.txt; echo "pmc summary rc=$?"
cat $OUT/r01_v16_pmc_summary.txt
timeout -k 10 400 python tools/bench_configs.py --configs C3,C5 > $OUT/configs_r01_v16.jsonl 2> $OUT/configs_r01_v16.err; rc=$?
echo "configs rc=$rc"; cat $OUT/configs_r01_v16.jsonl
exit $rc
