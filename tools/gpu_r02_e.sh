#!/bin/bash
# r02 step E: knob sweep for the hit64 kernel + PMC passes of the bench kernel
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT
T=${TAG:-r02_e}
timeout -k 10 300 python -u tools/sweep.py --rounds 2 --grid "bvh_leaf=2,3,4,6,8" > $OUT/sweep_leaf_$T.jsonl 2>&1 || exit $?
timeout -k 10 300 python -u tools/sweep.py --rounds 2 --grid "group=8,14,24,32;persist=1024,2048" > $OUT/sweep_group_$T.jsonl 2>&1 || exit $?
cat $OUT/sweep_leaf_$T.jsonl $OUT/sweep_group_$T.jsonl | grep cfg
PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU;SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
  bash tools/profile.sh $T || exit $?
cd "$ROOT"
python3 tools/pmc_summary.py $OUT/prof_$T --traffic $OUT/${T}_traffic.json book1_simple_1200x800_500spp_depth50 > $OUT/${T}_pmc_summary.txt
cat $OUT/${T}_pmc_summary.txt $OUT/${T}_traffic.json
