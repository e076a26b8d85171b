#!/bin/bash
# rocprofv3 on the bench workload: kernel-trace stats + separate PMC passes
# (never combined with sys/runtime traces).  Usage: profile.sh TAG [bench args]
# PROG=tools/bench_configs.py profiles that program instead of bench.py (C3 / C5).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
TAG="$1"; shift
ARGS="${*:---steps 2 --warmup 2 --no-cpu-baseline --no-modes --configs none}"
PROG="$ROOT/${PROG:-bench.py}"
export TMPDIR=/tmp
cd /tmp
bad() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
if [ ! -f "$OUT/rocprof_counters.txt" ]; then
  timeout -k 10 120 rocprofv3 -L > "$OUT/rocprof_counters.txt" 2>&1; echo "list rc=$?"
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o trace --output-format csv \
  -- python3 "$PROG" $ARGS > "$OUT/prof_${TAG}_trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; if bad $rc; then exit $rc; fi
# counter sets separated by ';' (PMC_SETS overrides the default list)
# (the last two sets attribute the wave-cycles: cycles issuing each
# instruction type, LDS waits, branches; outstanding-instruction levels for
# the memory latencies -- tools/pmc_summary.py --attrib)
SETS="${PMC_SETS:-FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY;SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE;SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH;SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_INSTS_FLAT SQ_WAVE_CYCLES}"
i=0
IFS=';' read -ra SETLIST <<< "$SETS"
for set in "${SETLIST[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set -d "$OUT/prof_$TAG/pmc$i" -o pmc --output-format csv \
    -- python3 "$PROG" $ARGS > "$OUT/prof_${TAG}_pmc$i.log" 2>&1
  rc=$?; echo "pmc$i ($set) rc=$rc"; if bad $rc; then exit $rc; fi
done
# per-launch means + the traffic / fractions file bench.py reads, stamped with
# the ISA hash of the profiled kernel in the library that ran (WORKLOAD names
# the bench configuration)
python3 "$ROOT/tools/pmc_summary.py" "$OUT/prof_$TAG" --traffic "$OUT/prof_${TAG}_traffic.json" \
  "${WORKLOAD:-book1_simple_1200x800_500spp_depth50}" > "$OUT/prof_${TAG}_pmc_summary.txt"
rc=$?; echo "summary rc=$rc"; cat "$OUT/prof_${TAG}_pmc_summary.txt"
exit $rc
