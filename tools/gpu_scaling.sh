#!/bin/bash
# The strong-scaling projection of the f64 headline (C2 shares at N = 1, 2, 4, 8,
# cost-dealt split) and the C4 f64 8-way shares, each share timed on one GPU
#   tools/gpu_scaling.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; TAG=$1
timeout -k 10 400 python -u tools/rank_split_time.py --ns 1,2,4,8 --reps 3 > "$OUT/${TAG}_split_f64.jsonl" 2> "$OUT/${TAG}_split_f64.err" || exit $?
cut -c1-300 "$OUT/${TAG}_split_f64.jsonl"
timeout -k 10 500 python -u tools/rank_split_time.py --size 3840x2160 --spp 4096 --ns 8 --reps 1 > "$OUT/${TAG}_c4_split_f64.jsonl" 2> "$OUT/${TAG}_c4_split_f64.err" || exit $?
cut -c1-300 "$OUT/${TAG}_c4_split_f64.jsonl"
