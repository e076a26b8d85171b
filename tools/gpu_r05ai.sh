# round-5: f64 piece length sweep with per-trip pieces and dealt owner pdfs (tuning grid_piece)
set -u
OUT=gpurun_out; mkdir -p $OUT
run() {
  timeout -k 10 200 python tools/bench_configs.py --configs $1 --precision f64 --spp-scale 0.5 --steps 2 ${2:+--tuning $2} \
    2>> $OUT/ab_r05ai.err >> $OUT/ab_r05ai.jsonl || exit $?
}
for round in 1 2; do
  run C5 ""; run C5 grid_piece=16; run C5 grid_piece=32; run C5 grid_piece=44
  run C3 ""; run C3 grid_piece=8; run C3 grid_piece=16
  echo "round $round done"
done
