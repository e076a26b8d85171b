set -u
OUT=gpurun_out; mkdir -p $OUT
for P in 4 8 11 16 22 32; do
  for p in f64 f32; do
    timeout -k 10 200 python tools/bench_configs.py --configs C3,C5 --precision $p --spp-scale 0.5 --steps 2 \
      --tuning grid_piece=$P >> $OUT/piece_sweep.jsonl 2>> $OUT/piece_sweep.err || exit $?
  done
  echo "P=$P done"
done
