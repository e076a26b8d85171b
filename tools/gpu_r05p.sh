# round-5: clock profile of the light-grid walks' sections (RTW_CLOCK build)
set -u
OUT=gpurun_out; mkdir -p $OUT
for a in "--config C3 --precision f64 --spp 256" "--config C3 --precision f32 --spp 256" "--config C5 --precision f32 --spp 64" "--config C5 --precision f64 --spp 32"; do
  timeout -k 10 200 python tools/clock_profile.py run $a >> $OUT/clock_r05p.jsonl 2>> $OUT/clock_r05p.err || exit $?
done
