# round-5: clock sections of the f64 walk's owner phase (merges vs dealt pdfs)
set -u
OUT=gpurun_out; mkdir -p $OUT
for a in "--config C5 --precision f64 --spp 32" "--config C3 --precision f64 --spp 256"; do
  timeout -k 10 200 python tools/clock_profile.py run $a >> $OUT/clock_r05z.jsonl 2>> $OUT/clock_r05z.err || exit $?
done
