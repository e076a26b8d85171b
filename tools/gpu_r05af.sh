# round-5 final: PMC of the light-grid kernels (C3 / C5, both precisions), then the bench line
set -u
for c in C3 C5; do for p in f64 f32; do
  bash tools/gpu_prof_c3.sh r05af_${c}_$p $c $p || exit $?
done; done
