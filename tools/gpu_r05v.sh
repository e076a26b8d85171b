# round-5 measurement session 2: C3 / C5 profiles in both precisions
set -u
for c in C3 C5; do for p in f64 f32; do
  bash tools/gpu_prof_c3.sh r05v_${c}_$p $c $p || exit $?
done; done
