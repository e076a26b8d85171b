#!/bin/bash
# WRITE_SIZE of the C2 render kernel for variant libraries / tunings:
#   tools/pmc_ab.sh "name:variant:grid" ...   (grid as tools/sweep.py --grid)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
cd /tmp
for spec in "$@"; do
  IFS=: read -r name var grid <<< "$spec"
  RTW_LIB_OVERRIDE=$R/build/variants/$var/librtw.so timeout -s KILL 120 rocprofv3 --pmc ${COUNTER:-WRITE_SIZE} \
    -d $R/gpurun_out/pmc_$name -o p --output-format csv -- python3 $R/tools/sweep.py --rounds 1 --grid "$grid" \
    > $R/gpurun_out/pmc_$name.log 2>&1 || exit 1
  python3 - $R/gpurun_out/pmc_$name/p_counter_collection.csv $name <<'PY'
import csv, sys, collections
per = collections.defaultdict(float)
for row in csv.DictReader(open(sys.argv[1])):
    if "render_kernel" in row["Kernel_Name"]:
        per[row["Dispatch_Id"]] += float(row["Counter_Value"])
v = list(per.values())
print(sys.argv[2], f"{sum(v) / len(v) * 1024 / 1e9:.2f} GB (KB units) per render launch")
PY
done
