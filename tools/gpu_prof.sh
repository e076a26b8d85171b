#!/bin/bash
# rocprofv3 kernel-trace + PMC passes of the headline bench (f64), tagged.
#   tools/gpu_prof.sh TAG [bench args]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
bash "$ROOT/tools/profile.sh" "$TAG" ${*:---steps 2 --warmup 2 --no-cpu-baseline --no-modes --configs none}
