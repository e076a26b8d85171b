#!/bin/bash
# r02 step M: GPU tests + C2 timing (hit64 on/off) + the f32 tolerance at C2
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT
T=${TAG:-r02_m}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/${T}_pytest.log 2>&1
rc=$?; tail -2 $OUT/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/${T}_pytest.log | head -30; exit $rc; }
timeout -k 10 200 python -u tools/sweep.py --rounds 2 --grid "hit64=1,0" 2>&1 | grep -E "cfg|segments" || exit 1
timeout -k 10 200 python -u tools/f32_tolerance.py > $OUT/${T}_tol.json 2>&1 || { tail -5 $OUT/${T}_tol.json; exit 1; }
tail -1 $OUT/${T}_tol.json
