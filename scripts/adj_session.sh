#!/bin/bash
# Adjoint checks: the adjoint parity tests, then scripts/time_adjoint.py at the headline shape
# (fused vs general) and at configs[2] (general). Each GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-adj}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_adjoint.py tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/time_adjoint.py > "$OUT/time_h.json" 2> "$OUT/time_h.err"
rc=$?; echo "time_h rc=$rc"; cat "$OUT/time_h.json"; [ $rc -eq 0 ] || exit $rc
if [ -n "${CFG2:-}" ]; then
  timeout -k 10 300 python3 scripts/time_adjoint.py $CFG2 > "$OUT/time_c2.json" 2> "$OUT/time_c2.err"
  rc=$?; echo "time_c2 rc=$rc"; cat "$OUT/time_c2.json"; [ $rc -eq 0 ] || exit $rc
fi
echo done
