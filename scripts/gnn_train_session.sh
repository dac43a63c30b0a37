#!/bin/bash
# GNN training path checks: the training-hypernetwork and GNN GPU tests, then the train-step timing
# (scripts/prof_gnn_train.py). Each GPU step has its own time limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-gtrain}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_hyper_train.py tests/test_gpu_gnn.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/prof_gnn_train.py 256 25 5 > "$OUT/train.txt" 2>&1
rc=$?; echo "train rc=$rc"; cat "$OUT/train.txt"; [ $rc -eq 0 ] || exit $rc
if [ "${PROF:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- \
      python3 scripts/prof_gnn_train.py 256 25 3 > "$OUT/prof.txt" 2>&1
  rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
echo done
