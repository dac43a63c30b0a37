#!/bin/bash
# Round-4 session S: small-batch GNN shapes after the gram fallback (P = 5: time_gnn at B = 1024 and
# 4096, the GNN GPU tests), then PMC passes over the headline training step (fused adjoint counters).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04s
timeout -k 10 600 python -u -m pytest tests/test_gpu_gnn.py tests/test_gpu_hyper_train.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04s/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04s/tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in "1024 5 256 64 25 3" "4096 5 256 64 25 3"; do
  timeout -k 10 300 python3 scripts/time_gnn.py $cfg >> gpurun_out/r04s/timing.txt || exit $?
done
cat gpurun_out/r04s/timing.txt
TAG=r04s_train bash scripts/pmc_cmd.sh scripts/prof_train.py || exit $?
exit 0
