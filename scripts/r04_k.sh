#!/bin/bash
# Round-4 session K: layer 1's Atb half hoisted out of the GNN iteration loop (dadmm_hyper_gcn_ex):
# GPU tests of the hypernetwork / GNN paths, then A/B timings of the configs[4] shard forward.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04k
timeout -k 10 900 python -u -m pytest tests/test_gpu_hyper.py tests/test_gpu_gnn.py tests/test_gpu_configs.py tests/test_abi.py -m "gpu or not gpu" -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04k/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04k/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for h in 0 1; do
    DADMM_HYPER_ATB_HOIST=$h timeout -k 10 300 python3 scripts/time_gnn.py 1024 50 1024 32 50 2 | sed "s/^/hoist=$h /" >> gpurun_out/r04k/timing.txt || exit $?
  done
done
cat gpurun_out/r04k/timing.txt
exit 0
