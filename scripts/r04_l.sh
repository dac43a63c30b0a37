#!/bin/bash
# Round-4 session L: gcn32_kernel (32x32x2 MFMA GCN layers): hypernetwork / GNN GPU tests, then A/B
# timing of the configs[4] shard forward (DADMM_GCN32=0/1) and a kernel trace of the new build.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04l
timeout -k 10 900 python -u -m pytest tests/test_gpu_hyper.py tests/test_gpu_gnn.py tests/test_gpu_configs.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04l/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04l/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for g in 0 1; do
    DADMM_GCN32=$g timeout -k 10 300 python3 scripts/time_gnn.py 1024 50 1024 32 50 2 | sed "s/^/gcn32=$g /" >> gpurun_out/r04l/timing.txt || exit $?
  done
done
cat gpurun_out/r04l/timing.txt
TAG=r04l_gnn PROF_T=300 bash scripts/prof_session.sh scripts/time_gnn.py 1024 50 1024 32 50 2 > /dev/null || exit $?
exit 0
