#!/bin/bash
# Round-4 session V: the P = 5 GNN forward at B = 4096 with the round-4 switches off / on
# (DADMM_GCN32, DADMM_HYPER_ATB_HOIST), the new GNN test case, and a kernel trace of the GNN train step.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04v
timeout -k 10 600 python -u -m pytest tests/test_gpu_gnn.py -k larger_shapes -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04v/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04v/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for g in 0 1; do for h in 0 1; do
    DADMM_GCN32=$g DADMM_HYPER_ATB_HOIST=$h timeout -k 10 300 python3 scripts/time_gnn.py 4096 5 256 64 25 3 | sed "s/^/gcn32=$g hoist=$h /" >> gpurun_out/r04v/timing.txt || exit $?
  done; done
done
cat gpurun_out/r04v/timing.txt
TAG=r04v_train PROF_T=300 bash scripts/prof_session.sh scripts/prof_gnn_train.py 256 25 3 > /dev/null || exit $?
exit 0
