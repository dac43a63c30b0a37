#!/bin/bash
# Round-4 session ZJ: the B = 256 GNN train step after the adjoint fusions — kernel trace, and a
# host-side cProfile of the same steps (is the step host- or device-bound?).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04zj
TAG=r04zj_train PROF_T=300 bash scripts/prof_session.sh scripts/prof_gnn_train.py 256 25 3 > /dev/null || exit $?
CPROF=1 timeout -k 10 300 python3 scripts/prof_gnn_train.py 256 25 5 > gpurun_out/r04zj/cprof.txt 2>&1 || exit $?
exit 0
