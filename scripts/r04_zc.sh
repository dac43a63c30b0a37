#!/bin/bash
# Round-4 session ZC: kernel traces of the configs[4]-shard GNN forward (B = 1024, P = 50, n = 1024,
# m = 32, K = 50) and of the B = 256 GNN train step at the current build.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=r04zc_c5 PROF_T=300 bash scripts/prof_session.sh scripts/prof_gnn.py 1024 50 1024 32 50 2 > /dev/null || exit $?
TAG=r04zc_train PROF_T=300 bash scripts/prof_session.sh scripts/prof_gnn_train.py 256 25 3 > /dev/null || exit $?
exit 0
