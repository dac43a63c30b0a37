#!/bin/bash
# Round-4 session W: kernel trace of the GNN train step at the headline batch (B = 4096, K = 25).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=r04w_train PROF_T=400 bash scripts/prof_session.sh scripts/prof_gnn_train.py 4096 25 2 > /dev/null || exit $?
exit 0
