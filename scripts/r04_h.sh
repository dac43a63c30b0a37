#!/bin/bash
# Round-4 session H: kernel traces of the general adjoint at configs[2] and the configs[4] shard GNN
# forward (per-kernel times for the next round of work).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=r04h_adj bash scripts/prof_session.sh scripts/time_adjoint.py 16 512 64 4096 25 || exit $?
TAG=r04h_gnn bash scripts/prof_session.sh scripts/time_gnn.py 1024 50 1024 32 50 2 || exit $?
exit 0
