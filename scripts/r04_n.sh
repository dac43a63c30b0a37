#!/bin/bash
# Round-4 session N: PMC passes over a short configs[4] shard GNN forward (gcn32_kernel, step_kernel,
# gram_lds_kernel counters).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=r04n_gnn bash scripts/pmc_cmd.sh scripts/time_gnn.py 1024 50 1024 32 4 1 || exit $?
exit 0
