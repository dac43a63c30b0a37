#!/bin/bash
# Round-4 session I: PMC passes over the configs[2] general adjoint (gram_kernel, adj_update_v4).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=r04i_adj bash scripts/pmc_cmd.sh scripts/time_adjoint.py 16 512 64 4096 5 || exit $?
exit 0
