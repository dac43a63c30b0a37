#!/bin/bash
# Agent-resident kernel variants (build/var/libdadmm_res_*.so) vs the product library at the
# headline shape (scripts/time_headline.py, DIVISIONS=agents), two interleaved rounds; then the
# product's row-divided kernel for reference. Each run under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
  for so in hyperparameter-gnn_unfolded-d-admm-main_amd/dadmm_hip/libdadmm.so build/var/libdadmm_res_*.so; do
    DIVISIONS=agents DADMM_LIB_VARIANT=$PWD/$so timeout -k 10 120 python3 scripts/time_headline.py 4096 5 256 64 25 1 20 || exit $?
  done
done
DIVISIONS=rows timeout -k 10 120 python3 scripts/time_headline.py 4096 5 256 64 25 2 20
