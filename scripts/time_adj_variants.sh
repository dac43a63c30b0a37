#!/bin/bash
# The fused adjoint's variants (build/var/libdadmm_*.so) vs the product library at the headline
# shape (scripts/time_adjoint.py), two interleaved rounds, each run under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
  for so in hyperparameter-gnn_unfolded-d-admm-main_amd/dadmm_hip/libdadmm.so build/var/libdadmm_*.so; do
    echo "== $so"
    DADMM_LIB_VARIANT=$PWD/$so timeout -k 10 120 python3 scripts/time_adjoint.py ${CFG:-} || exit $?
  done
done
