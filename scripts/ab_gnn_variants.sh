#!/bin/bash
# A/B of the product library against build/var variants (VARIANTS="name ...") on the GNN model
# forward (eval, no_grad; SHAPE: scripts/prof_gnn.py's B P n m K reps), two interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for r in 1 2; do
  for so in hyperparameter-gnn_unfolded-d-admm-main_amd/dadmm_hip/libdadmm.so ${VARIANTS:+$(for v in $VARIANTS; do echo build/var/libdadmm_$v.so; done)}; do
    out=$(DADMM_LIB_VARIANT=$PWD/$so timeout -k 10 200 python3 scripts/prof_gnn.py ${SHAPE:-1024 50 1024 32 10 2}) || exit $?
    echo "$(basename $so) $out"
  done
done
