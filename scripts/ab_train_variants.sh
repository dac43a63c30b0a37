#!/bin/bash
# A/B of the product library against build/var variants (VARIANTS="name ...") on the GNN train
# step (scripts/prof_gnn_train.py ARGS, default B=256 K=25, 5 steps), two interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for r in 1 2; do
  for so in hyperparameter-gnn_unfolded-d-admm-main_amd/dadmm_hip/libdadmm.so ${VARIANTS:+$(for v in $VARIANTS; do echo build/var/libdadmm_$v.so; done)}; do
    out=$(DADMM_LIB_VARIANT=$PWD/$so timeout -k 10 200 python3 scripts/prof_gnn_train.py ${ARGS:-256 25 5}) || exit $?
    echo "$(basename $so) $out"
  done
done
