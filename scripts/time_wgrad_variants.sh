#!/bin/bash
# wgrad2 variants (build/var/libdadmm_*.so) vs the product library on the train step's weight
# gradient shapes (scripts/time_wgrad.py R N K), two interleaved rounds, each run time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
# SHAPES: comma-separated "R N K" triples
IFS=, read -ra shapes <<< "${SHAPES:-512000 400 400,32000 400 400,32000 400 200,6400 400 2000,32000 100 512}"
for shape in "${shapes[@]}"; do
  for r in 1 2; do
    for so in hyperparameter-gnn_unfolded-d-admm-main_amd/dadmm_hip/libdadmm.so build/var/libdadmm_*.so; do
      out=$(DADMM_LIB_VARIANT=$PWD/$so timeout -k 10 120 python3 scripts/time_wgrad.py $shape 2>/dev/null | grep '^{') || exit $?
      echo "$(basename $so) $out"
    done
  done
done
