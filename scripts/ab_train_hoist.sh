#!/bin/bash
# A/B of the training forward's hoisted layer-1 Atb half (DADMM_HYPER_ATB_HOIST=0: the two-segment
# GEMM per iteration) on the B = 256 train step, interleaved, each run under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for h in 1 0 1 0; do
  out=$(DADMM_HYPER_ATB_HOIST=$h timeout -k 10 120 python3 scripts/prof_gnn_train.py ${ARGS:-256 25 5}) || exit $?
  echo "hoist=$h $out"
done
