#!/bin/bash
# Interleaved A/B of an environment switch on one timing command:
#   VAR=DADMM_HYPER_TAIL VALUES="1 0" CMD="python3 scripts/prof_gnn_train.py 256 25 5" bash scripts/ab_env.sh
# two rounds, each run under its own time limit; every output line is prefixed with VAR=value.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for r in 1 2; do
  for v in ${VALUES:-1 0}; do
    out=$(env "$VAR=$v" timeout -k 10 ${LIMIT:-200} $CMD) || exit $?
    echo "$VAR=$v $out"
  done
done
