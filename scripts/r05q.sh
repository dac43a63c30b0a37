#!/bin/bash
# Round-5 session q (the adjoint tests ran green first, 42 passed): the adjoint timing, the training Atb-hoist A/B and
# the configs[4]-shard forward A/B of the 64-column step variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=r05q STEPS="cmd:timeout -k 10 120 python3 scripts/time_adjoint.py && timeout -k 10 120 python3 scripts/time_adjoint.py && timeout -k 10 120 python3 scripts/time_adjoint.py \
| cmd:bash scripts/ab_train_hoist.sh \
| cmd:VARIANTS=step64 bash scripts/ab_gnn_variants.sh" bash scripts/session.sh
