#!/bin/bash
# Round-5 session q: adjoint tests on the new default, its timing, the training Atb-hoist A/B and
# the configs[4]-shard forward A/B of the 64-column step variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=r05q STEPS="tests:tests/test_gpu_adjoint.py tests/test_gpu_train.py \
| cmd:for i in 1 2 3; do timeout -k 10 120 python3 scripts/time_adjoint.py || exit 1; done \
| cmd:bash scripts/ab_train_hoist.sh \
| cmd:VARIANTS=step64 bash scripts/ab_gnn_variants.sh" bash scripts/session.sh
