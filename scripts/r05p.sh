#!/bin/bash
# Round-5 session p: product tests, the 64-column step variant's tests, adjoint variants,
# the training Atb-hoist A/B and the configs[4]-shard forward A/B of the step variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
V=$PWD/build/var
TAG=r05p STEPS="tests:tests/test_gpu_hyper_train.py tests/test_gpu_gnn.py \
| cmd:DADMM_LIB_VARIANT=$V/libdadmm_step64.so python -m pytest tests/test_gpu_gnn.py -q -x --timeout 120 --timeout-method thread \
| cmd:bash scripts/time_adj_variants.sh \
| cmd:bash scripts/ab_train_hoist.sh \
| cmd:VARIANTS=step64 bash scripts/ab_gnn_variants.sh" bash scripts/session.sh
