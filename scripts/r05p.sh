#!/bin/bash
# Round-5 session p: product tests, the 64-column step variant's tests, adjoint variants,
# the training Atb-hoist A/B and the configs[4]-shard forward A/B of the step variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
V=$PWD/build/var
TAG=r05p STEPS="tests:tests/test_gpu_hyper_train.py tests/test_gpu_gnn.py \
| cmd:DADMM_LIB_VARIANT=$V/libdadmm_step64.so python -m pytest tests/test_gpu_gnn.py -q -x --timeout 120 --timeout-method thread \
| cmd:bash scripts/time_adj_variants.sh \
| cmd:for h in 1 0 1 0; do DADMM_HYPER_ATB_HOIST=\$h python scripts/prof_gnn_train.py 256 25 5 | sed \"s/^/hoist=\$h /\" || exit 1; done \
| cmd:for r in 1 2; do for so in hyperparameter-gnn_unfolded-d-admm-main_amd/dadmm_hip/libdadmm.so build/var/libdadmm_step64.so; do DADMM_LIB_VARIANT=\$PWD/\$so python3 scripts/prof_gnn.py 1024 50 1024 32 10 2 | sed \"s|^|\$(basename \$so) |\" || exit 1; done; done" bash scripts/session.sh
