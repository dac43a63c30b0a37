#!/bin/bash
# Round-4 session D: parity of the one-wave gram (GNN + adjoint paths) and the capped stepwise
# visit lists (P = 100), then the gram A/B at configs[2]'s adjoint and configs[4]'s shard forward.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=r04d TESTS="tests/test_gpu_wide.py tests/test_gpu_adjoint.py tests/test_gpu_parity.py tests/test_gpu_gnn.py tests/test_gpu_configs.py tests/test_gpu_hyper_train.py tests/test_gpu_train.py" bash scripts/r04_session.sh || exit $?
TAG=r04v5 VARS="build/var/libdadmm_gw*.so" SCRIPT=scripts/time_adjoint.py CFG="16 512 64 4096 25" ROUNDS=2 bash scripts/r04_variants.sh || exit $?
TAG=r04v6 VARS="build/var/libdadmm_gw*.so" SCRIPT=scripts/time_gnn.py ROUNDS=2 bash scripts/r04_variants.sh || exit $?
TAG=r04v7 VARS="build/var/libdadmm_bwd*.so" SCRIPT=scripts/time_adjoint.py CFG="5 256 64 4096 25" ROUNDS=2 bash scripts/r04_variants.sh || exit $?
exit 0
