#!/bin/bash
# Round-4 session O: GNN step with U kept in registers between its phases (DADMM_STEP_KEEPU) and the
# row-norm kernel sized to its rows (CH by C): GNN / hypernetwork GPU tests, A/B of the step variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04o
timeout -k 10 900 python -u -m pytest tests/test_gpu_gnn.py tests/test_gpu_hyper.py tests/test_gpu_hyper_train.py tests/test_gpu_configs.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04o/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04o/tests.log; [ $rc -ne 0 ] && exit $rc
TAG=r04o VARS="build/var/libdadmm_keepu0.so build/var/libdadmm_keepu1.so" SCRIPT=scripts/time_gnn.py CFG="1024 50 1024 32 50 2" ROUNDS=2 bash scripts/r04_variants.sh || exit $?
exit 0
