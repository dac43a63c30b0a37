#!/bin/bash
# Round-4 session J: the LDS-resident gram kernel — GPU tests of every gram user, then A/B timings
# (configs[2] general adjoint, configs[4] shard GNN forward) against the previous gram kernel.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04j
timeout -k 10 600 python -u -m pytest tests/test_gpu_adjoint.py tests/test_gpu_gnn.py tests/test_gpu_wide.py tests/test_gpu_configs.py tests/test_gpu_hyper_train.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04j/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04j/tests.log; [ $rc -ne 0 ] && exit $rc
TAG=r04j_adj VARS="build/var/libdadmm_gramlds0.so build/var/libdadmm_gramlds1.so" SCRIPT=scripts/time_adjoint.py CFG="16 512 64 4096 25" ROUNDS=2 bash scripts/r04_variants.sh || exit $?
TAG=r04j_gnn VARS="build/var/libdadmm_gramlds0.so build/var/libdadmm_gramlds1.so" SCRIPT=scripts/time_gnn.py CFG="1024 50 1024 32 50 2" ROUNDS=2 bash scripts/r04_variants.sh || exit $?
exit 0
