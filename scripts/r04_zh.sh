#!/bin/bash
# Round-4 session ZH: the fused GNN step pass with 3 / 4 row pairs in flight per wave
# (build/var/libdadmm_upch3 / upch4) against 2 (product): GNN tests per variant, then the
# configs[4] shard forward.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04zh
for v in upch3 upch4; do
  DADMM_LIB_VARIANT=$PWD/build/var/libdadmm_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_gnn.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04zh/tests_$v.log 2>&1
  rc=$?; tail -1 gpurun_out/r04zh/tests_$v.log; [ $rc -ne 0 ] && exit $rc
done
TAG=r04zh VARS="hyperparameter-gnn_unfolded-d-admm-main_amd/dadmm_hip/libdadmm.so build/var/libdadmm_upch3.so build/var/libdadmm_upch4.so" SCRIPT=scripts/time_gnn.py CFG="1024 50 1024 32 50 2" ROUNDS=2 bash scripts/r04_variants.sh || exit $?
exit 0
