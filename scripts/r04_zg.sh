#!/bin/bash
# Round-4 session ZG: gcn32's mix epilogue with 5 or 8 A_hat rows per task (build/var/libdadmm_mr5 /
# mr8) against 4 (product): GCN tests per variant, single configs[4] layers, the configs[4] shard.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04zg
for v in mr5 mr8; do
  DADMM_LIB_VARIANT=$PWD/build/var/libdadmm_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_hyper.py -k gcn -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04zg/tests_$v.log 2>&1
  rc=$?; tail -1 gpurun_out/r04zg/tests_$v.log; [ $rc -ne 0 ] && exit $rc
done
for r in 1 2; do
for v in "" build/var/libdadmm_mr5.so build/var/libdadmm_mr8.so; do
  for cfg in "1024 50 400 400" "1024 50 200 400" "1024 50 100 200" "1024 50 1024 100"; do
    DADMM_LIB_VARIANT=${v:+$PWD/$v} timeout -k 10 120 python3 scripts/time_gcn_layer.py $cfg >> gpurun_out/r04zg/layers.txt || exit $?
  done
done
done
cat gpurun_out/r04zg/layers.txt
TAG=r04zg VARS="hyperparameter-gnn_unfolded-d-admm-main_amd/dadmm_hip/libdadmm.so build/var/libdadmm_mr5.so build/var/libdadmm_mr8.so" SCRIPT=scripts/time_gnn.py CFG="1024 50 1024 32 50 2" ROUNDS=2 bash scripts/r04_variants.sh || exit $?
exit 0
