#!/bin/bash
# Round-4 session U: gcn32 mix with the A_hat loads pipelined one node group ahead (DADMM_G32_MIX_PF):
# hypernetwork GPU tests, single layers and the configs[4] shard forward, A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04u
timeout -k 10 600 python -u -m pytest tests/test_gpu_hyper.py -k gcn -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04u/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04u/tests.log; [ $rc -ne 0 ] && exit $rc
for v in mixpf0 mixpf1; do
  for cfg in "1024 50 400 400" "1024 50 100 200"; do
    DADMM_LIB_VARIANT=$PWD/build/var/libdadmm_$v.so timeout -k 10 120 python3 scripts/time_gcn_layer.py $cfg >> gpurun_out/r04u/layers.txt || exit $?
  done
done
cat gpurun_out/r04u/layers.txt
TAG=r04u VARS="build/var/libdadmm_mixpf0.so build/var/libdadmm_mixpf1.so" SCRIPT=scripts/time_gnn.py CFG="1024 50 1024 32 50 2" ROUNDS=2 bash scripts/r04_variants.sh || exit $?
exit 0
