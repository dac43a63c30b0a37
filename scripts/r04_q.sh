#!/bin/bash
# Round-4 session Q: the GCN mix on MFMA (gcn32_kernel, DADMM_G32_MFMA_MIX) — hypernetwork / GNN GPU
# tests, then A/B of the configs[4] shard forward against the VALU mix.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04q
timeout -k 10 900 python -u -m pytest tests/test_gpu_hyper.py tests/test_gpu_gnn.py tests/test_gpu_configs.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04q/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04q/tests.log; [ $rc -ne 0 ] && exit $rc
TAG=r04q VARS="build/var/libdadmm_mix_valu.so build/var/libdadmm_mix_mfma.so" SCRIPT=scripts/time_gnn.py CFG="1024 50 1024 32 50 2" ROUNDS=2 bash scripts/r04_variants.sh || exit $?
exit 0
