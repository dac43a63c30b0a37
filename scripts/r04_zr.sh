#!/bin/bash
# Round-4 session ZR: phase 2 of the GNN step with its U and eta loads unconditional too (product,
# product) against loads under their guards (build/var/libdadmm_p2old.so): GNN tests (bit-exact
# recurrence), then the configs[4] shard forward and the P = 5 headline-batch GNN forward.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04zr
timeout -k 10 600 python -u -m pytest tests/test_gpu_gnn.py tests/test_gpu_configs.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04zr/tests.log 2>&1
rc=$?; tail -1 gpurun_out/r04zr/tests.log; [ $rc -ne 0 ] && exit $rc
TAG=r04zr VARS="hyperparameter-gnn_unfolded-d-admm-main_amd/dadmm_hip/libdadmm.so build/var/libdadmm_p2old.so" SCRIPT=scripts/time_gnn.py CFG="1024 50 1024 32 50 2" ROUNDS=2 bash scripts/r04_variants.sh || exit $?
for r in 1 2; do
  for v in "" build/var/libdadmm_p2old.so; do
    DADMM_LIB_VARIANT=${v:+$PWD/$v} timeout -k 10 300 python3 scripts/time_gnn.py 4096 5 256 64 25 3 | sed "s|^|lib=${v:-default} |" >> gpurun_out/r04zr/p5.txt || exit $?
  done
done
cat gpurun_out/r04zr/p5.txt
exit 0
