#!/bin/bash
# Round-4 session C: parity tests of the new paths, then the A/Bs (fused LDS padding at H, the
# 16-byte-lane adjoint and the LDS-staged gram at configs[2]'s adjoint and configs[4]'s shard).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=r04c TESTS="tests/test_gpu_wide.py tests/test_gpu_adjoint.py tests/test_gpu_stream.py tests/test_gpu_gnn.py tests/test_gpu_configs.py tests/test_gpu_hyper_train.py" bash scripts/r04_session.sh || exit $?
TAG=r04v1 VARS="build/var/libdadmm_f_*.so" CFG="5 256 64 4096 25 0.5 0 auto" \
  PMC="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" bash scripts/r04_variants.sh || exit $?
TAG=r04v2 VARS="build/var/libdadmm_adj_*.so build/var/libdadmm_gram_*.so" SCRIPT=scripts/time_adjoint.py \
  CFG="16 512 64 4096 25" ROUNDS=2 bash scripts/r04_variants.sh || exit $?
TAG=r04v3 VARS="build/var/libdadmm_gram_*.so" SCRIPT=scripts/time_gnn.py ROUNDS=2 bash scripts/r04_variants.sh || exit $?
TAG=r04v4 VARS="build/var/libdadmm_st_*.so" ROUNDS=3 PMC="FETCH_SIZE" bash scripts/r04_variants.sh || exit $?
exit 0
