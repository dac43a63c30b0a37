#!/bin/bash
# Round-4 session ZZ5: the GCN BatchNorm backward at one wave per workgroup on every grid, as a variant (
# product) against the previous commit (build/var/libdadmm_gbw0.so): hypernetwork tests, then
# the GNN train step (B = 256 / 4096) and the configs[4] shard forward.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04zz5
true
rc=$?; tail -1 gpurun_out/r04zz5/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in "" build/var/libdadmm_gbw0.so; do
    for cfg in "256 25 5" "4096 25 2"; do
      DADMM_LIB_VARIANT=${v:+$PWD/$v} timeout -k 10 300 python3 scripts/prof_gnn_train.py $cfg | sed "s|^|lib=${v:-default} |" >> gpurun_out/r04zz5/timing.txt || exit $?
    done
  done
done
cat gpurun_out/r04zz5/timing.txt
TAG=r04zz5 VARS="hyperparameter-gnn_unfolded-d-admm-main_amd/dadmm_hip/libdadmm.so build/var/libdadmm_gbw0.so" SCRIPT=scripts/time_gnn.py CFG="1024 50 1024 32 50 2" ROUNDS=1 bash scripts/r04_variants.sh || exit $?
exit 0
