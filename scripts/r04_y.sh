#!/bin/bash
# Round-4 session Y: the batched 400 x 400 weight gradient in isolation (wgrad2 vs wgrad_kernel),
# its PMC counters, and a kernel trace of the B = 256 GNN train step with wgrad2.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04y
for cfg in "512000 400 400" "512000 200 400" "102400 400 2000" "32000 400 400"; do
  for v in "" build/var/libdadmm_wg0.so; do
    DADMM_LIB_VARIANT=${v:+$PWD/$v} timeout -k 10 120 python3 scripts/time_wgrad.py $cfg >> gpurun_out/r04y/timing.txt || exit $?
  done
done
cat gpurun_out/r04y/timing.txt
TAG=r04y_pmc bash scripts/pmc_cmd.sh scripts/time_wgrad.py || exit $?
TAG=r04y_train PROF_T=300 bash scripts/prof_session.sh scripts/prof_gnn_train.py 256 25 3 > /dev/null || exit $?
exit 0
