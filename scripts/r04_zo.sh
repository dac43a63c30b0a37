#!/bin/bash
# Round-4 session ZO: wgrad2 with mask-based branch-free rings (DADMM_W2_FAST=1, product; 80 VGPRs, 3 waves per
# SIMD) against the per-step tests (build/var/libdadmm_fast0.so; 80 VGPRs, 3 waves): weight-gradient
# tests, isolated gradients, the B = 4096 / 256 train steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04zo
timeout -k 10 600 python -u -m pytest tests/test_gpu_hyper_train.py tests/test_gpu_hyper.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04zo/tests.log 2>&1
rc=$?; tail -1 gpurun_out/r04zo/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for cfg in "512000 400 400" "102400 400 2000" "32000 400 400"; do
  for v in "" build/var/libdadmm_fast0.so; do
    DADMM_LIB_VARIANT=${v:+$PWD/$v} timeout -k 10 120 python3 scripts/time_wgrad.py $cfg >> gpurun_out/r04zo/timing.txt || exit $?
  done
done
done
for v in "" build/var/libdadmm_fast0.so; do
  for cfg in "4096 25 2" "256 25 5"; do
    DADMM_LIB_VARIANT=${v:+$PWD/$v} timeout -k 10 300 python3 scripts/prof_gnn_train.py $cfg | sed "s|^|lib=${v:-default} |" >> gpurun_out/r04zo/timing.txt || exit $?
  done
done
cat gpurun_out/r04zo/timing.txt
exit 0
