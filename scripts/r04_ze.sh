#!/bin/bash
# Round-4 session ZE: wgrad2 ring refilled one step late (DADMM_W2_LAG=1, the product build) against
# the consumed-slot refill (build/var/libdadmm_lag0.so), isolated gradients + PMC, then tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04ze
for r in 1 2; do
for cfg in "512000 400 400" "102400 400 2000" "32000 400 400"; do
  for v in "" build/var/libdadmm_lag0.so; do
    DADMM_LIB_VARIANT=${v:+$PWD/$v} timeout -k 10 120 python3 scripts/time_wgrad.py $cfg >> gpurun_out/r04ze/timing.txt || exit $?
  done
done
done
cat gpurun_out/r04ze/timing.txt
TAG=r04ze_pmc bash scripts/pmc_cmd.sh scripts/time_wgrad.py || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_hyper_train.py tests/test_gpu_hyper.py -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04ze/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04ze/tests.log; exit $rc
