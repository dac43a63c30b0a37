#!/bin/bash
# Round-4 session Z: wgrad2 with row cursors (no per-step division, unconditional ring loads) —
# weight-gradient tests, then the isolated gradient and the GNN train step against the previous
# wgrad2 (build/var/libdadmm_w2old.so) and wgrad_kernel (libdadmm_wg0.so).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04za
timeout -k 10 600 python -u -m pytest tests/test_gpu_hyper_train.py tests/test_gpu_hyper.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04za/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04za/tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in "512000 400 400" "102400 400 2000" "32000 400 400" "1280 400 400"; do
  for v in "" build/var/libdadmm_w2old.so build/var/libdadmm_wg0.so; do
    DADMM_LIB_VARIANT=${v:+$PWD/$v} timeout -k 10 120 python3 scripts/time_wgrad.py $cfg >> gpurun_out/r04za/timing.txt || exit $?
  done
done
for r in 1 2; do
  for v in "" build/var/libdadmm_w2old.so; do
    for cfg in "256 25 5" "4096 25 2"; do
      DADMM_LIB_VARIANT=${v:+$PWD/$v} timeout -k 10 300 python3 scripts/prof_gnn_train.py $cfg | sed "s|^|lib=${v:-default} |" >> gpurun_out/r04za/timing.txt || exit $?
    done
  done
done
cat gpurun_out/r04za/timing.txt
TAG=r04za_pmc bash scripts/pmc_cmd.sh scripts/time_wgrad.py || exit $?
exit 0
