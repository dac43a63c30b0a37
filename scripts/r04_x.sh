#!/bin/bash
# Round-4 session X: wgrad2 (64 x 64 tiles, 32x32x2 MFMA, row splits in the deferred pass) —
# the weight-gradient tests, then GNN train steps with wgrad2 (libdadmm.so) and the round-3
# wgrad_kernel (build/var/libdadmm_wg0.so, -DDADMM_WGRAD2=0) at B = 256 and B = 4096.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04x
timeout -k 10 600 python -u -m pytest tests/test_gpu_hyper_train.py tests/test_gpu_hyper.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04x/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04x/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in "" build/var/libdadmm_wg0.so; do
    for cfg in "256 25 5" "4096 25 2"; do
      DADMM_LIB_VARIANT=${v:+$PWD/$v} timeout -k 10 300 python3 scripts/prof_gnn_train.py $cfg | sed "s|^|lib=${v:-default} |" >> gpurun_out/r04x/timing.txt || exit $?
    done
  done
done
cat gpurun_out/r04x/timing.txt
TAG=r04x_train PROF_T=400 bash scripts/prof_session.sh scripts/prof_gnn_train.py 4096 25 2 > /dev/null || exit $?
exit 0
