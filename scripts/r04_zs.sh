#!/bin/bash
# Round-4 session ZS: the GNN step adjoint's recompute loop unrolled over agents with unconditional
# loads (product) against the previous commit (build/var/libdadmm_sbold.so): GNN / training tests,
# then the GNN train step at B = 256 and B = 4096.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04zs
timeout -k 10 600 python -u -m pytest tests/test_gpu_gnn.py tests/test_gpu_hyper_train.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04zs/tests.log 2>&1
rc=$?; tail -1 gpurun_out/r04zs/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in "" build/var/libdadmm_sbold.so; do
    for cfg in "256 25 5" "4096 25 2"; do
      DADMM_LIB_VARIANT=${v:+$PWD/$v} timeout -k 10 300 python3 scripts/prof_gnn_train.py $cfg | sed "s|^|lib=${v:-default} |" >> gpurun_out/r04zs/timing.txt || exit $?
    done
  done
done
cat gpurun_out/r04zs/timing.txt
TAG=r04zs_train PROF_T=300 bash scripts/prof_session.sh scripts/prof_gnn_train.py 256 25 3 > /dev/null || exit $?
exit 0
