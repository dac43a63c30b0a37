#!/bin/bash
# Round-4 session ZI: the GNN adjoint's accumulations moved into kernels (dadmm_gnn_gram_acc,
# dadmm_hyper_linear_ex's in-place addend, ABI 16): hypernetwork / GNN GPU tests, then the GNN
# train step at B = 256 and B = 4096 (K = 25).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04zi
timeout -k 10 600 python -u -m pytest tests/test_gpu_hyper.py tests/test_gpu_hyper_train.py tests/test_gpu_gnn.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04zi/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04zi/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for cfg in "256 25 5" "4096 25 2"; do
    timeout -k 10 300 python3 scripts/prof_gnn_train.py $cfg >> gpurun_out/r04zi/timing.txt || exit $?
  done
done
cat gpurun_out/r04zi/timing.txt
exit 0
