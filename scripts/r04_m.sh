#!/bin/bash
# Round-4 session M: gcn32_kernel with A_hat read through the vector cache (two workgroups per CU)
# vs staged in LDS (one per CU) vs the mix ablated, and linear_kernel (DADMM_GCN32=0).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04m
timeout -k 10 600 python -u -m pytest tests/test_gpu_hyper.py -k "gcn" -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04m/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04m/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in g32lds g32glob g32nomix; do
    DADMM_LIB_VARIANT=$PWD/build/var/libdadmm_$v.so timeout -k 10 300 python3 scripts/time_gnn.py 1024 50 1024 32 50 2 >> gpurun_out/r04m/timing.txt || exit $?
  done
  DADMM_GCN32=0 timeout -k 10 300 python3 scripts/time_gnn.py 1024 50 1024 32 50 2 | sed 's/^/gcn32=0 /' >> gpurun_out/r04m/timing.txt || exit $?
done
cat gpurun_out/r04m/timing.txt
DADMM_LIB_VARIANT=$PWD/build/var/libdadmm_g32glob.so TAG=r04m_gnn PROF_T=300 bash scripts/prof_session.sh scripts/time_gnn.py 1024 50 1024 32 10 2 > /dev/null || exit $?
exit 0
