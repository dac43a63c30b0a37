set -o pipefail
O=gpurun_out/r06p2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -q -x --timeout 120 --timeout-method thread > $O/split_tests.txt 2>&1 || exit $?
for r in 1 2; do
  echo "== main (prio GEMM1+GEMM2)" >> $O/split_prio.txt
  timeout -k 10 120 python -u scripts/time_split.py 1024 100 >> $O/split_prio.txt 2>&1 || exit $?
  echo "== p4 (GEMM2 only)" >> $O/split_prio.txt
  DADMM_LIB_VARIANT=$PWD/build/svar/libdadmm_p4.so timeout -k 10 120 python -u scripts/time_split.py 1024 100 >> $O/split_prio.txt 2>&1 || exit $?
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
