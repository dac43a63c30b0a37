set -o pipefail
O=gpurun_out/r06s
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gnn.py -q -x --timeout 120 --timeout-method thread > $O/gnn_tests.txt 2>&1 || exit $?
for v in 0 1 0 1; do
  DADMM_AB_STORE_DELTA=$v timeout -k 10 240 python -u scripts/time_gnn.py 1024 50 1024 32 50 3 >> $O/c5_recomp.txt 2>&1 || exit $?
done
for v in wv8 wv16 wv8 wv16; do
  echo "== $v" >> $O/split_wv.txt
  DADMM_LIB_VARIANT=$PWD/build/svar/libdadmm_$v.so timeout -k 10 120 python -u scripts/time_split.py 1024 50 >> $O/split_wv.txt 2>&1 || exit $?
done
DADMM_LIB_VARIANT=$PWD/build/svar/libdadmm_wv16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -q -x --timeout 120 --timeout-method thread > $O/split_tests_wv16.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/time_prologue.py 1024 5 256 50 > $O/prologue.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/time_prologue.py 4096 5 256 50 >> $O/prologue.txt 2>&1 || exit $?
