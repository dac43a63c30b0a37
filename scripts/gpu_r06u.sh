set -o pipefail
O=gpurun_out/r06u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "prologue or draw" --timeout 120 --timeout-method thread > $O/prologue_tests.txt 2>&1 || exit $?
for v in wv8 wv4 wv8 wv4; do
  echo "== $v" >> $O/split_wv.txt
  DADMM_LIB_VARIANT=$PWD/build/svar/libdadmm_$v.so timeout -k 10 120 python -u scripts/time_split.py 1024 50 >> $O/split_wv.txt 2>&1 || exit $?
done
echo "== main (new prologue)" >> $O/split_wv.txt
timeout -k 10 120 python -u scripts/time_split.py 1024 50 >> $O/split_wv.txt 2>&1 || exit $?
for lib in main rngold; do
  for B in 1024 4096; do
    if [ $lib = main ]; then V=""; else V="DADMM_LIB_VARIANT=$PWD/build/svar/libdadmm_rngold.so"; fi
    env $V timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_${lib}_$B -o run -- python3 scripts/time_prologue.py $B 5 256 50 > $O/prof_${lib}_$B.out 2>&1 || exit $?
  done
done
for d in $O/prof_*; do [ -d $d ] && python3 scripts/rocpd_stats.py $(ls $d/*/run_results.db $d/run_results.db 2>/dev/null | head -1) > $d.csv; done
DADMM_LIB_VARIANT=$PWD/build/svar/libdadmm_wv4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -q -x --timeout 120 --timeout-method thread > $O/split_tests_wv4.txt 2>&1 || exit $?
