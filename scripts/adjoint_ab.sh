set -u
mkdir -p gpurun_out/adjab
for r in 1 2; do for v in oldadj vsums; do
  DADMM_LIB_VARIANT=$PWD/build/var/libdadmm_$v.so timeout -k 10 240 python3 scripts/time_adjoint.py 16 512 64 4096 25 > gpurun_out/adjab/$v.$r.json 2>gpurun_out/adjab/$v.$r.err || exit $?
  echo "$v $(tail -1 gpurun_out/adjab/$v.$r.json)"
done; done
DADMM_LIB_VARIANT=$PWD/build/var/libdadmm_vsums.so timeout -k 10 400 python -u -m pytest tests/test_gpu_adjoint.py -x -q --timeout 200 --timeout-method thread > gpurun_out/adjab/tests.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/adjab/tests.log
