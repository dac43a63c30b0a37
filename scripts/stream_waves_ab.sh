#!/bin/bash
# A/B at configs[2] of the streamed forward's forms, interleaved: 8 waves (two agents per wave),
# 16 waves (one agent per wave, DADMM_STREAM_WAVES=16) and the 8-wave build with the visit-table
# prefetch (build/var/libdadmm_qpf.so); then the stream parity tests on the 16-wave form and on
# the prefetch build.
set -u
OUT=gpurun_out/${TAG:-wab}; mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 scripts/time_config.py 16 512 64 4096 25 0.3 1 tiled > $OUT/$name.json 2>$OUT/$name.err || exit $?
  echo "$name $(cat $OUT/$name.json)"
}
for r in 1 2; do
  run w8.$r DADMM_STREAM_WAVES=8
  run w16.$r DADMM_STREAM_WAVES=16
  run qpf.$r DADMM_LIB_VARIANT=$PWD/build/var/libdadmm_qpf.so
done
DADMM_STREAM_WAVES=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > $OUT/tests16.log 2>&1; echo "tests16 rc=$?"; tail -1 $OUT/tests16.log
DADMM_LIB_VARIANT=$PWD/build/var/libdadmm_qpf.so timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > $OUT/testsqpf.log 2>&1; echo "testsqpf rc=$?"; tail -1 $OUT/testsqpf.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > $OUT/tests8.log 2>&1; echo "tests8 rc=$?"; tail -1 $OUT/tests8.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_adjoint.py tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread > $OUT/tests_adj.log 2>&1; echo "tests_adj rc=$?"; tail -1 $OUT/tests_adj.log
