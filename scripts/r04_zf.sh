#!/bin/bash
# Round-4 session ZF: the prologue's direct-counter Philox (DADMM_RNG_DIRECT=1, product) against
# hiprand's state machine (build/var/libdadmm_rng0.so): bit-exactness tests, headline bench A/B,
# and which torch op runs a copy kernel in every headline forward; gram_acc (ABI 15) tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04zf
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gnn.py tests/test_gpu_hyper_train.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04zf/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04zf/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for v in "" build/var/libdadmm_rng0.so; do
    DADMM_LIB_VARIANT=${v:+$PWD/$v} timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-extras --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print('${v:-default}', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" >> gpurun_out/r04zf/bench.txt || exit $?
  done
done
cat gpurun_out/r04zf/bench.txt
TAG=r04zf_kt PROF_T=200 bash scripts/prof_session.sh scripts/find_copy.py > gpurun_out/r04zf/find_copy.txt 2>&1 || exit $?
exit 0
