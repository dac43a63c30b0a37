#!/bin/bash
# Round-4 session E: the general adjoint's two changes (gram out-row prefetch, phase-2 operand
# prefetch) - parity, then A/B at configs[2]'s adjoint.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=r04e TESTS="tests/test_gpu_adjoint.py tests/test_gpu_gnn.py tests/test_gpu_wide.py tests/test_gpu_stream.py" bash scripts/r04_session.sh || exit $?
TAG=r04v8 VARS="build/var/libdadmm_go*.so build/var/libdadmm_apf*.so" SCRIPT=scripts/time_adjoint.py CFG="16 512 64 4096 25" ROUNDS=2 bash scripts/r04_variants.sh || exit $?
exit 0
