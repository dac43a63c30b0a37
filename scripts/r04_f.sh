#!/bin/bash
# Round-4 session F: the whole GPU suite, the bench, the kernel-trace + HBM-counter profile of the
# headline (profiles/r04), then the general-adjoint A/B (session E's variants).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=r04f TESTS=tests BENCH=1 bash scripts/r04_session.sh || exit $?
TAG=r04f_prof BENCH_EXTRA=--no-extras bash scripts/profile_round.sh || exit $?
TAG=r04v8 VARS="build/var/libdadmm_go*.so build/var/libdadmm_apf*.so" SCRIPT=scripts/time_adjoint.py CFG="16 512 64 4096 25" ROUNDS=2 bash scripts/r04_variants.sh || exit $?
exit 0
