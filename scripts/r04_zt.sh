#!/bin/bash
# Round-4 session ZT: final checkpoint of the session — the whole GPU suite, the bench (with extras),
# the kernel-trace + HBM-counter profile of the headline.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=r04zt TESTS=tests BENCH=1 bash scripts/r04_session.sh || exit $?
TAG=r04zt_prof BENCH_EXTRA=--no-extras bash scripts/profile_round.sh || exit $?
exit 0
