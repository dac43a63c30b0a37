#!/bin/bash
# Round-4 session ZZ4: final checkpoint of the session (after the GCN BatchNorm backward and two-stage colsum changes) — the whole GPU suite, the bench (with extras),
# the kernel-trace + HBM-counter profile of the headline.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=r04zz4 TESTS=tests BENCH=1 bash scripts/r04_session.sh || exit $?
TAG=r04zz4_prof BENCH_EXTRA=--no-extras bash scripts/profile_round.sh || exit $?
timeout -k 10 300 python -u scripts/prof_gnn_train.py 256 25 5 > gpurun_out/r04zz4/train_b256.txt 2>&1 && timeout -k 10 300 python -u scripts/prof_gnn_train.py 4096 25 2 > gpurun_out/r04zz4/train_b4096.txt 2>&1 || exit $?
exit 0
