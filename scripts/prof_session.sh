#!/bin/bash
# rocprofv3 kernel-trace summary of one command (scripts/...py args), under a time limit.
#   TAG=x scripts/prof_session.sh scripts/prof_gnn_train.py 256 25 3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 ${PROF_T:-300} rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- \
    python3 "$@" > "$OUT/out.txt" 2> "$OUT/err.txt"
rc=$?; echo "rocprof rc=$rc"; cat "$OUT/out.txt"; tail -3 "$OUT/err.txt"
exit $rc
