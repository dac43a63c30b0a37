#!/bin/bash
# Round GPU session (TAG, TESTS, BENCH, BENCH2 env): GPU suite (no -x: a failing parity test must not hide the bench), then the
# 1-GPU bench, then a 2-rank rehearsal of the self-launching multi-rank bench (gloo on one GPU).
# Stops at the first step that times out, aborts or faults (exit >= 124).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-round}
mkdir -p "$OUT"
run() {  # name seconds cmd...
    local name=$1 secs=$2; shift 2
    echo "== $name" ; date +%T
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"
    if [ $rc -ge 124 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
    return 0
}
if [ -n "$TESTS" ]; then
    run tests 900 python -u -m pytest $TESTS -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
fi
if [ -n "$BENCH" ]; then
    run bench 600 python bench.py --steps 20 --warmup 5
fi
if [ -n "$BENCH2" ]; then
    DADMM_DIST_BACKEND=gloo run bench2 300 python bench.py --gpus 2 --steps 5 --warmup 2 --no-extras --no-cpu-baseline
fi
exit 0
