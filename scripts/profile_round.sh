#!/bin/bash
# Round profile: rocprofv3 kernel-trace summary of the bench command, then the two HBM counter
# passes (FETCH_SIZE, WRITE_SIZE: one counter per run, kernel trace only).
# Every GPU step has its own time limit; the first failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline ${BENCH_EXTRA:-}"
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- \
    python3 $BENCH > "$OUT/bench_kt.json" 2> "$OUT/kt.err"
rc=$?; echo "kernel-trace rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/kt.err"; exit $rc; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/pmc_$c" -o pmc -- \
      python3 scripts/prof_kernel.py ${SHAPE:-} > "$OUT/pmc_$c.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/pmc_$c.log"; exit $rc; }
done
# (profiles/traffic.json is written back home from the merged gpurun_out: scripts/traffic.py)
echo done
