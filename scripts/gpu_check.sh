#!/bin/bash
# One GPU session: parity tests, smoke, a short bench, and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/timeout/abort ends the script (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
stop_if_fatal() {  # $1 = exit status of a GPU step
  if [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; then
    echo "FATAL step status $1 — stopping" | tee -a "$OUT/status.txt"; exit "$1"; fi
}
rocm-smi --showproductname > "$OUT/rocm_smi.txt" 2>&1 || true
lscpu > "$OUT/lscpu.txt" 2>&1 || true
echo "== pytest -m gpu" | tee -a "$OUT/status.txt"
timeout -k 10 ${PYTEST_T:-900} python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a "$OUT/status.txt"; tail -5 "$OUT/pytest_gpu.log"; stop_if_fatal $rc
echo "== smoke" | tee -a "$OUT/status.txt"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a "$OUT/status.txt"; tail -3 "$OUT/smoke.log"; stop_if_fatal $rc
if [ "${SKIP_BENCH:-0}" = 0 ]; then
  echo "== bench" | tee -a "$OUT/status.txt"
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; echo "bench rc=$rc" | tee -a "$OUT/status.txt"; tail -c 3000 "$OUT/bench.json"; tail -5 "$OUT/bench.err"; stop_if_fatal $rc
fi
if [ "${SKIP_PROF:-0}" = 0 ]; then
  echo "== rocprofv3 kernel trace" | tee -a "$OUT/status.txt"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o kt -- \
     python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
  rc=$?; echo "rocprof rc=$rc" | tee -a "$OUT/status.txt"; stop_if_fatal $rc
  find "$OUT/prof" -name '*stats*' | head
fi
echo done | tee -a "$OUT/status.txt"
