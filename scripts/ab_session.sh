#!/bin/bash
# One GPU session for kernel A/B work: the fused-path parity tests with the in-tree library,
# every build/var variant timed on the headline shape (and CFG2 if given), then the whole GPU
# suite and a bench line. Each GPU step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a "$OUT/status.txt"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/status.txt"
  tail -4 "$OUT/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step parity 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
  for so in build/var/libdadmm_*.so; do
    DADMM_LIB_VARIANT=$PWD/$so timeout -k 10 120 python3 scripts/time_config.py 5 256 64 4096 25 0.5 0 auto >> "$OUT/variants.jsonl" 2>>"$OUT/variants.err" || { echo "variant $so failed"; exit 1; }
    if [ -n "${CFG2:-}" ]; then
      DADMM_LIB_VARIANT=$PWD/$so timeout -k 10 120 python3 scripts/time_config.py $CFG2 >> "$OUT/variants.jsonl" 2>>"$OUT/variants.err" || { echo "variant $so failed"; exit 1; }
    fi
  done
done
cat "$OUT/variants.jsonl"
[ "${SKIP_SUITE:-0}" = 1 ] || step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 600 python bench.py
echo done | tee -a "$OUT/status.txt"
