#!/bin/bash
# A/B of the build/var/libdadmm_*.so variants on one config: ROUNDS interleaved timing rounds
# (scripts/time_config.py, HIP events, median of 10, output checksum) and, with PMC set, one
# rocprofv3 counter pass per variant (PMC = the counter list). Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-var}
mkdir -p "$OUT"
export TMPDIR=/tmp
SCRIPT=${SCRIPT:-scripts/time_config.py}
VARS=${VARS:-build/var/libdadmm_*.so}
for r in $(seq 1 ${ROUNDS:-3}); do
  for so in $VARS; do
    DADMM_LIB_VARIANT=$PWD/$so timeout -k 10 180 python3 $SCRIPT ${CFG:-} >> "$OUT/variants.jsonl"
    rc=$?; [ $rc -ne 0 ] && { echo "FAILED $so rc=$rc"; exit $rc; }
  done
done
cat "$OUT/variants.jsonl"
if [ -n "${PMC:-}" ]; then
  for so in $VARS; do
    name=$(basename $so .so)
    DADMM_LIB_VARIANT=$PWD/$so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $PMC --output-format csv \
        -d "$OUT/pmc_$name" -o pmc -- python3 $SCRIPT ${CFG:-} > "$OUT/pmc_$name.log" 2>&1
    rc=$?; echo "pmc $name rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/pmc_$name.log"; exit $rc; }
  done
fi
exit 0
