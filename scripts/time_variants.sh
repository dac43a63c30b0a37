#!/bin/bash
# Time every build/var/libdadmm_*.so on one config (scripts/time_config.py), two rounds,
# each run under its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for so in build/var/libdadmm_*.so; do
    DADMM_LIB_VARIANT=$PWD/$so timeout -k 10 180 python3 scripts/time_config.py ${CFG:-} >> gpurun_out/variants.jsonl
    rc=$?; [ $rc -ne 0 ] && { echo "FAILED $so rc=$rc"; exit $rc; }
  done
done
cat gpurun_out/variants.jsonl
