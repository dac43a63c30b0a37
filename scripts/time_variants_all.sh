#!/bin/bash
# Time every build/var/libdadmm_*.so on one config (scripts/time_config.py), two interleaved
# rounds. A variant whose output check fails (rc 1: ablations compute wrong or nondeterministic
# results) is reported and skipped; a fatal status (timeout, abort, fault) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-variants}.jsonl
for r in 1 2; do
  for so in build/var/libdadmm_*.so; do
    DADMM_LIB_VARIANT=$PWD/$so timeout -k 10 180 python3 scripts/time_config.py ${CFG:-} >> $OUT 2>/dev/null
    rc=$?
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "FATAL $so rc=$rc"; exit $rc; fi
    [ $rc -ne 0 ] && echo "{\"lib\": \"$(basename $so)\", \"rc\": $rc}" >> $OUT
  done
done
cat $OUT
