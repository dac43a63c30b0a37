#!/bin/bash
# scripts/time_adjoint.py at the headline shape with every build/var/libdadmm_*.so, 3 rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2 3; do for so in build/var/libdadmm_*.so; do
  out=$(DADMM_LIB_VARIANT=$PWD/$so timeout -k 10 200 python3 scripts/time_adjoint.py 2>/dev/null | tail -1); rc=$?
  [ $rc -ne 0 ] && { echo "FAILED $so"; exit $rc; }
  echo "$(basename $so) $out"
done; done
