#!/bin/bash
# Round-4 session G: streamed-forward ablation matrix at configs[2] (DADMM_ST_ABL builds, wrong results
# by design, timing only): 0 base, 1 no walk, 2 no operator loads, 8 no stores, combinations.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
DADMM_ABLATION=1 TAG=r04g VARS="build/var/libdadmm_stabl0.so build/var/libdadmm_stabl1.so build/var/libdadmm_stabl2.so build/var/libdadmm_stabl3.so build/var/libdadmm_stabl8.so build/var/libdadmm_stabl11.so build/var/libdadmm_stabl27.so" \
  CFG="16 512 64 4096 25 0.3 1 tiled" ROUNDS=2 bash scripts/r04_variants.sh || exit $?
exit 0
