#!/bin/bash
# Round-4 session P: streamed forward with the tile stores delayed behind the next tile's loads
# (DADMM_ST_DELAY) vs as before, configs[2] (time_config.py, checksums must agree).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=r04p VARS="build/var/libdadmm_st_d0.so build/var/libdadmm_st_d1.so" CFG="16 512 64 4096 25 0.3 1 tiled" ROUNDS=3 bash scripts/r04_variants.sh || exit $?
exit 0
