#!/bin/bash
# Timing variants of the column-split forward (never shipped): libdadmm.so rebuilt with
# dadmm_split.hip compiled under -D<flags>, into build/svar/libdadmm_<name>.so; select one with
# DADMM_LIB_VARIANT=<path> (dadmm_hip/_lib.py). Usage: scripts/split_variants.sh name "-DFLAG=1" ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/hyperparameter-gnn_unfolded-d-admm-main_amd/csrc
OUT=$ROOT/build/svar
mkdir -p $OUT
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -mllvm -pragma-unroll-threshold=1000000"
OBJS=$(ls $C/build/*.o | grep -v dadmm_split.hip.o)
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  ( /opt/rocm/bin/hipcc $FLAGS $defs -x hip -c $C/dadmm_split.hip -o $OUT/split_$name.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS $OUT/split_$name.o -o $OUT/libdadmm_$name.so ) &
done
wait
