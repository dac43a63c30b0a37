#!/bin/bash
# Build an alternative libdadmm (timing experiments, scripts/time_variants.sh):
#   scripts/build_variant.sh NAME "EXTRA HIPCC FLAGS" [SOURCE=dadmm_fused.hip]
# recompiles SOURCE with the extra flags (the rest from the in-tree build objects) into
# build/var/libdadmm_NAME.so. Timing builds only; the product library is csrc/Makefile's.
set -eu
cd "$(dirname "$0")/.."
NAME=$1; EXTRA=${2:-}; SRC=${3:-dadmm_fused.hip}
C=hyperparameter-gnn_unfolded-d-admm-main_amd/csrc
make -s -C $C >/dev/null
mkdir -p build/var
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -mllvm -pragma-unroll-threshold=1000000 -Wall -Wno-unused-function"
/opt/rocm/bin/hipcc $FLAGS $EXTRA -x hip -c $C/$SRC -o build/var/${NAME}_$SRC.o
OBJS=""
for o in $C/build/*.o; do
  b=$(basename $o)
  [ "$b" = "$SRC.o" ] && continue
  OBJS="$OBJS $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS build/var/${NAME}_$SRC.o -o build/var/libdadmm_$NAME.so
echo build/var/libdadmm_$NAME.so
