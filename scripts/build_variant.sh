#!/bin/bash
# Build an alternative libdadmm (timing experiments, scripts/time_variants.sh):
#   scripts/build_variant.sh NAME "EXTRA HIPCC FLAGS" [SOURCE=dadmm_fused.hip]
# recompiles SOURCE with the extra flags (the rest from the in-tree build objects) into
# build/var/libdadmm_NAME.so. Timing builds only; the product library is csrc/Makefile's.
# SOURCE may be a path under csrc/ (e.g. var/dadmm_gnn.hip, an older copy): the in-tree object of
# the same file name is the one replaced.
set -eu
cd "$(dirname "$0")/.."
NAME=$1; EXTRA=${2:-}; SRC=${3:-dadmm_fused.hip}
C=hyperparameter-gnn_unfolded-d-admm-main_amd/csrc
make -s -C $C >/dev/null
mkdir -p build/var
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -mllvm -pragma-unroll-threshold=1000000 -Wall -Wno-unused-function"
BASE=$(basename $SRC)
/opt/rocm/bin/hipcc $FLAGS $EXTRA -I$C -x hip -c $C/$SRC -o build/var/${NAME}_$BASE.o
OBJS=""
for o in $C/build/*.o; do
  b=$(basename $o)
  [ "$b" = "$BASE.o" ] && continue
  OBJS="$OBJS $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS build/var/${NAME}_$BASE.o -o build/var/libdadmm_$NAME.so
echo build/var/libdadmm_$NAME.so
