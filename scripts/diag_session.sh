#!/bin/bash
# Diagnostics of the fused kernel at the headline shape: per-phase stamps (diagnostic build
# build/ablate/libdadmm_stamps.so) and the two SQ counter groups of scripts/pmc.sh on the
# in-tree library (or the build/var variant named by LIBV, e.g. LIBV=sync). Each GPU step has
# its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-diag}
mkdir -p "$OUT"
export TMPDIR=/tmp
[ -n "${LIBV:-}" ] && export DADMM_LIB_VARIANT=$PWD/build/var/libdadmm_$LIBV.so
if [ -z "${LIBV:-}" ] && [ -f build/ablate/libdadmm_stamps.so ]; then
  timeout -k 10 120 python3 scripts/stamps.py > "$OUT/stamps.json" 2> "$OUT/stamps.err"
  rc=$?; echo "stamps rc=$rc"; cat "$OUT/stamps.json"; [ $rc -eq 0 ] || exit $rc
fi
i=0
for group in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" \
             "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
             "GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $group --output-format csv -d "$OUT/p$i" -o pmc -- \
      python3 scripts/prof_kernel.py ${SHAPE:-} > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.log"; exit $rc; }
done
echo done
