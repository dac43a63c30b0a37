#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel trace only) over an arbitrary python script:
#   TAG=x scripts/pmc_cmd.sh scripts/time_adjoint.py 16 512 64 4096 25
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmccmd}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $group --output-format csv -d "$OUT/p$i" -o pmc -- \
      python3 "$@" > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($group) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done <<'GROUPS'
SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM
SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS
TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum
GROUPS
echo done
