#!/bin/bash
# Stream-kernel GPU session: its parity tests, configs[2] timing (streamed vs per-iteration
# launches, interleaved), and PMC passes over the streamed launch. Each GPU step is time-limited;
# the first fatal status ends the script.
set -u
OUT=gpurun_out/${TAG:-s3}; mkdir -p $OUT
export TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_stream.log 2>&1
rc=$?; echo "stream tests rc=$rc"; tail -3 $OUT/pytest_stream.log; fatal $rc && exit $rc
for f in 1 0 1 0; do DADMM_TILED_STREAM=$f timeout -k 10 120 python scripts/time_config.py 16 512 64 4096 25 0.3 1 auto >> $OUT/time.jsonl 2>>$OUT/time.err || exit $?; done
cat $OUT/time.jsonl
[ "${PMC:-1}" = 0 ] && exit 0
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  DADMM_TILED_STREAM=1 timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $group --output-format csv -d "$OUT/p$i" -o pmc -- \
      python3 scripts/prof_config.py 16 512 64 4096 25 0.3 1 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($group) rc=$rc"; [ $rc -ne 0 ] && { tail -3 "$OUT/p$i.log"; exit $rc; }
done <<'GROUPS'
SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM
SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU
TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
GROUPS
echo done
