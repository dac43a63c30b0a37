#!/bin/bash
# A/B of the streamed forward's 8-wave (two agents per wave) and 16-wave (one agent per wave)
# forms at configs[2], interleaved, then the stream parity tests on the 16-wave form.
set -u
OUT=gpurun_out/${TAG:-wab}; mkdir -p $OUT
for r in 1 2; do for w in 8 16; do
  DADMM_STREAM_WAVES=$w timeout -k 10 120 python3 scripts/time_config.py 16 512 64 4096 25 0.3 1 tiled > $OUT/w$w.$r.json 2>$OUT/w$w.$r.err || exit $?
  echo "waves=$w $(cat $OUT/w$w.$r.json)"
done; done
DADMM_STREAM_WAVES=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > $OUT/tests16.log 2>&1; echo "tests16 rc=$?"; tail -2 $OUT/tests16.log
