#!/bin/bash
# bench.py (headline only) with every build/var/libdadmm_*.so, interleaved rounds; one JSON line each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for so in build/var/libdadmm_*.so; do
    out=$(DADMM_LIB_VARIANT=$PWD/$so timeout -k 10 240 python3 bench.py --steps 50 --warmup 10 --no-extras --no-cpu-baseline 2>/dev/null | tail -1)
    rc=$?; [ $rc -ne 0 ] && { echo "FAILED $so rc=$rc"; exit $rc; }
    echo "$(basename $so) $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["kernel_ms"],4), round(d["ms_per_step"],4), round(d["value"]/1e6,1))')" | tee -a gpurun_out/bench_variants.txt
  done
done
