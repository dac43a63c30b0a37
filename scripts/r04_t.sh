#!/bin/bash
# Round-4 session T: single GCN layers of configs[4] in isolation (time_gcn_layer.py): gcn32_kernel,
# linear_kernel (DADMM_GCN32=0) and gcn32 with the mix ablated (timing only).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r04t
for cfg in "1024 50 400 400" "1024 50 200 400" "1024 50 100 200" "1024 50 1024 100"; do
  timeout -k 10 120 python3 scripts/time_gcn_layer.py $cfg >> gpurun_out/r04t/layers.txt || exit $?
  DADMM_GCN32=0 timeout -k 10 120 python3 scripts/time_gcn_layer.py $cfg >> gpurun_out/r04t/layers.txt || exit $?
  DADMM_LIB_VARIANT=$PWD/build/var/libdadmm_g32nomix.so timeout -k 10 120 python3 scripts/time_gcn_layer.py $cfg >> gpurun_out/r04t/layers.txt || exit $?
done
cat gpurun_out/r04t/layers.txt
exit 0
