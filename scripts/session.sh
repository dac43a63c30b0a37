#!/bin/bash
# One GPU session: each step under its own time limit, chained with &&; the first failure ends
# the session (no retries). Output under gpurun_out/$TAG/.
#   TAG=name STEPS="tests:<pytest args> | prologue | bench:<args> | prof:<bench args> | cmd:<shell>" bash scripts/session.sh
# (steps are split on "|": a cmd step must not contain one — chain with && instead)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:?TAG}
mkdir -p "$O"
IFS='|' read -ra ST <<< "${STEPS:?STEPS}"
i=0
for st in "${ST[@]}"; do
  st="$(echo "$st" | sed 's/^ *//;s/ *$//')"
  kind=${st%%:*}; arg=""; [[ "$st" == *:* ]] && arg=${st#*:}
  i=$((i + 1))
  case "$kind" in
    tests)    timeout -k 10 900 python -u -m pytest $arg -x -v --timeout 120 --timeout-method thread > "$O/tests_$i.txt" 2>&1 ;;
    prologue) for so in hyperparameter-gnn_unfolded-d-admm-main_amd/dadmm_hip/libdadmm.so build/var/libdadmm_rngold.so; do
                DADMM_LIB_VARIANT=$PWD/$so timeout -k 10 120 python -u scripts/time_prologue.py >> "$O/prologue_$i.txt" 2>&1 || exit $?
              done ;;
    bench)    timeout -k 10 600 python -u bench.py $arg > "$O/bench_$i.json" 2> "$O/bench_$i.err" ;;
    prof)     timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$i" -o run -- python3 bench.py $arg > "$O/prof_$i.out" 2>&1 ;;
    cmd)      timeout -k 10 600 bash -c "$arg" > "$O/cmd_$i.txt" 2>&1 ;;
    *)        echo "unknown step $kind"; exit 2 ;;
  esac
  rc=$?
  echo "step $i ($kind) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
