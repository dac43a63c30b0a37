# Round checkpoint: GPU suite, smoke, bench, kernel stats of the bench, HBM traffic passes.
set -o pipefail
O=gpurun_out/${TAG:-final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $O/prof.out 2>&1 || exit $?
python3 scripts/rocpd_stats.py $(ls $O/prof/*/run_results.db $O/prof/run_results.db 2>/dev/null | head -1) > $O/kernel_stats.csv || exit $?
rm -rf $O/prof   # the rocpd database is tens of MB; gpurun copies back at most 64 MiB
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 scripts/prof_kernel.py > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 scripts/prof_kernel.py > $O/pmc_write.log 2>&1 || exit $?
python3 scripts/traffic.py $O > $O/traffic.txt 2>&1 || exit $?
rm -rf $O/pmc_fetch $O/pmc_write
echo done > $O/done.txt
