set -u
OUT=gpurun_out/${TAG:-s1}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_stream.log 2>&1
rc=$?; echo "stream tests rc=$rc"; tail -5 $OUT/pytest_stream.log
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -5 $OUT/pytest_parity.log
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
for f in 1 0 1 0; do DADMM_TILED_STREAM=$f timeout -k 10 120 python scripts/time_config.py 16 512 64 4096 25 0.3 1 auto >> $OUT/time.jsonl 2>>$OUT/time.err || exit $?; done
cat $OUT/time.jsonl
DADMM_TILED_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o kt -- python3 scripts/time_config.py 16 512 64 4096 25 0.3 1 auto > $OUT/prof.log 2>&1
echo "prof rc=$?"
