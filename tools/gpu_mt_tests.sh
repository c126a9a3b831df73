# GPU pass for the device MT19937 path: its tests, the streamed-codec tests, full-size Aggregator rates.
set -e
OUT=gpurun_out/${1:-mt}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_mt19937.py tests/test_stream_codecs.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 python -u -m pytest "tests/test_fullsize_parity.py::test_configs4_device_aggregator_other_codecs" \
  -x -q -s --timeout 300 --timeout-method thread > $OUT/fullsize.log 2>&1 || { tail -40 $OUT/fullsize.log; exit 1; }
grep "GB/s" $OUT/fullsize.log
tail -1 $OUT/fullsize.log
