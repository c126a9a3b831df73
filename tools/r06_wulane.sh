# Round-6 A/B: the compaction's slot-offset readlane with a wave-uniform index.
set -o pipefail
mkdir -p gpurun_out
cp tools/variants/lib_wulane.so openmsftl_amd/libfedcodec.so &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -x -q \
  -k "encode_decode or single_client or dense or batch or configs2 or philox or mask or dropout" --timeout 300 --timeout-method thread > gpurun_out/r06_wulane_tests.log 2>&1 &&
tail -2 gpurun_out/r06_wulane_tests.log &&
timeout -k 10 1000 python tools/ab.py --out gpurun_out/r06_ab_wulane.jsonl --reps 3 \
  --var base=tools/variants/lib_final.so --var wulane=tools/variants/lib_wulane.so \
  --probe "tools/c2_probe.py --steps 100" --probe "tools/encdec_probe.py --n 134217728" \
  --probe "tools/randk_probe.py --n 16777216" \
  --probe "bench.py --steps 40 --no-cpu-baseline --no-single --no-matrix" > gpurun_out/r06_ab_wulane.log 2>&1
