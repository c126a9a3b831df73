# Round-6: lone rand-k binning its candidates in the compaction (no k_resolve<true>) + the own
# pilot in k_fused_mag: parity subset, then the same-box A/B against the previous library.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_f64_boundary.py tests/test_stream_codecs.py -m gpu -x -q \
  -k "philox or rand or encode_decode or fused or concurrent" --timeout 120 --timeout-method thread > gpurun_out/r06_randbin_tests.log 2>&1 &&
tail -3 gpurun_out/r06_randbin_tests.log &&
timeout -k 10 900 python tools/ab.py --out gpurun_out/r06_ab_randbin.jsonl --reps 4 \
  --var base=tools/variants/lib_base.so --var new= \
  --probe "tools/randk_probe.py --n 16777216" --probe "tools/encdec_probe.py --n 16777216" > gpurun_out/r06_ab_randbin.log 2>&1
